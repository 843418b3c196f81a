// Probe 3: random e4m3 values, checks which value classes / scale ranges the
// host model of v_mfma_scale_f32_16x16x128_f8f6f4 gets right (dev tool).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void run(const uint8_t* imgA, const uint8_t* imgB, const int* scA, const int* scB, float* out) {
  const int l = threadIdx.x;
  i32x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = ((const int*)(imgA + l * 32))[j]; b[j] = ((const int*)(imgB + l * 32))[j]; }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, scA[l], 0, scB[l]);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];
}
static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float x = e == 0 ? (m / 8.0f) * std::ldexp(1.0f, -6) : (1.0f + m / 8.0f) * std::ldexp(1.0f, e - 7);
  return s ? -x : x;
}
int main() {
  uint8_t *dA, *dB; int *dsA, *dsB; float* dO;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsA, 256); hipMalloc(&dsB, 256); hipMalloc(&dO, 1024);
  for (int mode = 0; mode < 6; ++mode) {
    uint8_t A[2048], B[2048]; int sA[64], sB[64]; float O[256];
    srand(mode + 1);
    for (int i = 0; i < 2048; ++i) {
      int lo = mode == 1 ? 0x08 : 0, hi = (mode == 2) ? 0x40 : 0x70;   // 1: no subnormals; 2: small exponents
      A[i] = (rand() % 2 ? 0x80 : 0) | (lo + rand() % (hi - lo));
      B[i] = (rand() % 2 ? 0x80 : 0) | (lo + rand() % (hi - lo));
      if (mode == 5) { A[i] &= 0x7f; B[i] &= 0x7f; }                     // 5: positive only
    }
    for (int l = 0; l < 64; ++l) {
      sA[l] = mode >= 3 ? 125 + rand() % 5 : 127;
      sB[l] = mode == 4 ? 127 : (mode >= 3 ? 125 + rand() % 5 : 127);
    }
    hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
    hipMemcpy(dsA, sA, 256, hipMemcpyHostToDevice); hipMemcpy(dsB, sB, 256, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dB, dsA, dsB, dO);
    hipMemcpy(O, dO, 1024, hipMemcpyDeviceToHost);
    double maxerr = 0, maxref = 0; int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 4; ++r) {
        int row = 4 * (l >> 4) + r, col = l & 15;
        double ref = 0;
        for (int k = 0; k < 128; ++k) {
          int la = row + 16 * (k / 32), lb = col + 16 * (k / 32);
          ref += (double)e4m3(A[la * 32 + k % 32]) * std::ldexp(1.0, sA[la] - 127) *
                 (double)e4m3(B[lb * 32 + k % 32]) * std::ldexp(1.0, sB[lb] - 127);
        }
        double e = fabs(ref - O[l * 4 + r]);
        if (e > 1e-5 * fabs(ref) + 1e-9) bad++;
        maxerr = fmax(maxerr, e); maxref = fmax(maxref, fabs(ref));
      }
    printf("mode %d: max|ref| %.6g max|err| %.6g bad %d/256\n", mode, maxref, maxerr, bad);
  }
  return 0;
}
