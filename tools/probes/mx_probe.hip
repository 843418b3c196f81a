// Probe: operand / scale / output layout of v_mfma_scale_f32_16x16x128_f8f6f4
// (e4m3 x e4m3, E8M0 block scales) on gfx950, checked against a host model with
// exactly representable data.  Development tool (tools/probes/), not product.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

__global__ void probe(const uint8_t* A, const uint8_t* Bt, const uint8_t* sA, const uint8_t* sB, float* C) {
  const int l = threadIdx.x, c = l & 15, g = l >> 4;
  i32x8 a, b;
  const int* pa = (const int*)(A + c * 128 + 32 * g);
  const int* pb = (const int*)(Bt + c * 128 + 32 * g);
  for (int j = 0; j < 8; ++j) { a[j] = pa[j]; b[j] = pb[j]; }
  const int scale_a = sA[c * 4 + g];  // byte 0 (opsel 0)
  const int scale_b = sB[c * 4 + g];
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, scale_a, 0, scale_b);
  for (int r = 0; r < 4; ++r) C[(4 * g + r) * 16 + c] = acc[r];
}

static float e4m3(uint8_t v) {
  int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float x = e == 0 ? (m / 8.0f) * std::ldexp(1.0f, -6) : (1.0f + m / 8.0f) * std::ldexp(1.0f, e - 7);
  return s ? -x : x;
}

int main() {
  uint8_t A[16 * 128], Bt[16 * 128], sA[64], sB[64];
  srand(7);
  for (int i = 0; i < 16 * 128; ++i) { A[i] = (rand() % 2 ? 0x80 : 0) | (rand() % 0x70); Bt[i] = (rand() % 2 ? 0x80 : 0) | (rand() % 0x70); }
  for (int i = 0; i < 64; ++i) { sA[i] = 125 + rand() % 5; sB[i] = 125 + rand() % 5; }
  uint8_t *dA, *dB, *dsA, *dsB; float* dC;
  hipMalloc(&dA, sizeof A); hipMalloc(&dB, sizeof Bt); hipMalloc(&dsA, 64); hipMalloc(&dsB, 64); hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(dB, Bt, sizeof Bt, hipMemcpyHostToDevice);
  hipMemcpy(dsA, sA, 64, hipMemcpyHostToDevice); hipMemcpy(dsB, sB, 64, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dsA, dsB, dC);
  float C[256];
  hipMemcpy(C, dC, sizeof C, hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double ref = 0;
      for (int k = 0; k < 128; ++k)
        ref += (double)e4m3(A[r * 128 + k]) * std::ldexp(1.0, sA[r * 4 + k / 32] - 127) *
               (double)e4m3(Bt[c * 128 + k]) * std::ldexp(1.0, sB[c * 4 + k / 32] - 127);
      maxerr = fmax(maxerr, fabs(ref - C[r * 16 + c]));
      maxref = fmax(maxref, fabs(ref));
    }
  printf("mx_probe: max|ref| %.6g  max|err| %.6g  -> %s\n", maxref, maxerr, maxerr <= 1e-6 * maxref ? "LAYOUT OK" : "MISMATCH");
  return maxerr <= 1e-6 * maxref ? 0 : 1;
}
