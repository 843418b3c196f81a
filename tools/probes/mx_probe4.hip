// Probe 4: which lane's scale byte scales A[row][k-block] (dev tool).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
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
int main() {
  uint8_t *dA, *dB; int *dsA, *dsB; float* dO;
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsA, 256); hipMalloc(&dsB, 256); hipMalloc(&dO, 1024);
  uint8_t A[2048], B[2048]; int sA[64], sB[64]; float O[256];
  memset(B, 0x38, sizeof B);
  for (int which = 0; which < 2; ++which) {
    printf(which == 0 ? "scale_a mapping:\n" : "scale_b mapping:\n");
    for (int lane_data : {0, 16, 32, 48, 1, 17, 33, 49, 5, 53, 15, 63}) {   // data lane: row/col = lane&15, block = lane>>4
      memset(A, 0, sizeof A);
      uint8_t* D = which == 0 ? A : B;
      if (which == 1) { memset(A, 0x38, sizeof A); memset(B, 0, sizeof B); }
      D[lane_data * 32 + 3] = 0x38;                          // one element = 1.0
      int hits[256], nh = 0;
      for (int L = 0; L < 64; ++L)
        for (int byte = 0; byte < 4; ++byte) {
          for (int i = 0; i < 64; ++i) sA[i] = sB[i] = 0x7F7F7F7F;
          int* S = which == 0 ? sA : sB;
          S[L] = (int)((0x7F7F7F7Fu & ~(0xFFu << (8 * byte))) | (128u << (8 * byte)));
          hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
          hipMemcpy(dsA, sA, 256, hipMemcpyHostToDevice); hipMemcpy(dsB, sB, 256, hipMemcpyHostToDevice);
          hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dB, dsA, dsB, dO);
          hipMemcpy(O, dO, 1024, hipMemcpyDeviceToHost);
          float mx = 0; for (int i = 0; i < 256; ++i) mx = O[i] > mx ? O[i] : mx;
          if (mx == 2.0f) hits[nh++] = L * 4 + byte;
        }
      printf("  data lane %2d (row/col %2d, block %d) scaled by (lane,byte):", lane_data, lane_data & 15, lane_data >> 4);
      for (int i = 0; i < nh; ++i) printf(" (%d,%d)", hits[i] / 4, hits[i] % 4);
      printf("\n");
    }
  }
  return 0;
}
