// Diagnostic probe for v_mfma_scale_f32_16x16x128_f8f6f4 layouts (dev tool).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstdlib>
#include <cstring>

typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// img: per-lane 32-byte register images for A and B; scales: per-lane int
__global__ void run(const uint8_t* imgA, const uint8_t* imgB, const int* scA, const int* scB, float* out) {
  const int l = threadIdx.x;
  i32x8 a, b;
  const int* pa = (const int*)(imgA + l * 32);
  const int* pb = (const int*)(imgB + l * 32);
  for (int j = 0; j < 8; ++j) { a[j] = pa[j]; b[j] = pb[j]; }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, scA[l], 0, scB[l]);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = acc[r];  // raw per-lane accumulator
}

static uint8_t *dA, *dB; static int *dsA, *dsB; static float* dO;
static void go(const uint8_t* A, const uint8_t* B, const int* sA, const int* sB, float* O) {
  hipMemcpy(dA, A, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, B, 2048, hipMemcpyHostToDevice);
  hipMemcpy(dsA, sA, 256, hipMemcpyHostToDevice); hipMemcpy(dsB, sB, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, dA, dB, dsA, dsB, dO);
  hipMemcpy(O, dO, 1024, hipMemcpyDeviceToHost);
}

int main() {
  hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dsA, 256); hipMalloc(&dsB, 256); hipMalloc(&dO, 1024);
  uint8_t A[2048], B[2048]; int sA[64], sB[64]; float O[256];
  for (int l = 0; l < 64; ++l) sA[l] = sB[l] = 127;
  // 1. B all ones; one-hot A byte (lane l, byte j) -> which output (row, col) light up
  memset(B, 0x38, sizeof B);
  printf("A one-hot -> output rows (C layout assumed col=lane&15,row=4*(lane>>4)+reg):\n");
  for (int l : {0, 1, 15, 16, 17, 32, 48, 63})
    for (int j : {0, 1, 7, 8, 15, 16, 31}) {
      memset(A, 0, sizeof A); A[l * 32 + j] = 0x38;
      go(A, B, sA, sB, O);
      int rows = 0, cnt = 0; float v = 0;
      for (int ol = 0; ol < 64; ++ol) for (int r = 0; r < 4; ++r) if (O[ol * 4 + r] != 0) { rows |= 1 << (4 * (ol >> 4) + r); cnt++; v = O[ol*4+r]; }
      printf("  A lane %2d byte %2d: rows mask %05x nonzero %d val %g\n", l, j, rows, cnt, v);
    }
  // 2. A all ones; one-hot B byte -> which columns
  memset(A, 0x38, sizeof A);
  printf("B one-hot -> output cols:\n");
  for (int l : {0, 1, 15, 16, 32, 63})
    for (int j : {0, 16, 31}) {
      memset(B, 0, sizeof B); B[l * 32 + j] = 0x38;
      go(A, B, sA, sB, O);
      int cols = 0, cnt = 0;
      for (int ol = 0; ol < 64; ++ol) for (int r = 0; r < 4; ++r) if (O[ol * 4 + r] != 0) { cols |= 1 << (ol & 15); cnt++; }
      printf("  B lane %2d byte %2d: cols mask %04x nonzero %d\n", l, j, cols, cnt);
    }
  // 3. k pairing: A one-hot (lane la, byte ja) x B one-hot (lane lb, byte jb): nonzero iff same k
  printf("k pairing (A lane0 byte j vs B lane l byte j2):\n");
  for (int ja : {0, 1, 8, 16, 31}) {
    memset(A, 0, sizeof A); A[0 * 32 + ja] = 0x38;
    int found = 0;
    for (int lb = 0; lb < 64 && !found; lb += 16)
      for (int jb = 0; jb < 32 && !found; ++jb) {
        memset(B, 0, sizeof B); B[lb * 32 + jb] = 0x38;
        go(A, B, sA, sB, O);
        float s = 0; for (int i = 0; i < 256; ++i) s += fabsf(O[i]);
        if (s != 0) { printf("  A(l0,b%d) pairs with B(l%d,b%d)\n", ja, lb, jb); found = 1; }
      }
    if (!found) printf("  A(l0,b%d): no partner among B lanes {0,16,32,48}\n", ja);
  }
  // 4. scales: A all ones, B all ones, vary one lane's scale
  memset(A, 0x38, sizeof A); memset(B, 0x38, sizeof B);
  go(A, B, sA, sB, O);
  printf("all ones, unit scales: out[0]=%g (expect 128)\n", O[0]);
  for (int l : {0, 1, 16, 17, 48}) {
    for (int i = 0; i < 64; ++i) sA[i] = 127;
    sA[l] = 128;
    go(A, B, sA, sB, O);
    int rows = 0; for (int ol = 0; ol < 64; ++ol) for (int r = 0; r < 4; ++r) if (O[ol*4+r] != 128.0f) rows |= 1 << (4*(ol>>4)+r);
    printf("  scaleA lane %2d = 2: changed rows mask %05x out[0]=%g\n", l, rows, O[0]);
  }
  return 0;
}
