// Probe: streaming read bandwidth of one MI355X over a 32 GiB buffer (the
// bytes of a 1M-doc bf16 index), three ways, to size the B=1 scan's ceiling:
//   vgpr  : every wave streams its own contiguous range with global_load_dwordx4
//           into VGPRs, U loads in flight per lane (the direct scan's pattern);
//   lds   : every wave streams its range with global_load_lds_dwordx4 (1 KiB per
//           instruction) into a private LDS ring of S slots, vmcnt-throttled;
//   ldsr  : as lds, and the wave also reads each landed KiB back from LDS
//           (ds_read_b128: the scan's A-fragment reads).
// "nt" rows: the same with the non-temporal cache policy (nt loads; aux = 2
// on the LDS-DMA), the streaming hint for bytes read once.
// Grid = CUs x WPC waves (256-thread workgroups).  Development tool
// (tools/probes/), not product.  usage: bw_probe [GiB]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

#define CHECK(x)                                                                      \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

template <int U, bool NT = false>
__global__ __launch_bounds__(256) void vgpr_stream(const uint8_t* __restrict__ buf, size_t per_wave,
                                                   unsigned* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint8_t* base = buf + w * per_wave;
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (size_t off = 0; off < per_wave; off += (size_t)U * 1024) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const u32x4* p = reinterpret_cast<const u32x4*>(base + off + u * 1024 + lane * 16);
      v[u] = NT ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  const unsigned r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (r == 0x12345678u) sink[w] = r;   // practically never: keeps the loads live
}

// S slots of 1 KiB per wave; vmcnt(S-1) keeps S-1 pieces in flight.
template <int S, bool READ, int AUX = 0>
__global__ __launch_bounds__(256) void lds_stream(const uint8_t* __restrict__ buf, size_t per_wave,
                                                  unsigned* __restrict__ sink) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[4 * S * 1024];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const size_t w = (size_t)blockIdx.x * 4 + wave;
  const uint8_t* base = buf + w * per_wave;
  uint8_t* ring = smem + wave * S * 1024;
  u32x4 acc = {0u, 0u, 0u, 0u};
  const size_t n = per_wave / 1024;
  for (size_t i = 0; i < n; ++i) {
    const int slot = (int)(i % S);
    __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + i * 1024 + lane * 16),
                                     (lds_void_t*)(ring + slot * 1024), 16, 0, AUX);
    if (i + 1 >= (size_t)S) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(S - 1) : "memory");
      if (READ) acc ^= *reinterpret_cast<const u32x4*>(ring + ((i + 1) % S) * 1024 + lane * 16);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned r = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  if (r == 0x12345678u) sink[w] = r;
}

template <typename K>
float time_it(K kern, int grid, const uint8_t* buf, size_t per_wave, unsigned* sink) {
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, per_wave, sink);   // warm
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHECK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, buf, per_wave, sink);
    CHECK(hipEventRecord(b, 0));
    CHECK(hipEventSynchronize(b));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  return best;
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 30.0;
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  size_t bytes = (size_t)(gib * (1ull << 30));
  uint8_t* buf;
  unsigned* sink;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&sink, 1 << 24));
  CHECK(hipMemset(buf, 1, bytes));
  printf("buffer %.1f GiB, %d CUs\n", gib, cus);
  for (int wpc : {4, 8, 16}) {
    const int grid = cus * wpc / 4;
    const size_t waves = (size_t)grid * 4;
    const size_t per_wave = (bytes / waves) & ~(size_t)(16 * 1024 - 1);
    const double moved = (double)per_wave * waves;
    auto rep = [&](const char* what, float ms) {
      printf("waves/CU %2d  %-14s %8.3f ms  %7.1f GB/s\n", wpc, what, ms, moved / ms / 1e6);
    };
    rep("vgpr U=4", time_it(vgpr_stream<4>, grid, buf, per_wave, sink));
    rep("vgpr U=8", time_it(vgpr_stream<8>, grid, buf, per_wave, sink));
    rep("vgpr U=16", time_it(vgpr_stream<16>, grid, buf, per_wave, sink));
    rep("vgpr U=8 nt", time_it(vgpr_stream<8, true>, grid, buf, per_wave, sink));
    rep("vgpr U=16 nt", time_it(vgpr_stream<16, true>, grid, buf, per_wave, sink));
    if (wpc <= 8) {
      rep("lds S=8", time_it(lds_stream<8, false>, grid, buf, per_wave, sink));
      rep("lds S=16", time_it(lds_stream<16, false>, grid, buf, per_wave, sink));
      rep("lds S=32", time_it(lds_stream<32, false>, grid, buf, per_wave, sink));
      rep("ldsr S=16", time_it(lds_stream<16, true>, grid, buf, per_wave, sink));
      rep("lds S=16 nt", time_it(lds_stream<16, false, 2>, grid, buf, per_wave, sink));
      rep("lds S=32 nt", time_it(lds_stream<32, false, 2>, grid, buf, per_wave, sink));
    }
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(sink));
  return 0;
}
