// alloc_probe — does the B=1 streaming scan's rate depend on how its index
// memory was allocated?  Several 1M-doc bf16 token buffers (32.8 GB each) from
// hipMalloc and from hipExtMallocWithFlags(hipDeviceMallocContiguous), each
// scanned through its own cbv2_index (cbv2_score, B = 1) with the scan timed
// by the library's own events (cbv2_index_time_scans).  Values are a fixed
// pattern (the scan's time does not depend on them).  One line per buffer:
// mode, virtual address, median scan ms over 3 x 10 launches.
//   build: hipcc -O2 -I include tools/probes/alloc_probe.cpp
//          hybrid-rag-colbertv2_amd/libcolbert_mi355x.so -Wl,-rpath,... -o tools/_build/alloc_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "colbert_mi355x.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                              \
    }                                                                            \
  } while (0)

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? std::atoll(argv[1]) : 1000000;
  const std::string modes = argc > 2 ? argv[2] : "mmmcc";   // m = hipMalloc, c = contiguous
  const size_t bytes = (size_t)n * 128 * 128 * 2;
  int32_t* dl = nullptr;
  uint16_t* Q = nullptr;
  float* out = nullptr;
  CK(hipMalloc(&dl, n * 4));
  CK(hipMalloc(&Q, 32 * 128 * 2));
  CK(hipMalloc(&out, n * 4));
  std::vector<int32_t> h(n, 128);
  CK(hipMemcpy(dl, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemsetD16((hipDeviceptr_t)Q, 0x3c00, 32 * 128));
  struct Buf {
    char mode;
    void* p;
  };
  std::vector<Buf> bufs;
  for (char m : modes) {
    void* p = nullptr;
    hipError_t e = m == 'c' ? hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) : hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      std::printf("{\"mode\": \"%c\", \"error\": \"%s\"}\n", m, hipGetErrorString(e));
      (void)hipGetLastError();
      continue;
    }
    CK(hipMemsetD16((hipDeviceptr_t)p, 0x3b80, bytes / 2));
    bufs.push_back({m, p});
  }
  CK(hipDeviceSynchronize());
  for (int round = 0; round < 3; ++round) {
    for (auto& b : bufs) {
      cbv2_index* ix = nullptr;
      if (cbv2_index_create(0, b.p, CBV2_DTYPE_BF16, n, 128, 128, dl, 0, &ix)) {
        std::printf("create: %s\n", cbv2_last_error());
        return 1;
      }
      cbv2_score(ix, CBV2_SCORER_MAXSIM, Q, CBV2_DTYPE_BF16, 1, 32, out, n, nullptr);   // warm
      cbv2_index_time_scans(ix, 1);
      for (int i = 0; i < 10; ++i) cbv2_score(ix, CBV2_SCORER_MAXSIM, Q, CBV2_DTYPE_BF16, 1, 32, out, n, nullptr);
      cbv2_index_time_scans(ix, 0);
      float ms[16];
      int32_t cnt = 0;
      cbv2_index_scan_times(ix, ms, 16, &cnt);
      std::sort(ms, ms + cnt);
      std::printf("{\"round\": %d, \"mode\": \"%s\", \"ptr\": \"%p\", \"scan_ms_median\": %.4f, \"min\": %.4f}\n", round,
                  b.mode == 'c' ? "contiguous" : "hipMalloc", b.p, ms[cnt / 2], ms[0]);
      std::fflush(stdout);
      cbv2_index_destroy(ix);
    }
  }
  for (auto& b : bufs) CK(hipFree(b.p));
  return 0;
}
