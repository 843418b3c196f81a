// Block-max top-k lab (development tool, not part of the product ABI).
// Includes the product source and runs the production one-launch block-max
// top-k (bmax_topk_kernel, the B <= 8 latency path) with its lab stamps on:
// s_memrealtime (100 MHz) at every workgroup's start, at the row's last
// arrival and at the select's phase ends (topk_bmax_row: keys in LDS,
// threshold, qualifying blocks, gather, ranked + written).  One row's stamps
// (row 0), so run it at B = 1.
#define CBV2_LAB 1
#include "../hybrid-rag-colbertv2_amd/csrc/colbert_mi355x.hip"

// stamps: [16 + 2 grid.x] u64; done: B zeroed ints (re-zeroed by the kernel)
extern "C" int lab_bmax_topk(const float* scores, int32_t B, int64_t n, int32_t k, uint32_t* bm, float* out_s,
                             int32_t* out_i, int32_t* done, uint64_t* stamps, void* stream) {
  const hipStream_t st = (hipStream_t)stream;
  const int64_t nb = bm_blocks(n), ns = bm_supers(n);
  const int lds_max = (int)(kBmFixedLds + (size_t)kBmMaxBlocks * 4);
  if (hipFuncSetAttribute((const void*)bmax_topk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max) !=
      hipSuccess)
    return -3;
  const size_t lds = bm_select_lds(n, k);
  hipLaunchKernelGGL(bmax_topk_kernel, dim3((unsigned)((nb + kBmFusedBlocksPerWg - 1) / kBmFusedBlocksPerWg),
                                             (unsigned)B),
                     dim3(kTkThreads), lds, st, scores, n, n, k, (int64_t)0, bm, nb, bm_super_keys(bm, B, n), ns,
                     done, (int64_t)1, out_s, out_i, Mirror(), stamps);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
extern "C" int lab_bmax_grid(int64_t n) { return (int)((bm_blocks(n) + kBmFusedBlocksPerWg - 1) / kBmFusedBlocksPerWg); }
