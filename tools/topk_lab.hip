// Block-max top-k lab (development tool, not part of the product ABI).
// Includes the product source; exports lab_topk_bmax(), which runs the
// production block maxima (block_max_kernel) and then one of:
//   variant 0: an instrumented copy of topk_bmax_kernel (the production
//              select) that records s_memrealtime (100 MHz) at its phase
//              boundaries -- start, keys in LDS, radix pass 0, pass 1,
//              qualifying blocks, gather, ranked + written -- per row;
//   variant 2: the production topk_bmax (round 4: radix over the superblock
//              keys block_max_kernel also writes; no stamps);
//   variant 1: the same as 0 with the radix passes over 256-doc superblock keys
//              (the max of 4 block keys, 4x fewer keys in the atomics): the
//              kk-th largest superblock key t' bounds the kk-th score from
//              below as well, and every doc >= t' lies in a 64-doc block
//              whose key is >= t', so qualifying 64-doc blocks and the gather
//              are unchanged in kind (t' <= t: a few more of them).
// Both write the production's exact result (same keys, same tie rule).
#define CBV2_LAB 1
#include "../hybrid-rag-colbertv2_amd/csrc/colbert_mi355x.hip"

namespace {

template <int SUPER>
__global__ __launch_bounds__(kTkThreads) void topk_bmax_lab_kernel(const float* __restrict__ scores, int64_t n,
                                                                   int64_t ld, int k, int64_t id_base,
                                                                   const uint32_t* __restrict__ bm, int64_t bm_ld,
                                                                   float* __restrict__ out_s,
                                                                   int32_t* __restrict__ out_i,
                                                                   uint64_t* __restrict__ stamps) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bm_dyn[];
  uint64_t* const sel = reinterpret_cast<uint64_t*>(bm_dyn);
  uint32_t* const hist = reinterpret_cast<uint32_t*>(sel + kBmCand);
  uint32_t* const qual = hist + 2048;
  uint32_t* const misc = qual + kBmQual;
  uint32_t* const keys = misc + 16;
  const int tid = threadIdx.x, nth = blockDim.x, wave = tid >> 6;
  const int row = blockIdx.x;
  uint64_t st[8];
  st[0] = __builtin_amdgcn_s_memrealtime();
  const int nb = (int)((n + 63) >> 6);
  const int ns = (nb + SUPER - 1) / SUPER;   // radix keys (superblocks of SUPER blocks)
  const float* x = scores + (size_t)row * ld;
  const uint32_t* brow = bm + (size_t)row * bm_ld;
  const int kk = (int)((int64_t)k < n ? k : n);
  for (int i = tid; i < nb; i += nth) keys[i] = brow[i];
  if (tid < 16) misc[tid] = 0;
  __syncthreads();
  uint32_t* skeys = keys + nb;   // superblock keys (SUPER > 1)
  if (SUPER > 1) {
    for (int i = tid; i < ns; i += nth) {
      uint32_t m = 0;
      for (int j = 0; j < SUPER && i * SUPER + j < nb; ++j) m = max(m, keys[i * SUPER + j]);
      skeys[i] = m;
    }
    __syncthreads();
  }
  const uint32_t* rk = SUPER > 1 ? skeys : keys;
  st[1] = __builtin_amdgcn_s_memrealtime();
  uint32_t prefix = 0, mask = 0, kleft = (uint32_t)(kk < ns ? kk : ns);
  for (int p = 0; p < 2; ++p) {
    const int shift = 21 - 11 * p;
    for (int b = tid; b < 2048; b += nth) hist[b] = 0;
    __syncthreads();
    for (int i = tid; i < ns; i += nth) {
      const uint32_t u = rk[i];
      hist_add(hist, (u >> shift) & 2047u, (u & mask) == prefix);
    }
    __syncthreads();
    if (wave == 0) find_bin(hist, 2048, kleft, &misc[4], &misc[5], &misc[6]);
    __syncthreads();
    kleft -= misc[5];
    prefix |= misc[4] << shift;
    mask |= 2047u << shift;
    __syncthreads();
    st[2 + p] = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t t = prefix;
  for (int i = tid; i < nb; i += nth)
    if (keys[i] >= t) {
      const uint32_t pos = atomicAdd(&misc[0], 1u);
      if (pos < (uint32_t)kBmQual) qual[pos] = (uint32_t)i;
    }
  __syncthreads();
  st[4] = __builtin_amdgcn_s_memrealtime();
  const uint32_t nqual = misc[0];
  if (nqual <= (uint32_t)kBmQual) {
    constexpr int U = 4;
    const uint32_t total = nqual * 64;
    for (uint32_t w0 = tid; w0 < total; w0 += (uint32_t)nth * U) {
      float v[U];
      int64_t idx[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t w = w0 + (uint32_t)(u * nth);
        idx[u] = w < total ? (int64_t)qual[w >> 6] * 64 + (w & 63) : n;
        v[u] = idx[u] < n ? x[idx[u]] : neg_inf();
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (idx[u] < n && f2u(v[u]) >= t) {
          const uint32_t pos = atomicAdd(&misc[1], 1u);
          if (pos < (uint32_t)kBmCand) sel[pos] = rank_key(v[u], (uint32_t)idx[u]);
        }
    }
  }
  __syncthreads();
  st[5] = __builtin_amdgcn_s_memrealtime();
  const uint32_t ncand = misc[1];
  int m = (int)ncand;
  if (nqual > (uint32_t)kBmQual || ncand < (uint32_t)kk || ncand > (uint32_t)kBmCand) {
    __syncthreads();
    topk_exact_row(x, n, kk, sel, hist, &misc[4], &misc[5], &misc[6], &misc[7]);
    m = kk;
  }
  float* os = out_s + (size_t)row * k;
  int32_t* oi = out_i + (size_t)row * k;
  if (m <= kBmRankMax) {
    for (int i = tid; i < m; i += nth) {
      const uint64_t key = sel[i];
      int r = 0;
      for (int j = 0; j < m; ++j) r += sel[j] > key ? 1 : 0;
      if (r < k) {
        os[r] = u2f((uint32_t)(key >> 32));
        oi[r] = (int32_t)(id_base + (int64_t)(~(uint32_t)key));
      }
    }
    for (int j = m + tid; j < k; j += nth) {
      os[j] = neg_inf();
      oi[j] = -1;
    }
  } else {
    sort_and_write(sel, m, k, id_base, os, oi);
  }
  __syncthreads();
  st[6] = __builtin_amdgcn_s_memrealtime();
  st[7] = ((uint64_t)nqual << 32) | ncand;
  if (tid < 8) stamps[(size_t)row * 8 + tid] = st[tid];
}

}  // namespace

extern "C" int lab_topk_bmax(const float* scores, int32_t B, int64_t n, int32_t k, uint32_t* bm, float* out_s,
                             int32_t* out_i, uint64_t* stamps, int32_t variant, void* stream) {
  const hipStream_t st = (hipStream_t)stream;
  const int64_t nb = bm_blocks(n);
  if (variant == 2) {   // the production path: block + superblock maxima, superblock-key select
    int dev = 0;
    (void)hipGetDevice(&dev);
    return topk_bmax(scores, B, n, n, k, 0, bm, out_s, out_i, st, dev);
  }
  hipLaunchKernelGGL(block_max_kernel, dim3((unsigned)((nb + kBmBlocksPerWg - 1) / kBmBlocksPerWg), (unsigned)B),
                     dim3(256), 0, st, scores, n, n, bm, nb, bm_super_keys(bm, B, n), bm_supers(n));
  const size_t lds = kBmFixedLds + (size_t)nb * 4 + (variant == 1 ? (size_t)(nb + 3) / 4 * 4 : 0);
  auto kern = variant == 1 ? topk_bmax_lab_kernel<4> : topk_bmax_lab_kernel<1>;
  if (hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -3;
  hipLaunchKernelGGL(kern, dim3((unsigned)B), dim3(kTkThreads), lds, st, scores, n, n, k, (int64_t)0, bm, nb, out_s,
                     out_i, stamps);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
