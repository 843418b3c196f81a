// colbert_mi355x.hip — MI355X (gfx950 / CDNA4) kernels + C ABI for the ColBERT
// late-interaction retrieval path.  See include/colbert_mi355x.h for the
// contract and DESIGN.md for the roofline of each kernel.
//
// Kernels
//   maxsim_scan_kernel   S[b,i] = sum_{q<lq} max_{t<len_i} <Q[b,q], D_i[t]>  (bf16 MFMA,
//                        fp32 accumulate).  Replaces _maxsim_score (local_rag_complete.py:802-831)
//                        in its north-star (true MaxSim) form.  Query-stationary: each
//                        workgroup keeps 16 queries' fragments in VGPRs and streams a
//                        contiguous doc chunk HBM -> LDS (global_load_lds, XOR-swizzled,
//                        double-buffered); every doc tile is read once per workgroup.
//   topk_rows_kernel     torch.topk (local_rag_complete.py:767): exact radix select on
//                        order-preserving score bits, ties by lower doc index, bitonic sort.
//   rerank_kernel        rerank (local_rag_complete.py:779-800) on precomputed tiles:
//                        gather candidate docs by id straight into VGPRs, MaxSim, rank.
//   select_small_kernel  argsort + [:k] (local_rag_complete.py:789-792) of a short row.
//   merge_topk_kernel    cross-shard merge of sorted per-shard top-k lists.
//   meanpool_*           the reference's literal arithmetic (mean-pool + cosine,
//                        local_rag_complete.py:821-829) with doc means built once.
#include <hip/hip_runtime.h>

#include <stdarg.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <type_traits>
#include <vector>
#include <stdio.h>
#include <string.h>

#include "colbert_mi355x.h"

namespace {

constexpr int kDim = 128;                         // embedding dim (Jina-ColBERT-v2)
constexpr int kLd = 128;                          // token slots per doc
constexpr int kLqMax = 32;                        // query tokens per MFMA column block
constexpr int kRowBytes = kDim * 2;               // 256 B per bf16 token row
constexpr int kDocBytes = kLd * kRowBytes;        // 32 KiB per doc tile
constexpr int kTopkMax = 1024;                    // largest k any selection supports
constexpr int kSmallMax = 1024;                   // longest row for select_small / rerank C
constexpr int kMergeMax = 8192;                   // G * k limit of the merge kernel

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

__device__ __forceinline__ float neg_inf() { return -__builtin_inff(); }

// Order-preserving map float -> uint32 (larger float <=> larger uint).
__device__ __forceinline__ uint32_t f2u(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float u2f(uint32_t u) {
  u = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
  return __uint_as_float(u);
}
// Ranking key: score descending, then lower index first.
__device__ __forceinline__ uint64_t rank_key(float s, uint32_t idx) {
  return ((uint64_t)f2u(s) << 32) | (uint32_t)(~idx);
}

// Max / min over the 64 lanes, wave-uniform: 16-lane rows by DPP, then the
// four rows' lane 0.  Full EXEC.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
  return max(max((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
             max((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
  v = min(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
  return min(min((uint32_t)__builtin_amdgcn_readlane((int)v, 0), (uint32_t)__builtin_amdgcn_readlane((int)v, 16)),
             min((uint32_t)__builtin_amdgcn_readlane((int)v, 32), (uint32_t)__builtin_amdgcn_readlane((int)v, 48)));
}


__device__ __forceinline__ float max16(const f32x16& a) {
  float m0 = fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3]));
  float m1 = fmaxf(fmaxf(a[4], a[5]), fmaxf(a[6], a[7]));
  float m2 = fmaxf(fmaxf(a[8], a[9]), fmaxf(a[10], a[11]));
  float m3 = fmaxf(fmaxf(a[12], a[13]), fmaxf(a[14], a[15]));
  return fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
}

// Accumulator init for a partially valid 32-token block: 0 for doc rows < dl,
// -inf for padding rows.  Rows held by this lane for a 32x32x16 MFMA:
// row(reg) = row0 + (reg&3) + 8*(reg>>2), row0 = 32*blk + 4*h.
__device__ __forceinline__ f32x16 row_mask_init(int row0, int dl) {
  f32x16 a;
#pragma unroll
  for (int reg = 0; reg < 16; ++reg) a[reg] = (row0 + (reg & 3) + 8 * (reg >> 2) < dl) ? 0.0f : neg_inf();
  return a;
}

// Sum over the 32 query-token columns after folding the two row halves.
// Every lane ends with the identical value (xor butterfly of commutative adds).
__device__ __forceinline__ float col_reduce(float m, int r, int lq) {
  float v = fmaxf(m, __shfl_xor(m, 32));
  v = (r < lq) ? v : 0.0f;
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return v;
}

// Cross-lane helpers without LDS traffic (gfx950): v_permlane32_swap /
// v_permlane16_swap exchange half-waves / 16-lane rows; DPP row ops do the rest.
__device__ __forceinline__ float fold32_max(float v) {  // max over lanes l, l^32
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float fold16_max(float v) {  // max over lanes l, l^16 (rows 0<->1, 2<->3)
  const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float fold16_add(float v) {  // sum over lanes l, l^16 row pairs
  const auto t = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(t[0]) + __uint_as_float(t[1]);
}
__device__ __forceinline__ float dpp_row_sum16(float v) {  // sum over each 16-lane row, in every lane
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));   // quad_perm [1,0,3,2]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true));   // quad_perm [2,3,0,1]
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, true));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, true));  // row_mirror
  return v;
}
// 32x32 epilogue, DPP form: same result set as col_reduce, no ds_bpermute.
__device__ __forceinline__ float col_reduce_dpp(float m, int r, int lq) {
  float v = fold32_max(m);
  v = (r < lq) ? v : 0.0f;
  return fold16_add(dpp_row_sum16(v));
}

// B-operand fragments of one query for v_mfma_f32_32x32x16_bf16.  Lane l
// (r = l&31 query token, h = l>>5) holds, for k-step s, dims 64h+8s .. 64h+8s+7
// of token r.  The doc A-operand uses the same permutation of the 128 dims, so
// the 8 k-steps still sum every dim exactly once.
__device__ __forceinline__ void load_qfrag(const uint16_t* __restrict__ Q, int qi, int B, int lq,
                                           int lane, bf16x8 (&qf)[8]) {
  const int r = lane & 31, h = lane >> 5;
  const bool ok = (qi < B) && (r < lq);
  const u32x4* src = reinterpret_cast<const u32x4*>(Q + ((size_t)(ok ? qi : 0) * lq + (ok ? r : 0)) * kDim + 64 * h);
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    u32x4 v = ok ? src[s] : u32x4{0u, 0u, 0u, 0u};
    qf[s] = __builtin_bit_cast(bf16x8, v);
  }
}

// ---------------------------------------------------------------------------
// MaxSim scan.  Grid = n_qgroups * n_chunks workgroups of WAVES waves; each
// wave owns QW queries.  Doc tiles: LDS image [128 tokens][16 slots of 16 B],
// slot p of token t holding logical slot p ^ (t & 15) (conflict-free
// ds_read_b128 for the A-fragment pattern; filled by lane-linear LDS-DMA with
// the XOR applied to the per-lane SOURCE address).
// ---------------------------------------------------------------------------
template <int WAVES, int QW, bool DPP>
__global__ __launch_bounds__(WAVES * 64, 2) void maxsim_scan_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out,
    int64_t chunk_docs) {
  constexpr int QPB = WAVES * QW;
  constexpr int kPieces = kDocBytes / 1024;       // 1-KiB LDS-DMA pieces per doc
  constexpr int kPiecesPerWave = kPieces / WAVES;
  static_assert(kPieces % WAVES == 0, "pieces must split evenly over waves");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * kDocBytes];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;

  // XCD-aware, bijective block -> (query group, chunk): the blocks dealt to one
  // XCD (b % 8) cover consecutive linear ids, query group fastest, so all query
  // groups of a chunk stream the same docs through the same L2 at once.
  const int nq_groups = (B + QPB - 1) / QPB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, idx = bid >> 3, qd = nwg >> 3, rm = nwg & 7;
  const int lin = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + idx;
  const int g = lin % nq_groups;
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;  // uniform over the workgroup
  const int nd = (int)(d_end - d_begin);

  bf16x8 qf[QW][8];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag(Q, g * QPB + wave * QW + q, B, lq, lane, qf[q]);

  // LDS-DMA source offsets of this lane's pieces (same for every doc).
  uint32_t src_off[kPiecesPerWave];
#pragma unroll
  for (int j = 0; j < kPiecesPerWave; ++j) {
    const int piece = wave * kPiecesPerWave + j;
    const int t = 4 * piece + (lane >> 4);
    const int p = lane & 15;
    src_off[j] = t * kRowBytes + 16 * (p ^ (t & 15));
  }
  auto issue = [&](int i, int buf) {
    const uint8_t* dbase = tokens + (size_t)(d_begin + i) * kDocBytes;
#pragma unroll
    for (int j = 0; j < kPiecesPerWave; ++j) {
      const int piece = wave * kPiecesPerWave + j;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(dbase + src_off[j]),
                                       (lds_void_t*)(smem + buf * kDocBytes + piece * 1024), 16, 0, 0);
    }
  };

  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;

  issue(0, 0);
  for (int i = 0; i < nd; ++i) {
    // doc i landed (own pieces) -> barrier (everyone's pieces; everyone done with i-1)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + 1 < nd) issue(i + 1, (i + 1) & 1);

    const uint8_t* buf = smem + (i & 1) * kDocBytes;
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > kLd ? kLd : dl);
    float m[QW];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q] = neg_inf();
#pragma unroll
    for (int c = 0; c < kLd / 32; ++c) {
      if (dl > 32 * c) {
        bf16x8 af[8];
        const uint8_t* row = buf + (32 * c + r) * kRowBytes;
#pragma unroll
        for (int s = 0; s < 8; ++s)
          af[s] = *reinterpret_cast<const bf16x8*>(row + 16 * ((8 * h + s) ^ (r & 15)));
        // Padding rows (t >= dl) start their accumulation at -inf, so they can
        // never win the max: masking costs nothing on full blocks.
        const f32x16 init = (dl >= 32 * c + 32) ? f32x16{} : row_mask_init(32 * c + 4 * h, dl);
#pragma unroll
        for (int q = 0; q < QW; ++q) {
          f32x16 acc = init;
#pragma unroll
          for (int s = 0; s < 8; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], qf[q][s], acc, 0, 0, 0);
          m[q] = fmaxf(m[q], max16(acc));
        }
      }
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = DPP ? col_reduce_dpp(m[q], r, lq) : col_reduce(m[q], r, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = g * QPB + wave * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// MaxSim scan on v_mfma_f32_16x16x32_bf16.  Per (query, doc): 8 doc row tiles
// (16 tokens) x 2 query column tiles (16 tokens) x 4 k-steps (32 dims) = 64
// MFMAs.  Lane l: c = l&15, g = l>>4.  A (doc): token 16*rt + c, dims
// 32g + 8s .. +7 of k-step s;  B (query): token 16*ct + c, same dims.  C/D:
// column c (query token), rows 4g + reg (doc tokens).  Accumulators are 4
// registers, so the A fragments of the NEXT row tile are read from LDS while
// the current tile's MFMAs run (16 VGPRs per tile, double-buffered).
// LDS image: 16-B slot p of token t holds logical slot p ^ swz16(t), which is
// conflict-free for this fragment pattern in every ds_read_b128 lane group.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int swz16(int t) { return ((t & 1) << 3) | (t & 2) | ((t >> 2) & 1); }

__device__ __forceinline__ void load_qfrag16(const uint16_t* __restrict__ Q, int qi, int B, int lq, int lane,
                                             bf16x8 (&qf)[2][4]) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int tok = 16 * ct + c;
    const bool ok = (qi < B) && (tok < lq);
    const u32x4* src = reinterpret_cast<const u32x4*>(Q + ((size_t)(ok ? qi : 0) * lq + (ok ? tok : 0)) * kDim + 32 * g);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u32x4 v = ok ? src[s] : u32x4{0u, 0u, 0u, 0u};
      qf[ct][s] = __builtin_bit_cast(bf16x8, v);
    }
  }
}

// A fragments of row tile rt from the swizzled LDS image.
__device__ __forceinline__ void lds_afrag16(const uint8_t* buf, int rt, int lane, bf16x8 (&a)[4]) {
  const int c = lane & 15, g = lane >> 4;
  const int t = 16 * rt + c;
  const uint8_t* row = buf + t * kRowBytes;
  const int sw = swz16(t);
#pragma unroll
  for (int s = 0; s < 4; ++s) a[s] = *reinterpret_cast<const bf16x8*>(row + 16 * ((4 * g + s) ^ sw));
}

// A fragments of row tile rt straight from global memory (rerank gather).
__device__ __forceinline__ void gbl_afrag16(const uint8_t* doc, int rt, int lane, bf16x8 (&a)[4]) {
  const int c = lane & 15, g = lane >> 4;
  const u32x4* src = reinterpret_cast<const u32x4*>(doc + (16 * rt + c) * kRowBytes + 64 * g);
#pragma unroll
  for (int s = 0; s < 4; ++s) a[s] = __builtin_bit_cast(bf16x8, src[s]);
}

__device__ __forceinline__ f32x4 row_mask_init16(int row0, int dl) {
  f32x4 a;
#pragma unroll
  for (int reg = 0; reg < 4; ++reg) a[reg] = (row0 + reg < dl) ? 0.0f : neg_inf();
  return a;
}

// One row tile against QW queries: m[q][ct] = max(m, max over this lane's 4 rows).
template <int QW>
__device__ __forceinline__ void tile16(const bf16x8 (&a)[4], const bf16x8 (&qf)[QW][2][4], const f32x4& init,
                                       float (&m)[QW][2]) {
#pragma unroll
  for (int q = 0; q < QW; ++q) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      f32x4 acc = init;
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], qf[q][ct][s], acc, 0, 0, 0);
      m[q][ct] = fmaxf(fmaxf(m[q][ct], fmaxf(acc[0], acc[1])), fmaxf(acc[2], acc[3]));
    }
  }
}

// Per-(query, doc) epilogue of the 16x16 tiling: max over the 4 row groups,
// then sum over the lq query tokens (2 column tiles x 16 lanes).
__device__ __forceinline__ float reduce16(float m0, float m1, int lane, int lq) {
  const int c = lane & 15;
  m0 = fold16_max(fold32_max(m0));
  m1 = fold16_max(fold32_max(m1));
  const float v = (c < lq ? m0 : 0.0f) + (16 + c < lq ? m1 : 0.0f);
  return dpp_row_sum16(v);
}

// Full (query, doc) MaxSim for the 16x16 tiling; FRAG(rt, a) loads row tile rt.
template <int QW, typename Frag>
__device__ __forceinline__ void doc16(Frag frag, const bf16x8 (&qf)[QW][2][4], int dl, int lane, float (&m)[QW][2]) {
  const int g = lane >> 4;
#pragma unroll
  for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
  if (dl >= kLd) {
    // Full doc (the common case): straight-line, so hipcc counts the LDS reads
    // exactly and the next tile's fragments load under the current tile's MFMAs.
    bf16x8 a0[4], a1[4];
    frag(0, a0);
#pragma unroll
    for (int rt = 0; rt < kLd / 16; rt += 2) {
      frag(rt + 1, a1);
      tile16<QW>(a0, qf, f32x4{}, m);
      if (rt + 2 < kLd / 16) frag(rt + 2, a0);
      tile16<QW>(a1, qf, f32x4{}, m);
    }
    return;
  }
  const int nrt = (dl + 15) >> 4;
  bf16x8 a0[4], a1[4];
  if (nrt > 0) frag(0, a0);
#pragma unroll
  for (int rt = 0; rt < kLd / 16; rt += 2) {
    if (rt < nrt) {
      if (rt + 1 < nrt) frag(rt + 1, a1);
      const f32x4 init = (dl >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dl);
      tile16<QW>(a0, qf, init, m);
    }
    if (rt + 1 < nrt) {
      if (rt + 2 < nrt) frag(rt + 2, a0);
      const f32x4 init = (dl >= 16 * rt + 32) ? f32x4{} : row_mask_init16(16 * rt + 16 + 4 * g, dl);
      tile16<QW>(a1, qf, init, m);
    }
  }
}

template <int WAVES, int QW, int OCC = 2>
__global__ __launch_bounds__(WAVES * 64, OCC) void maxsim_scan16_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out,
    int64_t chunk_docs) {
  constexpr int QPB = WAVES * QW;
  constexpr int kPieces = kDocBytes / 1024;
  constexpr int kPiecesPerWave = kPieces / WAVES;
  static_assert(kPieces % WAVES == 0, "pieces must split evenly over waves");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * kDocBytes];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);

  const int nq_groups = (B + QPB - 1) / QPB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, idx = bid >> 3, qd = nwg >> 3, rm = nwg & 7;
  const int lin = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + idx;
  const int g = lin % nq_groups;
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;
  const int nd = (int)(d_end - d_begin);

  bf16x8 qf[QW][2][4];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag16(Q, g * QPB + wave * QW + q, B, lq, lane, qf[q]);

  uint32_t src_off[kPiecesPerWave];
#pragma unroll
  for (int j = 0; j < kPiecesPerWave; ++j) {
    const int piece = wave * kPiecesPerWave + j;
    const int t = 4 * piece + (lane >> 4);
    src_off[j] = t * kRowBytes + 16 * ((lane & 15) ^ swz16(t));
  }
  auto issue = [&](int i, int buf) {
    const uint8_t* dbase = tokens + (size_t)(d_begin + i) * kDocBytes;
#pragma unroll
    for (int j = 0; j < kPiecesPerWave; ++j) {
      const int piece = wave * kPiecesPerWave + j;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(dbase + src_off[j]),
                                       (lds_void_t*)(smem + buf * kDocBytes + piece * 1024), 16, 0, 0);
    }
  };

  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;

  issue(0, 0);
  for (int i = 0; i < nd; ++i) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + 1 < nd) issue(i + 1, (i + 1) & 1);

    const uint8_t* buf = smem + (i & 1) * kDocBytes;
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > kLd ? kLd : dl);
    float m[QW][2];
    doc16<QW>([&](int rt, bf16x8 (&a)[4]) { lds_afrag16(buf, rt, lane, a); }, qf, dl, lane, m);
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = g * QPB + wave * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// The production B >= 3 scan: doc-interleaved row tiles.  A 16-row A tile
// holds 4 consecutive tokens of each of 4 docs (rows 4g..4g+3 = doc g), so
// the lanes of MFMA output group g accumulate exactly doc g's row maxima:
// the per-doc epilogue needs no cross-group fold (no permlane swaps), just one
// 16-lane DPP sum per query per 4 docs — ~8x less epilogue VALU than
// maxsim_scan16_kernel, whose epilogue ran with no MFMA work to hide under.
// Each iteration streams 32 tokens of 4 docs (32 KiB) HBM -> LDS by LDS-DMA
// into a 3-deep ring (the next iteration's pieces stay in flight across the
// barrier); 4 iterations per doc group.  Within an iteration the 8 tiles x
// 2*QW MFMA chains run as one software pipeline: chain k's row max is taken
// after chains k+1..k+D have issued, so the MFMA->VALU read hazard is covered
// by MFMAs instead of s_nop.  LDS image [4 docs][32 tokens][16 slots of 16 B]
// with slot p of row R at p ^ swz4(R): the 16 rows a ds_read_b128 lane group
// touches get 16 distinct slots (conflict-free).  Per (query, doc) the dot
// products, the max and the column-sum order are those of doc16 + reduce16,
// so scores are bit-identical to every other scan and to the rerank kernel.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int swz4(int R) { return (((R >> 5) & 3) << 2) | (R & 3); }

// Full iteration (all 4 docs valid for its 32 tokens): 8 tiles, pipelined.
// (Moving chain k-D's max one MFMA later removes hipcc's s_nop pads for the
// MFMA -> VALU hazard, 26 -> 2 per iteration, and gains nothing measurable:
// the partner wave covers them.  Lab, round 1.)
struct NoTileHook {
  __device__ __forceinline__ void operator()(int) const {}
};

// hook(t) runs right after tile t's first MFMA chain has issued (SPREAD: the
// next iteration's DMA pieces; NoTileHook = nothing).
// PROBE (lab energy probe, INVALID scores): 1 = odd tiles reuse the even
// tile's A fragments (half the LDS read bytes, same MFMAs); 2 (kernel) = no
// doc streaming after the ring's first fill (no L2 -> LDS traffic).
// PROBE 3 (lab power probe, INVALID scores): the same FLOPs on
// v_mfma_f32_32x32x16_bf16 -- each pair of 16-row tiles as one 32-row tile of
// 8 k-steps, one 16-register chain per query, its 16 values folded into the
// running max (the same v_max3 count per FLOP as the 16x16 chains) -- with the
// same LDS reads; half the register-operand bytes per FLOP of the 16x16x32
// form.  Timing only: is the mid-batch scan's held clock (power) sensitive
// to the operand path?
template <int QW, int D, int NT>
__device__ __forceinline__ void iter4_full_probe32(const uint8_t* buf, int lane, const bf16x8 (&qf)[QW][2][4],
                                                   float (&m)[QW][2]) {
  static_assert(NT % 2 == 0, "tile pairs");
  constexpr int NT2 = NT / 2, NK = NT2 * QW;
  const int c = lane & 15, g = lane >> 4;
  const uint8_t* rowp = buf + (4 * NT * (c >> 2) + (c & 3)) * kRowBytes;
  auto frag = [&](int t, bf16x8 (&af)[8]) {   // tiles 2t, 2t + 1
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < 4; ++s)
        af[4 * h + s] = *reinterpret_cast<const bf16x8*>(rowp + 4 * (2 * t + h) * kRowBytes + 16 * ((4 * g + s) ^ c));
  };
  // one A buffer (a second does not fit beside 4 queries' fragments): the next
  // tile's fragments load right after the tile's last chain has issued, under
  // that chain's MFMAs
  bf16x8 a[8];
  f32x16 acc[D + 1];
  frag(0, a);
#pragma unroll
  for (int k = 0; k < NK + D; ++k) {
    if (k < NK) {
      const int t = k / QW, q = k % QW;
      f32x16 x = f32x16{};
#pragma unroll
      for (int s = 0; s < 8; ++s)
        x = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[s], qf[q][s >> 2][s & 3], x, 0, 0, 0);
      acc[k % (D + 1)] = x;
      if (q == QW - 1 && t + 1 < NT2) frag(t + 1, a);
    }
    if (k >= D) {
      const int q = (k - D) % QW;
      const f32x16& y = acc[(k - D) % (D + 1)];
      float& mm = m[q][0];
#pragma unroll
      for (int r = 0; r < 16; r += 2) mm = fmaxf(fmaxf(mm, y[r]), y[r + 1]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int QW, int D, int NT = 8, typename Hook = NoTileHook, int PROBE = 0>
__device__ __forceinline__ void iter4_full(const uint8_t* buf, int lane, const bf16x8 (&qf)[QW][2][4],
                                           float (&m)[QW][2], Hook hook = Hook{}) {
  if constexpr (PROBE == 3) {
    iter4_full_probe32<QW, D, NT>(buf, lane, qf, m);
    return;
  }
  constexpr int NC = 2 * QW;
  constexpr int NK = NT * NC;
  const int c = lane & 15, g = lane >> 4;
  const uint8_t* rowp = buf + (4 * NT * (c >> 2) + (c & 3)) * kRowBytes;  // row of tile t: + 4t rows
  auto frag = [&](int t, bf16x8 (&a)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      a[s] = *reinterpret_cast<const bf16x8*>(rowp + 4 * t * kRowBytes + 16 * ((4 * g + s) ^ c));
  };
  bf16x8 a[2][4];
  f32x4 acc[D + 1];
  frag(0, a[0]);
#pragma unroll
  for (int k = 0; k < NK + D; ++k) {
    if (k < NK) {
      const int t = k / NC, cc = k % NC;
      if (cc == 0 && t + 1 < NT && (PROBE != 1 || ((t + 1) & 1) == 0)) frag(t + 1, a[((t + 1) & 1) * (PROBE != 1)]);
      if (PROBE == 1 && cc == 0) {   // opaque: the reused fragments must not fold the MFMAs
#pragma unroll
        for (int s = 0; s < 4; ++s) asm volatile("" : "+v"(a[0][s]));
      }
      f32x4 x = f32x4{};
#pragma unroll
      for (int s = 0; s < 4; ++s)
        x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[(t & 1) * (PROBE != 1)][s], qf[cc >> 1][cc & 1][s], x, 0, 0, 0);
      acc[k % (D + 1)] = x;
      if (cc == 0) hook(t);
    }
    if (k >= D) {
      const int kk = k - D, pc = kk % NC;
      const f32x4& y = acc[kk % (D + 1)];
      float& mm = m[pc >> 1][pc & 1];
      mm = fmaxf(fmaxf(fmaxf(fmaxf(mm, y[0]), y[1]), y[2]), y[3]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// k-step-major order (lab, MORDER 1): the NC chains of a tile advance one
// k-step at a time with NC live accumulators, so NC consecutive MFMAs share
// their A fragment (doc rows) and only B (the query) changes; tile t-1's row
// maxima are taken between tile t's k-step-0 MFMAs (the accumulator a max
// reads is rewritten by the MFMA right after it).  Per chain the same k order
// and the same max: bit-identical to iter4_full.
template <int QW, int NT = 8>
__device__ __forceinline__ void iter4_full_kmajor(const uint8_t* buf, int lane, const bf16x8 (&qf)[QW][2][4],
                                                  float (&m)[QW][2]) {
  constexpr int NC = 2 * QW;
  const int c = lane & 15, g = lane >> 4;
  const uint8_t* rowp = buf + (4 * NT * (c >> 2) + (c & 3)) * kRowBytes;
  auto frag = [&](int t, bf16x8 (&a)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s)
      a[s] = *reinterpret_cast<const bf16x8*>(rowp + 4 * t * kRowBytes + 16 * ((4 * g + s) ^ c));
  };
  auto fold = [&](int cc, const f32x4& y) {
    float& mm = m[cc >> 1][cc & 1];
    mm = fmaxf(fmaxf(fmaxf(fmaxf(mm, y[0]), y[1]), y[2]), y[3]);
  };
  bf16x8 a[2][4];
  f32x4 acc[NC];
  frag(0, a[0]);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t + 1 < NT) frag(t + 1, a[(t + 1) & 1]);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int cc = 0; cc < NC; ++cc) {
        if (s == 0 && t > 0) fold(cc, acc[cc]);
        acc[cc] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[t & 1][s], qf[cc >> 1][cc & 1][s],
                                                          s == 0 ? f32x4{} : acc[cc], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) fold(cc, acc[cc]);
}

// Iteration j with ragged docs: per-lane-group -inf C-init masks padding rows.
template <int QW, int NT = 8>
__device__ __forceinline__ void iter4_ragged(const uint8_t* buf, int lane, int j, int dl_g, int dl_max,
                                             const bf16x8 (&qf)[QW][2][4], float (&m)[QW][2]) {
  const int c = lane & 15, g = lane >> 4;
  const uint8_t* rowp = buf + (4 * NT * (c >> 2) + (c & 3)) * kRowBytes;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int tok0 = 4 * NT * j + 4 * t;
    if (tok0 >= dl_max) break;
    bf16x8 a[4];
#pragma unroll
    for (int s = 0; s < 4; ++s)
      a[s] = *reinterpret_cast<const bf16x8*>(rowp + 4 * t * kRowBytes + 16 * ((4 * g + s) ^ c));
    f32x4 init;
#pragma unroll
    for (int r = 0; r < 4; ++r) init[r] = (tok0 + r < dl_g) ? 0.0f : neg_inf();
    tile16<QW>(a, qf, init, m);
  }
}

// Wait until flags[0 .. n) >= target (LDS counters of the ARRIVE ring; n <= 64).
__device__ __forceinline__ void lds_wait_all_ge(int* flags, int n, int target, int lane) {
  for (;;) {
    const int v = lane < n ? __hip_atomic_load(flags + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : target;
    if (__ballot(v < target) == 0) break;
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------
// Fused top-k (SURVEY §7 hard part (ii)): instead of writing the [B, n] score
// matrix, each wave keeps, per query it owns, a buffer of up to FK ranking
// keys (score bits << 32 | ~local doc index: unique, larger = better) in its
// own LDS region, with a threshold key and a count beside it (LDS too: the
// scan kernels have no SGPRs or VGPRs to spare).  A 64-doc epilogue block
// offers its keys; those above the threshold are appended.  When a buffer
// would overflow, the wave finds its k-th largest key by a bitwise binary
// search over ballot counts (64 steps, scalar work: 2 keys per lane, no sort,
// ~4 VGPRs) and keeps the k keys >= it, which becomes the threshold.  No
// barrier is involved: a buffer belongs to one wave.  After its last doc range
// the workgroup writes its best k keys per query to part[query][slot][k]
// (slot = its chunk in its query group; key 0 = padding) and
// select_keys_kernel picks each query's top-k over the slots.  Keys compare as
// the unfused (score desc, index asc) rule does, so the ids equal the unfused
// path's bit for bit.
// ---------------------------------------------------------------------------
constexpr int kFusedCap = 120;                    // keys per (wave, query) buffer (<= 128: 2 per lane)
constexpr int kFusedMaxK = kFusedCap - 16;        // appends go in 16-lane batches after a compaction
constexpr int kFusedStateBytes = 16;              // per (wave, query): threshold u64, count i32

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)v);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// Keep the best min(cnt, k) keys of buf[0..cnt) (this wave's LDS buffer, cnt
// <= 128) at buf[0..), unordered; thr = the k-th largest key once k are held.
__device__ __forceinline__ void topk_compact(uint64_t* buf, int& cnt, uint64_t& thr, int k, int lane) {
  if (cnt <= k) {
    if (cnt == k) {  // threshold = the smallest held key
      uint64_t m = lane < cnt ? buf[lane] : ~0ull;
      const uint64_t m2 = lane + 64 < cnt ? buf[lane + 64] : ~0ull;
      m = m < m2 ? m : m2;
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(m >> 32), off) << 32) |
                           (uint32_t)__shfl_xor((int)(uint32_t)m, off);
        m = m < o ? m : o;
      }
      thr = uniform64(m);
    }
    return;
  }
  const uint64_t a = lane < cnt ? buf[lane] : 0ull;
  const uint64_t b = lane + 64 < cnt ? buf[lane + 64] : 0ull;
  uint64_t T = 0;  // largest T with count(key >= T) >= k: the k-th largest (keys are unique)
#pragma unroll 1
  for (int bit = 63; bit >= 0; --bit) {
    const uint64_t t = T | (1ull << bit);
    const int c = __popcll(__ballot(a >= t)) + __popcll(__ballot(b >= t));
    if (c >= k) T = t;
  }
  const uint64_t below = (1ull << lane) - 1ull;
  const uint64_t ma = __ballot(a >= T), mb = __ballot(b >= T);
  if (a >= T) buf[__popcll(ma & below)] = a;
  if (b >= T) buf[__popcll(ma) + __popcll(mb & below)] = b;
  thr = T;
  cnt = k;
}

// Offer one key per lane (0 = none) to the buffer of one (wave, query).
template <int FK>
__device__ __forceinline__ void topk_offer(uint64_t* buf, uint8_t* state, int k, uint64_t key, int lane) {
  uint64_t thr = uniform64(*reinterpret_cast<const uint64_t*>(state));
  const uint64_t mask = __ballot(key > thr);
  const int np = __popcll(mask);
  if (np == 0) return;
  int cnt = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(state + 8));
  const uint64_t below = (1ull << lane) - 1ull;
  if (cnt + np <= FK) {
    if (key > thr) buf[cnt + __popcll(mask & below)] = key;
    cnt += np;
  } else {
#pragma unroll 1
    for (int h = 0; h < 4; ++h) {  // 16 lanes at a time: cnt <= k + 16 <= FK after a compaction
      const bool mine = (lane >> 4) == h;
      const int nh = __popcll(__ballot(mine && key > thr));
      if (nh == 0) continue;
      if (cnt + nh > FK) topk_compact(buf, cnt, thr, k, lane);
      const uint64_t m3 = __ballot(mine && key > thr);
      if (mine && key > thr) buf[cnt + __popcll(m3 & below)] = key;
      cnt += __popcll(m3);
    }
    if (lane == 0) *reinterpret_cast<uint64_t*>(state) = thr;
  }
  if (lane == 0) *reinterpret_cast<int*>(state + 8) = cnt;
}

// End of a workgroup's work: its best k keys of one query to dst[0..k) (0-padded).
__device__ __forceinline__ void topk_flush(uint64_t* buf, uint8_t* state, int k, uint64_t* dst, int lane) {
  uint64_t thr = uniform64(*reinterpret_cast<const uint64_t*>(state));
  int cnt = __builtin_amdgcn_readfirstlane(*reinterpret_cast<const int*>(state + 8));
  if (cnt > k) topk_compact(buf, cnt, thr, k, lane);
  for (int e = lane; e < k; e += 64) dst[e] = e < cnt ? buf[e] : 0ull;
}

// Dynamic-tail task grab (one thread): writes (doc offset into the tail, size;
// size 0 = done) to slot[0..1].  task_docs > 0: fixed tasks, the counter counts
// tasks; task_docs < 0: guided, by ticket: one atomicAdd draws ticket t, and
// round r = the r-th group of P tickets (P = workgroups per query group) hands
// out tasks of max(-task_docs, dyn / 2^(r+1) / P) docs (round r covers at most
// half of what rounds 0..r-1 left), so the offset of every ticket is a closed
// form and no grab ever retries.  (The earlier CAS form took remaining / 2P per
// grab: with 64 workgroups on one counter, one CAS won per round trip, and the
// serialized grants cost B=8 at 125k docs 0.78 -> 1.93 ms at a 30 % tail.
// CBV2_TAIL_CAS=1 rebuilds it for lab A/Bs.)
#ifndef CBV2_TAIL_CAS
#define CBV2_TAIL_CAS 0
#endif
__device__ __forceinline__ void ticket_task(int t, int dyn, int P, int minsz, int& o, int& sz) {
  int off = 0, s = minsz;
  for (int r = 0; r < 31; ++r) {
    s = ((dyn >> (r + 1)) / P) & ~15;
    if (s <= minsz) {   // this round and all later ones: minsz-doc tasks
      s = minsz;
      break;
    }
    if (t < P) break;
    off += s * P;
    t -= P;
  }
  const int64_t o64 = (int64_t)off + (int64_t)t * s;
  o = o64 < dyn ? (int)o64 : dyn;
  sz = o < dyn ? (dyn - o < s ? dyn - o : s) : 0;
}
__device__ __forceinline__ void next_task(int* ctr, int task_docs, int dyn, int P, int* slot) {
  int o, sz;
  if (task_docs > 0) {
    o = atomicAdd(ctr, 1) * task_docs;
    sz = o < dyn ? (dyn - o < task_docs ? dyn - o : task_docs) : 0;
  } else if (!CBV2_TAIL_CAS) {
    ticket_task(atomicAdd(ctr, 1), dyn, P, -task_docs, o, sz);
  } else {
    o = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
      const int rem = dyn - o;
      if (rem <= 0) { sz = 0; break; }
      sz = ((rem / (2 * P)) + 15) & ~15;
      sz = sz > -task_docs ? sz : -task_docs;
      sz = sz < rem ? sz : rem;
      const int prev = atomicCAS(ctr, o, o + sz);
      if (prev == o) break;
      o = prev;
    }
  }
  slot[0] = o;
  slot[1] = sz;
}

// The tail in nsl XCD-local slices (nsl = 8, or 1 = one shared tail): slice s
// = [lo(s), lo(s+1)) with its own counter ctr[s] per query group.  A
// workgroup drains the slice of its XCD (blockIdx % 8: blocks b and b + 8
// share an XCD) before the others', so the query groups reading the same
// tail docs on one XCD share its L2 (with one shared tail the tasks of a doc
// range land on up to 8 XCDs: PMC, r02h, +3.3 GB per 1M-doc launch).
__device__ __forceinline__ int tail_slice_lo(int s, int nsl, int dyn) {
  return s >= nsl ? dyn : (int)(((int64_t)dyn * s / nsl) & ~15LL);
}
__device__ __forceinline__ void next_task_sliced(int* ctr, int nsl, int xcd, int task_docs, int dyn, int P,
                                                 int* slot) {
  for (int r = 0; r < nsl; ++r) {
    const int sl = (xcd + r) % nsl;
    const int lo = tail_slice_lo(sl, nsl, dyn);
    // guided sizes as if every workgroup of the query group shared the slice:
    // small tasks, so the fast XCDs' steals at the end stay fine-grained
    next_task(ctr + sl, task_docs, tail_slice_lo(sl + 1, nsl, dyn) - lo, P, slot);
    if (slot[1] > 0) {
      slot[0] += lo;
      return;
    }
  }
  slot[0] = 0;
  slot[1] = 0;
}
// The task of ticket t of the first slice next_task_sliced would try (the
// scan's task hand-off draws it an iteration before it needs the task); size
// -1: that slice is drained -- the caller takes the drained path, whose
// next_task_sliced goes on to the other slices (no atomic with a return in
// the scan's loop but the one ticket: the waitcnt pass would otherwise keep
// its pending return against the VGPRs the loop's LDS reads reuse).
__device__ __forceinline__ void task_from_ticket(int t, int nsl, int xcd, int task_docs, int dyn, int P, int* slot) {
  const int sl = xcd % nsl;
  const int lo = tail_slice_lo(sl, nsl, dyn);
  const int sdyn = tail_slice_lo(sl + 1, nsl, dyn) - lo;
  int o, sz;
  if (task_docs > 0) {
    o = t * task_docs;
    sz = o < sdyn ? (sdyn - o < task_docs ? sdyn - o : task_docs) : 0;
  } else {
    ticket_task(t, sdyn, P, -task_docs, o, sz);
  }
  slot[0] = o + lo;
  slot[1] = sz > 0 ? sz : -1;
}

// Work split (per query group of QPB queries): docs [0, static_docs) in equal
// chunks, one per workgroup, XCD-aware as above; then, if task_ctr is given,
// docs [static_docs, n) as tasks of task_docs grabbed with one atomicAdd on
// the query group's counter until exhausted.  The XCDs hold different clocks
// under this load (1.98-2.11 GHz measured on one device, lab --stamps), so a
// static split ends when the slowest XCD does; the dynamic tail lets the fast
// ones take the remainder.  Every doc range runs the same pipelined loop.
// STAMPS (lab only): per-workgroup s_memrealtime / s_memtime at start and end.
// SPREAD (2-deep ring): a full iteration issues its wave's DMA pieces of the
// next iteration one per tile from inside the MFMA stream, instead of all at
// once after the barrier, where every wave of the CU queues on the address
// path at the same moment (lab phase stamps: ~1.2k issue cycles/iteration).
// FK > 0: fused top-k (see topk_offer): no score matrix; each workgroup writes
// its best topk_k keys per query to part[qi][slot][topk_k] (slot = its chunk).
// SPLITLOAD: only waves 0 .. WAVES/2-1 (one per SIMD) issue the ring's LDS-DMA
// pieces (twice as many each), so after each barrier the partner wave on the
// SIMD (waves WAVES/2 ..) starts its MFMAs at once instead of both waves
// spending the issue phase with the MFMA pipe idle.
// ARRIVE (with SPLITLOAD): no workgroup barrier per iteration.  Each loading
// wave publishes "iteration g landed" in LDS after its own vmcnt wait, every
// wave publishes "done with iteration g" after its last read of the slot, and
// a loader refills the slot of iteration g-1 once every wave is done with it.
// A wave waits only for what it reads or overwrites, so the partner waves
// cross iteration boundaries without draining the MFMA pipe at a barrier, and
// an NBUF-deep ring lets the loaders run up to NBUF-2 iterations ahead.
#ifndef CBV2_F8_D47
#define CBV2_F8_D47 1   // lab A/B builds set 3
#endif
#ifndef CBV2_SCAN_HANDOFF
#define CBV2_SCAN_HANDOFF 1   // lab A/B builds set 0: drained task switches (before round 6)
#endif
#ifndef CBV2_SCAN_QSKIP
#define CBV2_SCAN_QSKIP 1   // lab A/B builds set 0
#endif
constexpr bool kScanQSkip = CBV2_SCAN_QSKIP != 0;
// AUX: the doc stream's cache policy (0 cached: the query groups of a chunk
// share its tiles through L2; 2 non-temporal, for a launch of ONE query
// group, where every byte is read once).
// BMK: the block-max top-k's 64-doc block keys and 256-doc superblock keys
// folded in (bmk [B][bmk_ld], sbk [B][sbk_ld], zeroed before the launch): at
// each 64-doc group's store, the wave's max of the group's keys by atomic max
// -- a group of a range that does not start on a block boundary spans two
// blocks (and at most two superblocks), so its two parts go separately.  The
// keys equal block_max_kernel's.
// The bench's clock probe (cbv2_index_time_scans(ix, 2), product kernels,
// a runtime-null pointer otherwise): each workgroup adds (end - start) of
// s_memtime (shader clock) and s_memrealtime (100 MHz) to p[0] / p[1] (start
// subtracted at entry, end added at exit: nothing held across the loop) and
// counts its entry / exit in p[2] / p[3]; sum(dt) / sum(dr) x 0.1 GHz is the
// clock the launch's workgroups held, weighted by their run time.  The stamp
// waits its own lgkmcnt inside the asm (no LDS read is in flight here).
__device__ __forceinline__ void clock_probe(uint64_t* p, bool end) {
  unsigned long long t, r;
  asm volatile("s_memtime %0\n\ts_memrealtime %1\n\ts_waitcnt lgkmcnt(0)" : "=s"(t), "=s"(r)::"memory");
  atomicAdd(reinterpret_cast<unsigned long long*>(p), end ? t : 0ull - t);
  atomicAdd(reinterpret_cast<unsigned long long*>(p) + 1, end ? r : 0ull - r);
  atomicAdd(reinterpret_cast<unsigned long long*>(p) + (end ? 3 : 2), 1ull);
}

template <int WAVES, int QW, int D = 2, int NBUF = 3, bool STAMPS = false, int TPI = 32, int OCC = 2,
          bool SPREAD = false, int FK = 0, bool SPLITLOAD = false, bool ARRIVE = false, int PROBE = 0, int LD = kLd,
          int MORDER = 0, int AUX = 0, bool BMK = false>
__global__ __launch_bounds__(WAVES * 64, OCC) void maxsim_scan16x4_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out,
    int64_t chunk_docs, int64_t static_docs, int* __restrict__ task_ctr, int task_docs,
    uint64_t* __restrict__ stamps, int topk_k = 0, uint64_t* __restrict__ part = nullptr, int nslots = 0,
    int tail_slices = 1, uint32_t* __restrict__ bmk = nullptr, int64_t bmk_ld = 0, uint32_t* __restrict__ sbk = nullptr,
    int64_t sbk_ld = 0) {
  // TPI tokens of 4 docs per iteration (32: 32 KiB, 64: 64 KiB), IPG per group
  constexpr int QPB = WAVES * QW;
  constexpr int kIterBytes = 4 * TPI * kRowBytes;
  // LD token slots per doc (128; 256 / 512 / 1024 for long documents: a doc
  // group then spans LD / TPI iterations, the row maxima carried across them)
  static_assert(LD % TPI == 0 && LD >= 128 && LD <= 1024, "LD: 128, 256, 512 or 1024 token slots");
  constexpr int IPG = LD / TPI, NT = TPI / 4;
  constexpr size_t kDocStride = (size_t)LD * kRowBytes;
  constexpr int kPieces = kIterBytes / 1024;
  constexpr int kLoadWaves = SPLITLOAD ? WAVES / 2 : WAVES;
  constexpr int kPiecesPerWave = kPieces / kLoadWaves;   // per loading wave
  static_assert(TPI == 32 || TPI == 64, "32 or 64 tokens per iteration");
  static_assert(kPieces % kLoadWaves == 0, "pieces must split evenly over the loading waves");
  static_assert(NBUF >= 2 && NBUF <= 4, "2- to 4-deep ring");
  static_assert(!(SPREAD && SPLITLOAD), "SPREAD spreads every wave's pieces; SPLITLOAD moves them");
  static_assert(!ARRIVE || (SPLITLOAD && !SPREAD && kLoadWaves + WAVES <= 16), "ARRIVE needs SPLITLOAD");
  // one LDS object only: with a second __shared__ array hipcc starts putting
  // vmcnt(0) before the ring's ds_reads (LDS-DMA alias tracking)
  // fused top-k: one key buffer + state per (wave, query), after the task slots
  // (and, with ARRIVE, the landed / done counters)
  constexpr int kCandBytes = FK > 0 ? QPB * (FK * 8 + kFusedStateBytes) : 0;
  constexpr int kSyncBytes = ARRIVE ? 64 : 0;
  __shared__ __attribute__((aligned(1024))) uint8_t smem[NBUF * kIterBytes + 16 + kSyncBytes + kCandBytes];
  int* const task_slot = reinterpret_cast<int*>(smem + NBUF * kIterBytes);
  int* const sync_landed = reinterpret_cast<int*>(smem + NBUF * kIterBytes + 16);  // [loading waves]
  int* const sync_done = sync_landed + kLoadWaves;                                // [WAVES]
  uint8_t* const after_sync = smem + NBUF * kIterBytes + 16 + kSyncBytes;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  uint64_t* const cand = reinterpret_cast<uint64_t*>(after_sync) + (size_t)wave * QW * (FK > 0 ? FK : 1);
  uint8_t* const tk_state = after_sync + (FK > 0 ? QPB * FK * 8 : 0) + wave * QW * kFusedStateBytes;
  if (FK > 0 && lane < 2 * QW) reinterpret_cast<uint64_t*>(tk_state)[lane] = 0ull;  // thr = 0, cnt = 0
  if constexpr (ARRIVE) {
    if (threadIdx.x < kLoadWaves + WAVES) sync_landed[threadIdx.x] = 0;
    __syncthreads();
  }
  uint32_t gbase = 0;   // ARRIVE: iterations of the earlier doc ranges (ring slot of iteration it = (gbase+it) % NBUF)
  const int nq_groups = (B + QPB - 1) / QPB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, idx = bid >> 3, qd = nwg >> 3, rm = nwg & 7;
  const int lin = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + idx;
  const int qg = lin % nq_groups;
  const int64_t chunk = lin / nq_groups;
  uint64_t t_start = 0, r_start = 0;
  if constexpr (STAMPS) {
    t_start = __builtin_amdgcn_s_memtime();
    r_start = __builtin_amdgcn_s_memrealtime();
  } else {
    if (stamps != nullptr && threadIdx.x == 0) clock_probe(stamps, false);   // product: the clock probe
  }

  bf16x8 qf[QW][2][4];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag16(Q, qg * QPB + wave * QW + q, B, lq, lane, qf[q]);
  // (kHandoff: the fragments are in VGPRs before any range starts, as the
  // waitcnt pass sees it -- a range entered with its ring pre-issued issues
  // no load of its own, and the pass would otherwise wait vmcnt(0) before
  // every iteration's first MFMA)
  if constexpr (CBV2_SCAN_HANDOFF && NBUF == 3 && TPI == 32 && SPLITLOAD && !ARRIVE && !SPREAD)
    __builtin_amdgcn_s_waitcnt(0);

  // LDS-DMA piece p = rows 4p..4p+3 of the image [4 docs][TPI tokens] = doc
  // 4p / TPI, tokens TPI*j + 4p % TPI + 0..3; slot XOR (doc << 2 | R & 3)
  const bool loader = !SPLITLOAD || wave < kLoadWaves;   // wave-uniform
  const int lwave = loader ? wave : 0;
  // SPLITLOAD (16 pieces per loading wave): offsets on the fly instead of held
  // in VGPRs.  With R0 = 4 * piece (uniform) and L = lane >> 4: doc = R0 / TPI,
  // offset = (R0 % TPI + L) * 256 + 16 * (((lane & 15) ^ L) ^ (doc << 2)).
  constexpr int kHeld = SPLITLOAD ? 1 : kPiecesPerWave;
  uint32_t src_off[kHeld];
  int src_doc[kHeld];
  const uint32_t lb1 = (uint32_t)(lane >> 4) * kRowBytes, lb2 = 16u * (uint32_t)((lane & 15) ^ (lane >> 4));
#pragma unroll
  for (int jj = 0; jj < kHeld; ++jj) {
    const int R = 4 * (lwave * kPiecesPerWave + jj) + (lane >> 4);
    const int doc = R / TPI;
    src_off[jj] = (R % TPI) * kRowBytes + 16 * ((lane & 15) ^ ((doc << 2) | (R & 3)));
    src_doc[jj] = doc;
  }
  auto piece_src = [&](int jj, int& doc) -> uint32_t {
    if constexpr (SPLITLOAD) {
      const int R0 = 4 * (lwave * kPiecesPerWave + jj);
      doc = R0 / TPI;
      return (uint32_t)(R0 % TPI) * kRowBytes + lb1 + (lb2 ^ (uint32_t)(doc << 6));
    } else {
      doc = src_doc[jj];
      return src_off[jj];
    }
  };

  // STAMPS (lab only): per-wave s_memtime cycles in three phases of the ring
  // loop -- wait (vmcnt + barrier), issue (next DMA + doc lengths), compute
  // (tiles + epilogue, to the next iteration's top) -- and the iteration count
  uint64_t ph_wait = 0, ph_issue = 0, ph_comp = 0, ph_n = 0, ph_t = 0;

  // Task hand-off (3-deep ring, loading waves 0 .. WAVES/2-1: the dense B <= 2
  // one-per-CU scan): the next range is grabbed by the last (never loading)
  // wave four iterations before the current range ends, read after the
  // barrier of the second-last iteration, and its first two iterations go
  // into the ring where the current range's would have gone -- a task switch
  // drains nothing.  Lab, same box, interleaved (profiles/r06/handoff3_*):
  // B = 1 125k docs 0.594 -> 0.591 ms, 100k 0.486 -> 0.481, 1M 4.454 ->
  // 4.445; bit-identical scores.
  constexpr bool kHandoff =
      CBV2_SCAN_HANDOFF && !CBV2_TAIL_CAS && NBUF == 3 && TPI == 32 && SPLITLOAD && !ARRIVE && !SPREAD;
  // iteration it of the range [rb, rb + rnd) into ring slot buf
  auto issue_piece_at = [&](int64_t rb, int rnd, int it, int buf, int jj) {
    const int G = it / IPG, j = it % IPG;
    const int piece = lwave * kPiecesPerWave + jj;
    int pdoc;
    const uint32_t poff = piece_src(jj, pdoc);
    int d = 4 * G + pdoc;
    d = d < rnd ? d : rnd - 1;  // the last group's missing docs: any valid doc (rows masked)
    const uint8_t* src = tokens + (size_t)(rb + d) * kDocStride + (size_t)j * TPI * kRowBytes + poff;
    __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(smem + buf * kIterBytes + piece * 1024), 16, 0,
                                     AUX);
  };

  // the first range: this workgroup's static chunk (may be empty)
  int64_t d_begin = chunk * chunk_docs;
  int64_t d_end = d_begin + chunk_docs < static_docs ? d_begin + chunk_docs : static_docs;
  int cur = 0;               // ring slot of iteration it
  bool pre_issued = false;   // kHandoff: this range's first two iterations are in the ring already
  int grab_t = 0;            // kHandoff: the ticket drawn (last wave, lane 0)
  for (int k = 0;; ++k) {
    bool handed = false;                  // kHandoff: the next range was grabbed inside this one
    int64_t nx_begin = 0, nx_end = 0;     // ... and it is [nx_begin, nx_end) (empty: none)
    if (d_begin < d_end) {
      const int nd = (int)(d_end - d_begin);
      const int ngr = (nd + 3) >> 2;
      auto issue_piece = [&](int it, int buf, int jj) { issue_piece_at(d_begin, nd, it, buf, jj); };
      auto issue = [&](int it, int buf) {
        if (!loader || (PROBE == 2 && it >= NBUF)) return;   // PROBE 2 (INVALID): no streaming after the first fill
#pragma unroll
        for (int jj = 0; jj < kPiecesPerWave; ++jj) issue_piece(it, buf, jj);
      };

      float sc[QW];
      float m[QW][2];
#pragma unroll
      for (int q = 0; q < QW; ++q) sc[q] = 0.0f, m[q][0] = m[q][1] = neg_inf();
      int dl_g = 0, dl_min = 0, dl_max = 0;

      const int nit = IPG * ngr;   // (kHandoff: >= 4)
      if constexpr (ARRIVE) {   // the first NBUF-1 iterations (every earlier iteration is done: range barrier)
        for (int j0 = 0; j0 < NBUF - 1 && j0 < nit; ++j0) issue(j0, (int)((gbase + (uint32_t)j0) % NBUF));
      } else if (!pre_issued) {
        cur = 0;
        issue(0, 0);
        if (NBUF >= 3 && nit > 1) issue(1, 1);
        if (NBUF >= 4 && nit > 2) issue(2, 2);
      }
      pre_issued = false;
      const bool grab = kHandoff && task_ctr != nullptr;   // block-uniform
      const int grab_it = nit - 4;                         // (>= 0)
      bool stored = false;   // global stores issued last iteration (they count in vmcnt)
      for (int it = 0; it < nit; ++it) {
        uint64_t ph_a = 0;
        if constexpr (STAMPS) {
          ph_a = __builtin_amdgcn_s_memtime();
          if (ph_t) ph_comp += ph_a - ph_t;
        }
        const uint32_t gi = gbase + (uint32_t)it;   // ARRIVE: global iteration number
        int nslot = 0;
        const uint8_t* buf;
        if constexpr (ARRIVE) {
          if (loader) {   // this iteration's pieces of this wave landed -> publish
            const int ahead = min(NBUF - 2, nit - 1 - it);   // younger iterations already issued
            if (stored || ahead <= 0)
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            else if (ahead == 1)
              asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPiecesPerWave) : "memory");
            else
              asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPiecesPerWave) : "memory");
            if (lane == 0)
              __hip_atomic_store(sync_landed + lwave, (int)(gi + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          lds_wait_all_ge(sync_landed, kLoadWaves, (int)(gi + 1), lane);   // every loader's pieces
          if (loader && it + NBUF - 1 < nit) {   // refill iteration gi-1's slot once every wave is done with it
            lds_wait_all_ge(sync_done, WAVES, (int)gi, lane);
            issue(it + NBUF - 1, (int)((gi + NBUF - 1) % NBUF));
          }
          buf = smem + (gi % NBUF) * kIterBytes;
        } else {
          // it landed; the younger iterations issued (NBUF - 2 at most) stay in flight
          // (a hand-off: the next range's first iteration is the younger one
          // at it = nit - 1; a wait behind stores drains the ring: round 6
          // lab, not draining there measured neutral)
          const bool drain = stored;
          if (NBUF == 4 && it + 2 < nit && !drain)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPiecesPerWave) : "memory");
          else if (NBUF >= 3 && (it + 1 < nit || nx_begin < nx_end) && !drain)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPiecesPerWave) : "memory");
          else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
          asm volatile("" ::: "memory");
        }
        uint64_t ph_b = 0;
        if constexpr (STAMPS) {
          ph_b = __builtin_amdgcn_s_memtime();
          ph_wait += ph_b - ph_a;
        }
        stored = false;
        if constexpr (!ARRIVE) {
          nslot = cur ^ 1;  // 2-deep ring: iteration it+1's slot
          if (NBUF == 2 && !SPREAD && it + 1 < nit) issue(it + 1, nslot);
          if (NBUF == 3 && it + 2 < nit) issue(it + 2, cur == 0 ? 2 : cur - 1);
          if (grab && it + 2 >= nit) {   // the next range's iteration it + 2 - nit (its own issue site:
            if (it + 2 == nit) {         // the common one keeps its hoisted addresses)
              const int o = __builtin_amdgcn_readfirstlane(task_slot[2 * (k & 1)]);
              const int sz = __builtin_amdgcn_readfirstlane(task_slot[2 * (k & 1) + 1]);
              handed = sz >= 0;   // (-1: the own tail slice is drained -- the drained switch)
              nx_begin = static_docs + (int64_t)o;
              nx_end = sz > 0 && nx_begin < n ? (nx_begin + sz < n ? nx_begin + sz : n) : nx_begin;
            }
            if (nx_begin < nx_end && loader) {
#pragma unroll
              for (int jj = 0; jj < kPiecesPerWave; ++jj)
                issue_piece_at(nx_begin, (int)(nx_end - nx_begin), it + 2 - nit, cur == 0 ? 2 : cur - 1, jj);
            }
          }
          if (NBUF == 4 && it + 3 < nit) issue(it + 3, (cur + 3) & 3);
          buf = smem + cur * kIterBytes;
          cur = NBUF == 2 ? (cur ^ 1) : NBUF == 3 ? (cur == 2 ? 0 : cur + 1) : ((cur + 1) & 3);
        }

        const int G = it / IPG, j = it % IPG;
        if (j == 0) {
          int dl4[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            const int v = (4 * G + x < nd) ? doclens[d_begin + 4 * G + x] : 0;
            dl4[x] = v < 0 ? 0 : (v > LD ? LD : v);
          }
          dl_min = min(min(dl4[0], dl4[1]), min(dl4[2], dl4[3]));
          dl_max = max(max(dl4[0], dl4[1]), max(dl4[2], dl4[3]));
          dl_g = g == 0 ? dl4[0] : (g == 1 ? dl4[1] : (g == 2 ? dl4[2] : dl4[3]));
#pragma unroll
          for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
        }
        if constexpr (STAMPS) {
          ph_t = __builtin_amdgcn_s_memtime();
          ph_issue += ph_t - ph_b;
          ++ph_n;
        }
        const bool full = TPI * j + TPI <= dl_min;
        // small shapes (QW <= 2, the B <= 8 launches): a wave's padded query
        // slots (queries >= B) skip their MFMAs -- at B = 5 on the 4 x 2 shape
        // 3 of 8 -- which at these batches, HBM- and power-bound, buy clock;
        // the live queries' chains are the same instructions in the same order
        // (the 4 x 4 shape too, B = 9-16; never the 8 x 4 shape of large batches)
        constexpr bool kSkipShape = QW <= 2 || (QW == 4 && WAVES == 4);
        const int nlive = kSkipShape ? max(0, min(QW, B - (qg * QPB + wave * QW))) : QW;
        if constexpr (kScanQSkip && kSkipShape && !SPREAD && MORDER == 0) {
          // the first nlive query slots of the wave, as arrays of their own
          auto live = [&](auto nq) {
            constexpr int L = decltype(nq)::value;
            auto& q = reinterpret_cast<const bf16x8(&)[L][2][4]>(qf[0]);
            auto& mm = reinterpret_cast<float(&)[L][2]>(m[0]);
            if (full)
              iter4_full<L, D, NT, NoTileHook, PROBE>(buf, lane, q, mm);
            else if (TPI * j < dl_max)
              iter4_ragged<L, NT>(buf, lane, j, dl_g, dl_max, q, mm);
          };
          if (nlive == QW) live(std::integral_constant<int, QW>{});
          else if (QW >= 4 && nlive == 3) live(std::integral_constant<int, (QW >= 4 ? 3 : 1)>{});
          else if (QW >= 3 && nlive == 2) live(std::integral_constant<int, (QW >= 3 ? 2 : 1)>{});
          else if (QW >= 2 && nlive == 1) live(std::integral_constant<int, 1>{});
        } else {
        if constexpr (SPREAD && NBUF == 2) {
          static_assert(NT >= kPiecesPerWave, "one piece per tile");
          if (it + 1 < nit && !full) issue(it + 1, nslot);   // ragged or empty iteration: all at once
        }
        if (full) {
          if constexpr (SPREAD && NBUF == 2) {
            if (it + 1 < nit)
              iter4_full<QW, D, NT>(buf, lane, qf, m, [&](int t) {
                if (t < kPiecesPerWave) issue_piece(it + 1, nslot, t);
              });
            else
              iter4_full<QW, D, NT>(buf, lane, qf, m);
          } else {
            if constexpr (MORDER == 1)
              iter4_full_kmajor<QW, NT>(buf, lane, qf, m);
            else
              iter4_full<QW, D, NT, NoTileHook, PROBE>(buf, lane, qf, m);
          }
        } else if (TPI * j < dl_max)
          iter4_ragged<QW, NT>(buf, lane, j, dl_g, dl_max, qf, m);
        }
        if (j == IPG - 1) {
          // doc 4G+g's score in every lane of group g; lane c of the 64-doc block
          // register keeps doc group c, so lane (c, g) holds doc 4c+g of the block
#pragma unroll
          for (int q = 0; q < QW; ++q) {
            const float v = dpp_row_sum16((c < lq ? m[q][0] : 0.0f) + (16 + c < lq ? m[q][1] : 0.0f));
            sc[q] = (c == (G & 15)) ? v : sc[q];
          }
          if ((G & 15) == 15 || G == ngr - 1) {
            const int dd = 64 * (G >> 4) + 4 * c + g;
            if constexpr (FK > 0) {
#pragma unroll
              for (int q = 0; q < QW; ++q) {
                if (qg * QPB + wave * QW + q >= B) continue;   // wave-uniform
                const uint32_t loc = (uint32_t)(d_begin + dd);
                const uint64_t key = (c <= (G & 15) && dd < nd) ? ((uint64_t)f2u(sc[q]) << 32) | (uint32_t)~loc : 0ull;
                topk_offer<FK>(cand + q * FK, tk_state + q * kFusedStateBytes, topk_k, key, lane);
              }
            } else {
#pragma unroll
              for (int q = 0; q < QW; ++q) {
                const int qi = qg * QPB + wave * QW + q;
                if (qi < B && c <= (G & 15) && dd < nd) out[(size_t)qi * ld_out + d_begin + dd] = sc[q];
              }
              stored = true;
              if constexpr (BMK) {
                const int64_t d0 = d_begin + 64 * (G >> 4);   // the group's first doc
                const int64_t bb = ((d0 >> 6) + 1) << 6;       // the next block boundary
                const bool valid = c <= (G & 15) && dd < nd;
#pragma unroll
                for (int q = 0; q < QW; ++q) {
                  const int qi = qg * QPB + wave * QW + q;
                  if (qi >= B) continue;   // wave-uniform
                  const uint32_t v = valid ? f2u(sc[q]) : 0u;
                  const uint32_t ulo = wave_max_u32(d_begin + dd < bb ? v : 0u);
                  const uint32_t uhi = wave_max_u32(d_begin + dd >= bb ? v : 0u);
                  if (lane == 0) {
                    uint32_t* br = bmk + (size_t)qi * bmk_ld;
                    uint32_t* sr = sbk + (size_t)qi * sbk_ld;
                    const int64_t b0 = d0 >> 6, s0 = d0 >> 8;
                    if (ulo != 0u) atomicMax(br + b0, ulo);
                    if (uhi != 0u) atomicMax(br + b0 + 1, uhi);
                    if ((bb & 255) == 0) {   // the block boundary is a superblock boundary
                      if (ulo != 0u) atomicMax(sr + s0, ulo);
                      if (uhi != 0u) atomicMax(sr + s0 + 1, uhi);
                    } else if ((ulo | uhi) != 0u) {
                      atomicMax(sr + s0, max(ulo, uhi));
                    }
                  }
                }
              }
            }
          }
        }
        if constexpr (ARRIVE) {   // this wave's reads of the slot are issued (LDS serves a wave in order)
          asm volatile("" ::: "memory");
          if (lane == 0) __hip_atomic_store(sync_done + wave, (int)(gi + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        // the hand-off's grab by the last wave (never a loader: waiting for
        // its atomic drains no ring; a wave-uniform branch, so no other wave
        // executes that wait): the ticket at grab_it, the task in LDS before
        // that wave's barrier of iteration nit - 2
        if (grab && wave == WAVES - 1 && (it == grab_it || it == grab_it + 1)) {
          if (it == grab_it) {
            if (lane == 0) grab_t = atomicAdd(task_ctr + tail_slices * qg + (bid & 7) % tail_slices, 1);
          } else {
            if (lane == 0)
              task_from_ticket(grab_t, tail_slices, bid & 7, task_docs, (int)(n - static_docs), nwg / nq_groups,
                               task_slot + 2 * (k & 1));
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          }
        }
      }
      if constexpr (ARRIVE) gbase += (uint32_t)nit;
    }
    if (task_ctr == nullptr) break;
    if (kHandoff && handed) {   // the next range was grabbed and its first two iterations issued above
      if (nx_begin >= nx_end) break;
      d_begin = nx_begin;
      d_end = nx_end;
      pre_issued = true;   // (cur is its first slot)
      continue;
    }
    // next dynamic task; the barrier also retires every wave's reads of the
    // ring before the next range refills it (two slots: a slow wave may still
    // read slot k&1 while thread 0 fills slot (k+1)&1).
    if (threadIdx.x == 0)
      next_task_sliced(task_ctr + tail_slices * qg, tail_slices, bid & 7, task_docs, (int)(n - static_docs),
                       nwg / nq_groups, task_slot + 2 * (k & 1));
    __syncthreads();
    const int o = __builtin_amdgcn_readfirstlane(task_slot[2 * (k & 1)]);
    const int sz = __builtin_amdgcn_readfirstlane(task_slot[2 * (k & 1) + 1]);
    d_begin = static_docs + (int64_t)o;
    if (sz <= 0 || d_begin >= n) break;
    d_end = d_begin + sz < n ? d_begin + sz : n;
  }
  if constexpr (FK > 0) {  // this workgroup's best topk_k per query; key 0 pads
#pragma unroll 1
    for (int q = 0; q < QW; ++q) {
      const int qi = qg * QPB + wave * QW + q;
      if (qi >= B) continue;
      topk_flush(cand + q * FK, tk_state + q * kFusedStateBytes, topk_k,
                 part + ((size_t)qi * nslots + (size_t)chunk) * topk_k, lane);
    }
  }
  if constexpr (!STAMPS) {
    if (stamps != nullptr) {   // block-uniform
      __syncthreads();
      if (threadIdx.x == 0) clock_probe(stamps, true);
    }
  }
  if constexpr (STAMPS) {
    if (ph_t) ph_comp += __builtin_amdgcn_s_memtime() - ph_t;
    if (threadIdx.x == 0) {
      uint64_t* st = stamps + 4 * (size_t)bid;
      st[0] = r_start;
      st[1] = __builtin_amdgcn_s_memrealtime();
      st[2] = t_start;
      st[3] = __builtin_amdgcn_s_memtime();
    }
    if (lane == 0) {  // phase sums: rows 16384 + 8 * bid + wave of the [rows][4] stamp buffer
      uint64_t* ph = stamps + 4 * ((size_t)16384 + 8 * (size_t)bid + wave);
      ph[0] = ph_wait;
      ph[1] = ph_issue;
      ph[2] = ph_comp;
      ph[3] = ph_n;
    }
  }
}

// ---------------------------------------------------------------------------
// Small-batch scan (B <= 2 per query group): HBM-bound, so no LDS staging —
// every wave owns a contiguous doc range and streams each doc (32 KiB, 128 B
// per lane per row tile) straight into VGPRs; 8 waves per CU keep ~256 KiB in
// flight per CU.  Same tile order, masking and epilogue as doc16, so scores are
// bit-identical to the LDS kernel's and the rerank kernel's.
// ---------------------------------------------------------------------------
// LONG: docs of ld = 256 / 512 / 1024 token slots, scored 128 tokens at a time
// with the row maxima carried across the blocks (same tile order: the bits of
// a doc of <= 128 tokens do not depend on ld).
template <int QW, bool LONG = false>
__global__ __launch_bounds__(256, 2) void maxsim_scan_direct_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out,
    int64_t chunk_docs, int ld = kLd) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t lin = (int64_t)blockIdx.x * 4 + wave;      // one doc chunk per wave
  const int qg = (int)(lin % nq_groups);
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;  // uniform over the wave; no block-level sync below
  const int nd = (int)(d_end - d_begin);

  bf16x8 qf[QW][2][4];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag16(Q, qg * QW + q, B, lq, lane, qf[q]);
  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;

  for (int i = 0; i < nd; ++i) {
    const int lmax = LONG ? ld : kLd;
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > lmax ? lmax : dl);
    float m[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    for (int blk = 0; blk == 0 || (LONG && kLd * blk < dl); ++blk) {   // one block unless LONG
      const int dlb = dl - kLd * blk;
      const uint8_t* dbase = tokens + (size_t)(d_begin + i) * (size_t)lmax * kRowBytes + (size_t)blk * kDocBytes;
      bf16x8 af[kLd / 16][4];
#pragma unroll
      for (int rt = 0; rt < kLd / 16; ++rt)
        if (16 * rt < dlb) gbl_afrag16(dbase, rt, lane, af[rt]);
#pragma unroll
      for (int rt = 0; rt < kLd / 16; ++rt) {
        if (16 * rt < dlb) {
          const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
          tile16<QW>(af[rt], qf, init, m);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = qg * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Streaming small-batch scan (B <= 2, the production bf16 path; variants
// 14-16): HBM-bound, so the kernel is built around the stream.  Every wave
// owns a contiguous doc range and 1-2 queries (fragments in VGPRs), as the
// direct scan below, but the docs' 16-row tiles arrive by LDS-DMA -- 1 KiB
// per wave-instruction, 4 per tile, with the non-temporal policy (AUX = 2:
// the bytes are read once) -- into a private ring of 8 tile slots per wave
// (32 KiB; 128 KiB per 4-wave workgroup, one workgroup per CU).  Only the
// tiles that hold tokens are streamed: the wave walks the sequence of (doc,
// tile < ceil(doclen / 16)) pairs of its range with an issue cursor 8 tiles
// ahead of the compute cursor, tile k in slot k % 8; after tile k is read
// from its slot, tile k + 8 is issued into it, so the wait for the oldest
// tile is a constant vmcnt(28) until the issue cursor runs out.  Same tiles,
// masks, max order and epilogue as the direct scan: bit-identical scores.
// Lab (same process, 1M docs): B=1 5.201 -> 4.704 ms (6.30 -> 6.97 TB/s),
// B=2 5.262 -> 4.711, 125k B=1 0.656 -> 0.587; the same kernel without the
// nt policy runs at the direct scan's rate (profiles/r03ae_*).
// ---------------------------------------------------------------------------
constexpr int kStreamSlots = 8;                    // tile slots per wave ring
// A doc length through the scalar unit (s_load): a vector load of it would be
// counted by vmcnt, and waiting for it would drain the LDS-DMA ring.
__device__ __forceinline__ int sload_len(const int32_t* p) {
  int v;
  asm volatile("s_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v) : "s"(p) : "memory");
  return v;
}
// TW2 (lab): two tiles of one doc per wait, as the MXFP8 streaming scan;
// neutral here (1M B=1 4.722 vs 4.708 ms, profiles/r03z_lab_bf16_tw2.log).
// bm (nullable): the block maxima of the block-max top-k (block_max_kernel's
// keys: max of f2u(score) over each 64-doc block) folded into the epilogue --
// a wave writes its scores 64 docs at a time, which with chunks of a multiple
// of 64 docs (the launcher's rounding) are exactly one block: one wave max and
// one store per block, and the separate block-max launch is skipped.
// PF (lab): the next tile's fragments are read from the ring while this
// tile's MFMAs run (the LDS read latency off the critical path).
template <int QW, int AUX, int WAVES = 4, int SLOTS = kStreamSlots, bool TW2 = false, bool PF = false>
__global__ __launch_bounds__(WAVES * 64, 1) void maxsim_scan_stream_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out, int64_t chunk_docs,
    int ld, uint32_t* __restrict__ bm, int64_t bm_ld, uint32_t* __restrict__ sb, int64_t sb_ld) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[WAVES * SLOTS * 4096];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t lin = (int64_t)blockIdx.x * WAVES + wave;      // one doc chunk per wave
  const int qg = (int)(lin % nq_groups);
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;  // uniform over the wave; no block-level sync below
  const int nd = (int)(d_end - d_begin);
  uint8_t* ring = smem + wave * (SLOTS * 4096);
  const size_t doc_bytes = (size_t)ld * kRowBytes;
  const int32_t* dls = doclens + d_begin;
  // 32-bit cursor arithmetic keeps every comparison on the scalar unit (a
  // 64-bit compare goes to the VALU, the loop turns "divergent" and hipcc
  // loads the lengths through the vector path, whose vmcnt(0) would drain
  // the ring at every doc)
  auto ntiles = [&](int d) -> int {
    int dl = sload_len(dls + d);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    return (dl + 15) >> 4;
  };
  // piece q of a tile = its rows 4q .. 4q + 3; lane l writes LDS slot (row
  // 4q + (l >> 4), position l & 15), so it fetches the logical 16-B slot
  // stored there: position ^ swz16(row) (the layout lds_afrag16 reads)
  uint32_t src_off[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int t = 4 * q + g;
    src_off[q] = (uint32_t)(t * kRowBytes + 16 * (c ^ swz16(t)));
  }
  // issue cursor: the next (doc, tile) to stream, and tiles issued so far
  int idoc = 0;
  int itile = 0, intl = ntiles(0);
  while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
  int issued = 0;
  const uint8_t* tbase = tokens + (size_t)d_begin * doc_bytes;
  auto issue_next = [&]() {
    if (idoc >= nd) return;
    const uint8_t* base = tbase + (size_t)idoc * doc_bytes + (size_t)itile * 16 * kRowBytes;
    uint8_t* dst = ring + (issued & (SLOTS - 1)) * 4096;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + src_off[q]), (lds_void_t*)(dst + q * 1024), 16, 0, AUX);
    ++issued;
    if (++itile >= intl) {
      itile = 0;
      intl = 0;
      while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
    }
  };
  bf16x8 qf[QW][2][4];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag16(Q, qg * QW + q, B, lq, lane, qf[q]);
  float sc[QW];
  uint32_t smax[QW];   // running superblock key (bm != nullptr)
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f, smax[q] = 0u;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the query fragments: out of the ring's count
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) issue_next();

  int consumed = 0;
  // PF: the ring's next tile, read ahead (c: this lane's row of the tile)
  auto read_tile = [&](bf16x8 (&a)[4]) {
    if (issued - consumed >= SLOTS)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SLOTS - 1)) : "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint8_t* row = ring + (consumed & (SLOTS - 1)) * 4096 + c * kRowBytes;
    const int sw = swz16(c);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) a[s4] = *reinterpret_cast<const bf16x8*>(row + 16 * ((4 * g + s4) ^ sw));
  };
  bf16x8 a_cur[4];
  if (PF && issued > 0) {
    read_tile(a_cur);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    ++consumed;
    issue_next();
  }
  for (int i = 0; i < nd; ++i) {
    int dl = sload_len(dls + i);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    const int nt = (dl + 15) >> 4;
    float m[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    for (int t = 0; t < nt; ++t) {
      if (PF) {
        bf16x8 a_nx[4];
        const bool more = consumed < issued;   // the ring holds a later tile (issued ahead of every read)
        if (more) read_tile(a_nx);
        const f32x4 init = (dl >= 16 * t + 16) ? f32x4{} : row_mask_init16(16 * t + 4 * g, dl);
        tile16<QW>(a_cur, qf, init, m);
        if (more) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // its slot is read: refill it
          ++consumed;
          issue_next();
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) a_cur[s4] = a_nx[s4];
        }
        continue;
      }
      if (TW2 && t + 1 < nt) {
        if (issued - consumed >= SLOTS)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SLOTS - 2)) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        bf16x8 a2[2][4];
        const int sw = swz16(c);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint8_t* row = ring + ((consumed + u) & (SLOTS - 1)) * 4096 + c * kRowBytes;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            a2[u][s4] = *reinterpret_cast<const bf16x8*>(row + 16 * ((4 * g + s4) ^ sw));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // both slots read: refill them
        consumed += 2;
        issue_next();
        issue_next();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int tt = t + u;
          const f32x4 init = (dl >= 16 * tt + 16) ? f32x4{} : row_mask_init16(16 * tt + 4 * g, dl);
          tile16<QW>(a2[u], qf, init, m);
        }
        ++t;
        continue;
      }
      // 8 tiles in flight: the oldest 4 pieces are this tile's (later loads
      // and stores only make the wait stricter); fewer: the stream is ending
      if (issued - consumed >= SLOTS)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SLOTS - 1)) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bf16x8 a[4];
      const uint8_t* row = ring + (consumed & (SLOTS - 1)) * 4096 + c * kRowBytes;
      const int sw = swz16(c);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) a[s4] = *reinterpret_cast<const bf16x8*>(row + 16 * ((4 * g + s4) ^ sw));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot is read: refill it
      ++consumed;
      issue_next();
      const f32x4 init = (dl >= 16 * t + 16) ? f32x4{} : row_mask_init16(16 * t + 4 * g, dl);
      tile16<QW>(a, qf, init, m);
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = qg * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
        if (bm != nullptr) {
          uint32_t u = lane < cnt ? f2u(sc[q]) : 0u;
#pragma unroll
          for (int off = 1; off < 64; off <<= 1) u = max(u, (uint32_t)__shfl_xor((int)u, off));
          const int64_t gi = (d_begin + i0) >> 6;   // this 64-doc block; chunks are whole superblocks
          smax[q] = max(smax[q], u);
          if (lane == 0 && qi < B) bm[(size_t)qi * bm_ld + gi] = u;
          if ((gi & 3) == 3 || i == nd - 1) {
            if (lane == 0 && qi < B) sb[(size_t)qi * sb_ld + (gi >> 2)] = smax[q];
            smax[q] = 0u;
          }
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Paired streaming scan (mid batches, B = 3..8; lab variants 22-24): the B <= 2
// streaming scan's LDS-DMA ring, SHARED by the 2 waves of a 128-thread
// workgroup, each wave scoring its own QW queries on every tile -- so the
// corpus is streamed once per 2*QW queries while the SIMD interleaves two
// waves' MFMA chains (one wave per SIMD with all of a mid batch's queries
// cannot hide them: lab variants 18/19).  Both waves walk the same (doc,
// tile) sequence; wave h fetches pieces 2h, 2h + 1 of each tile (rows 8h ..
// 8h + 7), waits for its own pieces, and an s_barrier publishes the whole tile
// to both.  Tile k lives in slot k % SLOTS; after the barrier of tile t both
// waves have finished reading tile t - 1 (each reads a tile completely before
// computing it), so tile t + SLOTS - 1 is issued into that slot.  Same tiles,
// masks, max order and epilogue as the streaming scan: bit-identical scores.
// Four such workgroups per CU (32 KiB of LDS each) = 2 waves per SIMD.
template <int QW, int AUX, int SLOTS = kStreamSlots>
__global__ __launch_bounds__(128, 2) void maxsim_scan_pair_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out, int64_t chunk_docs,
    int ld) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring[SLOTS * 4096];
  const int lane = threadIdx.x & 63;
  const int h = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  constexpr int QPB = 2 * QW;
  const int nq_groups = (B + QPB - 1) / QPB;
  const int qg = (int)(blockIdx.x % nq_groups);
  const int64_t chunk = blockIdx.x / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;  // workgroup-uniform
  const int nd = (int)(d_end - d_begin);
  const size_t doc_bytes = (size_t)ld * kRowBytes;
  const int32_t* dls = doclens + d_begin;
  auto ntiles = [&](int d) -> int {
    int dl = sload_len(dls + d);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    return (dl + 15) >> 4;
  };
  uint32_t src_off[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int t = 4 * (2 * h + j) + g;
    src_off[j] = (uint32_t)(t * kRowBytes + 16 * (c ^ swz16(t)));
  }
  int idoc = 0;
  int itile = 0, intl = ntiles(0);
  while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
  int issued = 0;
  const uint8_t* tbase = tokens + (size_t)d_begin * doc_bytes;
  auto issue_next = [&]() {
    if (idoc >= nd) return;
    const uint8_t* base = tbase + (size_t)idoc * doc_bytes + (size_t)itile * 16 * kRowBytes;
    uint8_t* dst = ring + (issued % SLOTS) * 4096;
#pragma unroll
    for (int j = 0; j < 2; ++j)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(base + src_off[j]), (lds_void_t*)(dst + (2 * h + j) * 1024), 16,
                                       0, AUX);
    ++issued;
    if (++itile >= intl) {
      itile = 0;
      intl = 0;
      while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
    }
  };
  bf16x8 qf[QW][2][4];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag16(Q, qg * QPB + h * QW + q, B, lq, lane, qf[q]);
  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the query fragments: out of the ring's count
#pragma unroll
  for (int k = 0; k < SLOTS - 1; ++k) issue_next();
  int consumed = 0;
  for (int i = 0; i < nd; ++i) {
    int dl = sload_len(dls + i);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    const int nt = (dl + 15) >> 4;
    float m[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    for (int t = 0; t < nt; ++t) {
      // SLOTS - 1 tiles in flight: this tile's 2 pieces are the oldest
      if (issued - consumed >= SLOTS - 1)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (SLOTS - 2)) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();   // both waves' pieces of the tile have landed
      bf16x8 a[4];
      const uint8_t* row = ring + (consumed % SLOTS) * 4096 + c * kRowBytes;
      const int sw = swz16(c);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) a[s4] = *reinterpret_cast<const bf16x8*>(row + 16 * ((4 * g + s4) ^ sw));
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      ++consumed;
      issue_next();   // into the slot of tile consumed - 2, read by both waves before this barrier
      const f32x4 init = (dl >= 16 * t + 16) ? f32x4{} : row_mask_init16(16 * t + 4 * g, dl);
      tile16<QW>(a, qf, init, m);
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = qg * QPB + h * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ===========================================================================
// MXFP8 path (config 5): doc and query tokens as e4m3 bytes with one E8M0
// power-of-two scale per token per 64 dims, scored on the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate on gfx950).
// Operand map (verified on MI355X by tools/probes/mx_probe{2,3,4}.hip):
//   lane l (c = l&15, g = l>>4) holds 32 bytes = K range [32g, 32g+32) of
//   row/column c; lane c + 16h (h = 0, 1) supplies byte 0 of its scale VGPR
//   for K range [64h, 64h+64) of row/column c; lanes 32..63's scales are unused.
// One MFMA covers the whole 128-dim contraction of a 16x16 token tile.
// ===========================================================================
typedef __attribute__((ext_vector_type(8))) int i32x8;
constexpr int kF8DocBytes = kLd * kDim;            // 16 KiB of e4m3 per doc
constexpr int kF8ScaleBytes = kLd * 2;             // 256 B of E8M0 per doc
constexpr int kF8Stage = kF8DocBytes + kF8ScaleBytes;

// LDS image of a doc: 128 rows x 8 slots of 16 B, slot s of row t stored at
// s ^ swz8(t) (conflict-free for the two ds_read_b128 of a fragment), then the
// 256 scale bytes.
__device__ __forceinline__ int swz8(int t) { return (((t >> 1) & 1) << 2) | ((t >> 2) & 1); }

// E8M0 exponent for a half-row with max magnitude m: smallest e with m <= 448 * 2^e.
__device__ __forceinline__ int mx_exp(float m) {
  if (!(m > 0.0f)) return 0;
  int p;
  const float f = frexpf(m, &p);  // m = f * 2^p, f in [0.5, 1); 448 = 0.875 * 2^9
  int e = (f <= 0.875f) ? p - 9 : p - 8;
  return e < -127 ? -127 : (e > 127 ? 127 : e);
}

template <typename T>
__device__ __forceinline__ float to_f32(T v);
template <>
__device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f32<uint16_t>(uint16_t v) { return __uint_as_float((uint32_t)v << 16); }

template <typename T>
__device__ __forceinline__ void quantize_row(const T* __restrict__ x, int64_t row, int lane, uint8_t* __restrict__ q,
                                             uint8_t* __restrict__ sc);

// One wave per 128-value row: bytes q[row][128] (e4m3, RNE) and scales[row][2].
template <typename T>
__global__ __launch_bounds__(256) void quantize_mxfp8_kernel(const T* __restrict__ x, int64_t rows,
                                                             uint8_t* __restrict__ q, uint8_t* __restrict__ sc) {
  const int lane = threadIdx.x & 63;
  // grid-stride over rows: a dispatch's grid is a 32-bit work-item count
  for (int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); row < rows; row += (int64_t)gridDim.x * 4)
    quantize_row<T>(x, row, lane, q, sc);
}

template <typename T>
__device__ __forceinline__ void quantize_row(const T* __restrict__ x, int64_t row, int lane, uint8_t* __restrict__ q,
                                             uint8_t* __restrict__ sc) {
  const float a = to_f32<T>(x[row * kDim + 2 * lane]);
  const float b = to_f32<T>(x[row * kDim + 2 * lane + 1]);
  float m = fmaxf(fabsf(a), fabsf(b));
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0xB1, 0xF, 0xF, true)));
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x4E, 0xF, 0xF, true)));
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x141, 0xF, 0xF, true)));
  m = fmaxf(m, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(m), 0x140, 0xF, 0xF, true)));
  m = fold16_max(m);  // max over the 32 lanes of this half (dims 64h .. 64h+63)
  const int e = mx_exp(m);
  const int packed = __builtin_amdgcn_cvt_pk_fp8_f32(ldexpf(a, -e), ldexpf(b, -e), 0, false);
  *reinterpret_cast<uint16_t*>(q + row * kDim + 2 * lane) = (uint16_t)(packed & 0xffff);
  if ((lane & 31) == 0) sc[row * 2 + (lane >> 5)] = (uint8_t)(127 + e);
}

// Query fragments for the f8 tiling: 32 bytes + the scale byte of half g&1.
__device__ __forceinline__ void load_qfrag_f8(const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int qi,
                                              int B, int lq, int lane, i32x8 (&qa)[2], int (&qs)[2]) {
  const int c = lane & 15, g = lane >> 4;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    const int tok = 16 * ct + c;
    const bool ok = (qi < B) && (tok < lq);
    const size_t row = ok ? (size_t)qi * lq + tok : 0;
    const i32x8* src = reinterpret_cast<const i32x8*>(Qb + row * kDim + 32 * g);
    qa[ct] = ok ? *src : i32x8{0, 0, 0, 0, 0, 0, 0, 0};
    qs[ct] = ok ? (int)Qs[row * 2 + (g & 1)] : 127;
  }
}

__device__ __forceinline__ void lds_afrag_f8(const uint8_t* buf, int rt, int lane, i32x8& a, int& as) {
  const int c = lane & 15, g = lane >> 4;
  const int t = 16 * rt + c;
  const uint8_t* row = buf + t * kDim;
  const int sw = swz8(t);
  const u32x4 lo = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g) ^ sw));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g + 1) ^ sw));
  a = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  as = buf[kF8DocBytes + t * 2 + (g & 1)];
}

__device__ __forceinline__ void gbl_afrag_f8(const uint8_t* doc, const uint8_t* dsc, int rt, int lane, i32x8& a,
                                             int& as) {
  const int c = lane & 15, g = lane >> 4;
  const int t = 16 * rt + c;
  a = *reinterpret_cast<const i32x8*>(doc + t * kDim + 32 * g);
  as = dsc[t * 2 + (g & 1)];
}

template <int QW>
__device__ __forceinline__ void tile_f8(const i32x8& a, int as, const i32x8 (&qa)[QW][2], const int (&qs)[QW][2],
                                        const f32x4& init, float (&m)[QW][2]) {
#pragma unroll
  for (int q = 0; q < QW; ++q) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const f32x4 acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, qa[q][ct], init, 0, 0, 0, as, 0, qs[q][ct]);
      m[q][ct] = fmaxf(fmaxf(m[q][ct], fmaxf(acc[0], acc[1])), fmaxf(acc[2], acc[3]));
    }
  }
}

// Query scale bytes of the doc-interleaved f8 scan: one VGPR per (query,
// column tile) (PQS = false), or four packed per VGPR with the MFMA's op_sel
// picking the byte (PQS = true: 12 fewer VGPRs at 8 queries per wave).  i =
// 2 * query + column tile; a compile-time constant once the loops unroll.
template <int QW, bool PQS>
constexpr int kQsRegs = PQS ? (2 * QW + 3) / 4 : 2 * QW;

template <bool PQS>
__device__ __forceinline__ f32x4 mfma_f8q(const i32x8& a, int as, const i32x8& b, const int* qsv, int i,
                                          const f32x4& c) {
  if constexpr (!PQS) {
    return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, as, 0, qsv[i]);
  } else {
    const int v = qsv[i >> 2];
    switch (i & 3) {
      case 0: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, as, 0, v);
      case 1: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, as, 1, v);
      case 2: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, as, 2, v);
      default: return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, as, 3, v);
    }
  }
}

template <int QW, bool PQS>
__device__ __forceinline__ void pack_qscales(const int (&qs)[QW][2], int (&qsv)[kQsRegs<QW, PQS>]) {
#pragma unroll
  for (int r = 0; r < kQsRegs<QW, PQS>; ++r) qsv[r] = 0;
#pragma unroll
  for (int i = 0; i < 2 * QW; ++i) {
    const int v = qs[i >> 1][i & 1];
    if constexpr (PQS) qsv[i >> 2] |= (v & 0xff) << (8 * (i & 3));
    else qsv[i] = v;
  }
}

template <int QW, bool PQS>
__device__ __forceinline__ void tile_f8q(const i32x8& a, int as, const i32x8 (&qa)[QW][2], const int* qsv,
                                         const f32x4& init, float (&m)[QW][2]) {
#pragma unroll
  for (int q = 0; q < QW; ++q) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const f32x4 acc = mfma_f8q<PQS>(a, as, qa[q][ct], qsv, 2 * q + ct, init);
      m[q][ct] = fmaxf(fmaxf(m[q][ct], fmaxf(acc[0], acc[1])), fmaxf(acc[2], acc[3]));
    }
  }
}

// Whole (query, doc) pass of the f8 tiling; FRAG(rt, a, as) loads row tile rt.
template <int QW, typename Frag>
__device__ __forceinline__ void doc_f8(Frag frag, const i32x8 (&qa)[QW][2], const int (&qs)[QW][2], int dl, int lane,
                                       float (&m)[QW][2]) {
  const int g = lane >> 4;
#pragma unroll
  for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
  if (dl >= kLd) {
    i32x8 a0, a1;
    int s0, s1;
    frag(0, a0, s0);
#pragma unroll
    for (int rt = 0; rt < kLd / 16; rt += 2) {
      frag(rt + 1, a1, s1);
      tile_f8<QW>(a0, s0, qa, qs, f32x4{}, m);
      if (rt + 2 < kLd / 16) frag(rt + 2, a0, s0);
      tile_f8<QW>(a1, s1, qa, qs, f32x4{}, m);
    }
    return;
  }
  const int nrt = (dl + 15) >> 4;
  for (int rt = 0; rt < nrt; ++rt) {
    i32x8 a;
    int as;
    frag(rt, a, as);
    const f32x4 init = (dl >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dl);
    tile_f8<QW>(a, as, qa, qs, init, m);
  }
}

// LDS-staged f8 scan: 8 waves x 8 queries = 64 queries per workgroup.
template <int WAVES, int QW>
__global__ __launch_bounds__(WAVES * 64, 2) void maxsim_scan_f8_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int B, int lq,
    float* __restrict__ out, int64_t ld_out, int64_t chunk_docs) {
  constexpr int QPB = WAVES * QW;
  constexpr int kPieces = kF8DocBytes / 1024;
  constexpr int kPiecesPerWave = kPieces / WAVES;
  static_assert(kPieces % WAVES == 0, "pieces must split evenly over waves");
  __shared__ __attribute__((aligned(1024))) uint8_t smem[2 * kF8Stage + 256];

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nq_groups = (B + QPB - 1) / QPB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, idx = bid >> 3, qd = nwg >> 3, rm = nwg & 7;
  const int lin = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + idx;
  const int g = lin % nq_groups;
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;
  const int nd = (int)(d_end - d_begin);

  i32x8 qa[QW][2];
  int qs[QW][2];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag_f8(Qb, Qs, g * QPB + wave * QW + q, B, lq, lane, qa[q], qs[q]);

  uint32_t src_off[kPiecesPerWave];
#pragma unroll
  for (int j = 0; j < kPiecesPerWave; ++j) {
    const int piece = wave * kPiecesPerWave + j;
    const int t = 8 * piece + (lane >> 3);
    src_off[j] = t * kDim + 16 * ((lane & 7) ^ swz8(t));
  }
  auto issue = [&](int i, int buf) {
    const uint8_t* dbase = tokens + (size_t)(d_begin + i) * kF8DocBytes;
    uint8_t* sbuf = smem + buf * kF8Stage;
#pragma unroll
    for (int j = 0; j < kPiecesPerWave; ++j) {
      const int piece = wave * kPiecesPerWave + j;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(dbase + src_off[j]), (lds_void_t*)(sbuf + piece * 1024), 16, 0,
                                       0);
    }
    if (wave == 0)  // the doc's 256 scale bytes: one dword per lane
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(tscales + (size_t)(d_begin + i) * kF8ScaleBytes + 4 * lane),
                                       (lds_void_t*)(sbuf + kF8DocBytes), 4, 0, 0);
  };

  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;

  issue(0, 0);
  for (int i = 0; i < nd; ++i) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i + 1 < nd) issue(i + 1, (i + 1) & 1);
    const uint8_t* buf = smem + (i & 1) * kF8Stage;
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > kLd ? kLd : dl);
    float m[QW][2];
    doc_f8<QW>([&](int rt, i32x8& a, int& as) { lds_afrag_f8(buf, rt, lane, a, as); }, qa, qs, dl, lane, m);
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = g * QPB + wave * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// Doc-interleaved f8 scan (the production B > 8 MXFP8 path; same design as
// maxsim_scan16x4_kernel): each iteration stages TPI tokens of 4 docs (TPI x
// 512 B of e4m3 + TPI x 8 B of scales) into an LDS ring; row tile t holds
// tokens 4t..4t+3 of docs 0..3 in rows 4g..4g+3, so output lane group g is doc
// g and the epilogue is one 16-lane DPP sum per query per 4 docs.  Image: row
// R = TPI*doc + token, 8 slots of 16 B with slot s at s ^ swz_f8(R) =
// s ^ (doc << 1 | (R >> 1) & 1) (the 8 rows of one parity a lane group reads
// get 8 distinct slots); then the 2 scale bytes of every row at
// 4 * TPI * 128 + 2R.
template <int TPI>
__device__ __forceinline__ int swz_f8(int R) { return (((R / TPI) & 3) << 1) | ((R >> 1) & 1); }

template <int TPI = 32>
__device__ __forceinline__ void lds_afrag_f8x4(const uint8_t* buf, int t, int lane, i32x8& a, int& as) {
  const int c = lane & 15, g = lane >> 4;
  const int R = TPI * (c >> 2) + 4 * t + (c & 3);
  const uint8_t* row = buf + R * kDim;
  const int sw = swz_f8<TPI>(R);
  const u32x4 lo = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g) ^ sw));
  const u32x4 hi = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g + 1) ^ sw));
  a = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  as = buf[4 * TPI * kDim + R * 2 + (g & 1)];
}

// PF (prefetch-after-first-MFMA): tile t+1's LDS reads issue after tile t's
// first MFMA, so the lgkmcnt wait that tile t's fragments need does not also
// wait for them (hipcc waits lgkmcnt(0) there), and the fold of chain k-D is
// fenced after MFMA k (hipcc otherwise hoists the fold above it and pads the
// MFMA -> VALU hazard with s_nop).
// PROBE (lab only, INVALID scores): 1 = no per-MFMA fold (each accumulator
// chains its MFMAs and is folded once per iteration), to bound the fold's cost.
template <int QW, int D, int TPI = 32, bool PF = false, bool PQS = false, int PROBE = 0>
__device__ __forceinline__ void iter_f8x4_full(const uint8_t* buf, int lane, const i32x8 (&qa)[QW][2],
                                               const int* qsv, float (&m)[QW][2]) {
  constexpr int NC = 2 * QW;
  static_assert(D >= 1 && NC % (D + 1) == 0, "ring slot of chain k must be k % (D+1) across tiles");
  constexpr int NT = TPI / 4;
  i32x8 a[2];
  int as[2];
  f32x4 acc[D + 1];
  lds_afrag_f8x4<TPI>(buf, 0, lane, a[0], as[0]);
  auto fold = [&](int k) {  // row max of chain k (k = t * NC + cc), issued D chains later
    const int pc = k % NC;
    const f32x4& y = acc[k % (D + 1)];
    float& mm = m[pc >> 1][pc & 1];
    mm = fmaxf(fmaxf(fmaxf(fmaxf(mm, y[0]), y[1]), y[2]), y[3]);
  };
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int cc = 0; cc < NC; ++cc) {
      const int k = t * NC + cc;
      if (!PF && cc == 0 && t + 1 < NT) lds_afrag_f8x4<TPI>(buf, t + 1, lane, a[(t + 1) & 1], as[(t + 1) & 1]);
      if constexpr (PROBE == 1)
        acc[k % (D + 1)] = mfma_f8q<PQS>(a[t & 1], as[t & 1], qa[cc >> 1][cc & 1], qsv, cc,
                                         k < D + 1 ? f32x4{} : acc[k % (D + 1)]);
      else
        acc[k % (D + 1)] = mfma_f8q<PQS>(a[t & 1], as[t & 1], qa[cc >> 1][cc & 1], qsv, cc, f32x4{});
      if constexpr (PF) {
        __builtin_amdgcn_sched_barrier(0);
        if (cc == 0 && t + 1 < NT) lds_afrag_f8x4<TPI>(buf, t + 1, lane, a[(t + 1) & 1], as[(t + 1) & 1]);
      }
      if (PROBE != 1 && k >= D) fold(k - D);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  if constexpr (PROBE == 1) {
#pragma unroll
    for (int k = NT * NC - D - 1; k < NT * NC; ++k) fold(k);
  } else {
#pragma unroll
    for (int k = NT * NC - D; k < NT * NC; ++k) fold(k);
  }
}

template <int QW, int TPI = 32, bool PQS = false>
__device__ __forceinline__ void iter_f8x4_ragged(const uint8_t* buf, int lane, int j, int dl_g, int dl_max,
                                                 const i32x8 (&qa)[QW][2], const int* qsv, float (&m)[QW][2]) {
  const int nt = min(TPI / 4, (dl_max - TPI * j + 3) >> 2);
#pragma unroll 1
  for (int t = 0; t < nt; ++t) {
    const int tok0 = TPI * j + 4 * t;
    i32x8 a;
    int as;
    lds_afrag_f8x4<TPI>(buf, t, lane, a, as);
    f32x4 init;
#pragma unroll
    for (int r = 0; r < 4; ++r) init[r] = (tok0 + r < dl_g) ? 0.0f : neg_inf();
    tile_f8q<QW, PQS>(a, as, qa, qsv, init, m);
  }
}

// PAIR: two TPI-token iterations per barrier (4 ring slots = 2 pair buffers;
// pair p+1 is issued right after the barrier that retires pair p-1, so its
// loads get one pair's compute to land) -- half the barriers and pipeline
// drains of the 3-deep ring, the same 32-token body (and VGPRs) per step.
// Lab only (round 3, bit-identical, profiles/r03i_lab_f8_spread_*): SPREAD2
// (with PAIR) issues pair p+1's second iteration after the first iteration of
// pair p instead of right after the barrier (-0.3 %); SPLIT has only waves
// 0 .. WAVES/2 - 1 issue the DMA pieces (+0.2 %, within noise, 4 VGPR spills).
template <int WAVES, int QW, int D = 1, int NBUF = 3, int TPI = 32, bool PF = false, int OCC = 2,   // D = 2 spills at QW = 8
          int FK = 0, int LD = kLd, bool PQS = false, bool PAIR = false, bool SPREAD2 = false, bool SPLIT = false,
          bool QUAD = false, int PROBE = 0, int AUX = 0>
__global__ __launch_bounds__(WAVES * 64, OCC) void maxsim_scan_f8x4_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int B, int lq,
    float* __restrict__ out, int64_t ld_out, int64_t chunk_docs, int64_t static_docs, int* __restrict__ task_ctr,
    int task_docs, int topk_k = 0, uint64_t* __restrict__ part = nullptr, int nslots = 0, int tail_slices = 1,
    uint64_t* __restrict__ clk = nullptr) {
  if (clk != nullptr && threadIdx.x == 0) clock_probe(clk, false);   // the bench's clock probe (null otherwise)
  constexpr int QPB = WAVES * QW;
  constexpr int kIterBytes = 4 * TPI * kDim;                 // e4m3 bytes per iteration
  constexpr int kIterStage = kIterBytes + 4 * TPI * 2;        // + 2 scale bytes per row
  // LD token slots per doc (128; 256 / 512 / 1024 for long documents: a doc
  // group then spans LD / TPI iterations, the row maxima carried across them)
  static_assert(LD % TPI == 0 && LD >= 128 && LD <= 1024, "LD: 128, 256, 512 or 1024 token slots");
  constexpr int IPG = LD / TPI;
  constexpr size_t kDocStride = (size_t)LD * kDim, kScaleStride = (size_t)LD * 2;
  constexpr int kScaleDma = 4 * TPI * 2 / 256;                // 256-B scale DMAs per iteration
  constexpr int kPieces = kIterBytes / 1024;
  constexpr int kLoadWaves = SPLIT ? WAVES / 2 : WAVES;
  constexpr int kPiecesPerWave = kPieces / kLoadWaves;
  static_assert(TPI == 32 || TPI == 64 || TPI == 128, "32, 64 or 128 tokens per iteration");
  static_assert(kPieces % kLoadWaves == 0 && kScaleDma <= kLoadWaves, "pieces must split evenly over waves");
  constexpr int kGrp = QUAD ? 4 : 2;   // PAIR: iterations per barrier (QUAD, lab: four)
  static_assert(!SPREAD2 || (PAIR && !QUAD), "SPREAD2 spreads a PAIR ring's issue");
  static_assert(!QUAD || PAIR, "QUAD is a PAIR ring of four");
  static_assert(PAIR ? (NBUF == 2 * kGrp && IPG % kGrp == 0 && FK == 0) : (NBUF == 2 || NBUF == 3),
                "2- or 3-deep ring; PAIR: 2 x kGrp slots, whole groups per doc group, unfused");
  constexpr int kCandBytes = FK > 0 ? QPB * (FK * 8 + kFusedStateBytes) : 0;   // fused top-k buffers + state
  __shared__ __attribute__((aligned(1024))) uint8_t smem[NBUF * kIterStage + 256 + 16 + kCandBytes];
  int* const task_slot = reinterpret_cast<int*>(smem + NBUF * kIterStage + 256);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  uint64_t* const cand =
      reinterpret_cast<uint64_t*>(smem + NBUF * kIterStage + 256 + 16) + (size_t)wave * QW * (FK > 0 ? FK : 1);
  uint8_t* const tk_state =
      smem + NBUF * kIterStage + 256 + 16 + (FK > 0 ? QPB * FK * 8 : 0) + wave * QW * kFusedStateBytes;
  if (FK > 0 && lane < 2 * QW) reinterpret_cast<uint64_t*>(tk_state)[lane] = 0ull;
  const int nq_groups = (B + QPB - 1) / QPB;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, idx = bid >> 3, qd = nwg >> 3, rm = nwg & 7;
  const int lin = (xcd < rm ? xcd * (qd + 1) : rm * (qd + 1) + (xcd - rm) * qd) + idx;
  const int qg = lin % nq_groups;
  const int64_t chunk = lin / nq_groups;

  i32x8 qa[QW][2];
  int qsv[kQsRegs<QW, PQS>];
  {
    int qs[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) load_qfrag_f8(Qb, Qs, qg * QPB + wave * QW + q, B, lq, lane, qa[q], qs[q]);
    pack_qscales<QW, PQS>(qs, qsv);
  }

  // piece p = image rows 8p..8p+7 (128 B each) = doc 8p / TPI (uniform per
  // piece), tokens TPI*j + 8p % TPI + 0..7.  Offsets are recomputed per issue
  // (a few VALU) rather than held: at 8 queries per wave the VGPR file is full.
  // the same static chunks + guided dynamic tail as maxsim_scan16x4_kernel
  int64_t d_begin = chunk * chunk_docs;
  int64_t d_end = d_begin + chunk_docs < static_docs ? d_begin + chunk_docs : static_docs;
  for (int kt = 0;; ++kt) {
  if (d_begin < d_end) {
  const int nd = (int)(d_end - d_begin);
  const int ngr = (nd + 3) >> 2;
  auto clamp_doc = [&](int d) { return d < nd ? d : nd - 1; };  // the last group's missing docs: rows masked
  auto issue = [&](int it, int buf) {
    const int G = it / IPG, j = it % IPG;
    uint8_t* sbuf = smem + buf * kIterStage;
    if (SPLIT && wave >= kLoadWaves) return;   // the partner waves load nothing (wave-uniform)
#pragma unroll
    for (int jj = 0; jj < kPiecesPerWave; ++jj) {
      const int piece = wave * kPiecesPerWave + jj;
      const int R = 8 * piece + (lane >> 3);
      const uint32_t off = (R % TPI) * kDim + 16 * ((lane & 7) ^ swz_f8<TPI>(R));
      const int d = clamp_doc(4 * G + 8 * piece / TPI);
      const uint8_t* src = tokens + (size_t)(d_begin + d) * kDocStride + (size_t)j * TPI * kDim + off;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(sbuf + piece * 1024), 16, 0, AUX);
    }
    if (wave < kScaleDma) {  // scale bytes b = 256 * wave + 4L: row b/2 = TPI * doc + token
      const int R = (256 * wave + 4 * lane) / 2;
      const int d = clamp_doc(4 * G + R / TPI);
      const uint8_t* src = tscales + (size_t)(d_begin + d) * kScaleStride + (size_t)(j * TPI + R % TPI) * 2;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)src, (lds_void_t*)(sbuf + kIterBytes + 256 * wave), 4, 0, AUX);
    }
  };
  // vector-memory ops per wave per iteration (the vmcnt that leaves one iteration in flight)
  const bool loader = wave < kScaleDma;

  float sc[QW];
  float m[QW][2];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f, m[q][0] = m[q][1] = neg_inf();
  int dl_g = 0, dl_min = 0, dl_max = 0;

  const int nit = IPG * ngr;
  bool stored = false;
  // one TPI-token iteration on the landed slot buf: doc-group start, tiles, epilogue
  auto step = [&](int it, const uint8_t* buf) {
    const int G = it / IPG, j = it % IPG;
    if (j == 0) {
      int dl4[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int v = (4 * G + x < nd) ? doclens[d_begin + 4 * G + x] : 0;
        dl4[x] = v < 0 ? 0 : (v > LD ? LD : v);
      }
      dl_min = min(min(dl4[0], dl4[1]), min(dl4[2], dl4[3]));
      dl_max = max(max(dl4[0], dl4[1]), max(dl4[2], dl4[3]));
      dl_g = g == 0 ? dl4[0] : (g == 1 ? dl4[1] : (g == 2 ? dl4[2] : dl4[3]));
#pragma unroll
      for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    }
    // the 4-wave shapes of batches <= 16: a wave's padded query slots (>= B)
    // skip their MFMAs, as in maxsim_scan16x4_kernel (same chains, same order)
    constexpr bool kSkipF8 = kScanQSkip && WAVES == 4 && (QW <= 2 || QW == 4) && PROBE == 0 && FK == 0;
    if constexpr (kSkipF8) {
      const int nlive = max(0, min(QW, B - (qg * QPB + wave * QW)));
      auto live = [&](auto nq) {
        constexpr int L = decltype(nq)::value;
        constexpr int DL = (2 * L) % (D + 1) == 0 ? D : 1;   // the accumulator ring must divide the chains
        auto& q = reinterpret_cast<const i32x8(&)[L][2]>(qa[0]);
        auto& mm = reinterpret_cast<float(&)[L][2]>(m[0]);
        if (TPI * j + TPI <= dl_min)
          iter_f8x4_full<L, DL, TPI, PF, PQS, 0>(buf, lane, q, qsv, mm);
        else if (TPI * j < dl_max)
          iter_f8x4_ragged<L, TPI, PQS>(buf, lane, j, dl_g, dl_max, q, qsv, mm);
      };
      if (nlive == QW) live(std::integral_constant<int, QW>{});
      else if (QW >= 4 && nlive == 3) live(std::integral_constant<int, (QW >= 4 ? 3 : 1)>{});
      else if (QW >= 3 && nlive == 2) live(std::integral_constant<int, (QW >= 3 ? 2 : 1)>{});
      else if (QW >= 2 && nlive == 1) live(std::integral_constant<int, 1>{});
    } else {
      if (TPI * j + TPI <= dl_min)
        iter_f8x4_full<QW, D, TPI, PF, PQS, PROBE == 1 ? 1 : 0>(buf, lane, qa, qsv, m);
      else if (TPI * j < dl_max)
        iter_f8x4_ragged<QW, TPI, PQS>(buf, lane, j, dl_g, dl_max, qa, qsv, m);
    }
    if (j == IPG - 1) {
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        if constexpr (PROBE == 2) {   // INVALID: no cross-lane sum (bounds the epilogue's cost)
          sc[q] = (c == (G & 15)) ? m[q][0] + m[q][1] : sc[q];
          continue;
        }
        const float v = dpp_row_sum16((c < lq ? m[q][0] : 0.0f) + (16 + c < lq ? m[q][1] : 0.0f));
        sc[q] = (c == (G & 15)) ? v : sc[q];
      }
      if ((G & 15) == 15 || G == ngr - 1) {
        const int dd = 64 * (G >> 4) + 4 * c + g;
        if constexpr (FK > 0) {
#pragma unroll
          for (int q = 0; q < QW; ++q) {
            if (qg * QPB + wave * QW + q >= B) continue;   // wave-uniform
            const uint32_t loc = (uint32_t)(d_begin + dd);
            const uint64_t key = (c <= (G & 15) && dd < nd) ? ((uint64_t)f2u(sc[q]) << 32) | (uint32_t)~loc : 0ull;
            topk_offer<FK>(cand + q * FK, tk_state + q * kFusedStateBytes, topk_k, key, lane);
          }
        } else {
#pragma unroll
          for (int q = 0; q < QW; ++q) {
            const int qi = qg * QPB + wave * QW + q;
            if (qi < B && c <= (G & 15) && dd < nd) out[(size_t)qi * ld_out + d_begin + dd] = sc[q];
          }
          stored = true;
        }
      }
    }
  };
  if constexpr (PAIR && !QUAD) {
    issue(0, 0);
    if (nit > 1) issue(1, 1);
    for (int it = 0; it < nit; ++it) {
      const int pb = (it >> 1) & 1;   // this pair's buffer: slots 2pb, 2pb + 1
      if ((it & 1) == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this pair landed (the next is not issued yet)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (it + 2 < nit) issue(it + 2, 2 * (pb ^ 1));   // into the pair every wave finished before the barrier
        if (!SPREAD2 && it + 3 < nit) issue(it + 3, 2 * (pb ^ 1) + 1);
      } else if (SPREAD2 && it + 2 < nit) {
        issue(it + 2, 2 * (pb ^ 1) + 1);                   // the same free pair buffer, one iteration later
      }
      step(it, smem + (2 * pb + (it & 1)) * kIterStage);
    }
  } else if constexpr (QUAD) {   // the same with four iterations per barrier (slots 4qb .. 4qb + 3)
#pragma unroll
    for (int x = 0; x < 4; ++x)
      if (x < nit) issue(x, x);
    for (int it = 0; it < nit; ++it) {
      const int qb = (it >> 2) & 1;
      if ((it & 3) == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
#pragma unroll
        for (int x = 0; x < 4; ++x)
          if (it + 4 + x < nit) issue(it + 4 + x, 4 * (qb ^ 1) + x);
      }
      step(it, smem + (4 * qb + (it & 3)) * kIterStage);
    }
  } else {
    issue(0, 0);
    if (NBUF == 3 && nit > 1) issue(1, 1);
    int cur = 0;
    for (int it = 0; it < nit; ++it) {
      if (NBUF == 3 && it + 1 < nit && !stored) {
        if (loader)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPiecesPerWave + 1) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kPiecesPerWave) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      stored = false;
      if (NBUF == 2 && it + 1 < nit) issue(it + 1, cur ^ 1);
      if (NBUF == 3 && it + 2 < nit) issue(it + 2, cur == 0 ? 2 : cur - 1);
      const uint8_t* buf = smem + cur * kIterStage;
      cur = NBUF == 2 ? (cur ^ 1) : (cur == 2 ? 0 : cur + 1);
      step(it, buf);
    }
  }
  }
    if (task_ctr == nullptr) break;
    if (threadIdx.x == 0)
      next_task_sliced(task_ctr + tail_slices * qg, tail_slices, bid & 7, task_docs, (int)(n - static_docs),
                       nwg / nq_groups, task_slot + 2 * (kt & 1));
    __syncthreads();
    const int o = __builtin_amdgcn_readfirstlane(task_slot[2 * (kt & 1)]);
    const int sz = __builtin_amdgcn_readfirstlane(task_slot[2 * (kt & 1) + 1]);
    d_begin = static_docs + (int64_t)o;
    if (sz <= 0 || d_begin >= n) break;
    d_end = d_begin + sz < n ? d_begin + sz : n;
  }
  if constexpr (FK > 0) {
#pragma unroll 1
    for (int q = 0; q < QW; ++q) {
      const int qi = qg * QPB + wave * QW + q;
      if (qi >= B) continue;
      topk_flush(cand + q * FK, tk_state + q * kFusedStateBytes, topk_k,
                 part + ((size_t)qi * nslots + (size_t)chunk) * topk_k, lane);
    }
  }
  if (clk != nullptr) {   // block-uniform
    __syncthreads();
    if (threadIdx.x == 0) clock_probe(clk, true);
  }
}

// Small-batch f8 scan: one doc chunk per wave, docs streamed to VGPRs.
// LONG: docs of ld = 256 / 512 / 1024 token slots, 128 tokens at a time with
// the row maxima carried (same tile order: a doc of <= 128 tokens scores the
// same bits whatever ld).
template <int QW, bool LONG = false>
__global__ __launch_bounds__(256, 2) void maxsim_scan_f8_direct_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int B, int lq,
    float* __restrict__ out, int64_t ld_out, int64_t chunk_docs, int ld = kLd) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4;
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t lin = (int64_t)blockIdx.x * 4 + wave;
  const int qg = (int)(lin % nq_groups);
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;
  const int nd = (int)(d_end - d_begin);
  i32x8 qa[QW][2];
  int qs[QW][2];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag_f8(Qb, Qs, qg * QW + q, B, lq, lane, qa[q], qs[q]);
  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;
  const int lmax = LONG ? ld : kLd;
  for (int i = 0; i < nd; ++i) {
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > lmax ? lmax : dl);
    float m[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    for (int blk = 0; blk == 0 || (LONG && kLd * blk < dl); ++blk) {   // one block unless LONG
      const int dlb = dl - kLd * blk;
      const uint8_t* dbase = tokens + ((size_t)(d_begin + i) * lmax + (size_t)kLd * blk) * kDim;
      const uint8_t* dsc = tscales + ((size_t)(d_begin + i) * lmax + (size_t)kLd * blk) * 2;
      i32x8 af[kLd / 16];
      int as[kLd / 16];
#pragma unroll
      for (int rt = 0; rt < kLd / 16; ++rt)
        if (16 * rt < dlb) gbl_afrag_f8(dbase, dsc, rt, lane, af[rt], as[rt]);
#pragma unroll
      for (int rt = 0; rt < kLd / 16; ++rt) {
        if (16 * rt < dlb) {
          const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
          tile_f8<QW>(af[rt], as[rt], qa, qs, init, m);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = qg * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// MXFP8 streaming small-batch scan (B <= 2, QW = 2; production): the bf16
// streaming scan's design on e4m3 tiles.  A 16-row tile is 2 KiB of tokens
// (two 1 KiB LDS-DMA pieces, rows 8p .. 8p + 7, XOR-swizzled into the layout
// lds_afrag_f8 reads) plus its 32 scale bytes (one 4-byte-per-lane LDS-DMA:
// lanes 0-7 fetch the tile's scales, lanes 8-63 repeat them, so no lane reads
// past the scale array); 3 ops per tile, SLOTS tile slots per wave, the oldest
// tile waited with a constant vmcnt(3 (SLOTS - 1)).  The direct scan's tiles,
// masks, max order and epilogue: bit-identical scores.  An f8 tile is half
// the bytes of a bf16 one for the same per-tile waits, so the production
// shape runs 8 waves x 8 slots (147 KiB per CU): lab, same process, 1.25M
// docs B=1 3.346 -> 3.071 ms (direct -> 8 x 8; 4 x 16: 3.33 on another box,
// 16 x 4: 3.098), B=2 3.417 -> 3.115, 125k 0.349 -> 0.311
// (profiles/r03ai_*).
// ---------------------------------------------------------------------------
constexpr int kF8SlotBytes = 2048 + 256;
// TW2 (production since r03z): two tiles of one doc per wait (one vmcnt
// wait, one lgkmcnt wait and one refill of two slots per pair; odd tails take
// the one-tile step).  Lab, same process, bit-identical
// (profiles/r03z_lab_f8_tw2.log: variant 10 = one tile per wait, 32 = TW2 at
// 8 x 8, 33 = TW2 at 4 x 16): 1.25M docs B=1 3.320 -> 3.282 ms, B=2 3.178 ->
// 3.155, 125k B=1 0.318 -> 0.316; at 4 x 16 B=2 and 125k lose (3.342 / 0.423).
template <int QW, int AUX, int WAVES = 4, int SLOTS = 16, bool TW2 = true>
__global__ __launch_bounds__(WAVES * 64, 1) void maxsim_scan_f8_stream_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int B, int lq,
    float* __restrict__ out, int64_t ld_out, int64_t chunk_docs, int ld) {
  __shared__ __attribute__((aligned(1024))) uint8_t smem[WAVES * SLOTS * kF8SlotBytes];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane & 15, g = lane >> 4;
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t lin = (int64_t)blockIdx.x * WAVES + wave;      // one doc chunk per wave
  const int qg = (int)(lin % nq_groups);
  const int64_t chunk = lin / nq_groups;
  const int64_t d_begin = chunk * chunk_docs;
  const int64_t d_end = (d_begin + chunk_docs < n) ? d_begin + chunk_docs : n;
  if (d_begin >= d_end) return;  // uniform over the wave; no block-level sync below
  const int nd = (int)(d_end - d_begin);
  uint8_t* ring = smem + wave * (SLOTS * kF8SlotBytes);
  const int32_t* dls = doclens + d_begin;
  auto ntiles = [&](int d) -> int {
    int dl = sload_len(dls + d);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    return (dl + 15) >> 4;
  };
  // token piece p of a tile = its rows 8p .. 8p + 7; lane l writes position
  // l & 7 of row 8p + (l >> 3), so it fetches logical slot position ^ swz8(row)
  uint32_t src_off[2];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int t = 8 * p + (lane >> 3);
    src_off[p] = (uint32_t)(t * kDim + 16 * ((lane & 7) ^ swz8(t)));
  }
  const uint32_t sc_off = 4u * (uint32_t)(lane & 7);
  int idoc = 0, itile = 0, intl = ntiles(0);
  while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
  int issued = 0;
  const uint8_t* tb = tokens + (size_t)d_begin * ld * kDim;
  const uint8_t* sb = tscales + (size_t)d_begin * ld * 2;
  auto issue_next = [&]() {
    if (idoc >= nd) return;
    const size_t row0 = (size_t)idoc * ld + (size_t)itile * 16;
    uint8_t* dst = ring + (issued & (SLOTS - 1)) * kF8SlotBytes;
#pragma unroll
    for (int p = 0; p < 2; ++p)
      __builtin_amdgcn_global_load_lds((gbl_void_t*)(tb + row0 * kDim + src_off[p]), (lds_void_t*)(dst + p * 1024), 16,
                                       0, AUX);
    __builtin_amdgcn_global_load_lds((gbl_void_t*)(sb + row0 * 2 + sc_off), (lds_void_t*)(dst + 2048), 4, 0, AUX);
    ++issued;
    if (++itile >= intl) {
      itile = 0;
      intl = 0;
      while (intl == 0 && ++idoc < nd) intl = ntiles(idoc);
    }
  };
  i32x8 qa[QW][2];
  int qs[QW][2];
#pragma unroll
  for (int q = 0; q < QW; ++q) load_qfrag_f8(Qb, Qs, qg * QW + q, B, lq, lane, qa[q], qs[q]);
  float sc[QW];
#pragma unroll
  for (int q = 0; q < QW; ++q) sc[q] = 0.0f;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the query fragments: out of the ring's count
#pragma unroll
  for (int k = 0; k < SLOTS; ++k) issue_next();

  int consumed = 0;
  for (int i = 0; i < nd; ++i) {
    int dl = sload_len(dls + i);
    dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    const int nt = (dl + 15) >> 4;
    float m[QW][2];
#pragma unroll
    for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
    for (int t = 0; t < nt; ++t) {
      if (TW2 && t + 1 < nt) {
        // the ring is full unless the stream is ending: the oldest two tiles
        // have landed once at most SLOTS - 2 tiles (3 ops each) are in flight
        if (issued - consumed >= SLOTS)
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (SLOTS - 2)) : "memory");
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        u32x4 lo[2], hi[2];
        int as2[2];
        const int sw = swz8(c);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const uint8_t* slot = ring + ((consumed + u) & (SLOTS - 1)) * kF8SlotBytes;
          const uint8_t* row = slot + c * kDim;
          lo[u] = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g) ^ sw));
          hi[u] = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g + 1) ^ sw));
          as2[u] = slot[2048 + c * 2 + (g & 1)];
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // both slots read: refill them
        consumed += 2;
        issue_next();
        issue_next();
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const i32x8 a = i32x8{(int)lo[u][0], (int)lo[u][1], (int)lo[u][2], (int)lo[u][3],
                                (int)hi[u][0], (int)hi[u][1], (int)hi[u][2], (int)hi[u][3]};
          const int tt = t + u;
          const f32x4 init = (dl >= 16 * tt + 16) ? f32x4{} : row_mask_init16(16 * tt + 4 * g, dl);
          tile_f8<QW>(a, as2[u], qa, qs, init, m);
        }
        ++t;
        continue;
      }
      if (issued - consumed >= SLOTS)
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * (SLOTS - 1)) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint8_t* slot = ring + (consumed & (SLOTS - 1)) * kF8SlotBytes;
      const uint8_t* row = slot + c * kDim;
      const int sw = swz8(c);
      const u32x4 lo = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g) ^ sw));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(row + 16 * ((2 * g + 1) ^ sw));
      const int as = slot[2048 + c * 2 + (g & 1)];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot is read: refill it
      ++consumed;
      issue_next();
      const i32x8 a = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2],
                            (int)hi[3]};
      const f32x4 init = (dl >= 16 * t + 16) ? f32x4{} : row_mask_init16(16 * t + 4 * g, dl);
      tile_f8<QW>(a, as, qa, qs, init, m);
    }
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (i & 63)) ? v : sc[q];
    }
    if ((i & 63) == 63 || i == nd - 1) {
      const int i0 = i & ~63;
      const int cnt = i - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = qg * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Row top-k: exact radix select (11/11/10-bit digits of the order-preserving
// score key; if the k-th score is tied, a second radix select over ~index picks
// the lowest indices), then a bitonic sort of the k winners in LDS.
// ---------------------------------------------------------------------------
constexpr int kTkThreads = 1024;

// Wave 0 finds bin b with count(bins > b) < kleft <= count(bins >= b).
__device__ void find_bin(const uint32_t* hist, int nb, uint32_t kleft, uint32_t* s_bin,
                         uint32_t* s_above, uint32_t* s_bincount) {
  const int lane = threadIdx.x & 63;
  const int per = nb / 64;
  uint32_t tot = 0;
  for (int j = 0; j < per; ++j) tot += hist[lane * per + j];
  uint32_t incl = tot;  // inclusive suffix sum over lanes >= lane
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    uint32_t t = __shfl_down(incl, off);
    if (lane + off < 64) incl += t;
  }
  const uint32_t above = incl - tot;
  const bool mine = (above < kleft) && (kleft <= incl);
  if (mine) {
    uint32_t cum = above;
    for (int j = per - 1; j >= 0; --j) {
      const uint32_t c = hist[lane * per + j];
      if (cum + c >= kleft) {
        *s_bin = lane * per + j;
        *s_above = cum;
        *s_bincount = c;
        break;
      }
      cum += c;
    }
  }
}

// find_bin for 1024 bins (16 per lane): each lane's bins in registers (four
// 16-B LDS reads, hist 16-B aligned), the suffix sums across lanes, then the
// owning lane's own registers -- no dependent LDS reads.
__device__ void find_bin1024(const uint32_t* hist, uint32_t kleft, uint32_t* s_bin, uint32_t* s_above,
                             uint32_t* s_bincount) {
  const int lane = threadIdx.x & 63;
  uint32_t h[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const uint4 v = reinterpret_cast<const uint4*>(hist + lane * 16)[q];
    h[4 * q] = v.x, h[4 * q + 1] = v.y, h[4 * q + 2] = v.z, h[4 * q + 3] = v.w;
  }
  uint32_t tot = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) tot += h[j];
  uint32_t incl = tot;  // inclusive suffix sum over lanes >= lane
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t t = __shfl_down(incl, off);
    if (lane + off < 64) incl += t;
  }
  const uint32_t above = incl - tot;
  if (above < kleft && kleft <= incl) {
    uint32_t cum = above;
    int bin = 0;
    uint32_t cnt = 0, abv = 0;
    bool found = false;
#pragma unroll
    for (int j = 15; j >= 0; --j) {
      if (!found && cum + h[j] >= kleft) {
        found = true;
        bin = lane * 16 + j;
        abv = cum;
        cnt = h[j];
      }
      cum += h[j];
    }
    *s_bin = (uint32_t)bin;
    *s_above = abv;
    *s_bincount = cnt;
  }
}

__device__ void bitonic_desc(uint64_t* keys, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      __syncthreads();
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const uint64_t a = keys[i], b = keys[j];
          const bool desc = (i & size) == 0;
          if (desc ? (a < b) : (a > b)) {
            keys[i] = b;
            keys[j] = a;
          }
        }
      }
    }
  }
  __syncthreads();
}

// LDS histogram add with wave aggregation: lanes whose bins agree add once
// (up to 4 rounds, led by the lowest remaining lane's bin), the rest by plain
// atomics.  Score keys of similar magnitude share their top digit, so in a
// radix select's first pass one bin takes most of a wave: 64 serialised LDS
// atomics on one address become one add.
__device__ __forceinline__ void hist_add(uint32_t* hist, uint32_t bin, bool take) {
  const int lane = threadIdx.x & 63;
  uint64_t rem = __ballot(take);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (rem == 0) break;   // wave-uniform
    const int leader = __ffsll((unsigned long long)rem) - 1;
    const uint32_t lb = __shfl(bin, leader);
    const uint64_t same = rem & __ballot(take && bin == lb);
    if (lane == leader) atomicAdd(&hist[lb], (uint32_t)__popcll(same));
    rem &= ~same;
  }
  if ((rem >> lane) & 1ull) atomicAdd(&hist[bin], 1u);
}

// Exact selection of the kk largest keys of row x into sel[0..kk) (unordered).
// Radix select on the 32-bit score key (11/11/10-bit digits); if the kk-th
// score is tied, a second radix select over ~index keeps the lowest indices.
// BOUNDED: only entries whose ranking key is < bound take part (the next
// pass of a multi-pass selection: bound = the previous pass's smallest key).
template <bool BOUNDED = false>
__device__ void topk_exact_row(const float* __restrict__ x, int64_t n, int kk, uint64_t* sel, uint32_t* hist,
                               uint32_t* s_bin, uint32_t* s_above, uint32_t* s_bincount, uint32_t* s_cnt,
                               uint64_t bound = ~0ull) {
  const int tid = threadIdx.x, nth = blockDim.x;
  const int wave = tid >> 6;
  auto live = [&](float v, int64_t i) { return !BOUNDED || rank_key(v, (uint32_t)i) < bound; };
  if (!BOUNDED && kk == n) {
    for (int i = tid; i < kk; i += nth) sel[i] = rank_key(x[i], (uint32_t)i);
    __syncthreads();
    return;
  }
  const int shifts[3] = {21, 10, 0};
  const int bits[3] = {11, 11, 10};
  uint32_t prefix = 0, mask = 0, kleft = (uint32_t)kk, last_count = 0;
#pragma unroll 1
  for (int p = 0; p < 3; ++p) {
    const int nb = 1 << bits[p];
    for (int b = tid; b < nb; b += nth) hist[b] = 0;
    __syncthreads();
    for (int64_t i = tid; i < n; i += nth) {
      const float v = x[i];
      const uint32_t u = f2u(v);
      hist_add(hist, (u >> shifts[p]) & (nb - 1), (u & mask) == prefix && live(v, i));
    }
    __syncthreads();
    if (wave == 0) find_bin(hist, nb, kleft, s_bin, s_above, s_bincount);
    __syncthreads();
    kleft -= *s_above;
    prefix |= *s_bin << shifts[p];
    mask |= (uint32_t)(nb - 1) << shifts[p];
    last_count = *s_bincount;
    __syncthreads();
  }
  const uint32_t ustar = prefix;
  uint32_t id_thr = 0xffffffffu;  // ties at ustar with index <= id_thr are taken
  if (kleft < last_count) {
    uint32_t iprefix = 0, imask = 0, kl2 = kleft;
#pragma unroll 1
    for (int p = 0; p < 3; ++p) {
      const int nb = 1 << bits[p];
      for (int b = tid; b < nb; b += nth) hist[b] = 0;
      __syncthreads();
      for (int64_t i = tid; i < n; i += nth) {
        const uint32_t key2 = ~(uint32_t)i;
        const float v = x[i];
        hist_add(hist, (key2 >> shifts[p]) & (nb - 1), f2u(v) == ustar && (key2 & imask) == iprefix && live(v, i));
      }
      __syncthreads();
      if (wave == 0) find_bin(hist, nb, kl2, s_bin, s_above, s_bincount);
      __syncthreads();
      kl2 -= *s_above;
      iprefix |= *s_bin << shifts[p];
      imask |= (uint32_t)(nb - 1) << shifts[p];
      __syncthreads();
    }
    id_thr = ~iprefix;
  }
  if (tid == 0) *s_cnt = 0;
  __syncthreads();
  for (int64_t i = tid; i < n; i += nth) {
    const float v = x[i];
    const uint32_t u = f2u(v);
    if ((u > ustar || (u == ustar && (uint32_t)i <= id_thr)) && live(v, i)) {
      const uint32_t pos = atomicAdd(s_cnt, 1u);
      if (pos < (uint32_t)kk) sel[pos] = ((uint64_t)u << 32) | (uint32_t)(~(uint32_t)i);
    }
  }
  __syncthreads();
}

// Sort sel[0..cnt) descending (padding to a power of two) and write the best k.
// The ids of a selection also written straight to host memory (the latency
// path's device-mapped buffer, read by the host after the stream's event):
// system-scope write-through stores, so the host sees them once the kernel
// has completed.
// The words are 8 bytes, {id, seq} (seq in the high half), LL-style: a word
// is whole or absent, so the host polling them needs no ordering between the
// stores -- every word of the call carries the call's seq once written.
// soff (words, > 0): the score of word i also at w[soff + i] ({score bits,
// seq}; the latency path's host rerank takes stage 2's scores from there).
struct Mirror {
  uint64_t* w = nullptr;
  uint32_t seq = 0;
  int64_t soff = 0;
  __device__ __forceinline__ void put(size_t i, int32_t id, float s) const {
    const uint64_t t = (uint64_t)seq << 32;
    __hip_atomic_store(w + i, t | (uint32_t)id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (soff > 0) __hip_atomic_store(w + soff + i, t | __float_as_uint(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __device__ __host__ __forceinline__ Mirror row(size_t b, int k) const {
    return Mirror{w ? w + b * (size_t)k : nullptr, seq, soff};
  }
};

// The pre-armed rerank of the latency path (retrieve.cpp): the rerank is
// launched before the host has fused stage 1 and 2, and its candidates arrive
// in a device-mapped host buffer as 8-byte words {id, seq} (whole or absent),
// written by the host after the launch.  Thread 0 of a workgroup polls its
// candidate's word (system-scope loads, s_sleep between polls) until the tag
// is the call's seq -- so the host's fusion -> rerank hop costs a PCIe read,
// not a kernel launch.  It never waits forever: after `ticks` of
// s_memrealtime (100 MHz; kCandWaitTicks = 1 s) it gives up through the
// call's wait gate (below) and the candidate reads as -1 (scores -inf); the
// host, which writes the words whatever happens (-1 words on its own
// failure), then fails the call.
//
// The wait gate: two tagged words of the call's mapped buffer, gate[0]
// written by a kernel that is about to give up, gate[1] by the host just
// before it publishes the words the kernel waits for.  Each side stores its
// own word, fences (seq_cst, system scope), then loads the other's (Dekker):
// of a kernel that gave up (read no host word) and a host that then
// published, at least one read the other's -- so a host whose load misses
// the kernel's word knows no kernel gave up, and a kernel that reads the
// host's word withdraws and waits on (kBackstopTicks: the host is past its
// last wait and writing).  A host that reads the kernel's word fails the call
// (CBV2_EHIP): no call returns after a timed-out device wait.
struct TaggedCand {
  const uint64_t* w = nullptr;
  uint32_t seq = 0;
  uint64_t* gate = nullptr;   // [0] kernel's word, [1] host's word (nullable: a timeout gives up at once)
  uint64_t ticks = 0;         // the wait's bound (s_memrealtime ticks)
};

// The FINAL top-k of a retrieve call, also written to host memory by the
// select that produces it (the latency path's device-mapped buffer, tagged
// words as Mirror's): per row [k] score words, [k] id words, [k] position
// words, {value bits, seq}.  The host polls them and has its results as soon
// as the select stored them -- no D2H copy, no stream wait.
struct FinalMirror {
  uint64_t* w = nullptr;
  uint32_t seq = 0;
  int k = 0;
  __device__ __forceinline__ void put(size_t b, int r, float s, int32_t id, int32_t pos) const {
    uint64_t* row = w + b * 3 * (size_t)k;
    const uint64_t t = (uint64_t)seq << 32;
    __hip_atomic_store(row + r, t | __float_as_uint(s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(row + k + r, t | (uint32_t)id, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(row + 2 * k + r, t | (uint32_t)pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
};
constexpr uint64_t kCandWaitTicks = 100000000ull;    // 1 s
constexpr uint64_t kBackstopTicks = 3000000000ull;   // 30 s: the host committed to publish (gate) yet nothing came
// Added to a row's band count by a collect workgroup whose wait for phase 1
// gave up: above any real count (<= k + n < 2^28), so the row overflows.
constexpr int32_t kWaitTimedOut = 1 << 28;
// The kernel's side of the wait gate: true = give up (the host had not
// committed to publish), false = the host is publishing: wait on.
__device__ __forceinline__ bool gate_give_up(uint64_t* gate, uint32_t seq) {
  if (gate == nullptr) return true;
  const uint64_t t = ((uint64_t)seq << 32) | 1u;
  __hip_atomic_store(gate, t, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  return __hip_atomic_load(gate + 1, __ATOMIC_SEQ_CST, __HIP_MEMORY_SCOPE_SYSTEM) != t;
}
// Polls one tagged word until it carries seq; -1 once the gate says give up.
__device__ __forceinline__ bool poll_tagged(const uint64_t* w, uint32_t seq, uint64_t* gate, uint64_t ticks,
                                            uint64_t* out) {
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool committed = false;
  for (;;) {
    const uint64_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if ((uint32_t)(v >> 32) == seq) {
      *out = v;
      return true;
    }
    if (__builtin_amdgcn_s_memrealtime() - t0 > ticks) {
      if (committed || gate_give_up(gate, seq)) return false;
      committed = true;   // the host is writing: a generous bound of its own
      ticks = kBackstopTicks;
      t0 = __builtin_amdgcn_s_memrealtime();
    }
    __builtin_amdgcn_s_sleep(2);
  }
}
__device__ __forceinline__ int32_t wait_tagged(const uint64_t* w, const TaggedCand& tc) {
  uint64_t v;
  return poll_tagged(w, tc.seq, tc.gate, tc.ticks, &v) ? (int32_t)(uint32_t)v : -1;
}
// The latency path's final top-k picked by the HOST (retrieve.cpp's host
// rerank: every fused candidate's score is already known -- stage 2's own, or
// stage 1's prescore -- so the host selects it): this one-workgroup kernel is
// launched before the host has the result, polls its tagged words in the
// call's mapped buffer (FinalMirror's layout: per row [k] score, [k] id, [k]
// position words) and writes the device outputs.  A word that never comes
// (ticks, then the wait gate) is written -inf / -1 and the host fails the call.
__global__ __launch_bounds__(256) void host_result_kernel(const uint64_t* __restrict__ w, uint32_t seq, int B, int k,
                                                          float* __restrict__ out_s, int32_t* __restrict__ out_i,
                                                          int32_t* __restrict__ out_p, uint64_t* gate,
                                                          uint64_t ticks) {
  bool gave_up = false;   // (one give-up per thread: its later words are not waited for)
  for (int i = threadIdx.x; i < 3 * B * k; i += blockDim.x) {
    const int b = i / (3 * k), r = i - b * 3 * k;
    uint64_t v = 0;
    const bool ok = !gave_up && poll_tagged(w + i, seq, gate, ticks, &v);
    gave_up = !ok;
    const uint32_t x = (uint32_t)v;
    if (r < k)
      out_s[(size_t)b * k + r] = ok ? __uint_as_float(x) : neg_inf();
    else if (r < 2 * k)
      out_i[(size_t)b * k + r - k] = ok ? (int32_t)x : -1;
    else
      out_p[(size_t)b * k + r - 2 * k] = ok ? (int32_t)x : -1;
  }
}
__device__ __forceinline__ int32_t read_tagged(const uint64_t* w) {
  return (int32_t)(uint32_t)__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// mirror (w nullable): out_i's values also to mirror's words [0, k)
__device__ void sort_and_write(uint64_t* sel, int cnt, int k, int64_t id_base, float* out_s, int32_t* out_i,
                               Mirror mirror = Mirror()) {
  int P = 1;
  while (P < cnt) P <<= 1;
  for (int i = cnt + threadIdx.x; i < P; i += blockDim.x) sel[i] = 0;
  bitonic_desc(sel, P);
  for (int j = threadIdx.x; j < k; j += blockDim.x) {
    float s = neg_inf();
    int32_t id = -1;
    if (j < cnt) {
      const uint64_t key = sel[j];
      s = u2f((uint32_t)(key >> 32));
      id = (int32_t)(id_base + (int64_t)(~(uint32_t)key));
    }
    out_s[j] = s;
    out_i[j] = id;
    if (mirror.w != nullptr) mirror.put(j, id, s);
  }
}

__global__ __launch_bounds__(kTkThreads) void topk_rows_kernel(const float* __restrict__ scores, int64_t n,
                                                               int64_t ld, int k, int64_t id_base,
                                                               float* __restrict__ out_s,
                                                               int32_t* __restrict__ out_i,
                                                               const int32_t* __restrict__ only_neg = nullptr,
                                                               Mirror mirror = Mirror()) {
  __shared__ uint32_t hist[2048];
  __shared__ uint64_t sel[kTopkMax];
  __shared__ uint32_t s_bin, s_above, s_bincount, s_cnt;
  if (only_neg != nullptr && only_neg[blockIdx.x] >= 0) return;  // block-uniform: rows flagged < 0 only
  const float* x = scores + (size_t)blockIdx.x * ld;
  const int kk = (int)((int64_t)k < n ? k : n);
  topk_exact_row(x, n, kk, sel, hist, &s_bin, &s_above, &s_bincount, &s_cnt);
  sort_and_write(sel, kk, k, id_base, out_s + (size_t)blockIdx.x * k, out_i + (size_t)blockIdx.x * k,
                 mirror.row(blockIdx.x, k));
}

// ---------------------------------------------------------------------------
// Multi-pass selection for k beyond one LDS sort (torch.topk takes any k,
// local_rag_complete.py:767; argsort any C, :789): passes of up to PASS keys,
// each an exact selection restricted to keys below the previous pass's
// smallest (topk_exact_row<true>), sorted in LDS and written at its offset.
// Same keys and tie rule (score desc, lower index first) as every other path.
// ids_row (nullable) maps index -> id (else id_base + index); out_i / out_p
// (nullable) receive ids / indices.  Slots past min(k, n): -inf / -1 / -1.
// ---------------------------------------------------------------------------
template <int PASS>
__device__ void topk_multi_row(const float* x, int64_t n, int k, const int32_t* ids_row, int64_t id_base,
                               float* out_s, int32_t* out_i, int32_t* out_p, uint64_t* sel, uint32_t* hist,
                               uint32_t* misc) {
  const int kk_total = (int)((int64_t)k < n ? k : n);
  uint64_t bound = ~0ull;
  for (int off = 0; off < kk_total; off += PASS) {
    const int kk = kk_total - off < PASS ? kk_total - off : PASS;
    topk_exact_row<true>(x, n, kk, sel, hist, misc, misc + 1, misc + 2, misc + 3, bound);
    int P = 1;
    while (P < kk) P <<= 1;
    for (int i = kk + threadIdx.x; i < P; i += blockDim.x) sel[i] = 0;
    bitonic_desc(sel, P);
    for (int j = threadIdx.x; j < kk; j += blockDim.x) {
      const uint64_t key = sel[j];
      const uint32_t idx = ~(uint32_t)key;
      out_s[off + j] = u2f((uint32_t)(key >> 32));
      if (out_i) out_i[off + j] = ids_row ? ids_row[idx] : (int32_t)(id_base + (int64_t)idx);
      if (out_p) out_p[off + j] = (int32_t)idx;
    }
    bound = sel[kk - 1];
    __syncthreads();  // every thread has read sel before the next pass refills it
  }
  for (int j = kk_total + threadIdx.x; j < k; j += blockDim.x) {
    out_s[j] = neg_inf();
    if (out_i) out_i[j] = -1;
    if (out_p) out_p[j] = -1;
  }
}

constexpr int kMultiPass = 4096;  // keys sorted per pass (32 KiB of LDS)
__global__ __launch_bounds__(kTkThreads) void topk_multi_kernel(const float* __restrict__ scores, int64_t n,
                                                                int64_t ld, int k, int64_t id_base,
                                                                const int32_t* __restrict__ ids, int64_t ids_ld,
                                                                float* __restrict__ out_s, int32_t* __restrict__ out_i,
                                                                int32_t* __restrict__ out_p,
                                                                const int32_t* __restrict__ only_neg = nullptr) {
  __shared__ uint32_t hist[2048];
  __shared__ uint64_t sel[kMultiPass];
  __shared__ uint32_t misc[4];
  if (only_neg != nullptr && only_neg[blockIdx.x] >= 0) return;  // block-uniform: rows flagged < 0 only
  const size_t b = blockIdx.x;
  topk_multi_row<kMultiPass>(scores + b * ld, n, k, ids ? ids + b * ids_ld : nullptr, id_base, out_s + b * k,
                             out_i ? out_i + b * k : nullptr, out_p ? out_p + b * k : nullptr, sel, hist, misc);
}

// ---------------------------------------------------------------------------
// Sampled top-k for long rows (n >= kSampledMinN), two launches:
//  1. topk_filter_kernel, grid (S splits, B rows): every workgroup of a row
//     derives the SAME threshold t = the m-th largest key of a fixed strided
//     sample (m sized for ~8k expected survivors), then streams its 1/S of the
//     row once, gathers every element with key >= t in LDS and appends them
//     to the row's candidate list with ONE global atomic per workgroup.  (One
//     device-scope atomic per survivor serialised on the counters' cache
//     line, ~12 ns each: B=16 x ~800 survivors took the filter to 142 us at
//     100k docs, 205 us at 1M; rocprofv3, r02ah.)
//  2. topk_select_kernel, one workgroup per row: if count(key >= t) is in
//     [k, capacity] the top-k are exactly the top-k of the candidates (every
//     element >= the k-th largest is >= t), sorted in LDS; otherwise the row
//     falls back to the exact full-row radix select.  Results are identical to
//     topk_rows_kernel in every case.
// ---------------------------------------------------------------------------
constexpr int kSampleN = 8192;
constexpr int kCandCap = 8192;
constexpr int64_t kSampledMinN = 65536;

__global__ __launch_bounds__(256) void topk_filter_kernel(const float* __restrict__ scores, int64_t n, int64_t ld,
                                                          int k, uint32_t* __restrict__ cnt,
                                                          uint64_t* __restrict__ cand) {
  __shared__ __attribute__((aligned(16))) uint32_t skeys[kSampleN];
  __shared__ uint32_t hist[256];
  __shared__ uint32_t s_bin, s_above, s_bincount;
  const int tid = threadIdx.x;
  const int row = blockIdx.y;
  const float* x = scores + (size_t)row * ld;
  const int64_t stride = n / kSampleN;
  {   // all 32 strided sample loads of a thread in flight at once (a load-store
      // loop kept ~1 in flight: the sample, not the stream, set the B=1 time)
    constexpr int SPT = kSampleN / 256;
    float sv[SPT];
#pragma unroll
    for (int u = 0; u < SPT; ++u) sv[u] = x[(int64_t)(tid + 256 * u) * stride];
#pragma unroll
    for (int u = 0; u < SPT; ++u) skeys[tid + 256 * u] = f2u(sv[u]);
  }
  int64_t m64 = (8LL * k * kSampleN + n - 1) / n;
  const uint32_t m = (uint32_t)(m64 < 1 ? 1 : (m64 > kSampleN ? kSampleN : m64));
  uint32_t prefix = 0, mask = 0, kleft = m;
  for (int p = 0; p < 4; ++p) {
    const int shift = 24 - 8 * p;
    hist[tid] = 0;
    __syncthreads();
    for (int j = tid; j < kSampleN; j += 256) {
      const uint32_t u = skeys[j];
      if ((u & mask) == prefix) atomicAdd(&hist[(u >> shift) & 255], 1u);   // (wave-aggregated adds: slower here)
    }
    __syncthreads();
    if (tid < 64) find_bin(hist, 256, kleft, &s_bin, &s_above, &s_bincount);
    __syncthreads();
    kleft -= s_above;
    prefix |= s_bin << shift;
    mask |= 255u << shift;
    __syncthreads();
  }
  const uint32_t t = prefix;
  // slices of a multiple of 4 scores, so a row that starts 16-B aligned
  // (aligned base, ld % 4 == 0) streams as float4: 16 scores per thread in flight (4 KiB
  // per workgroup with scalar loads left the B=256 filter at 2.1 TB/s)
  const int64_t per = ((n + gridDim.x - 1) / gridDim.x + 3) & ~3LL;
  const int64_t a = (int64_t)blockIdx.x * per;
  const int64_t b = (a + per < n) ? a + per : n;
  uint64_t* crow = cand + (size_t)row * kCandCap;
  // survivors staged in LDS (the sample's space, free after the select above);
  // past the stage's capacity (a row with many ties at t) straight to global
  constexpr uint32_t kStage = kSampleN / 2;
  uint64_t* stage = reinterpret_cast<uint64_t*>(skeys);
  if (tid == 0) s_above = 0;   // reused: the workgroup's survivor count
  __syncthreads();
  auto offer = [&](int64_t i, float v) {
    const uint32_t key = f2u(v);
    if (key >= t) {
      const uint64_t kv = ((uint64_t)key << 32) | (uint32_t)(~(uint32_t)i);
      const uint32_t lp = atomicAdd(&s_above, 1u);
      if (lp < kStage) {
        stage[lp] = kv;
      } else {
        const uint32_t pos = atomicAdd(&cnt[row], 1u);
        if (pos < (uint32_t)kCandCap) crow[pos] = kv;
      }
    }
  };
  if ((ld & 3) == 0 && ((uintptr_t)scores & 15) == 0) {
    constexpr int U = 4;
    for (int64_t i = a + 4 * tid; i < b; i += 4 * 256 * U) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t j = i + (int64_t)u * 1024;
        if (j + 3 < b) {
          v[u] = *reinterpret_cast<const f32x4*>(x + j);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[u][e] = (j + e < b) ? x[j + e] : neg_inf();
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t j = i + (int64_t)u * 1024 + e;
          if (j < b) offer(j, v[u][e]);
        }
    }
  } else {
    for (int64_t i = a + tid; i < b; i += 4 * 256) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = (i + u * 256 < b) ? x[i + u * 256] : neg_inf();
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (i + u * 256 < b) offer(i + u * 256, v[u]);
    }
  }
  __syncthreads();
  const uint32_t nloc = s_above < kStage ? s_above : kStage;
  if (tid == 0 && nloc > 0) s_bin = atomicAdd(&cnt[row], nloc);   // reused: this workgroup's base
  __syncthreads();
  if (nloc > 0) {
    const uint32_t base = s_bin;
    for (uint32_t j = tid; j < nloc; j += 256)
      if (base + j < (uint32_t)kCandCap) crow[base + j] = stage[j];
  }
}

__global__ __launch_bounds__(kTkThreads) void topk_select_kernel(const float* __restrict__ scores, int64_t n,
                                                                 int64_t ld, int k, int64_t id_base,
                                                                 const uint32_t* __restrict__ cnt,
                                                                 const uint64_t* __restrict__ cand,
                                                                 float* __restrict__ out_s,
                                                                 int32_t* __restrict__ out_i) {
  __shared__ uint64_t sel[kCandCap];
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_bin, s_above, s_bincount, s_cnt;
  const int row = blockIdx.x;
  const int kk = (int)((int64_t)k < n ? k : n);
  const uint32_t c = cnt[row];
  int m = kk;
  if (c >= (uint32_t)kk && c <= (uint32_t)kCandCap) {
    const uint64_t* crow = cand + (size_t)row * kCandCap;
    for (uint32_t i = threadIdx.x; i < c; i += kTkThreads) sel[i] = crow[i];
    __syncthreads();
    m = (int)c;
  } else {
    topk_exact_row(scores + (size_t)row * ld, n, kk, sel, hist, &s_bin, &s_above, &s_bincount, &s_cnt);
  }
  sort_and_write(sel, m, k, id_base, out_s + (size_t)row * k, out_i + (size_t)row * k);
}

// ---------------------------------------------------------------------------
// Block-max top-k for long rows (kSampledMinN <= n <= 64 * kBmMaxBlocks), two
// launches (replaces the sampled filter + select):
//  1. block_max_kernel: bm[row][j] = max key of docs [64j, 64j + 64), one wave
//     per block, the whole chip streaming the score matrix once.
//  2. topk_bmax_kernel, one workgroup per row: t = the kk-th largest block key
//     rounded down to its top 22 bits (two 11-bit radix passes in LDS).  At
//     least kk blocks have a max >= t, so the kk-th largest score is >= t:
//     every doc of the top-kk is >= t and lies in a block whose max is >= t.
//     Only those blocks (about kk) are read; their docs >= t are gathered as
//     ranking keys (score desc, index asc) and ranked by counting (<= 512
//     keys) or a bitonic sort.  Fewer than kk or more than kBmCand gathered
//     (ties at t), or more than kBmQual qualifying blocks: the row falls back
//     to the exact full-row radix select.  The result equals topk_rows_kernel's
//     in every case, and the correctness argument never depends on bm being
//     tight -- only on every entry being >= its block's true max.
// ---------------------------------------------------------------------------
constexpr int kBmCand = 4096;          // gathered ranking keys (32 KiB)
constexpr int kBmQual = 2048;          // qualifying blocks
constexpr int kBmMaxBlocks = 24576;    // rows of n <= 1,572,864 (superblock keys in LDS: 24 KiB)
constexpr int kBmRankMax = 512;        // gathered keys ranked by counting (else bitonic)
constexpr int kBmBins = 1024;          // threshold bins (find_bin1024); qualifying superblocks listed in hist
static_assert(kBmRankMax <= 1024, "the counting rank takes one key per thread at most (1024-thread selects)");
constexpr size_t kBmFixedLds = kBmCand * 8 + 2048 * 4 + kBmQual * 4 + 64;
__host__ __device__ inline int64_t bm_blocks(int64_t n) { return (n + 63) >> 6; }   // 64-doc blocks of a row
__host__ __device__ inline int64_t bm_supers(int64_t n) { return (n + 255) >> 8; }  // 256-doc superblocks of a row
// kk large against the superblock count (kk * 8 > ns: rows of 65k-262k docs
// with k up to 1,024): the kk-th superblock key would sit near the row's
// bottom and qualify nearly every doc (then the full-row fallback), so the
// select's threshold comes from the 64-doc block keys instead
__host__ __device__ inline bool bm_by_block(int64_t n, int k) {
  const int64_t kk = (int64_t)k < n ? k : n;
  return kk * 8 > bm_supers(n);
}
// dynamic LDS of a row select: the fixed part + its threshold keys
inline size_t bm_select_lds(int64_t n, int k) {
  return kBmFixedLds + (size_t)(bm_by_block(n, k) ? bm_blocks(n) : bm_supers(n)) * 4;
}
// Workspace of the block-max top-k: block keys [B][nb], then superblock keys [B][ns].
inline uint32_t* bm_super_keys(uint32_t* bm, int32_t B, int64_t n) { return bm + (size_t)B * bm_blocks(n); }

// 16 lanes per 64-doc block (a float4 each), 4 blocks per wave-load, 4 loads
// in flight per lane: a wave covers 16 blocks, a workgroup 64.  Rows that do
// not start 16-B aligned (n % 4 != 0) load their floats one by one.
// sb (superblock keys, row stride sb_ld): the max of each 4 consecutive block
// keys = one 256-doc superblock (a wave's 4 rows of one load step).
__device__ __forceinline__ uint32_t umax_over_rows(uint32_t v) {   // max over lanes l, l^16, l^32, l^48
  auto t = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = max(t[0], t[1]);
  t = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return max(t[0], t[1]);
}
constexpr int kBmBlocksPerWg = 64;
__global__ __launch_bounds__(256) void block_max_kernel(const float* __restrict__ scores, int64_t n, int64_t ld,
                                                        uint32_t* __restrict__ bm, int64_t bm_ld,
                                                        uint32_t* __restrict__ sb, int64_t sb_ld) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.y;
  const int64_t nb = (n + 63) >> 6;
  const int c = lane & 15, r = lane >> 4;
  const int64_t b0 = (int64_t)blockIdx.x * kBmBlocksPerWg + wave * 16;
  const float* x = scores + (size_t)row * ld;
  const bool vec = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(scores) & 15) == 0);
  uint32_t key[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // block b0 + 4u + r, docs 64 * blk + 4c .. + 3
    const int64_t blk = b0 + 4 * u + r;
    const int64_t i = blk * 64 + 4 * c;
    uint32_t m = 0u;
    if (blk < nb) {
      if (vec && i + 3 < n) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
        m = max(max(f2u(v[0]), f2u(v[1])), max(f2u(v[2]), f2u(v[3])));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) m = (i + e < n) ? max(m, f2u(x[i + e])) : m;
      }
    }
    key[u] = m;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // max over each 16-lane row = one block
    uint32_t v = key[u];
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
    const int64_t blk = b0 + 4 * u + r;
    if (c == 0 && blk < nb) bm[(size_t)row * bm_ld + blk] = v;
    const uint32_t s4 = umax_over_rows(v);   // blocks b0 + 4u .. + 3 (b0 is a multiple of 16)
    if (lane == 0 && b0 + 4 * u < nb) sb[(size_t)row * sb_ld + (b0 >> 2) + u] = s4;
  }
}

// In-launch hand-off to the row's LAST workgroup (the workgroups of a row
// each store part of the row, the last one to finish reads all of it), by
// the write-through protocol of MI355X_MICROARCH.md's hand-off table, row 1 --
// no fences (an agent-scope __threadfence costs ~3.5 us per workgroup, more
// than the kernel boundary it would save):
//  * every handed-off store is an sc1 store (st_sc1) and every load of those
//    bytes in the last workgroup an sc1 load (ld_sc1: global_*, never flat_);
//  * each storing wave drains its stores (s_waitcnt vmcnt(0)) before the
//    workgroup barrier, then ONE lane adds to an agent-scope counter; the
//    workgroup whose add returned the last count is told so by the value;
//  * shards = 8 (launches of up to ~1k workgroups per row): the counter is
//    kept per XCD (blockIdx.x mod 8 -- a row's workgroups x and x + 8 share an
//    XCD), each on a 128-B line of its own, and each shard's last adder adds
//    to the row's top counter: ~1/8 of the serialised same-address atomics
//    (~12 ns each, "fanin" row of the price table).  shards = 1: one counter.
// The counters are zero before the launch; the last adders re-zero them, so
// the next launch on the stream finds them zero again.  Every workgroup of
// the row calls this exactly once (block-uniform); returns block-uniform.
constexpr int kArriveInts = 9 * 32;   // one row's sharded counters: 8 XCD shards + the top, 128 B apart
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __uint_as_float(
      __hip_atomic_load(reinterpret_cast<const uint32_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool row_last_arrival(int32_t* __restrict__ ctr, int nwg, int shards, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's sc1 stores have landed
  __syncthreads();
  if (threadIdx.x == 0) {
    int last = 0;
    if (shards == 1) {
      last = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nwg - 1;
      if (last) __hip_atomic_store(ctr, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      const int sh = (int)(blockIdx.x & 7u);
      const int per = (nwg - sh + 7) / 8;   // this shard's workgroups: x = sh (mod 8), x < nwg
      int32_t* c = ctr + 32 * sh;
      if (__hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == per - 1) {
        __hip_atomic_store(c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int used = nwg < 8 ? nwg : 8;
        last = __hip_atomic_fetch_add(ctr + 256, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == used - 1;
        if (last) __hip_atomic_store(ctr + 256, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    *s_flag = last;
  }
  __syncthreads();
  return *s_flag != 0;
}

// The select of one row (topk_bmax_kernel's work; run by a whole workgroup):
// bm / sb = the row's block and superblock keys, lds = bm_select_lds(n, k)
// bytes of LDS.
// SC1: bm / sb were stored in this launch (bmax_topk_kernel): read them with
// sc1 loads (the write-through hand-off, row_last_arrival).
// stamps (lab only, nullable): s_memrealtime at the phase ends -- [0] keys in
// LDS, [1] threshold, [2] qualifying blocks, [3] gather, [4] ranked + written;
// inside the threshold: [7] key range, [8] histogram, [9] bin found
constexpr int kLabWgs = 4096;                          // workgroups with start / end stamps
[[maybe_unused]] constexpr size_t kLabStride = 16 + 2 * (size_t)kLabWgs;   // u64 per stamped launch kind
__device__ __forceinline__ void lab_stamp(uint64_t* stamps, int i) {
  if (stamps != nullptr && threadIdx.x == 0) stamps[i] = __builtin_amdgcn_s_memrealtime();
}
template <bool SC1 = false>
__device__ void topk_bmax_row(const float* __restrict__ x, int64_t n, int k, int64_t id_base,
                              const uint32_t* __restrict__ brow, const uint32_t* __restrict__ srow, float* os,
                              int32_t* oi, uint8_t* lds, Mirror mirror = Mirror(), uint64_t* stamps = nullptr) {
  uint64_t* const sel = reinterpret_cast<uint64_t*>(lds);   // [kBmCand]
  uint32_t* const hist = reinterpret_cast<uint32_t*>(sel + kBmCand);   // [2048]
  uint32_t* const qual = hist + 2048;                              // [kBmQual]
  uint32_t* const misc = qual + kBmQual;                           // [16]
  uint32_t* const keys = misc + 16;                                // [ns] superblock keys
  const int tid = threadIdx.x, nth = blockDim.x, wave = tid >> 6;
  const int nb = (int)((n + 63) >> 6);
  const int ns = (int)((n + 255) >> 8);
  const int kk = (int)((int64_t)k < n ? k : n);
  // (bm_by_block: the threshold over the 64-doc block keys)
  const bool by_block = bm_by_block(n, k);
  const int nk = by_block ? nb : ns;
  const uint32_t kleft = (uint32_t)(kk < nk ? kk : nk);
  // the threshold's keys into LDS (superblock keys, or the block keys when
  // by_block: lds = bm_select_lds), with this thread's range of them
  uint32_t mx = 0u, mn = ~0u;
  for (int i = tid; i < nk; i += nth) {
    const uint32_t u = by_block ? (SC1 ? ld_sc1(brow + i) : brow[i]) : (SC1 ? ld_sc1(srow + i) : srow[i]);
    keys[i] = u;
    mx = max(mx, u);
    mn = min(mn, u);
  }
  for (int b = tid; b < kBmBins; b += nth) hist[b] = 0;
  if (tid < 16) misc[tid] = (tid == 9 || tid == 10) ? ~0u : 0u;   // [8] max, [9] min, [10] t
  mx = wave_max_u32(mx);
  mn = wave_min_u32(mn);
  __syncthreads();   // misc zeroed before the atomics below
  if ((tid & 63) == 0) {
    atomicMax(&misc[8], mx);
    atomicMin(&misc[9], mn);
  }
  __syncthreads();
  lab_stamp(stamps, 0);
  // 1. t = a key that at least kleft = min(kk, keys) of the keys reach:
  //    kleft superblocks (blocks) have a max >= t, so the kk-th largest score
  //    is >= t, and every doc >= t lies in a 64-doc block whose key is >= t.
  //    Any such t is correct -- the kleft-th largest key itself or one below
  //    it (a lower t only gathers more candidates) -- so no exact selection:
  //    the keys' range [lo, hi] in kBmBins linear bins, the bin at which the
  //    count from the top reaches kleft (find_bin), t = the smallest key of
  //    that bin and the bins above it.  Keys in LDS, one histogram pass, one
  //    minimum pass.  (Lab, B=1 at 125k docs: 7.2 us for two exact radix
  //    passes over the block keys in L2; 24 us for one wave bisecting them.)
  const uint32_t khi = misc[8];
  // larger key -> higher bin (find_bin counts from the top bin down); the
  // bin index in float arithmetic (no 64-bit division): only its
  // monotonicity matters, and float conversion, scaling and truncation are
  // monotone
  const float bscale = (float)kBmBins / ((float)(khi - misc[9]) + 1.0f);
  auto bin_of = [&](uint32_t u) {
    const uint32_t d = (uint32_t)((float)(khi - u) * bscale);
    return (uint32_t)(kBmBins - 1) - (d < (uint32_t)kBmBins ? d : (uint32_t)(kBmBins - 1));
  };
  for (int i = tid; i < nk; i += nth) atomicAdd(&hist[bin_of(keys[i])], 1u);   // linear bins: few collisions
  __syncthreads();
  if (wave == 0) find_bin1024(hist, kleft, &misc[4], &misc[5], &misc[6]);
  __syncthreads();
  {
    const uint32_t bstar = misc[4];
    uint32_t tm = ~0u;
    for (int i = tid; i < nk; i += nth) {
      const uint32_t u = keys[i];
      if (bin_of(u) >= bstar) tm = min(tm, u);
    }
    tm = wave_min_u32(tm);
    if ((tid & 63) == 0) atomicMin(&misc[10], tm);
  }
  __syncthreads();
  const uint32_t t = misc[10];
  lab_stamp(stamps, 1);
  // 2. the 64-doc blocks whose max reaches t: by superblock, the superblocks
  //    >= t first (their keys in LDS; listed in hist, free again), then the
  //    <= 4 block keys of each, all loads in flight at once (not a pass over
  //    every block key: ~4 dependent load rounds per thread at 1M docs)
  if (by_block) {
    for (int j = tid; j < nb; j += nth)
      if (keys[j] >= t) {
        const uint32_t pos = atomicAdd(&misc[0], 1u);
        if (pos < (uint32_t)kBmQual) qual[pos] = (uint32_t)j;
      }
  } else {
    for (int i = tid; i < ns; i += nth)
      if (keys[i] >= t) {
        const uint32_t pos = atomicAdd(&misc[2], 1u);
        if (pos < (uint32_t)kBmBins) hist[pos] = (uint32_t)i;
      }
    __syncthreads();
    const uint32_t nsq = misc[2];
    if (nsq > (uint32_t)kBmBins) {
      if (tid == 0) misc[0] = (uint32_t)kBmQual + 1;   // too many: the exact fallback below
    } else {
      for (uint32_t w = tid; w < 4 * nsq; w += (uint32_t)nth) {
        const int j = 4 * (int)hist[w >> 2] + (int)(w & 3);
        if (j < nb && (SC1 ? ld_sc1(brow + j) : brow[j]) >= t) {
          const uint32_t pos = atomicAdd(&misc[0], 1u);
          if (pos < (uint32_t)kBmQual) qual[pos] = (uint32_t)j;
        }
      }
    }
  }
  __syncthreads();
  lab_stamp(stamps, 2);
  const uint32_t nqual = misc[0];
  if (nqual <= (uint32_t)kBmQual) {
    // 4 scores per thread per step (a float4 when the row is 16-B aligned),
    // U steps of loads in flight: a 64-doc block = 16 threads
    constexpr int U = 2;
    const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    const uint32_t total = nqual * 16;
    for (uint32_t w0 = tid; w0 < total; w0 += (uint32_t)nth * U) {
      float v[U][4];
      int64_t i0[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint32_t w = w0 + (uint32_t)(u * nth);
        i0[u] = w < total ? (int64_t)qual[w >> 4] * 64 + 4 * (w & 15) : n;
        if (vec && i0[u] + 3 < n) {
          const f32x4 q = *reinterpret_cast<const f32x4*>(x + i0[u]);
          v[u][0] = q[0], v[u][1] = q[1], v[u][2] = q[2], v[u][3] = q[3];
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[u][e] = i0[u] + e < n ? x[i0[u] + e] : neg_inf();
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (i0[u] + e < n && f2u(v[u][e]) >= t) {
            const uint32_t pos = atomicAdd(&misc[1], 1u);
            if (pos < (uint32_t)kBmCand) sel[pos] = rank_key(v[u][e], (uint32_t)(i0[u] + e));
          }
    }
  }
  __syncthreads();
  lab_stamp(stamps, 3);
  const uint32_t ncand = misc[1];
  int m = (int)ncand;
  if (nqual > (uint32_t)kBmQual || ncand < (uint32_t)kk || ncand > (uint32_t)kBmCand) {
    __syncthreads();
    topk_exact_row(x, n, kk, sel, hist, &misc[4], &misc[5], &misc[6], &misc[7]);
    m = kk;
  }
  if (m <= kBmRankMax) {   // rank by counting: keys are unique, rank = #greater
    // T threads per key (consecutive lanes), each counting m / T of the keys
    int T = 1;
    while (T < 64 && 2 * T * m <= nth) T <<= 1;
    const int i = tid / T, p = tid & (T - 1);
    const uint64_t key = i < m ? sel[i] : 0ull;
    int r = 0;
    if (i < m)
      for (int j = p; j < m; j += T) r += sel[j] > key ? 1 : 0;
    for (int o = 1; o < T; o <<= 1) r += __shfl_xor(r, o);
    if (i < m && p == 0 && r < k) {
      os[r] = u2f((uint32_t)(key >> 32));
      oi[r] = (int32_t)(id_base + (int64_t)(~(uint32_t)key));
      if (mirror.w != nullptr) mirror.put(r, oi[r], os[r]);
    }
    for (int j = m + tid; j < k; j += nth) {
      os[j] = neg_inf();
      oi[j] = -1;
      if (mirror.w != nullptr) mirror.put(j, -1, neg_inf());
    }
  } else {
    sort_and_write(sel, m, k, id_base, os, oi, mirror);
  }
  if (stamps != nullptr) {
    __syncthreads();
    lab_stamp(stamps, 4);
    if (tid == 0) stamps[5] = ((uint64_t)nqual << 32) | ncand;
  }
}

__global__ __launch_bounds__(kTkThreads) void topk_bmax_kernel(const float* __restrict__ scores, int64_t n, int64_t ld,
                                                               int k, int64_t id_base, const uint32_t* __restrict__ bm,
                                                               int64_t bm_ld, const uint32_t* __restrict__ sb,
                                                               int64_t sb_ld, float* __restrict__ out_s,
                                                               int32_t* __restrict__ out_i,
                                                               Mirror mirror = Mirror(),
                                                               uint64_t* __restrict__ stamps = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bm_dyn[];
  const int row = blockIdx.x;
  if (stamps != nullptr && row == 0 && threadIdx.x == 0) {   // lab: row 0 (start = its select's start)
    const uint64_t t = __builtin_amdgcn_s_memrealtime();
    stamps[16] = t;
    stamps[17] = t;
    stamps[6] = t;
  }
  topk_bmax_row(scores + (size_t)row * ld, n, k, id_base, bm + (size_t)row * bm_ld, sb + (size_t)row * sb_ld,
                out_s + (size_t)row * k, out_i + (size_t)row * k, bm_dyn, mirror.row(row, k),
                row == 0 ? stamps : nullptr);
}

// Block-max top-k in ONE launch (small batches, the latency path): grid (P, B)
// of 1024-thread workgroups, each writing the block and superblock keys of 256
// blocks (16,384 docs) of row b as block_max_kernel does, then the row's last
// workgroup to finish (row_last_arrival on done[b]) runs the row's select
// (topk_bmax_row).  Same keys, same select: the same results as block_max +
// topk_bmax_kernel, one launch and its gap fewer.
constexpr int kBmFusedBlocksPerWg = 16 * (kTkThreads / 64);   // 16 blocks per wave
__global__ __launch_bounds__(kTkThreads) void bmax_topk_kernel(const float* __restrict__ scores, int64_t n, int64_t ld,
                                                               int k, int64_t id_base, uint32_t* __restrict__ bm,
                                                               int64_t bm_ld, uint32_t* __restrict__ sb, int64_t sb_ld,
                                                               int32_t* __restrict__ done, int64_t done_ld,
                                                               float* __restrict__ out_s, int32_t* __restrict__ out_i,
                                                               Mirror mirror, uint64_t* __restrict__ stamps = nullptr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t bm_dyn[];
  __shared__ int s_last;
  // stamps (lab only): [16 + 2x] / [17 + 2x] workgroup x's start / keys
  // stored, [6] the last arrival
  if (stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs)
    stamps[16 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.y;
  const int64_t nb = (n + 63) >> 6;
  const int c = lane & 15, r = lane >> 4;
  const int64_t b0 = (int64_t)blockIdx.x * kBmFusedBlocksPerWg + wave * 16;
  const float* x = scores + (size_t)row * ld;
  uint32_t* brow = bm + (size_t)row * bm_ld;
  uint32_t* srow = sb + (size_t)row * sb_ld;
  const bool vec = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(scores) & 15) == 0);
  uint32_t key[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // block b0 + 4u + r, docs 64 * blk + 4c .. + 3
    const int64_t blk = b0 + 4 * u + r;
    const int64_t i = blk * 64 + 4 * c;
    uint32_t m = 0u;
    if (blk < nb) {
      if (vec && i + 3 < n) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(x + i);
        m = max(max(f2u(v[0]), f2u(v[1])), max(f2u(v[2]), f2u(v[3])));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) m = (i + e < n) ? max(m, f2u(x[i + e])) : m;
      }
    }
    key[u] = m;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {   // max over each 16-lane row = one block
    uint32_t v = key[u];
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, true));
    v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, true));
    const int64_t blk = b0 + 4 * u + r;
    if (c == 0 && blk < nb) st_sc1(brow + blk, v);
    const uint32_t s4 = umax_over_rows(v);   // blocks b0 + 4u .. + 3 (b0 is a multiple of 16)
    if (lane == 0 && b0 + 4 * u < nb) st_sc1(srow + (b0 >> 2) + u, s4);
  }
  // <= 96 workgroups per row (n <= 64 * kBmMaxBlocks): one counter
  if (stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs)
    stamps[17 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (!row_last_arrival(done + (size_t)row * done_ld, (int)gridDim.x, 1, &s_last)) return;
  lab_stamp(stamps, 6);
  topk_bmax_row<true>(x, n, k, id_base, brow, srow, out_s + (size_t)row * k, out_i + (size_t)row * k, bm_dyn,
                      mirror.row(row, k), stamps);
}

// ---------------------------------------------------------------------------
// Top-k of the fused scan's per-workgroup lists: row b holds M = slots * k
// unique 64-bit ranking keys (0 = padding).  Exact radix select of the
// kk = min(k, M)-th largest key (8 passes of 8-bit digits over the keys in
// global memory / L2), then the kk keys >= it (exactly kk: keys are unique)
// sorted in LDS; a 0 key is written as (-inf, -1).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kTkThreads) void select_keys_kernel(const uint64_t* __restrict__ keys, int64_t M,
                                                                 int64_t row_stride, int k, int64_t id_base,
                                                                 float* __restrict__ out_s,
                                                                 int32_t* __restrict__ out_i) {
  __shared__ uint32_t hist[256];
  __shared__ uint64_t sel[kTopkMax];
  __shared__ uint32_t s_bin, s_above, s_bincount, s_cnt;
  const int tid = threadIdx.x, wave = tid >> 6;
  const uint64_t* x = keys + (size_t)blockIdx.x * row_stride;
  const int kk = (int)((int64_t)k < M ? k : M);
  uint64_t prefix = 0, mask = 0;
  uint32_t kleft = (uint32_t)kk;
  for (int p = 0; p < 8; ++p) {
    const int shift = 56 - 8 * p;
    if (tid < 256) hist[tid] = 0;
    __syncthreads();
    for (int64_t i = tid; i < M; i += kTkThreads) {
      const uint64_t u = x[i];
      hist_add(hist, (u >> shift) & 255, (u & mask) == prefix);
    }
    __syncthreads();
    if (wave == 0) find_bin(hist, 256, kleft, &s_bin, &s_above, &s_bincount);
    __syncthreads();
    kleft -= s_above;
    prefix |= (uint64_t)s_bin << shift;
    mask |= 255ull << shift;
    __syncthreads();
  }
  // the kk keys >= the kk-th largest (unique, except padding zeros: when the
  // kk-th largest is 0 only the nonzero keys are collected, the rest pad)
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for (int64_t i = tid; i < M; i += kTkThreads) {
    const uint64_t u = x[i];
    if (u >= prefix && u != 0ull) {
      const uint32_t pos = atomicAdd(&s_cnt, 1u);
      if (pos < (uint32_t)kk) sel[pos] = u;
    }
  }
  __syncthreads();
  const int got = (int)(s_cnt < (uint32_t)kk ? s_cnt : (uint32_t)kk);
  int P = 1;
  while (P < kk) P <<= 1;
  for (int i = got + tid; i < P; i += kTkThreads) sel[i] = 0;
  bitonic_desc(sel, P);
  float* os = out_s + (size_t)blockIdx.x * k;
  int32_t* oi = out_i + (size_t)blockIdx.x * k;
  for (int j = tid; j < k; j += kTkThreads) {
    const uint64_t key = j < kk ? sel[j] : 0ull;
    os[j] = key ? u2f((uint32_t)(key >> 32)) : neg_inf();
    oi[j] = key ? (int32_t)(id_base + (int64_t)(~(uint32_t)key)) : -1;
  }
}

// ---------------------------------------------------------------------------
// Small-row selection (rank counting; rows of C <= 1024).
// ---------------------------------------------------------------------------
// fin (w nullable): the row's result also to fin's host words (row b; an id
// the caller does not take is written -1)
__device__ void select_from_lds(const float* sc, const uint64_t* keys, int C, int k, const int32_t* ids_row,
                                float* out_s, int32_t* out_i, int32_t* out_p, FinalMirror fin = FinalMirror(),
                                size_t b = 0) {
  for (int t = threadIdx.x; t < C; t += blockDim.x) {
    const uint64_t kt = keys[t];
    int rank = 0;
    for (int j = 0; j < C; ++j) rank += (keys[j] > kt);
    if (rank < k) {
      const int32_t id = ids_row ? ids_row[t] : t;
      out_s[rank] = sc[t];
      if (out_i) out_i[rank] = id;
      if (out_p) out_p[rank] = t;
      if (fin.w != nullptr) fin.put(b, rank, sc[t], out_i ? id : -1, t);
    }
  }
  for (int j = C + threadIdx.x; j < k; j += blockDim.x) {
    out_s[j] = neg_inf();
    if (out_i) out_i[j] = -1;
    if (out_p) out_p[j] = -1;
    if (fin.w != nullptr) fin.put(b, j, neg_inf(), -1, -1);
  }
}

// ids_tagged (nullable): the ids as the pre-armed rerank's tagged words (all
// present: the rerank that ran before on the stream waited for them)
__global__ __launch_bounds__(256) void select_small_kernel(const float* __restrict__ scores,
                                                           const int32_t* __restrict__ ids, int C, int k,
                                                           float* __restrict__ out_s,
                                                           int32_t* __restrict__ out_i,
                                                           int32_t* __restrict__ out_p,
                                                           const uint64_t* __restrict__ ids_tagged = nullptr,
                                                           FinalMirror fin = FinalMirror()) {
  __shared__ float sc[kSmallMax];
  __shared__ uint64_t keys[kSmallMax];
  __shared__ int32_t tid_ids[kSmallMax];
  const size_t b = blockIdx.x;
  for (int t = threadIdx.x; t < C; t += blockDim.x) {
    sc[t] = scores[b * C + t];
    keys[t] = rank_key(sc[t], (uint32_t)t);
    if (ids_tagged != nullptr) tid_ids[t] = read_tagged(ids_tagged + b * C + t);
  }
  __syncthreads();
  const int32_t* idr = ids_tagged != nullptr ? tid_ids : (ids ? ids + b * C : nullptr);
  select_from_lds(sc, keys, C, k, idr, out_s + b * k, out_i ? out_i + b * k : nullptr,
                  out_p ? out_p + b * k : nullptr, fin, b);
}

// The sharded stage 3 without a collective (sharded.cpp,
// cbv2_rerank_sharded_prescored): every fused candidate's rerank score is
// already in the stage-2 all-gather -- its owner's local top-k list (the
// scan's / band's score of the doc: the rerank's bits, test_gpu_fp8 /
// DESIGN §3.7) or its owner's stage-1 prescore (the rerank of the rank's own
// BM25 top-kb, run before the all-gather).  Row b of the gathered blocks
// (rank g's block at recv + g * blk words: [B][k] scores | [B][k] ids | [B][kb]
// BM25 scores | [B][kb] BM25 ids | [B][kb] prescores): the row's candidates go
// into an LDS id table (open addressing), every gathered (id, score) entry
// probes it, and the row's top-k is selected as select_small_kernel does
// (score desc, position asc).  A candidate found nowhere (not from these
// lists) scores -inf and is counted in *misses; a negative id scores -inf,
// as the rerank scores it.  C <= kSmallMax.
constexpr int kPreTab = 2 * kSmallMax;   // id table slots (a power of two >= 2 C)
__global__ __launch_bounds__(256) void prescored_select_kernel(
    const int32_t* __restrict__ recv, int G, int64_t blk, int B, int k, int kb, const int32_t* __restrict__ cand,
    int C, int fk, float* __restrict__ out_s, int32_t* __restrict__ out_i, int32_t* __restrict__ out_p,
    int32_t* __restrict__ misses) {
  __shared__ float sc[kSmallMax];
  __shared__ uint64_t keys[kSmallMax];
  __shared__ int32_t tab_id[kPreTab];
  __shared__ uint32_t tab_sc[kPreTab];
  __shared__ int32_t tab_hit[kPreTab];
  const int b = blockIdx.x;
  const int32_t* crow = cand + (size_t)b * C;
  int bits = 4;
  while ((1 << bits) < 2 * C) ++bits;
  const uint32_t mask = (1u << bits) - 1;
  auto slot0 = [&](int32_t id) { return ((uint32_t)id * 2654435761u) >> (32 - bits); };
  for (int t = threadIdx.x; t <= (int)mask; t += blockDim.x) {
    tab_id[t] = -1;
    tab_hit[t] = 0;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < C; t += blockDim.x) {   // the row's candidates (duplicates share a slot)
    const int32_t id = crow[t];
    if (id < 0) continue;
    for (uint32_t h = slot0(id);; h = (h + 1) & mask) {
      const int32_t prev = atomicCAS(&tab_id[h], -1, id);
      if (prev == -1 || prev == id) break;
    }
  }
  __syncthreads();
  const int per = k + kb;
  for (int e = threadIdx.x; e < G * per; e += blockDim.x) {   // every gathered (id, score) of row b
    const int g = e / per, j = e - g * per;
    const int32_t* base = recv + (size_t)g * blk;
    int32_t id;
    uint32_t sb;
    if (j < k) {
      id = base[(size_t)B * k + (size_t)b * k + j];
      sb = (uint32_t)base[(size_t)b * k + j];
    } else {
      const size_t jj = (size_t)b * kb + (j - k);
      id = base[2 * (size_t)B * k + (size_t)B * kb + jj];
      sb = (uint32_t)base[2 * (size_t)B * k + 2 * (size_t)B * kb + jj];
    }
    if (id < 0) continue;
    for (uint32_t h = slot0(id);; h = (h + 1) & mask) {
      const int32_t t = tab_id[h];
      if (t == -1) break;
      if (t == id) {   // (an id in both of its owner's lists carries the same bits in each)
        tab_sc[h] = sb;
        tab_hit[h] = 1;
        break;
      }
    }
  }
  __syncthreads();
  int miss = 0;
  for (int t = threadIdx.x; t < C; t += blockDim.x) {
    const int32_t id = crow[t];
    float v = neg_inf();
    if (id >= 0) {
      uint32_t h = slot0(id);
      while (tab_id[h] != id) h = (h + 1) & mask;
      if (tab_hit[h]) v = __uint_as_float(tab_sc[h]);
      else ++miss;
    }
    sc[t] = v;
    keys[t] = rank_key(v, (uint32_t)t);
  }
  if (miss != 0 && misses != nullptr) atomicAdd(misses, miss);
  __syncthreads();
  select_from_lds(sc, keys, C, fk, crow, out_s + (size_t)b * fk, out_i + (size_t)b * fk,
                  out_p ? out_p + (size_t)b * fk : nullptr);
}

// ---------------------------------------------------------------------------
// Rerank: one workgroup per query; each wave gathers whole candidate docs
// (32 KiB, contiguous) straight into VGPRs and scores them with the same MFMA
// tiling as the scan; then rank-select top-k in LDS.  BIG (C > kSmallMax): the
// C raw scores live in dynamic LDS (C <= kRerankMaxC) and the selection is the
// multi-pass one (any k).
// ---------------------------------------------------------------------------
constexpr int kRrWaves = 8;
constexpr int kRerankMaxC = 32768;   // BIG: 128 KiB of scores + 16 KiB of selection state

__device__ __forceinline__ float rerank_one_bf16(const uint8_t* __restrict__ tokens,
                                                 const int32_t* __restrict__ doclens, int64_t n, int64_t id_base,
                                                 const bf16x8 (&qf)[1][2][4], int lq, int32_t id, int lane,
                                                 int ld) {
  const int64_t loc = (int64_t)id - id_base;
  if (id < 0 || loc < 0 || loc >= n) return neg_inf();
  const int g = lane >> 4;
  int dl = doclens[loc];
  dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
  float m[1][2] = {{neg_inf(), neg_inf()}};
  // 128 tokens at a time (one block unless the index holds long docs): the
  // whole block in flight at once (32 KiB per wave), then the scan's math
  for (int blk = 0; blk == 0 || kLd * blk < dl; ++blk) {
    const int dlb = dl - kLd * blk;
    const uint8_t* dbase = tokens + (size_t)loc * (size_t)ld * kRowBytes + (size_t)blk * kDocBytes;
    bf16x8 af[kLd / 16][4];
#pragma unroll
    for (int rt = 0; rt < kLd / 16; ++rt)
      if (16 * rt < dlb) gbl_afrag16(dbase, rt, lane, af[rt]);
#pragma unroll
    for (int rt = 0; rt < kLd / 16; ++rt) {
      if (16 * rt < dlb) {
        const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
        tile16<1>(af[rt], qf, init, m);
      }
    }
  }
  return reduce16(m[0][0], m[0][1], lane, lq);
}

// The selection tail shared by the bf16 and MXFP8 rerank kernels: sc[0..C) raw
// candidate scores (LDS) -> raw output (k == 0) or the top-k by position rule.
template <bool BIG>
__device__ __forceinline__ void rerank_finish(float* sc, uint64_t* keys, uint32_t* hist, uint32_t* misc, int b,
                                              const int32_t* crow, int C, int k, float* __restrict__ out_s,
                                              int32_t* __restrict__ out_i, int32_t* __restrict__ out_p) {
  __syncthreads();
  if (k == 0) {
    for (int t = threadIdx.x; t < C; t += blockDim.x) out_s[(size_t)b * C + t] = sc[t];
    return;
  }
  if constexpr (BIG) {
    topk_multi_row<kTopkMax>(sc, C, k, crow, 0, out_s + (size_t)b * k, out_i + (size_t)b * k,
                             out_p ? out_p + (size_t)b * k : nullptr, keys, hist, misc);
  } else {
    for (int t = threadIdx.x; t < C; t += blockDim.x) keys[t] = rank_key(sc[t], (uint32_t)t);
    __syncthreads();
    select_from_lds(sc, keys, C, k, crow, out_s + (size_t)b * k, out_i + (size_t)b * k,
                    out_p ? out_p + (size_t)b * k : nullptr);
  }
}

template <bool BIG = false>
__global__ __launch_bounds__(kRrWaves * 64) void rerank_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n, int64_t id_base,
    const uint16_t* __restrict__ Q, int lq, const int32_t* __restrict__ cand, int C, int k,
    float* __restrict__ out_s, int32_t* __restrict__ out_i, int32_t* __restrict__ out_p, int ld) {
  extern __shared__ float sc_dyn[];
  __shared__ float sc_fix[BIG ? 1 : kSmallMax];
  __shared__ uint64_t keys[BIG ? kTopkMax : kSmallMax];
  __shared__ uint32_t hist[BIG ? 2048 : 1];
  __shared__ uint32_t misc[4];
  float* sc = BIG ? sc_dyn : sc_fix;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  bf16x8 qf[1][2][4];
  load_qfrag16(Q, b, b + 1, lq, lane, qf[0]);
  const int32_t* crow = cand + (size_t)b * C;
  for (int c = wave; c < C; c += kRrWaves) {
    const float v = rerank_one_bf16(tokens, doclens, n, id_base, qf, lq, crow[c], lane, ld);
    if (lane == 0) sc[c] = v;
  }
  rerank_finish<BIG>(sc, keys, hist, misc, b, crow, C, k, out_s, out_i, out_p);
}

__device__ __forceinline__ float rerank_one_f8(const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales,
                                               const int32_t* __restrict__ doclens, int64_t n, int64_t id_base,
                                               const i32x8 (&qa)[1][2], const int (&qs)[1][2], int lq, int32_t id,
                                               int lane, int ld) {
  const int64_t loc = (int64_t)id - id_base;
  if (id < 0 || loc < 0 || loc >= n) return neg_inf();
  const int g = lane >> 4;
  int dl = doclens[loc];
  dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
  float m[1][2] = {{neg_inf(), neg_inf()}};
  for (int blk = 0; blk == 0 || kLd * blk < dl; ++blk) {   // long documents: 128-token blocks
    const int dlb = dl - kLd * blk;
    const uint8_t* dbase = tokens + ((size_t)loc * ld + (size_t)kLd * blk) * kDim;
    const uint8_t* dsc = tscales + ((size_t)loc * ld + (size_t)kLd * blk) * 2;
    i32x8 af[kLd / 16];
    int as[kLd / 16];
#pragma unroll
    for (int rt = 0; rt < kLd / 16; ++rt)
      if (16 * rt < dlb) gbl_afrag_f8(dbase, dsc, rt, lane, af[rt], as[rt]);
#pragma unroll
    for (int rt = 0; rt < kLd / 16; ++rt) {
      if (16 * rt < dlb) {
        const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
        tile_f8<1>(af[rt], as[rt], qa, qs, init, m);
      }
    }
  }
  return reduce16(m[0][0], m[0][1], lane, lq);
}

template <bool BIG = false>
__global__ __launch_bounds__(kRrWaves * 64) void rerank_f8_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, int64_t id_base, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int lq,
    const int32_t* __restrict__ cand, int C, int k, float* __restrict__ out_s, int32_t* __restrict__ out_i,
    int32_t* __restrict__ out_p, int ld) {
  extern __shared__ float sc_dyn[];
  __shared__ float sc_fix[BIG ? 1 : kSmallMax];
  __shared__ uint64_t keys[BIG ? kTopkMax : kSmallMax];
  __shared__ uint32_t hist[BIG ? 2048 : 1];
  __shared__ uint32_t misc[4];
  float* sc = BIG ? sc_dyn : sc_fix;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x;
  i32x8 qa[1][2];
  int qs[1][2];
  load_qfrag_f8(Qb, Qs, b, b + 1, lq, lane, qa[0], qs[0]);
  const int32_t* crow = cand + (size_t)b * C;
  for (int c = wave; c < C; c += kRrWaves) {
    const float v = rerank_one_f8(tokens, tscales, doclens, n, id_base, qa, qs, lq, crow[c], lane, ld);
    if (lane == 0) sc[c] = v;
  }
  rerank_finish<BIG>(sc, keys, hist, misc, b, crow, C, k, out_s, out_i, out_p);
}

// Candidate-parallel rerank scores (small batches, raw): one wave per (query,
// candidate), grid (ceil(C / kRrWaves), B).  A B=1 rerank of 50 candidates
// then spreads over 7 CUs instead of running 7 candidates per wave in
// sequence on one; the same per-candidate math (rerank_one_*), so the same
// bits.  The top-k of the raw row is select_small_kernel (= rerank_finish).
template <bool F8>
__global__ __launch_bounds__(kRrWaves * 64) void rerank_raw_kernel(
    const uint8_t* __restrict__ tokens, const uint8_t* __restrict__ tscales, const int32_t* __restrict__ doclens,
    int64_t n, int64_t id_base, const uint8_t* __restrict__ Qb, const uint8_t* __restrict__ Qs, int lq,
    const int32_t* __restrict__ cand, int C, float* __restrict__ raw, int ld) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int c = blockIdx.x * kRrWaves + wave;
  if (c >= C) return;   // wave-uniform; no barriers below
  const int32_t id = cand[(size_t)b * C + c];
  float v;
  if constexpr (F8) {
    i32x8 qa[1][2];
    int qs[1][2];
    load_qfrag_f8(Qb, Qs, b, b + 1, lq, lane, qa[0], qs[0]);
    v = rerank_one_f8(tokens, tscales, doclens, n, id_base, qa, qs, lq, id, lane, ld);
  } else {
    bf16x8 qf[1][2][4];
    load_qfrag16(reinterpret_cast<const uint16_t*>(Qb), b, b + 1, lq, lane, qf[0]);
    v = rerank_one_bf16(tokens, doclens, n, id_base, qf, lq, id, lane, ld);
  }
  if (lane == 0) raw[(size_t)b * C + c] = v;
}

// bf16 rerank of small batches with one (query, candidate) per WORKGROUP: the
// doc's 128-token blocks split over the 4 waves (wave w: row tiles 2w, 2w + 1),
// each wave's column maxima max'ed in LDS and summed by wave 0 as reduce16
// does -- max is exact, so the bits equal rerank_one_bf16's (one wave walking
// all 8 tiles), at one 8 KiB HBM round trip per wave instead of 32 KiB.
__global__ __launch_bounds__(256, 2) void rerank_split_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n, int64_t id_base,
    const uint16_t* __restrict__ Q, int lq, const int32_t* __restrict__ cand, int C, float* __restrict__ raw, int ld,
    TaggedCand tc = TaggedCand(), Mirror raw_words = Mirror()) {
  __shared__ float s_m[4][32];
  __shared__ int32_t s_cid;
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y, c = blockIdx.x;
  int32_t id;
  if (tc.w != nullptr) {   // pre-armed: the host writes the candidate after this launch
    if (threadIdx.x == 0) s_cid = wait_tagged(tc.w + (size_t)b * C + c, tc);
    __syncthreads();
    id = s_cid;
  } else {
    id = cand[(size_t)b * C + c];
  }
  const int64_t loc = (int64_t)id - id_base;
  if (id < 0 || loc < 0 || loc >= n) {   // block-uniform
    if (threadIdx.x == 0) {
      raw[(size_t)b * C + c] = neg_inf();
      if (raw_words.w != nullptr) raw_words.put((size_t)b * C + c, (int32_t)__float_as_uint(neg_inf()), 0.0f);
    }
    return;
  }
  bf16x8 qf[1][2][4];
  load_qfrag16(Q, b, b + 1, lq, lane, qf[0]);
  int dl = doclens[loc];
  float m[1][2] = {{neg_inf(), neg_inf()}};
  for (int blk = 0; blk == 0 || kLd * blk < dl; ++blk) {
    const uint8_t* dbase = tokens + (size_t)loc * (size_t)ld * kRowBytes + (size_t)blk * kDocBytes;
    bf16x8 af[2][4];
#pragma unroll
    for (int t = 0; t < 2; ++t)   // the first block's loads do not wait for the doc length
      if (blk == 0 || 16 * (2 * wave + t) < dl - kLd * blk) gbl_afrag16(dbase, 2 * wave + t, lane, af[t]);
    if (blk == 0) dl = dl < 0 ? 0 : (dl > ld ? ld : dl);
    const int dlb = dl - kLd * blk;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int rt = 2 * wave + t;
      if (16 * rt < dlb) {
        const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
        tile16<1>(af[t], qf, init, m);
      }
    }
  }
  const float w0 = fold16_max(fold32_max(m[0][0])), w1 = fold16_max(fold32_max(m[0][1]));
  if (lane < 16) {
    s_m[wave][lane] = w0;
    s_m[wave][16 + lane] = w1;
  }
  __syncthreads();
  if (wave == 0) {
    const float m0 = fmaxf(fmaxf(s_m[0][c16], s_m[1][c16]), fmaxf(s_m[2][c16], s_m[3][c16]));
    const float m1 = fmaxf(fmaxf(s_m[0][16 + c16], s_m[1][16 + c16]), fmaxf(s_m[2][16 + c16], s_m[3][16 + c16]));
    const float v = dpp_row_sum16((c16 < lq ? m0 : 0.0f) + (16 + c16 < lq ? m1 : 0.0f));
    if (lane == 0) {
      raw[(size_t)b * C + c] = v;
      if (raw_words.w != nullptr) raw_words.put((size_t)b * C + c, (int32_t)__float_as_uint(v), 0.0f);
    }
  }
}

// ---------------------------------------------------------------------------
// fp32-faithful path (an index built from fp32 embeddings, as the reference
// stores them: local_rag_complete.py:735-746).  Each fp32 token x is split
// into hi = bf16(x) (round to nearest even; the index tokens every scan reads)
// and lo = bf16(x - hi) (the residual, read only for candidates).  A
// candidate's faithful score takes three bf16 MFMAs per product
// (lo.qhi + hi.qlo first, then hi.qhi; only lo.qlo ~2^-16 is dropped), fp32
// accumulate.  The bf16 scan's score T of any doc is within beta(q) of its
// exact score (Cauchy-Schwarz on the residuals, bounds below), so every doc
// of the exact top-k has T >= T_k - 2 beta(q): the band the search rescores.
// ---------------------------------------------------------------------------
constexpr float kBoundUp = 1.0f + 1.0f / 1024.0f;  // rounds fp32 norm sums up
constexpr float kAccSlack = 1.0f / 4096.0f;        // MFMA accumulation + dropped terms, per |q||d|

// 16 lanes per 128-value row, 8 values per lane: split into hi/lo, return the
// lane-group sums of x^2, (x - hi)^2 and hi^2 in every lane of the group.
__device__ __forceinline__ void split_row8(const float* __restrict__ src, uint16_t* __restrict__ hi,
                                           uint16_t* __restrict__ lo, int sub, float& xx, float& rr, float& hh) {
  const f32x4* s4 = reinterpret_cast<const f32x4*>(src + 8 * sub);
  const f32x4 v0 = s4[0], v1 = s4[1];
  float x[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
  uint16_t h[8], l[8];
  xx = rr = hh = 0.0f;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const __bf16 bh = (__bf16)x[e];
    const float fh = (float)bh;
    const float r = x[e] - fh;  // exact: hi is the rounding of x
    const __bf16 bl = (__bf16)r;
    h[e] = __builtin_bit_cast(uint16_t, bh);
    l[e] = __builtin_bit_cast(uint16_t, bl);
    xx += x[e] * x[e];
    rr += r * r;
    hh += fh * fh;
  }
  u32x4 ph, pl;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    ph[e] = (uint32_t)h[2 * e] | ((uint32_t)h[2 * e + 1] << 16);
    pl[e] = (uint32_t)l[2 * e] | ((uint32_t)l[2 * e + 1] << 16);
  }
  *reinterpret_cast<u32x4*>(hi + 8 * sub) = ph;
  *reinterpret_cast<u32x4*>(lo + 8 * sub) = pl;
#pragma unroll
  for (int off = 1; off < 16; off <<= 1) {
    xx += __shfl_xor(xx, off);
    rr += __shfl_xor(rr, off);
    hh += __shfl_xor(hh, off);
  }
}

// Index split: rows of 128 f32 -> hi, lo; bounds[0] = max ||x - hi||, bounds[1]
// = max ||hi|| over the rows that score (rounded up; atomic max on the
// non-negative bits).  doclens (nullable): rows are docs of ld rows and row t
// of doc i scores iff t < doclens[i] (padding is split but never bounds).
__global__ __launch_bounds__(256) void split_f32_kernel(const float* __restrict__ x, int64_t rows, int ld,
                                                        const int32_t* __restrict__ doclens,
                                                        uint16_t* __restrict__ hi, uint16_t* __restrict__ lo,
                                                        float* __restrict__ bounds) {
  const int sub = threadIdx.x & 15;
  float rmax = 0.0f, hmax = 0.0f;
  for (int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4; r < rows;
       r += ((int64_t)gridDim.x * blockDim.x) >> 4) {
    float xx, rr, hh;
    split_row8(x + r * kDim, hi + r * kDim, lo + r * kDim, sub, xx, rr, hh);
    if (doclens == nullptr || (int)(r % ld) < doclens[r / ld]) {
      rmax = fmaxf(rmax, sqrtf(rr) * kBoundUp);
      hmax = fmaxf(hmax, sqrtf(hh) * kBoundUp);
    }
  }
#pragma unroll
  for (int off = 16; off < 64; off <<= 1) {
    rmax = fmaxf(rmax, __shfl_xor(rmax, off));
    hmax = fmaxf(hmax, __shfl_xor(hmax, off));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMax(reinterpret_cast<unsigned int*>(bounds), __float_as_uint(rmax));
    atomicMax(reinterpret_cast<unsigned int*>(bounds) + 1, __float_as_uint(hmax));
  }
}

// Query split: one wave per query, 4 rows at a time.  beta[b] bounds
// |T - S| for every doc: sum_i ||q_i|| E + ||q_i - qhi_i|| M + slack (||q_i|| + ||q_i - qhi_i||) M
// with E = max ||x - hi||, M = max ||hi|| of the index.  A search's split also
// resets the row's band state (each nullable): count[b] = count0 (the band
// collect's counter; k when the band's first k slots are the bf16 top-k
// already rescored by phase 1), lbu[b] = ~0 (the atomic-min of the bf16 top-k's
// faithful scores, order-preserving bits), done[b] = 0 (the fallback's
// finished-workgroup counter), the row's arrival counters (arrive: narrive
// ints per row over kArriveSlotsK slots -- the launches that select in their
// last workgroup: the block-max select, the band select, the rerank select;
// and phase 1's finished-pair count of phase1_collect_kernel)
// and -- ctr, the search's scan -- the scan's task-counter block: launches
// fewer than separate memsets.
constexpr int kArriveSlotsK = 4;   // slots of the faithful workspace's arrival counters (kArriveSlots)
constexpr int kArrPhase1K = 3;     // (kArrPhase1) the phase-1 slot: done1's replicas, then at
constexpr int64_t kSplitZeroInts = 16384;   // block keys zeroed per extra workgroup of the query split
__global__ __launch_bounds__(512) void split_query_kernel(const float* __restrict__ Q, int lq,
                                                          uint16_t* __restrict__ qhi, uint16_t* __restrict__ qlo,
                                                          float E, float M, float* __restrict__ beta,
                                                          int32_t* __restrict__ count = nullptr,
                                                          uint32_t* __restrict__ lbu = nullptr,
                                                          int32_t* __restrict__ done = nullptr, int count0 = 0,
                                                          int32_t* __restrict__ arrive = nullptr, int narrive = 0,
                                                          int* __restrict__ ctr = nullptr, int nctr = 0,
                                                          uint32_t ready_seq = 0, int nrows = 0,
                                                          uint32_t* __restrict__ zkeys = nullptr, int64_t nz = 0,
                                                          int32_t* __restrict__ ready_words = nullptr) {
  // one 16-lane group per query token (lq <= 32: one pass, no loop -- the B=1
  // latency path waits on this launch); the per-token bound terms are summed
  // in the order of the round-3 one-wave kernel (4 strided partial sums, then
  // pairwise), so beta keeps its bits
  __shared__ float s_t[kLqMax];
  const int b = blockIdx.x, tid = threadIdx.x, r = tid >> 4, sub = tid & 15;
  if (nrows > 0 && b >= nrows) {   // workgroups past the rows: zero the scan-folded block keys (zkeys, 16-B aligned)
    const int64_t per = kSplitZeroInts, i0 = (int64_t)(b - nrows) * per;
    for (int64_t i = i0 + 4 * tid; i < i0 + per && i < nz; i += 4 * blockDim.x) {
      if (i + 3 < nz)
        *reinterpret_cast<uint4*>(zkeys + i) = make_uint4(0u, 0u, 0u, 0u);
      else
        for (int64_t e = i; e < nz; ++e) zkeys[e] = 0u;
    }
    return;
  }
  if (r < lq) {
    const size_t row = (size_t)b * lq + r;
    float xx, rr, hh;
    split_row8(Q + row * kDim, qhi + row * kDim, qlo + row * kDim, sub, xx, rr, hh);
    const float nq = sqrtf(xx) * kBoundUp, eq = sqrtf(rr) * kBoundUp;
    const float t = nq * E + eq * M + kAccSlack * (nq + eq) * M;
    if (sub == 0) s_t[r] = t;
  }
  __syncthreads();
  if (tid == 0) {
    float a[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      a[g] = 0.0f;
      for (int rr = g; rr < lq; rr += 4) a[g] += s_t[rr];
    }
    beta[b] = ((a[0] + a[1]) + (a[2] + a[3])) * kBoundUp;
    if (count != nullptr) count[b] = count0;
    if (lbu != nullptr) lbu[b] = 0xffffffffu;
    if (done != nullptr) done[b] = 0;
  }
  if (arrive != nullptr) {   // slot j of row b at (j * B + b) * per
    const int per = narrive / kArriveSlotsK;
    for (int i = tid; i < narrive; i += blockDim.x) {
      const int j = i / per, e = i - j * per;
      arrive[((size_t)j * nrows + b) * per + e] = 0;
    }
  }
  if (ctr != nullptr && b == 0)   // the scan's task counters (the scan that follows skips its memset)
    for (int i = tid; i < nctr; i += blockDim.x) ctr[i] = 0;
  if (ready_seq != 0 && ready_words != nullptr) {
    // the row's split is published to the host (ready_words[b], a word of the
    // call's mapped buffer): plain stores -> agent release -> relaxed flag
    // (MI355X_MICROARCH.md, the handoff-flag row; the vmcnt(0) after the
    // fence: its compiler-hazard fix).  The host launches the stage-1
    // prescore on another stream only once it has seen every row's flag.
    __syncthreads();
    if (tid == 0) {
      __threadfence();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(ready_words + b, (int32_t)ready_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// One row tile, faithful product: acc = init + lo.qhi + hi.qlo + hi.qhi.
__device__ __forceinline__ void tile16_x3(const bf16x8 (&ah)[4], const bf16x8 (&al)[4], const bf16x8 (&qh)[2][4],
                                          const bf16x8 (&ql)[2][4], const f32x4& init, float (&m)[2]) {
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    f32x4 acc = init;
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[s], qh[ct][s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s], ql[ct][s], acc, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[s], qh[ct][s], acc, 0, 0, 0);
    m[ct] = fmaxf(fmaxf(m[ct], fmaxf(acc[0], acc[1])), fmaxf(acc[2], acc[3]));
  }
}

// Faithful MaxSim of local doc `loc` (ld token slots, `dl` of them scoring)
// for one query whose split fragments are qh / ql: 128-token blocks of hi +
// lo, row maxima carried across blocks (LONG), then the sum over the query's
// lq tokens.  Every faithful rescoring kernel scores a pair through this one
// function, so a pair's bits never depend on which kernel scored it.
template <bool LONG>
__device__ __forceinline__ float faithful_doc16(const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo,
                                                int64_t loc, int ld, int dl, const bf16x8 (&qh)[2][4],
                                                const bf16x8 (&ql)[2][4], int lane, int lq) {
  const int g = lane >> 4;
  const int lmax = LONG ? ld : kLd;
  float m[2] = {neg_inf(), neg_inf()};
  for (int blk = 0; blk == 0 || (LONG && kLd * blk < dl); ++blk) {
    const int dlb = dl - kLd * blk;
    const size_t at = ((size_t)loc * lmax + (size_t)kLd * blk) * kRowBytes;
    const uint8_t* dh = hi + at;
    const uint8_t* dlo = lo + at;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      bf16x8 ah[4][4], al[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int rt = 4 * half + t;
        if (16 * rt < dlb) {
          gbl_afrag16(dh, rt, lane, ah[t]);
          gbl_afrag16(dlo, rt, lane, al[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int rt = 4 * half + t;
        if (16 * rt < dlb) {
          const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
          tile16_x3(ah[t], al[t], qh, ql, init, m);
        }
      }
    }
  }
  return reduce16(m[0], m[1], lane, lq);
}

// Faithful rescoring: query b = blockIdx.y against candidates c (cand == null:
// c is the local doc index), pw consecutive candidates per wave step (1 for
// small launches: one doc per wave, so a B=1 launch of 100 docs spreads over
// 100 waves instead of 25 walking 4 docs in sequence; kRsPerWave otherwise),
// grid-stride over blockIdx.x; out[b*ld_out + c].  count (nullable) bounds c
// per query (the band collected by the search); only_neg (nullable) skips
// every query whose status is >= 0 (the search's full-scan fallback).
// LONG: docs of ld = 256 / 512 / 1024 token slots (128-token blocks, the row
// maxima carried); the 128-slot build keeps its single-block code.  lb_min
// (nullable): every score is also atomic-min'ed into lb_min[b] as
// order-preserving bits (the two-pass band's lower bound: the minimum
// faithful score of the bf16 top-k, with no separate reduction launch).
constexpr int kRsPerWave = 4;
template <bool LONG = false>
__global__ __launch_bounds__(256, 2) void rescore_x3_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens, int64_t n,
    int64_t id_base, const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int lq,
    const int32_t* __restrict__ cand, const int32_t* __restrict__ count, int64_t limit, int64_t ld_c,
    float* __restrict__ out, int64_t ld_out, const int32_t* __restrict__ only_neg, int ld, int pw,
    uint32_t* __restrict__ lb_min) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (only_neg != nullptr && only_neg[b] >= 0) return;  // block-uniform; no block-level sync below
  int64_t lim = limit;
  if (count != nullptr) {
    const int64_t cb = count[b];
    lim = cb < lim ? cb : lim;
  }
  const int64_t step = (int64_t)gridDim.x * 4 * pw;
  int64_t c0 = ((int64_t)blockIdx.x * 4 + wave) * pw;
  if (c0 >= lim) return;  // wave-uniform
  bf16x8 qh[2][4], ql[2][4];
  load_qfrag16(qhi, b, b + 1, lq, lane, qh);
  load_qfrag16(qlo, b, b + 1, lq, lane, ql);
  for (; c0 < lim; c0 += step)
  for (int64_t c = c0; c < c0 + pw && c < lim; ++c) {
    const int64_t id = cand ? (int64_t)cand[b * ld_c + c] : id_base + c;
    const int64_t loc = id - id_base;
    float v = neg_inf();
    if (id >= 0 && loc >= 0 && loc < n) {
      const int lmax = LONG ? ld : kLd;
      int dl = doclens[loc];
      dl = dl < 0 ? 0 : (dl > lmax ? lmax : dl);
      v = faithful_doc16<LONG>(hi, lo, loc, ld, dl, qh, ql, lane, lq);
    }
    if (lane == 0) {
      out[(size_t)b * ld_out + c] = v;
      if (lb_min != nullptr) atomicMin(lb_min + b, f2u(v));
    }
  }
}

// Faithful rescoring, one (query, candidate) pair per WORKGROUP: the doc's
// token rows are split over the 4 waves (wave w takes row tiles 2w, 2w + 1
// of every 128-token block), each wave folds its rows' maxima to per-query-
// token column maxima, the workgroup takes the max of the 4 in LDS and wave 0
// sums them exactly as reduce16 does -- max is exact and order-free, so the
// score's bits equal rescore_x3_kernel's (one wave walking all 8 tiles).  A
// pair costs one HBM round trip of 16 KiB per wave and 48 MFMAs per wave
// instead of two round trips of 32 KiB and 192 MFMAs on one wave: the
// latency path's rescorings (the bf16 top-k, the band, the 50 candidates)
// are bound by that per-pair latency, not by bytes.  Same arguments as
// rescore_x3_kernel (pw unused); grid (pairs, B), grid-stride over pairs.
// The split pair's score (called by every thread of the workgroup; the result
// is valid in wave 0): waves' row maxima -> column maxima -> LDS -> max of
// the 4 -> reduce16's sum.
// dl: the doc's raw doclens entry (clamped here, after the first block's
// tile loads are issued: those do not wait for it).
// NW waves per doc (4: 2 row tiles each; 2: 4 row tiles each).
template <bool LONG, int NW = 4>
__device__ __forceinline__ float faithful_doc_split(const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo,
                                                    int64_t loc, int ld, int dl, const bf16x8 (&qh)[2][4],
                                                    const bf16x8 (&ql)[2][4], int lane, int wave, int lq,
                                                    float (&s_m)[4][32]) {
  constexpr int TPW = 8 / NW;   // row tiles per wave
  const int g = lane >> 4, c16 = lane & 15;
  const int lmax = LONG ? ld : kLd;
  float m[2] = {neg_inf(), neg_inf()};
  for (int blk = 0; blk == 0 || (LONG && kLd * blk < dl); ++blk) {
    const size_t at = ((size_t)loc * lmax + (size_t)kLd * blk) * kRowBytes;
    bf16x8 ah[TPW][4], al[TPW][4];
    // the first block's tiles are loaded whatever the doc length (its slots
    // exist; padding rows are loaded but never computed)
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int rt = TPW * wave + t;
      if (blk == 0 || 16 * rt < dl - kLd * blk) {
        gbl_afrag16(hi + at, rt, lane, ah[t]);
        gbl_afrag16(lo + at, rt, lane, al[t]);
      }
    }
    if (blk == 0) dl = dl < 0 ? 0 : (dl > lmax ? lmax : dl);
    const int dlb = dl - kLd * blk;
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      const int rt = TPW * wave + t;
      if (16 * rt < dlb) {
        const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
        tile16_x3(ah[t], al[t], qh, ql, init, m);
      }
    }
  }
  const float w0 = fold16_max(fold32_max(m[0])), w1 = fold16_max(fold32_max(m[1]));
  if (lane < 16) {
    s_m[wave][lane] = w0;
    s_m[wave][16 + lane] = w1;
  }
  __syncthreads();
  float v = 0.0f;
  if (wave == 0) {
    float m0 = s_m[0][c16], m1 = s_m[0][16 + c16];
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      m0 = fmaxf(m0, s_m[w][c16]);
      m1 = fmaxf(m1, s_m[w][16 + c16]);
    }
    v = dpp_row_sum16((c16 < lq ? m0 : 0.0f) + (16 + c16 < lq ? m1 : 0.0f));
  }
  __syncthreads();   // s_m is rewritten by the next pair
  return v;
}

// Selections run by a row's LAST workgroup (row_last_arrival, 8 shards) in
// the launch that scored the row, instead of a select launch after it.
struct RowSelect {
  int mode = 0;                  // kSelNone / kSelCand / kSelBand
  int32_t* arrive = nullptr;     // row b's counters at arrive + b * kArriveInts (zero before the launch)
  int k = 0;
  float* out_s = nullptr;
  int32_t* out_i = nullptr;
  int32_t* out_p = nullptr;      // kSelCand: positions in the candidate list (nullable)
  const float* lb = nullptr;     // kSelBand: a lower bound of the row's k-th score (nullable), or
  const uint32_t* lbu = nullptr; //   its order-preserving bits (the two-pass band's)
  int32_t* status = nullptr;     // kSelBand: the band size (the fallback writes -1 for overflowed rows)
  Mirror ids_mirror;             // kSelBand: [B][k] host mirror of the final ids (w nullable)
  FinalMirror fin;               // kSelCand: the host words of the call's final result (w nullable)
  Mirror raw;                    // kSelNone (w nullable): every pair's score also as the host word
                                 // raw.w[b * ld_c + c] ({score bits, seq}; the latency path's stage-1 prescore)
  uint64_t* stamps = nullptr;    // lab builds only (LAB_STAMPS): [16 + 2x] / [17 + 2x] workgroup x's start /
                                 // end of its pairs, [6] the row select's start, [4] its end
};
constexpr int kSelNone = 0, kSelCand = 1, kSelBand = 2;

// kSelCand (= select_small_kernel's work): the row's C <= kSmallMax raw
// scores (stored in this launch: sc1 loads), ranked with the position rule.
__device__ void select_cand_row(const float* raw, const int32_t* crow, int C, int k, float* os, int32_t* oi,
                                int32_t* op, float* sc, uint64_t* keys, FinalMirror fin = FinalMirror(),
                                size_t b = 0) {
  for (int t = threadIdx.x; t < C; t += blockDim.x) {
    sc[t] = ld_sc1(raw + t);
    keys[t] = rank_key(sc[t], (uint32_t)t);
  }
  __syncthreads();
  select_from_lds(sc, keys, C, k, crow, os, oi, op, fin, b);
}

// kSelBand (= band_select_kernel's result): the exact top-k of the row's cnt
// band keys (score desc, id asc; F stored in this launch or before it: sc1
// loads).  The keys reaching the lower bound lb hold the top-k (k docs score
// at least lb); when 1024 or fewer do, they alone are ranked by counting,
// otherwise (ties at the top, or a shard's band with fewer than k keys above
// a global bound) the kk-th largest key is found by six radix passes over all
// the keys and the kk keys at or above it are ranked.
__device__ void select_band_row(const float* F, const int32_t* cand, int cnt, int k, int64_t id_base, bool has_lb,
                                float lbv, float* os, int32_t* oi, uint64_t* sel, uint32_t* hist, uint32_t* misc,
                                Mirror mirror) {
  const int tid = threadIdx.x, nth = blockDim.x, wave = tid >> 6;
  const int kk = k < cnt ? k : cnt;
  auto key_at = [&](int i) { return rank_key(ld_sc1(F + i), (uint32_t)((int64_t)cand[i] - id_base)); };
  if (tid < 8) misc[tid] = 0;
  __syncthreads();
  const uint32_t ulb = has_lb ? f2u(lbv) : 0u;
  constexpr int U = 8;   // U keys' loads in flight per thread, then the filter
  for (int i0 = tid; i0 < cnt; i0 += nth * U) {
    uint64_t kv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) kv[u] = i0 + u * nth < cnt ? key_at(i0 + u * nth) : 0ull;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * nth < cnt && (uint32_t)(kv[u] >> 32) >= ulb) {
        const uint32_t pos = atomicAdd(&misc[0], 1u);
        if (pos < (uint32_t)kTopkMax) sel[pos] = kv[u];
      }
  }
  __syncthreads();
  int m = (int)misc[0];
  __syncthreads();
  if (m < kk || m > kTopkMax) {
    const int shifts[6] = {53, 42, 32, 21, 10, 0};
    const int bits[6] = {11, 11, 10, 11, 11, 10};
    uint64_t prefix = 0, mask = 0;
    uint32_t kleft = (uint32_t)kk;
    for (int p = 0; p < 6; ++p) {
      const int nb = 1 << bits[p];
      for (int i = tid; i < nb; i += nth) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < cnt; i += nth) {
        const uint64_t key = key_at(i);
        hist_add(hist, (uint32_t)(key >> shifts[p]) & (uint32_t)(nb - 1), (key & mask) == prefix);
      }
      __syncthreads();
      if (wave == 0) find_bin(hist, nb, kleft, &misc[4], &misc[5], &misc[6]);
      __syncthreads();
      kleft -= misc[5];
      prefix |= (uint64_t)misc[4] << shifts[p];
      mask |= (uint64_t)(nb - 1) << shifts[p];
      __syncthreads();
    }
    if (tid == 0) misc[0] = 0;
    __syncthreads();
    for (int i = tid; i < cnt; i += nth) {   // exactly kk keys reach the kk-th largest (keys are unique)
      const uint64_t key = key_at(i);
      if (key >= prefix) {
        const uint32_t pos = atomicAdd(&misc[0], 1u);
        if (pos < (uint32_t)kTopkMax) sel[pos] = key;
      }
    }
    __syncthreads();
    m = kk;
  }
  for (int i = tid; i < m; i += nth) {   // rank = #greater (unique keys)
    const uint64_t key = sel[i];
    int r = 0;
    for (int j = 0; j < m; ++j) r += sel[j] > key ? 1 : 0;
    if (r < k) {
      os[r] = u2f((uint32_t)(key >> 32));
      oi[r] = (int32_t)(id_base + (int64_t)(~(uint32_t)key));
      if (mirror.w != nullptr) mirror.put(r, oi[r], os[r]);
    }
  }
  for (int j = m + tid; j < k; j += nth) {
    os[j] = neg_inf();
    oi[j] = -1;
    if (mirror.w != nullptr) mirror.put(j, -1, neg_inf());
  }
}

template <bool LONG = false, int NW = 4>
__global__ __launch_bounds__(NW * 64, 2) void rescore_split_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens, int64_t n,
    int64_t id_base, const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int lq,
    const int32_t* __restrict__ cand, const int32_t* __restrict__ count, int64_t limit, int64_t ld_c,
    float* __restrict__ out, int64_t ld_out, const int32_t* __restrict__ only_neg, int ld,
    uint32_t* __restrict__ lb_min, int64_t c0, float* __restrict__ fb_T = nullptr, int32_t* __restrict__ fb_done = nullptr,
    int fb_k = 0, float* __restrict__ fb_s = nullptr, int32_t* __restrict__ fb_i = nullptr, RowSelect rs = RowSelect(),
    TaggedCand tc = TaggedCand()) {
  __shared__ float s_m[4][32];
  __shared__ uint64_t sel[kTopkMax];   // the fallback's / the row select's
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_bin, s_above, s_bincount, s_cnt;
  __shared__ uint32_t misc[8];
  __shared__ int s_last;
  __shared__ int32_t s_cid;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (rs.stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs)
    rs.stamps[16 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (only_neg != nullptr && only_neg[b] >= 0) return;  // block-uniform
  int64_t lim = limit;
  if (count != nullptr) {
    const int64_t cb = count[b];
    lim = cb < lim ? cb : lim;
    if (fb_T != nullptr && cb > limit) {   // block-uniform: the row's band overflowed its capacity
      // the full-scan fallback in this launch (fallback_split_kernel's work:
      // every doc's faithful score into fb_T, then the row's last workgroup
      // runs the exact top-k into fb_s / fb_i; band_select leaves such rows,
      // a row select in this launch (rs) marks them -1 here)
      bf16x8 qh[2][4], ql[2][4];
      load_qfrag16(qhi, b, b + 1, lq, lane, qh);
      load_qfrag16(qlo, b, b + 1, lq, lane, ql);
      float* row = fb_T + (size_t)b * n;
      for (int64_t c = blockIdx.x; c < n; c += gridDim.x) {   // block-uniform
        const float v = faithful_doc_split<LONG, NW>(hi, lo, c, ld, doclens[c], qh, ql, lane, wave, lq, s_m);
        if (threadIdx.x == 0) row[c] = v;
      }
      __threadfence();   // this workgroup's scores, visible device-wide before it is counted
      __syncthreads();
      if (threadIdx.x == 0) s_last = atomicAdd(fb_done + b, 1) == (int)gridDim.x - 1;
      __syncthreads();
      if (!s_last) return;
      __threadfence();   // every workgroup's scores of the row are in
      const int kk = (int)((int64_t)fb_k < n ? fb_k : n);
      topk_exact_row(row, n, kk, sel, hist, &s_bin, &s_above, &s_bincount, &s_cnt);
      sort_and_write(sel, kk, fb_k, id_base, fb_s + (size_t)b * fb_k, fb_i + (size_t)b * fb_k,
                     rs.ids_mirror.row(b, fb_k));
      if (rs.mode == kSelBand && threadIdx.x == 0) rs.status[b] = cb >= kWaitTimedOut ? -2 : -1;
      return;
    }
  }
  const bool idle = c0 + (int64_t)blockIdx.x >= lim;   // block-uniform
  if (idle && rs.mode == kSelNone) return;
  if (!idle) {
    bf16x8 qh[2][4], ql[2][4];
    load_qfrag16(qhi, b, b + 1, lq, lane, qh);
    load_qfrag16(qlo, b, b + 1, lq, lane, ql);
    for (int64_t c = c0 + blockIdx.x; c < lim; c += gridDim.x) {   // block-uniform trip count
      int64_t id;
      if (tc.w != nullptr) {   // pre-armed (the latency path's rerank): the host writes the candidate after the launch
        if (threadIdx.x == 0) {
          s_cid = wait_tagged(tc.w + (size_t)b * ld_c + c, tc);
          // handed to the row select through device memory (cand: the
          // caller's device array, unread on this path), not re-read from host
          if (rs.mode != kSelNone)
            st_sc1(reinterpret_cast<uint32_t*>(const_cast<int32_t*>(cand)) + (size_t)b * ld_c + c, (uint32_t)s_cid);
        }
        __syncthreads();
        id = s_cid;
        __syncthreads();   // s_cid is rewritten by the next pair
      } else {
        id = cand ? (int64_t)cand[b * ld_c + c] : id_base + c;
      }
      const int64_t loc = id - id_base;
      float v = neg_inf();
      if (id >= 0 && loc >= 0 && loc < n)                      // block-uniform
        v = faithful_doc_split<LONG, NW>(hi, lo, loc, ld, doclens[loc], qh, ql, lane, wave, lq, s_m);
      if (threadIdx.x == 0) {
        if (rs.mode != kSelNone)
          st_sc1(out + (size_t)b * ld_out + c, v);   // handed to the row's last workgroup
        else
          out[(size_t)b * ld_out + c] = v;
        if (rs.raw.w != nullptr) rs.raw.put((size_t)b * ld_c + c, (int32_t)__float_as_uint(v), 0.0f);
        if (lb_min != nullptr) atomicMin(lb_min + b, f2u(v));
      }
    }
  }
  if (rs.stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs)
    rs.stamps[17 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (rs.mode == kSelNone) return;
  if (!row_last_arrival(rs.arrive + (size_t)b * kArriveInts, (int)gridDim.x, 8, &s_last)) return;
  lab_stamp(rs.stamps, 6);
  if (rs.mode == kSelCand) {   // C = limit candidates, ids = the row's cand
    const int32_t* crow = cand + (size_t)b * ld_c;
    if (tc.w != nullptr) {       // the ids each workgroup stored for its candidate (sc1), not the host words
      int32_t* ids_lds = reinterpret_cast<int32_t*>(hist) + kSmallMax;
      for (int t = threadIdx.x; t < (int)limit; t += blockDim.x)
        ids_lds[t] = (int32_t)ld_sc1(reinterpret_cast<const uint32_t*>(crow) + t);
      crow = ids_lds;            // (published by select_cand_row's barrier)
    }
    select_cand_row(out + (size_t)b * ld_out, crow, (int)limit, rs.k, rs.out_s + (size_t)b * rs.k,
                    rs.out_i + (size_t)b * rs.k, rs.out_p ? rs.out_p + (size_t)b * rs.k : nullptr,
                    reinterpret_cast<float*>(hist), sel, rs.fin, (size_t)b);
  } else {                     // the band: lim keys (count[b] <= limit here)
    const bool has_lb = rs.lb != nullptr || rs.lbu != nullptr;
    const float lbv = rs.lbu != nullptr ? u2f(rs.lbu[b]) : (rs.lb != nullptr ? rs.lb[b] : 0.0f);
    select_band_row(out + (size_t)b * ld_out, cand + (size_t)b * ld_c, (int)lim, rs.k, id_base, has_lb, lbv,
                    rs.out_s + (size_t)b * rs.k, rs.out_i + (size_t)b * rs.k, sel, hist, misc,
                    rs.ids_mirror.row(b, rs.k));
    if (threadIdx.x == 0) rs.status[b] = (int32_t)lim;
  }
  if (rs.stamps != nullptr) {
    __syncthreads();
    lab_stamp(rs.stamps, 4);
    if (threadIdx.x == 0) rs.stamps[5] = (uint64_t)lim;
  }
}

// The faithful search's full-scan fallback in ONE launch (rows whose band
// overflowed its capacity, status < 0; every other row's workgroups exit at
// once): the rows' faithful scores of every doc into T (rescore_split_kernel's
// pairs), then the LAST workgroup of a row to finish -- a per-row counter
// (done[b], reset by the query split), agent-scope fences around it -- runs
// the exact top-k of the row (topk_exact_row + the bitonic sort, as
// topk_rows_kernel, with 256 threads).  k <= kTopkMax.
template <bool LONG = false>
__global__ __launch_bounds__(256, 2) void fallback_split_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens, int64_t n,
    int64_t id_base, const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int lq,
    float* __restrict__ T, const int32_t* __restrict__ status, int ld, int32_t* __restrict__ done, int k,
    float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  __shared__ float s_m[4][32];
  __shared__ uint64_t sel[kTopkMax];
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t s_bin, s_above, s_bincount, s_cnt;
  __shared__ int s_last;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y;
  if (status[b] >= 0) return;   // block-uniform: the band held the row's top-k
  bf16x8 qh[2][4], ql[2][4];
  load_qfrag16(qhi, b, b + 1, lq, lane, qh);
  load_qfrag16(qlo, b, b + 1, lq, lane, ql);
  float* row = T + (size_t)b * n;
  for (int64_t c = blockIdx.x; c < n; c += gridDim.x) {   // block-uniform
    const float v = faithful_doc_split<LONG>(hi, lo, c, ld, doclens[c], qh, ql, lane, wave, lq, s_m);
    if (threadIdx.x == 0) row[c] = v;
  }
  __threadfence();   // this workgroup's scores, visible device-wide before it is counted
  __syncthreads();
  if (threadIdx.x == 0) s_last = atomicAdd(done + b, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (!s_last) return;
  __threadfence();   // every workgroup's scores of the row are in
  const int kk = (int)((int64_t)k < n ? k : n);
  topk_exact_row(row, n, kk, sel, hist, &s_bin, &s_above, &s_bincount, &s_cnt);
  sort_and_write(sel, kk, k, id_base, out_s + (size_t)b * k, out_i + (size_t)b * k);
}

// ---------------------------------------------------------------------------
// Doc-major band rescoring.  The bands of a batch overlap (at B=256, 1M docs,
// ~0.9k band docs per query with the two-pass band: 0.23M (query, doc) pairs
// over ~0.2M distinct docs), so rescoring pair by pair would gather the shared
// band docs' hi+lo (64 KiB) more than once.  Instead the pairs are grouped by doc (counting sort: per-doc counts,
// wave-aggregated segment offsets, scatter) and one wave rescored every pair
// of a doc with the doc's tiles loaded once per half, the queries' fragments
// (16 KiB each, L2-resident) streamed per pair.  Same arithmetic and max
// order per pair as rescore_x3_kernel: identical bits.  Rows whose band
// overflowed cap are skipped (the search recomputes them in full).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void band_count_kernel(const int32_t* __restrict__ cand,
                                                         const int32_t* __restrict__ count, int cap,
                                                         int64_t id_base, int64_t n, int32_t* __restrict__ dcnt,
                                                         int c0) {
  const int b = blockIdx.y;
  const int tot = count[b];
  if (tot > cap) return;   // overflow row: full scan later
  for (int c = c0 + blockIdx.x * blockDim.x + threadIdx.x; c < tot; c += gridDim.x * blockDim.x) {
    const int64_t d = (int64_t)cand[(size_t)b * cap + c] - id_base;
    if (d >= 0 && d < n) atomicAdd(dcnt + d, 1);
  }
}

// Per doc with pairs: a segment [doff, doff + cnt) of the pair list and an
// entry in the active list.  Each workgroup owns a contiguous range of docs:
// pass 1 sums the range (one atomic per counter per WORKGROUP -- one per wave
// serialised ~30k atomics on two addresses, 0.36 ms at B=256), pass 2 walks it
// in 256-doc tiles with a block-wide exclusive scan.  Segment order across
// workgroups is arbitrary; every pair's (b, c) travels with it, so the scores
// land in the same places.  ctr[0] = pairs, ctr[1] = active docs.
__global__ __launch_bounds__(256) void band_offsets_kernel(const int32_t* __restrict__ dcnt, int64_t n,
                                                           int32_t* __restrict__ doff, int32_t* __restrict__ act,
                                                           int32_t* __restrict__ act_off,
                                                           int32_t* __restrict__ act_cnt, int32_t* __restrict__ ctr) {
  __shared__ int s_p[4], s_a[4];
  __shared__ int s_base[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t tiles = (n + 255) >> 8;
  const int64_t per = (tiles + gridDim.x - 1) / gridDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * per;
  const int64_t t1 = t0 + per < tiles ? t0 + per : tiles;
  if (t0 >= t1) return;   // block-uniform
  int sp = 0, sa = 0;
  for (int64_t t = t0; t < t1; ++t) {
    const int64_t d = (t << 8) + tid;
    const int c = d < n ? dcnt[d] : 0;
    sp += c;
    sa += c > 0 ? 1 : 0;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    sp += __shfl_xor(sp, off);
    sa += __shfl_xor(sa, off);
  }
  if (lane == 0) {
    s_p[wave] = sp;
    s_a[wave] = sa;
  }
  __syncthreads();
  if (tid == 0) {
    const int tp = s_p[0] + s_p[1] + s_p[2] + s_p[3], ta = s_a[0] + s_a[1] + s_a[2] + s_a[3];
    s_base[0] = tp > 0 ? atomicAdd(ctr, tp) : 0;
    s_base[1] = ta > 0 ? atomicAdd(ctr + 1, ta) : 0;
  }
  __syncthreads();
  int pb = s_base[0], ab = s_base[1];
  for (int64_t t = t0; t < t1; ++t) {
    const int64_t d = (t << 8) + tid;
    const int c = d < n ? dcnt[d] : 0;
    int incl = c;   // inclusive prefix sum over the wave
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int v = __shfl_up(incl, off);
      if (lane >= off) incl += v;
    }
    const uint64_t am = __ballot(c > 0);
    __syncthreads();   // the previous tile's s_p / s_a reads are done
    if (lane == 63) {
      s_p[wave] = incl;
      s_a[wave] = __popcll(am);
    }
    __syncthreads();
    int wp = 0, wa = 0;
    for (int w = 0; w < wave; ++w) {
      wp += s_p[w];
      wa += s_a[w];
    }
    if (c > 0) {
      const int o = pb + wp + incl - c;
      const int a = ab + wa + __popcll(am & ((1ull << lane) - 1ull));
      doff[d] = o;
      act[a] = (int32_t)d;
      act_off[a] = o;
      act_cnt[a] = c;
    }
    pb += s_p[0] + s_p[1] + s_p[2] + s_p[3];
    ab += s_a[0] + s_a[1] + s_a[2] + s_a[3];
  }
}

__global__ __launch_bounds__(256) void band_scatter_kernel(const int32_t* __restrict__ cand,
                                                           const int32_t* __restrict__ count, int cap,
                                                           int64_t id_base, int64_t n, int32_t* __restrict__ dcnt,
                                                           const int32_t* __restrict__ doff,
                                                           int32_t* __restrict__ pair_b, int32_t* __restrict__ pair_c,
                                                           int c0) {
  const int b = blockIdx.y;
  const int tot = count[b];
  if (tot > cap) return;
  for (int c = c0 + blockIdx.x * blockDim.x + threadIdx.x; c < tot; c += gridDim.x * blockDim.x) {
    const int64_t d = (int64_t)cand[(size_t)b * cap + c] - id_base;
    if (d < 0 || d >= n) continue;
    const int pos = doff[d] + atomicSub(dcnt + d, 1) - 1;   // leaves dcnt at 0
    pair_b[pos] = b;
    pair_c[pos] = c;
  }
}

constexpr int kDocPairs = 4;   // pairs of one doc held per pass (their running maxima in VGPRs)
// PAIR_OUTER: a wave takes the doc's pairs one at a time, each with its query
// fragments loaded once and the doc's tiles re-read per pair (cache-served
// after the first); otherwise the doc's tiles are loaded once per half and
// the query fragments re-read per pair and half.
template <bool PAIR_OUTER = false, bool LONG = false>
__global__ __launch_bounds__(256) void rescore_docs_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens,
    const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int B, int lq,
    const int32_t* __restrict__ act, const int32_t* __restrict__ act_off, const int32_t* __restrict__ act_cnt,
    const int32_t* __restrict__ ctr, const int32_t* __restrict__ pair_b, const int32_t* __restrict__ pair_c,
    float* __restrict__ F, int cap, int ld) {
  const int lane = threadIdx.x & 63, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n_act = ctr[1];
  for (int a = blockIdx.x * 4 + wave; a < n_act; a += gridDim.x * 4) {   // one doc per wave
    const int64_t d = act[a];
    const int o = act_off[a], cnt = act_cnt[a];
    const int lmax = LONG ? ld : kLd;
    int dl = doclens[d];
    dl = dl < 0 ? 0 : (dl > lmax ? lmax : dl);
    const uint8_t* dh0 = hi + (size_t)d * lmax * kRowBytes;
    const uint8_t* dlo0 = lo + (size_t)d * lmax * kRowBytes;
    const int nblk = LONG && dl > kLd ? (dl + kLd - 1) / kLd : 1;   // long documents: 128-token blocks
    if constexpr (PAIR_OUTER) {
#pragma unroll 1
      for (int p = 0; p < cnt; ++p) {
        const int b = pair_b[o + p];
        bf16x8 qh[2][4], ql[2][4];
        load_qfrag16(qhi, b, B, lq, lane, qh);
        load_qfrag16(qlo, b, B, lq, lane, ql);
        float m[2] = {neg_inf(), neg_inf()};
        for (int blk = 0; blk < nblk; ++blk) {
          const int dlb = dl - kLd * blk;
          const uint8_t* dh = dh0 + (size_t)blk * kDocBytes;
          const uint8_t* dlo = dlo0 + (size_t)blk * kDocBytes;
#pragma unroll
          for (int half = 0; half < 2; ++half) {
            bf16x8 ah[4][4], al[4][4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int rt = 4 * half + t;
              if (16 * rt < dlb) {
                gbl_afrag16(dh, rt, lane, ah[t]);
                gbl_afrag16(dlo, rt, lane, al[t]);
              }
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              const int rt = 4 * half + t;
              if (16 * rt < dlb) {
                const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
                tile16_x3(ah[t], al[t], qh, ql, init, m);
              }
            }
          }
        }
        const float v = reduce16(m[0], m[1], lane, lq);
        if (lane == 0) F[(size_t)b * cap + pair_c[o + p]] = v;
      }
      continue;
    }
    for (int p0 = 0; p0 < cnt; p0 += kDocPairs) {
      const int np = cnt - p0 < kDocPairs ? cnt - p0 : kDocPairs;
      float m[kDocPairs][2];
#pragma unroll
      for (int q = 0; q < kDocPairs; ++q) m[q][0] = m[q][1] = neg_inf();
      for (int blk = 0; blk < nblk; ++blk)
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const int dlb = dl - kLd * blk;
        const uint8_t* dh = dh0 + (size_t)blk * kDocBytes;
        const uint8_t* dlo = dlo0 + (size_t)blk * kDocBytes;
        bf16x8 ah[4][4], al[4][4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int rt = 4 * half + t;
          if (16 * rt < dlb) {
            gbl_afrag16(dh, rt, lane, ah[t]);
            gbl_afrag16(dlo, rt, lane, al[t]);
          }
        }
#pragma unroll 1
        for (int p = 0; p < np; ++p) {
          const int b = pair_b[o + p0 + p];
          bf16x8 qh[2][4], ql[2][4];
          load_qfrag16(qhi, b, B, lq, lane, qh);
          load_qfrag16(qlo, b, B, lq, lane, ql);
          float mm[2] = {neg_inf(), neg_inf()};
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int rt = 4 * half + t;
            if (16 * rt < dlb) {
              const f32x4 init = (dlb >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dlb);
              tile16_x3(ah[t], al[t], qh, ql, init, mm);
            }
          }
#pragma unroll
          for (int q = 0; q < kDocPairs; ++q)
            if (q == p) {
              m[q][0] = fmaxf(m[q][0], mm[0]);
              m[q][1] = fmaxf(m[q][1], mm[1]);
            }
        }
      }
#pragma unroll
      for (int q = 0; q < kDocPairs; ++q) {
        if (q < np) {
          const float v = reduce16(m[q][0], m[q][1], lane, lq);
          if (lane == 0) F[(size_t)pair_b[o + p0 + q] * cap + pair_c[o + p0 + q]] = v;
        }
      }
    }
  }
}

// Doc-major band rescoring with the doc split over the workgroup (128-slot
// docs): one band doc per workgroup of NW waves, wave w holding row tiles
// [w * 8/NW, (w + 1) * 8/NW) of hi and lo in VGPRs for all of the doc's pairs;
// per pair the query's split fragments (L2-resident) and the
// faithful_doc_split reduction (column maxima -> LDS -> max over the waves ->
// sum): the same bits as every other faithful rescoring.  NW = 4
// (CBV2_OPT_BAND_DOC_MAJOR = 3): ~170 VGPRs; NW = 2 (= 4): a half doc per
// wave, both halves in flight at once, 2 waves per SIMD -- where the
// one-wave-per-doc kernel (mode 1) walks the halves in turn at 1 wave per
// SIMD (254 VGPRs + accumulators).  The doc's tiles are loaded before its
// length is known (its 128 slots exist; rows past the length never enter a
// product), the next doc's list entry while this one computes.
template <int NW>
__global__ __launch_bounds__(NW * 64, NW == 4 ? 3 : 2) void rescore_docs_split_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens,
    const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int B, int lq,
    const int32_t* __restrict__ act, const int32_t* __restrict__ act_off, const int32_t* __restrict__ act_cnt,
    const int32_t* __restrict__ ctr, const int32_t* __restrict__ pair_b, const int32_t* __restrict__ pair_c,
    float* __restrict__ F, int cap) {
  constexpr int TPW = 8 / NW;   // row tiles per wave
  __shared__ float s_m[NW][32];
  const int lane = threadIdx.x & 63, g = lane >> 4, c16 = lane & 15;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int n_act = ctr[1];
  int a = blockIdx.x;
  if (a >= n_act) return;   // block-uniform
  int64_t d = act[a];
  for (; a < n_act; a += gridDim.x) {   // one doc per workgroup (block-uniform)
    const size_t at = (size_t)d * kLd * kRowBytes;
    bf16x8 ah[TPW][4], al[TPW][4];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
      gbl_afrag16(hi + at, TPW * wave + t, lane, ah[t]);
      gbl_afrag16(lo + at, TPW * wave + t, lane, al[t]);
    }
    const int o = act_off[a], cnt = act_cnt[a];
    int dl = doclens[d];
    dl = dl < 0 ? 0 : (dl > kLd ? kLd : dl);
    const int an = a + (int)gridDim.x;
    const int64_t d_next = an < n_act ? act[an] : 0;
    for (int p = 0; p < cnt; ++p) {
      const int b = pair_b[o + p];
      bf16x8 qh[2][4], ql[2][4];
      load_qfrag16(qhi, b, B, lq, lane, qh);
      load_qfrag16(qlo, b, B, lq, lane, ql);
      float m[2] = {neg_inf(), neg_inf()};
#pragma unroll
      for (int t = 0; t < TPW; ++t) {
        const int rt = TPW * wave + t;
        if (16 * rt < dl) {
          const f32x4 init = (dl >= 16 * rt + 16) ? f32x4{} : row_mask_init16(16 * rt + 4 * g, dl);
          tile16_x3(ah[t], al[t], qh, ql, init, m);
        }
      }
      const float w0 = fold16_max(fold32_max(m[0])), w1 = fold16_max(fold32_max(m[1]));
      if (lane < 16) {
        s_m[wave][lane] = w0;
        s_m[wave][16 + lane] = w1;
      }
      __syncthreads();
      if (wave == 0) {
        float m0 = s_m[0][c16], m1 = s_m[0][16 + c16];
#pragma unroll
        for (int w = 1; w < NW; ++w) {
          m0 = fmaxf(m0, s_m[w][c16]);
          m1 = fmaxf(m1, s_m[w][16 + c16]);
        }
        const float v = dpp_row_sum16((c16 < lq ? m0 : 0.0f) + (16 + c16 < lq ? m1 : 0.0f));
        if (lane == 0) F[(size_t)b * cap + pair_c[o + p]] = v;
      }
      __syncthreads();
    }
    d = d_next;
  }
}

// The band's threshold for row b: the exact lower bound of the k-th faithful
// score minus beta(b) -- from the caller (lb, floats: the sharded path's
// global bound) or from the atomic-min of the bf16 top-k's faithful scores
// (lbu, order-preserving bits) -- or, without either, T_k - 2 beta(b).
__device__ __forceinline__ float band_threshold(int b, const float* __restrict__ lb, const uint32_t* __restrict__ lbu,
                                                const float* __restrict__ topk_s, int k,
                                                const float* __restrict__ beta) {
  if (lbu != nullptr) return u2f(lbu[b]) - beta[b];
  if (lb != nullptr) return lb[b] - beta[b];
  return topk_s[(size_t)b * k + k - 1] - 2.0f * beta[b];
}

// Band collect: row b of the bf16 scan's scores T; every doc with T >= thr is
// appended (global id) to cand[b][0..cap); count[b] = the band size (may
// exceed cap: the search then recomputes that row in full).  thr = lb[b] -
// beta(b) when the exact lower bound lb of the k-th score is given (every doc
// of the exact top-k has T >= S - beta >= S_k - beta >= lb - beta), else T_k -
// 2 beta(b) (S_k >= T_k - beta).  Hits gather in an LDS list (LDS atomics; the
// global counter of a row is hit by one atomic per workgroup, not one per
// wave hit), flushed once at the end.
constexpr int kBandLds = 2048;
__global__ __launch_bounds__(256) void band_collect_kernel(const float* __restrict__ T, int64_t n,
                                                           const float* __restrict__ topk_s, int k,
                                                           const float* __restrict__ beta, int64_t id_base,
                                                           int cap, int32_t* __restrict__ cand,
                                                           int32_t* __restrict__ count,
                                                           const float* __restrict__ lb,
                                                           const uint32_t* __restrict__ lbu,
                                                           const int32_t* __restrict__ topk_i,
                                                           const uint32_t* __restrict__ bm,
                                                           uint64_t* __restrict__ stamps = nullptr) {
  __shared__ int32_t s_ids[kBandLds];
  __shared__ int s_n, s_base;
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  if (stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs)
    stamps[16 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const float thr = band_threshold(b, lb, lbu, topk_s, k, beta);
  const float* row = T + (size_t)b * n;
  int32_t* crow = cand + (size_t)b * cap;
  // topk_i (nullable): the band's slots [0, k) are the bf16 top-k (every one
  // of them is in the band: T_j >= F_j - beta >= lb - beta), already rescored
  // by phase 1 and count[b] started at k; the docs at or above the k-th key
  // are left out here
  uint64_t kth = 0;
  if (topk_i != nullptr) {
    kth = rank_key(topk_s[(size_t)b * k + k - 1], (uint32_t)((int64_t)topk_i[(size_t)b * k + k - 1] - id_base));
    if (blockIdx.x == 0)
      for (int j = threadIdx.x; j < k; j += blockDim.x) crow[j] = topk_i[(size_t)b * k + j];
  }
  // doc i (this lane's) with score v: appended when in the band (wave-uniform call)
  auto offer = [&](int64_t i, float v) {
    const bool take = i < n && v >= thr && (topk_i == nullptr || rank_key(v, (uint32_t)i) < kth);
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int nh = __popcll(mask);
    int base = 0;
    if (lane == 0) base = atomicAdd(&s_n, nh);
    base = __shfl(base, 0);
    const int pos = base + __popcll(mask & ((1ull << lane) - 1ull));
    if (take) {
      if (pos < kBandLds) {
        s_ids[pos] = (int32_t)(id_base + i);
      } else {  // LDS list full (a very wide band): straight to the global list
        const int gp = atomicAdd(count + b, 1);
        if (gp < cap) crow[gp] = (int32_t)(id_base + i);
      }
    }
  };
  if (bm != nullptr) {
    // bm (nullable): the row's 64-doc block maxima of the block-max top-k
    // (keys f2u(max), [B][ceil(n / 64)]) -- a block whose key is below the
    // threshold holds no band doc and its scores are never read: ~1 block in
    // 18 at 1M docs (883 band docs / query), instead of the whole 4 MB row.
    // A workgroup takes 64 consecutive block keys (one per lane, read by every
    // wave); the qualifying blocks are dealt to its waves in turn, and a wave
    // reads 4 of them per step (16 lanes per block, a float4 each): at a small
    // shard most blocks qualify (125k docs: the band spans most of the
    // 1,954 blocks) and ~31 workgroups share them.
    const int64_t nb = (n + 63) >> 6;
    const uint32_t* krow = bm + (size_t)b * nb;
    const uint32_t uthr = f2u(thr);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int c16 = lane & 15, r4 = lane >> 4;
    const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(T) & 15) == 0;
    for (int64_t g0 = (int64_t)blockIdx.x * 64; g0 < nb; g0 += (int64_t)gridDim.x * 64) {
      const int64_t kb = g0 + lane;   // one block key per lane
      const uint64_t qual = __ballot(kb < nb && krow[kb] >= uthr);
      uint64_t mine = 0;              // this wave's share: qualifying blocks q = wave (mod nw)
      int q = 0;
      for (uint64_t m = qual; m != 0; m &= m - 1, ++q)
        if (q % nw == wave) mine |= m & (~m + 1);
      while (mine != 0) {             // wave-uniform; 4 blocks per step, 4 steps' loads in flight
        int64_t i0[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          int64_t blk = -1;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int64_t bu = mine != 0 ? g0 + (__ffsll((long long)mine) - 1) : -1;
            if (mine != 0) mine &= mine - 1;
            if (u == r4) blk = bu;
          }
          i0[s4] = blk >= 0 ? (blk << 6) + 4 * c16 : n;
        }
        float v[4][4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          if (vec && i0[s4] + 3 < n) {
            const f32x4 x4 = *reinterpret_cast<const f32x4*>(row + i0[s4]);
            v[s4][0] = x4[0], v[s4][1] = x4[1], v[s4][2] = x4[2], v[s4][3] = x4[3];
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[s4][e] = i0[s4] + e < n ? row[i0[s4] + e] : 0.0f;
          }
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int e = 0; e < 4; ++e) offer(i0[s4] + e < n ? i0[s4] + e : n, v[s4][e]);
      }
    }
  } else {
    constexpr int U = 8;  // 8 coalesced loads in flight per thread, then the ballots
    const int64_t step = (int64_t)gridDim.x * blockDim.x * U;
    for (int64_t i0 = (int64_t)blockIdx.x * blockDim.x * U; i0 < n; i0 += step) {  // uniform trip count per wave
      float v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t i = i0 + (int64_t)u * blockDim.x + threadIdx.x;
        v[u] = i < n ? row[i] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) offer(i0 + (int64_t)u * blockDim.x + threadIdx.x, v[u]);
    }
  }
  __syncthreads();
  const int nl = s_n < kBandLds ? s_n : kBandLds;
  if (threadIdx.x == 0) s_base = nl > 0 ? atomicAdd(count + b, nl) : 0;
  __syncthreads();
  for (int t = threadIdx.x; t < nl; t += blockDim.x)
    if (s_base + t < cap) crow[s_base + t] = s_ids[t];
  if (stamps != nullptr && threadIdx.x == 0 && blockIdx.x < kLabWgs) {
    stamps[17 + 2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    atomicAdd(reinterpret_cast<unsigned long long*>(stamps + 5), (unsigned long long)s_n);
  }
}

// Phase 1 of the two-pass band and the band collect in ONE launch (the latency
// path, B <= kBandPairMaxB; band_collect_kernel's block-key path with the
// bf16 top-k reused): grid (k + S, B), 256 threads.
//  * workgroups x < k: phase 1's pair x -- the faithful score of the bf16
//    top-k's doc x into F[b][x] (sc1) and the atomic min into lbu[b] (for the
//    later launches), then counts it on done1[b]'s 8 replicas (one agent add
//    per replica);
//  * workgroups x >= k: the collect of 64-doc blocks [64 (x - k), +64).  While
//    phase 1 runs they load the 64 block keys and the scores of every block
//    that can hold a band doc at all (key >= T_k - 2 beta: lb >= T_k - beta,
//    since each of the k faithful scores is >= its bf16 score - beta); then
//    they wait for the row's phase 1 (thread 0 polls one replica of done1[b]
//    with sc1 loads until it reaches k), take lb = the minimum of F[b][0..k) (sc1 loads: the
//    same bits as the atomic min) and keep, as band_collect_kernel does, the
//    docs with T >= lb - beta below the k-th bf16 key.
// The hand-off is MI355X_MICROARCH.md's hand-off table, row 2 (sc1 stores,
// vmcnt(0), one wave instruction adding to every replica; sc1 poll of one
// replica, barrier, 4-B sc1 loads).  A collect
// workgroup waits only for phase-1 workgroups of its row, all of lower
// linear index -- dispatched before it, and never waiting themselves -- so the
// launch cannot deadlock whatever the occupancy.  done1 is zeroed by the query
// split.  Same band (as a set) as phase 1 + band_collect_kernel; the band's
// order is the collect's append order either way (the select ranks by key).
constexpr int kP1Replicas = 8;   // done1 replicas (32 ints apart, within one kArriveInts slot)
static_assert(32 * kP1Replicas <= kArriveInts, "done1's replicas fit one arrival slot");
__global__ __launch_bounds__(256, 2) void phase1_collect_kernel(
    const uint8_t* __restrict__ hi, const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens, int64_t n,
    int64_t id_base, const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int lq,
    const int32_t* __restrict__ topk_i, const float* __restrict__ topk_s, int k, float* __restrict__ F,
    int64_t ld_F, uint32_t* __restrict__ lbu, int32_t* __restrict__ done1, int64_t done_ld,
    const float* __restrict__ T, const float* __restrict__ beta, const uint32_t* __restrict__ bm, int cap,
    int32_t* __restrict__ cand, int32_t* __restrict__ count, uint64_t wait_ticks,
    uint64_t* __restrict__ stamps = nullptr) {
  __shared__ float s_m[4][32];
  __shared__ int32_t s_ids[kBandLds];
  __shared__ int s_n, s_base, s_timed_out;
  __shared__ uint32_t s_lb;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.y;
  const int x = blockIdx.x;
  if (stamps != nullptr && threadIdx.x == 0 && x < kLabWgs) stamps[16 + 2 * x] = __builtin_amdgcn_s_memrealtime();
  if (x < k) {   // ---- phase 1: pair x of row b
    bf16x8 qh[2][4], ql[2][4];
    load_qfrag16(qhi, b, b + 1, lq, lane, qh);
    load_qfrag16(qlo, b, b + 1, lq, lane, ql);
    const int64_t id = topk_i[(size_t)b * k + x];
    const int64_t loc = id - id_base;
    float v = neg_inf();
    if (id >= 0 && loc >= 0 && loc < n)   // block-uniform
      v = faithful_doc_split<false, 4>(hi, lo, loc, kLd, doclens[loc], qh, ql, lane, wave, lq, s_m);
    if (threadIdx.x == 0) {
      st_sc1(F + (size_t)b * ld_F + x, v);
      atomicMin(lbu + b, f2u(v));
    }
    if (wave == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the F store has landed
      // done1 in 8 replicas 128 B apart (hand-off table, row 2: one wave
      // instruction, one lane per replica): each collect workgroup polls one
      // of them, so ~1/8 of the pollers share a line with the adds
      if (lane < kP1Replicas)
        __hip_atomic_fetch_add(done1 + (size_t)b * done_ld + 32 * lane, 1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      if (stamps != nullptr && lane == 0 && x < kLabWgs) stamps[17 + 2 * x] = __builtin_amdgcn_s_memrealtime();
    }
    return;
  }
  // ---- the collect of blocks [64 g, 64 g + 64) of row b
  if (threadIdx.x == 0) s_n = 0;
  if (threadIdx.x == 0) s_lb = 0xffffffffu;
  const float* row = T + (size_t)b * n;
  int32_t* crow = cand + (size_t)b * cap;
  const uint64_t kth = rank_key(topk_s[(size_t)b * k + k - 1], (uint32_t)((int64_t)topk_i[(size_t)b * k + k - 1] - id_base));
  if (x == k)   // the band's slots [0, k): the bf16 top-k, rescored by phase 1 (count[b] starts at k)
    for (int j = threadIdx.x; j < k; j += blockDim.x) crow[j] = topk_i[(size_t)b * k + j];
  const int64_t nb = (n + 63) >> 6;
  const int64_t g0 = (int64_t)(x - k) * 64;
  const uint32_t uthr0 = f2u(topk_s[(size_t)b * k + k - 1] - 2.0f * beta[b]);   // <= any lb - beta
  const int nw = blockDim.x >> 6;
  const int c16 = lane & 15, r4 = lane >> 4;
  const bool vec = (n & 3) == 0 && (reinterpret_cast<uintptr_t>(T) & 15) == 0;
  const int64_t kb = g0 + lane;   // one block key per lane
  const uint64_t qual = __ballot(kb < nb && bm[(size_t)b * nb + kb] >= uthr0);
  uint64_t mine = 0;              // this wave's share: qualifying blocks q = wave (mod nw), <= 16
  {
    int q = 0;
    for (uint64_t m = qual; m != 0; m &= m - 1, ++q)
      if (q % nw == wave) mine |= m & (~m + 1);
  }
  int64_t i0[4];
  float v[4][4];
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4) {   // 4 blocks per step, 4 steps: every load in flight before the wait
    int64_t blk = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t bu = mine != 0 ? g0 + (__ffsll((long long)mine) - 1) : -1;
      if (mine != 0) mine &= mine - 1;
      if (u == r4) blk = bu;
    }
    i0[s4] = blk >= 0 ? (blk << 6) + 4 * c16 : n;
    if (vec && i0[s4] + 3 < n) {
      const f32x4 x4 = *reinterpret_cast<const f32x4*>(row + i0[s4]);
      v[s4][0] = x4[0], v[s4][1] = x4[1], v[s4][2] = x4[2], v[s4][3] = x4[3];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[s4][e] = i0[s4] + e < n ? row[i0[s4] + e] : 0.0f;
    }
  }
  // phase 1 of row b done: thread 0 polls (sc1), the barrier releases the rest.
  // The poll is bounded (wait_ticks; 0 = give up at once, the tests' knob): a
  // workgroup that gives up knows no lb, so it marks its row overflowed with
  // kWaitTimedOut -- the row then takes the full faithful scan in the
  // rescoring launch (exact whatever phase 1 did) and reports status -2.
  if (threadIdx.x == 0) {
    const int32_t* d = done1 + (size_t)b * done_ld + 32 * ((x - k) % kP1Replicas);
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool done = false;
    for (;;) {
      done = (int)__hip_atomic_load(d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= k;
      if (done || wait_ticks == 0 || __builtin_amdgcn_s_memrealtime() - t0 >= wait_ticks) break;
      __builtin_amdgcn_s_sleep(4);
    }
    s_timed_out = done ? 0 : 1;
    if (!done) atomicAdd(count + b, kWaitTimedOut);
  }
  __syncthreads();
  if (s_timed_out) return;   // block-uniform
  {   // lb = min over the k faithful scores (sc1 loads), as the atomic min has it
    uint32_t mn = ~0u;
    for (int j = threadIdx.x; j < k; j += blockDim.x) mn = min(mn, f2u(ld_sc1(F + (size_t)b * ld_F + j)));
    mn = wave_min_u32(mn);
    if (lane == 0) atomicMin(&s_lb, mn);
  }
  __syncthreads();
  const float thr = u2f(s_lb) - beta[b];
  auto offer = [&](int64_t i, float val) {
    const bool take = i < n && val >= thr && rank_key(val, (uint32_t)i) < kth;
    const uint64_t mask = __ballot(take);
    if (mask == 0) return;
    const int nh = __popcll(mask);
    int base = 0;
    if (lane == 0) base = atomicAdd(&s_n, nh);
    base = __shfl(base, 0);
    const int pos = base + __popcll(mask & ((1ull << lane) - 1ull));
    if (take) {
      if (pos < kBandLds) {
        s_ids[pos] = (int32_t)(id_base + i);
      } else {
        const int gp = atomicAdd(count + b, 1);
        if (gp < cap) crow[gp] = (int32_t)(id_base + i);
      }
    }
  };
#pragma unroll
  for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
    for (int e = 0; e < 4; ++e) offer(i0[s4] + e < n ? i0[s4] + e : n, v[s4][e]);
  __syncthreads();
  const int nl = s_n < kBandLds ? s_n : kBandLds;
  if (threadIdx.x == 0) s_base = nl > 0 ? atomicAdd(count + b, nl) : 0;
  __syncthreads();
  for (int t = threadIdx.x; t < nl; t += blockDim.x)
    if (s_base + t < cap) crow[s_base + t] = s_ids[t];
  if (stamps != nullptr && threadIdx.x == 0 && x < kLabWgs) {
    stamps[17 + 2 * x] = __builtin_amdgcn_s_memrealtime();
    atomicAdd(reinterpret_cast<unsigned long long*>(stamps + 5), (unsigned long long)s_n);
  }
}

// Band collect + rescoring in ONE launch, for batches of at most
// kBandPairMaxB queries over 128-slot docs (the latency path): workgroup x of
// row b scans docs [x * kBcrDocs, (x + 1) * kBcrDocs) of T, gathers the docs
// with T >= thr in LDS (never more than its slice: no overflow path),
// reserves their slots of the band with ONE atomic on count[b], then scores
// them one after another with the whole workgroup (faithful_doc_split: the
// same bits as every other faithful rescoring) and writes (global id, score)
// at the reserved slots.  Slots >= cap are dropped: count[b] > cap marks the
// row for the full faithful scan.
constexpr int kBcrDocs = 256 * 2;
__global__ __launch_bounds__(256, 2) void band_collect_rescore_kernel(
    const float* __restrict__ T, int64_t n, const float* __restrict__ topk_s, int k, const float* __restrict__ beta,
    const float* __restrict__ lb, const uint32_t* __restrict__ lbu, const uint8_t* __restrict__ hi,
    const uint8_t* __restrict__ lo, const int32_t* __restrict__ doclens, int64_t id_base,
    const uint16_t* __restrict__ qhi, const uint16_t* __restrict__ qlo, int lq, int cap, int32_t* __restrict__ cand,
    float* __restrict__ F, int32_t* __restrict__ count) {
  __shared__ int32_t s_loc[kBcrDocs];
  __shared__ float s_m[4][32];
  __shared__ int s_n, s_base;
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  {
    const float thr = band_threshold(b, lb, lbu, topk_s, k, beta);
    const float* row = T + (size_t)b * n;
    const int64_t i0 = (int64_t)blockIdx.x * kBcrDocs;
    constexpr int U = kBcrDocs / 256;
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * 256 + threadIdx.x;
      v[u] = i < n ? row[i] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + (int64_t)u * 256 + threadIdx.x;
      const bool take = i < n && v[u] >= thr;
      const uint64_t mask = __ballot(take);
      if (mask == 0) continue;   // wave-uniform
      int base = 0;
      if (lane == 0) base = atomicAdd(&s_n, __popcll(mask));
      base = __shfl(base, 0);
      if (take) s_loc[base + __popcll(mask & ((1ull << lane) - 1ull))] = (int32_t)i;
    }
  }
  __syncthreads();
  const int nl = s_n;
  if (nl == 0) return;   // block-uniform
  if (threadIdx.x == 0) s_base = atomicAdd(count + b, nl);
  __syncthreads();
  const int base = s_base;
  bf16x8 qh[2][4], ql[2][4];
  load_qfrag16(qhi, b, b + 1, lq, lane, qh);
  load_qfrag16(qlo, b, b + 1, lq, lane, ql);
  for (int j = 0; j < nl && base + j < cap; ++j) {   // block-uniform
    const int64_t loc = s_loc[j];
    const float v = faithful_doc_split<false>(hi, lo, loc, kLd, doclens[loc], qh, ql, lane, wave, lq, s_m);
    if (threadIdx.x == 0) {
      cand[(size_t)b * cap + base + j] = (int32_t)(id_base + loc);
      F[(size_t)b * cap + base + j] = v;
    }
  }
}

// k-th largest value of the union of G lists of k scores, list g of row b at
// fk[g * g_stride + b * k .. + k): the cross-shard lower bound of the global
// k-th faithful score (every shard's exact faithful scores of its bf16 top-k;
// k docs of the corpus score at least the union's k-th largest).  Radix select
// over the order-preserving score bits (11/11/10-bit digits), one workgroup
// per row; -inf padding (an empty shard) counts as a value like any other.
__global__ __launch_bounds__(kTkThreads) void union_kth_kernel(const float* __restrict__ fk, int G, int k,
                                                               size_t g_stride, float* __restrict__ lb) {
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t misc[8];
  const int b = blockIdx.x, tid = threadIdx.x, nth = blockDim.x;
  const int m = G * k;
  uint32_t prefix = 0, mask = 0, kleft = (uint32_t)k;
  for (int p = 0; p < 3; ++p) {
    const int shift = p == 0 ? 21 : (p == 1 ? 10 : 0);
    const uint32_t bits = p == 2 ? 1023u : 2047u;
    for (int i = tid; i < 2048; i += nth) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < m; i += nth) {
      const int g = i / k, j = i - g * k;
      const uint32_t u = f2u(fk[(size_t)g * g_stride + (size_t)b * k + j]);
      hist_add(hist, (u >> shift) & bits, (u & mask) == prefix);
    }
    __syncthreads();
    if ((tid >> 6) == 0) find_bin(hist, (int)bits + 1, kleft, &misc[4], &misc[5], &misc[6]);
    __syncthreads();
    kleft -= misc[5];
    prefix |= misc[4] << shift;
    mask |= bits << shift;
    __syncthreads();
  }
  if (tid == 0) lb[b] = u2f(prefix);
}

// Band select: exact top-k of the rescored band (score desc, id asc);
// status[b] = band size when certified, -1 when the band overflowed cap.
constexpr int kBandCapMax = 16384;
constexpr int kBandPairMaxB = 8;       // batches up to this rescore the band pair by pair (search_f32_phase2)
constexpr int kBandSelMax = 512;       // keys ranked by counting after the radix select (those reaching the k-th score)
// a band of at most this many keys is ranked by counting directly (each key
// counted against every other from LDS: 107 us for an 880-key band at 1M docs,
// B=1, vs 14 us through the radix select; profiles/r04e_*)
constexpr int kBandCountMax = 128;
// lb / lbu (nullable, as band_threshold): a lower bound of the row's k-th
// score; when at least kk band keys reach it and no more than kBandSelMax
// do, those keys alone are ranked (the top-kk is among them) -- no radix pass.
__global__ __launch_bounds__(kTkThreads) void band_select_kernel(const float* __restrict__ F,
                                                                 const int32_t* __restrict__ cand,
                                                                 const int32_t* __restrict__ count, int cap, int k,
                                                                 int64_t id_base, float* __restrict__ out_s,
                                                                 int32_t* __restrict__ out_i,
                                                                 int32_t* __restrict__ status,
                                                                 const float* __restrict__ lb,
                                                                 const uint32_t* __restrict__ lbu) {
  __shared__ uint64_t keys[kBandCapMax];
  __shared__ uint64_t sel[kBandSelMax];
  __shared__ uint32_t hist[2048];
  __shared__ uint32_t misc[8];
  const int b = blockIdx.x, tid = threadIdx.x, nth = blockDim.x;
  const int total = count[b];
  const int cnt = total < cap ? total : cap;
  if (total > cap) {   // block-uniform: the band overflowed -- the fallback writes this row
    if (tid == 0) status[b] = -1;
    return;
  }
  for (int t = tid; t < cnt; t += nth)
    keys[t] = rank_key(F[(size_t)b * cap + t], (uint32_t)((int64_t)cand[(size_t)b * cap + t] - id_base));
  if (tid < 8) misc[tid] = 0;
  __syncthreads();
  float* os = out_s + (size_t)b * k;
  int32_t* oi = out_i + (size_t)b * k;
  const uint64_t* src = keys;
  int m = cnt;
  const int kk0 = k < cnt ? k : cnt;
  if (cnt > kBandCountMax && (lb != nullptr || lbu != nullptr)) {
    // the keys whose score reaches the k-th score's lower bound
    const uint32_t ulb = f2u(lbu != nullptr ? u2f(lbu[b]) : lb[b]);
    for (int i = tid; i < cnt; i += nth)
      if ((uint32_t)(keys[i] >> 32) >= ulb) {
        const uint32_t pos = atomicAdd(&misc[0], 1u);
        if (pos < (uint32_t)kBandSelMax) sel[pos] = keys[i];
      }
    __syncthreads();
    if (misc[0] >= (uint32_t)kk0 && misc[0] <= (uint32_t)kBandSelMax) {
      src = sel;
      m = (int)misc[0];
    }
    __syncthreads();
    if (tid == 0) misc[0] = 0;
    __syncthreads();
  }
  if (src == keys && cnt > kBandCountMax) {
    // the kk-th largest score (the keys' top 32 bits) by radix select over
    // 11/11/10-bit digits, then the keys that reach it (the top-kk and its
    // score ties) into sel
    const uint32_t kk = (uint32_t)(k < cnt ? k : cnt);
    uint32_t prefix = 0, mask = 0, kleft = kk;
    for (int p = 0; p < 3; ++p) {
      const int shift = p == 0 ? 21 : (p == 1 ? 10 : 0);
      const uint32_t bits = p == 2 ? 1023u : 2047u;
      for (int i = tid; i < 2048; i += nth) hist[i] = 0;
      __syncthreads();
      for (int i = tid; i < cnt; i += nth) {
        const uint32_t u = (uint32_t)(keys[i] >> 32);
        hist_add(hist, (u >> shift) & bits, (u & mask) == prefix);
      }
      __syncthreads();
      if ((tid >> 6) == 0) find_bin(hist, (int)bits + 1, kleft, &misc[4], &misc[5], &misc[6]);
      __syncthreads();
      kleft -= misc[5];
      prefix |= misc[4] << shift;
      mask |= bits << shift;
      __syncthreads();
    }
    for (int i = tid; i < cnt; i += nth)
      if ((uint32_t)(keys[i] >> 32) >= prefix) {
        const uint32_t pos = atomicAdd(&misc[0], 1u);
        if (pos < (uint32_t)kBandSelMax) sel[pos] = keys[i];
      }
    __syncthreads();
    m = (int)misc[0];
    src = sel;
  }
  if (src == keys ? m <= kBandCountMax : m <= kBandSelMax) {   // keys are unique (distinct docs): rank = #greater
    for (int i = tid; i < m; i += nth) {
      const uint64_t key = src[i];
      int r = 0;
      for (int j = 0; j < m; ++j) r += src[j] > key ? 1 : 0;
      if (r < k) {
        os[r] = u2f((uint32_t)(key >> 32));
        oi[r] = (int32_t)(id_base + (int64_t)(~(uint32_t)key));
      }
    }
    for (int j = m + tid; j < k; j += nth) {
      os[j] = neg_inf();
      oi[j] = -1;
    }
  } else {                  // more than kBandSelMax keys tie at the k-th score: sort the whole band
    sort_and_write(keys, cnt, k, id_base, os, oi);
  }
  if (tid == 0) status[b] = total > cap ? -1 : total;
}

// ---------------------------------------------------------------------------
// Merge G sorted per-shard lists: rank = own position + #greater keys in every
// other list (binary search); ids are unique across shards so ranks are too.
// ---------------------------------------------------------------------------
// LDS_KEYS: the G*k keys are staged in LDS (G*k <= kMergeMax); otherwise the
// binary searches read the lists in place (any k).
template <bool LDS_KEYS = true>
__global__ __launch_bounds__(256) void merge_topk_kernel(const float* __restrict__ in_s,
                                                         const int32_t* __restrict__ in_i, int G, int B,
                                                         int k, size_t g_stride, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
  __shared__ uint64_t keys[LDS_KEYS ? kMergeMax : 1];
  __shared__ int nvalid[64];
  const int b = blockIdx.x;
  auto key_at = [&](int g, int j) -> uint64_t {
    if constexpr (LDS_KEYS) {
      return keys[g * k + j];
    } else {
      const size_t src = (size_t)g * g_stride + (size_t)b * k + j;
      const int32_t id = in_i[src];
      return id >= 0 ? rank_key(in_s[src], (uint32_t)id) : 0ull;
    }
  };
  if constexpr (LDS_KEYS) {
    for (int t = threadIdx.x; t < G * k; t += blockDim.x) {
      const int g = t / k, j = t % k;
      const size_t src = (size_t)g * g_stride + (size_t)b * k + j;
      const int32_t id = in_i[src];
      keys[t] = id >= 0 ? rank_key(in_s[src], (uint32_t)id) : 0ull;
    }
  }
  if (threadIdx.x < G) {  // valid entries form a prefix of each sorted list
    const size_t base = (size_t)threadIdx.x * g_stride + (size_t)b * k;
    int lo = 0, hi = k;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (in_i[base + mid] >= 0) lo = mid + 1; else hi = mid;
    }
    nvalid[threadIdx.x] = lo;
  }
  __syncthreads();
  int total = 0;
  for (int g = 0; g < G; ++g) total += nvalid[g];
  for (int64_t t = threadIdx.x; t < (int64_t)G * k; t += blockDim.x) {
    const int g = (int)(t / k), j = (int)(t % k);
    if (j >= nvalid[g]) continue;
    const uint64_t key = key_at(g, j);
    int rank = j;
    for (int g2 = 0; g2 < G; ++g2) {
      if (g2 == g) continue;
      int lo = 0, hi = nvalid[g2];  // count of entries > key (list sorted descending)
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (key_at(g2, mid) > key) lo = mid + 1; else hi = mid;
      }
      rank += lo;
    }
    if (rank < k) {
      out_s[(size_t)b * k + rank] = u2f((uint32_t)(key >> 32));
      out_i[(size_t)b * k + rank] = (int32_t)(~(uint32_t)key);
    }
  }
  for (int j = total + threadIdx.x; j < k; j += blockDim.x) {
    out_s[(size_t)b * k + j] = neg_inf();
    out_i[(size_t)b * k + j] = -1;
  }
}

// ---------------------------------------------------------------------------
// Literal reference scorer: cosine(mean_q, mean_d) as torch computes it
// (x / max(||x||, 1e-8), then sum of products).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(128) void meanpool_build_kernel(const float* __restrict__ tok, int ld_src,
                                                             const int32_t* __restrict__ doclens,
                                                             float* __restrict__ means) {
  __shared__ float red[2];
  const size_t doc = blockIdx.x;
  const int d = threadIdx.x;
  int dl = doclens[doc];
  dl = dl < 0 ? 0 : (dl > ld_src ? ld_src : dl);
  float s = 0.0f;
  for (int t = 0; t < dl; ++t) s += tok[(doc * ld_src + t) * kDim + d];
  const float mean = dl > 0 ? s / (float)dl : 0.0f;
  float sq = mean * mean;
  for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sq;
  __syncthreads();
  const float nrm = sqrtf(red[0] + red[1]);
  means[doc * kDim + d] = mean / fmaxf(nrm, 1e-8f);
}

constexpr int kMpDocs = 64, kMpQ = 16;
__global__ __launch_bounds__(256) void meanpool_scores_kernel(const float* __restrict__ means, int64_t n,
                                                              const float* __restrict__ Q, int B, int lq,
                                                              float* __restrict__ out, int64_t ld_out) {
  __shared__ float qn[kMpQ][kDim];
  __shared__ float dm[kMpDocs][kDim + 1];
  const int tid = threadIdx.x;
  const int64_t doc0 = (int64_t)blockIdx.x * kMpDocs;
  const int q0 = blockIdx.y * kMpQ;
  {  // normalised query means: 16 threads per query, 8 dims each
    const int qq = tid >> 4, part = tid & 15;
    const int qi = q0 + qq;
    float mv[8];
    float sq = 0.0f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.0f;
      if (qi < B)
        for (int t = 0; t < lq; ++t) s += Q[((size_t)qi * lq + t) * kDim + part * 8 + j];
      mv[j] = s / (float)lq;
      sq += mv[j] * mv[j];
    }
    for (int off = 8; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
    const float inv = 1.0f / fmaxf(sqrtf(sq), 1e-8f);
#pragma unroll
    for (int j = 0; j < 8; ++j) qn[qq][part * 8 + j] = mv[j] * inv;
  }
  for (int e = tid; e < kMpDocs * kDim; e += 256) {
    const int dd = e / kDim, c = e % kDim;
    dm[dd][c] = (doc0 + dd < n) ? means[(size_t)(doc0 + dd) * kDim + c] : 0.0f;
  }
  __syncthreads();
  const int dd = tid & 63;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int qq = (tid >> 6) * 4 + j;
    float s = 0.0f;
    for (int c = 0; c < kDim; ++c) s += qn[qq][c] * dm[dd][c];
    if (q0 + qq < B && doc0 + dd < n) out[(size_t)(q0 + qq) * ld_out + doc0 + dd] = s;
  }
}

}  // namespace

// ===========================================================================
// C ABI
// ===========================================================================
struct cbv2_index {
  int device;
  const uint8_t* tokens;
  int64_t n;
  int32_t ld, d;
  const int32_t* doclens;
  int64_t id_base;
  const float* doc_means;
  int32_t dtype;           // CBV2_DTYPE_BF16 or CBV2_DTYPE_MXFP8
  const uint8_t* scales;   // MXFP8: E8M0 [n][128][2]
  // Dynamic-tail task counters.  cbv2_search (and everything built on it)
  // takes them from the caller's workspace, so concurrent calls on distinct
  // streams never share a counter.  cbv2_score has no workspace: it uses a
  // ring of slots owned by the handle, one per launch, each zeroed on the
  // launch's stream; before a slot is reused, the new launch's stream waits
  // for the event recorded after the slot's previous launch (ring_ev), so
  // slot reuse is ordered across streams.  nullptr = static split only.
  int* task_ring = nullptr;
  uint32_t task_seq = 0;
  hipEvent_t ring_ev[128] = {};
  bool ring_ev_used[128] = {};
  // Work split of the most recent scan launch (cbv2_index_last_scan_plan).
  int64_t last_plan[4] = {0, 0, 0, 0};
  // CBV2_OPT_FUSED_TOPK: off by default.  In-process A/B on MI355X (round 2,
  // profiles/r02k_fused_ab.jsonl): cbv2_search fused 145.9 vs unfused 145.2 ms
  // at 1M docs B=256, 38.7 vs 38.2 at B=64, 18.6 vs 18.4 at 125k (the fused
  // scan runs ~1 % longer than the unfused scan + its radix top-k).
  bool fused_topk = false;   // CBV2_OPT_FUSED_TOPK != 0
  int fused_topk_mode = 0;   // its value (2: also the MXFP8 scan, A/B only)
  int dynamic_tail = 1;      // CBV2_OPT_DYNAMIC_TAIL (1: XCD-sliced tail, 2: one shared tail, 0: off)
  int topk_bmax = 1;         // CBV2_OPT_TOPK_BMAX (1: block-max top-k where eligible, 0: sampled filter + select)
  // CBV2_OPT_BAND_DOC_MAJOR: 0 pair by pair (round 4 default: with the split
  // rescoring the pair-by-pair gather beats grouping by doc -- band 2.64 vs
  // 2.78 ms at B=256, 0.72 vs 0.85 at 64, 0.22 vs 0.31 at 16, 1M docs,
  // profiles/r04u_band_ab.jsonl); 1 / 2 / 3 / 4 doc-major kernels (A/B)
  int band_doc_major = 0;
  bool band_lower_bound = true;  // CBV2_OPT_BAND_LOWER_BOUND
  // CBV2_OPT_BAND_FUSED (B <= 8: collect + rescore in one launch): off -- the
  // band collect (7.4 us) + the split rescoring (one band doc per workgroup)
  // beat the fused launch (39 us at 1M docs, B=1: its workgroups score their
  // few hits one after another; profiles/r04d_*)
  bool band_fused = false;
  bool rescore_split = true;     // CBV2_OPT_RESCORE_SPLIT (one pair per workgroup, rows over 4 waves)
  bool band_reuse = true;        // CBV2_OPT_BAND_REUSE (the band's first k slots: phase 1's top-k scores)
  bool band_block_skip = true;   // CBV2_OPT_BAND_BLOCK_SKIP (the collect reads only blocks whose max reaches it)
  int rescore_grid = 0;          // CBV2_OPT_RESCORE_GRID (workgroups per row of a split rescoring; 0: automatic)
  // CBV2_OPT_DENSE_DOCS: the docs fill (nearly) all 128 token slots -- B <= 2
  // then runs the 4 x 1 non-temporal scan (every slot streamed, 7.1 TB/s;
  // MXFP8 its 4 x 1 shape) instead of the streaming scan that skips empty
  // tiles (6.9 TB/s)
  bool dense_docs = false;
  bool p1_collect_fused = true;  // CBV2_OPT_P1_COLLECT_FUSED (phase1_collect_kernel)
  bool fold_keys = true;         // CBV2_OPT_FOLD_KEYS (scan_folds_bmax_zeroed)
  std::mutex mu;  // ring_ev_used, scan_ev / scan_ev_used
  // fp32-faithful index: bf16 residual lo = bf16(x - hi) of the fp32 corpus
  // whose rounding hi is `tokens`, and the split's bounds (max ||x - hi||,
  // max ||hi||); nullptr = plain bf16 index.
  const uint8_t* resid = nullptr;
  float resid_max = 0.0f, norm_max = 0.0f;
  // Scan timing (cbv2_index_time_scans): while enabled, every MaxSim scan
  // launch is bracketed by a pair of HIP events recorded on its own stream;
  // the pairs are reused across enable cycles and destroyed with the handle.
  bool time_scans = false;
  uint64_t* clk = nullptr;   // the scans' clock probe sums (cbv2_index_time_scans(ix, 2)), device [4]
  bool clock_on = false;
  size_t scan_ev_used = 0;
  std::vector<hipEvent_t> scan_ev;  // [2 * i] start, [2 * i + 1] stop
  // Band timing (same switch): a faithful search's work after the bf16 top-k
  // of its scan (band bound, collect, rescoring, select, fallback) is
  // bracketed by band_ev[2 * i] / [2 * i + 1]; band_open = a start recorded
  // whose stop is still to come (cbv2_search_f32_begin -> _finish).
  size_t band_ev_used = 0;
  bool band_open = false;
  std::vector<hipEvent_t> band_ev;
};

namespace {
thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define CBV2_HIP(call)                                                                    \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess) return fail(CBV2_EHIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#define CBV2_REQUIRE(cond, ...) \
  do {                          \
    if (!(cond)) return fail(CBV2_EINVAL, __VA_ARGS__); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) { ok = false; return; }
    if (prev != dev && hipSetDevice(dev) != hipSuccess) ok = false;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

constexpr int kRingSlots = 128;   // cbv2_score launches in flight before a slot is reused
constexpr int kTailSlices = 8;    // XCD-local slices of the dynamic tail (next_task_sliced)
constexpr int kRingInts = 64 * kTailSlices;  // counters per launch: 64 query groups x slices (B <= 64 * 32)
constexpr size_t kCtrBytes = kRingInts * sizeof(int);  // counter block at the head of a search workspace

// The handle's task-counter ring and its per-slot events (index creation;
// failure leaves cbv2_score on the static split).
void alloc_task_ring(cbv2_index* ix) {
  if (ix->n == 0) return;
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(ix->device) != hipSuccess) return;
  void* p = nullptr;
  if (hipMalloc(&p, (size_t)kRingSlots * kRingInts * sizeof(int)) == hipSuccess) {
    bool ok = true;
    for (int s = 0; s < kRingSlots && ok; ++s)
      ok = hipEventCreateWithFlags(&ix->ring_ev[s], hipEventDisableTiming) == hipSuccess;
    if (ok) {
      ix->task_ring = (int*)p;
    } else {
      for (int s = 0; s < kRingSlots; ++s)
        if (ix->ring_ev[s]) (void)hipEventDestroy(ix->ring_ev[s]), ix->ring_ev[s] = nullptr;
      (void)hipFree(p);
    }
  }
  (void)hipSetDevice(prev);
}

int cu_count(int dev) {
  static int cache[64] = {0};
  if (dev >= 0 && dev < 64 && cache[dev]) return cache[dev];
  int v = 256;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
  if (dev >= 0 && dev < 64) cache[dev] = v;
  return v;
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(CBV2_EHIP, "%s launch: %s", what, hipGetErrorString(e));
  return CBV2_OK;
}

// Scan variants (tools/scan_lab.py A/Bs them in one process; the default is
// the fastest measured).  id: kernel, waves/workgroup, queries/wave.
enum ScanVariant {
  kScan32Shfl = 0, kScan32Dpp = 1, kScan16W4 = 2, kScan16W8 = 3, kScan32DppW8 = 4,
  kScan16W4Q8 = 5, kScan16W8Q2 = 6, kScan16W8Q3 = 7, kScan16W4Q2 = 8,
  kScanDirectQ1 = 9, kScanDirectQ2 = 10, kScan16x4W8 = 11, kScan16x4W4 = 12, kScan16x4W4Q2 = 13,
  kScanStreamQ1 = 14, kScanStreamQ2 = 15, kScanStreamQ1Cached = 16, kScanStreamQ1W8 = 17, kScanStreamQ4 = 18,
  kScanStreamQ8 = 19, kScanStreamQ1Tw2 = 20, kScanStreamQ2Tw2 = 21, kScanPairQ1 = 22, kScanPairQ2 = 23,
  kScanPairQ4 = 24, kScanStreamQ4Pf = 25, kScanStreamQ1Pf = 26, kScanStreamQ2Pf = 27, kScan16x4W4Q1 = 28,
  kScan16x4W8Q1 = 30, kScan16x4W8Q1x2 = 31, kScan16x4W4Q1Nt = 33, kScan16x4W4Q2Nt = 34, kScan16x4W4Nt = 35,
  kScanAuto = -1
};
// Measured (tools/scan_lab.py, 200k docs, B=256, one MI355X): 0: 54.8 %,
// 1: 58.3 %, 2: 61.7 %, 3: 65.3 %, 4: 59.4 %, 5: 52.0 %, 6: 61.2 %, 8: 54.8 %
// of the bf16 dense peak.  rerank_kernel uses the same 16x16 math as 2/3/5-8.
// Tried and dropped: a 3-buffer variant that reads the next doc's first tile
// under the current doc's last MFMAs (carried fragments push the loop past 256
// VGPRs; hipcc spills the query fragments: 12 % of peak).
constexpr int kDefaultScan = kScanAuto;
// Auto dispatch (measured, tools/scan_lab.py, round 2, r02z): B <= 2 the
// direct scan (HBM-bound: B=1 5.3 ms, B=2 5.3 ms at 1M docs); 3 <= B <= 8 the
// 4-wave doc-interleaved scan with 2 queries per wave (B=8: 6.3 ms vs 13.8 for
// the direct scan, whose 4 query groups each stream every doc into VGPRs;
// B=3-4: ~6.3 vs 7.8 ms; at 125k docs 0.84 vs 1.79 ms at B=8); B <= 16 the
// same with 4 queries per wave; larger B the 8-wave scan.  Long documents
// keep the direct scan up to B=8 (kLongDirectMaxB).
constexpr int kDirectMaxB = 2;
constexpr int kOneWgMaxB = 2;   // the dense B <= 2 scan: one 4-wave workgroup per CU (scan_maxsim)
constexpr int kSmallLdsMaxB = 16;
constexpr int kLongDirectMaxB = 8;

// Auto shape for B > kDirectMaxB: the doc-interleaved shape with the least
// ceil(B / queries per workgroup) x (time per query group), from per-group
// times measured at 1M docs over B = 8..256 (lab r02af: every shape at every
// B, same process).  The query groups of a doc chunk share its tiles through
// L2, so a launch costs about its group count times the group time; ties go
// to the larger shape.  Checked against the measured best at every B of the
// sweep (bf16 B = 24/40/48/80/96/128: Q2/Q2/W4/W4/W8/W8; MXFP8 24/40/80/96/
// 128/192: 9/9/7/8/5/5).
struct ShapeCost {
  int qpb;      // queries per workgroup
  float ms;     // one query group over 1M docs
  int id;       // scan variant / f8 shape
};
template <int N>
int pick_shape(const ShapeCost (&c)[N], int B) {
  int best = c[0].id;
  float best_ms = 1e30f;
  for (int i = 0; i < N; ++i) {
    const float ms = (float)((B + c[i].qpb - 1) / c[i].qpb) * c[i].ms;
    if (ms <= best_ms) best_ms = ms, best = c[i].id;
  }
  return best;
}
// bf16: 4 waves x 1 query (round 4: 4.6 ms per group -- B = 3-4 without the
// 4 x 2 shape's padded query slots, which at 82 % MFMA-busy cost it the
// clock, and with the non-temporal doc stream of a one-group launch: 1M docs,
// same process, B=4 5.98 (4 x 2) -> 4.92 (4 x 1) -> 4.62 ms (4 x 1, nt), B=3
// 4.91 -> 4.62; profiles/r04m_lab_midbatch.log, r04n_lab_midbatch.log), 4 x 2
// (6.1; nt for B = 5-8: B=8 6.39 -> 6.34; padded query slots skip their MFMAs:
// B=5 5.92 -> 5.53, B=6 6.15 -> 5.81, profiles/r04p_lab_qskip.log), 4 x 4
// (9.6; B=16 alone 10.6; nt and padded-slot skipping for B <= 16: B=9 9.61 ->
// 8.60, B=12 10.05 -> 9.44, B=16 10.64 -> 10.56, profiles/r04s_lab.log), 8 x 4
// (17.4; B=256 = 8 groups 139 ms)
constexpr ShapeCost kBf16Shapes[] = {
    {4, 4.6f, kScan16x4W4Q1}, {8, 6.1f, kScan16x4W4Q2}, {16, 9.6f, kScan16x4W4}, {32, 17.4f, kScan16x4W8}};

template <int WAVES, int QW, int PER_CU, typename Kern>
int launch_scan(Kern kern, cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out,
                hipStream_t st, const char* name) {
  constexpr int QPB = WAVES * QW;
  const int nq_groups = (B + QPB - 1) / QPB;
  const int64_t target = (int64_t)PER_CU * cu_count(ix->device);  // resident workgroups
  int64_t n_chunks = target / nq_groups;   // never more workgroups than resident slots
  if (n_chunks < 1) n_chunks = 1;
  if (n_chunks > ix->n) n_chunks = ix->n;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t grid = (int64_t)nq_groups * n_chunks;
  if (grid > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(WAVES * 64), 0, st, ix->tokens, ix->doclens, ix->n, Q, B, lq,
                     out, ld_out, chunk_docs);
  return launch_check(name);
}

// The B > 16 doc-interleaved scan: one workgroup per CU; docs [0, static_docs)
// split statically, the last ~dyn_frac of the corpus as dynamic tasks of
// task_docs (see maxsim_scan16x4_kernel).  Defaults from tools/scan_lab.py on
// MI355X (B=256): static 146.7 -> guided 10 % tail 142.7 ms at 1M docs,
// 18.26 -> 17.73 ms at 125k (fixed 64-doc tasks: 143.1 / 17.92).
constexpr float kScanDynFrac = 0.10f;
constexpr int kScanTaskDocs = -16;     // guided: tasks shrink to 16 docs at the end
// B <= 16 (one query group, two 4-wave workgroups per CU): a larger dynamic
// share.  Lab, 1M docs, B=16: tail loss 9.7 % at 0.1 (per-workgroup stamps;
// clocks 1.57-1.70 GHz across XCDs under streaming); 12.41 -> 11.76 ms at 0.3
// (-5.2 %); 0.5 and 1.0 lose at 1M (14.2 / 16.2 ms).  B=64 is flat in the
// fraction (36.87-36.90 ms), so B > 16 keeps 0.1.  (Round 1's "125k: 1.479 ->
// 1.439 ms" was noise: the tail only switched on from 262,144 docs at B <= 16
// then; it now switches on whenever each static chunk keeps >= 64 docs.)
constexpr float kScanDynFracSmallB = 0.30f;
// The 4-wave x 4-query shape (B = 9-16) on the ticket tail (round 2, session
// 3; the 0.5 / 1.0 losses above were the CAS tail): lab, same process, 8
// interleaved rounds (profiles/r02s3_lab_dynfrac_b16.log): 1M docs B=16 10.64
// (0.3) -> 10.48 (0.45) -> 10.32 (0.6) -> 10.37 ms (0.75); 100k 1.080 ->
// 1.064 / 1.069 / 1.129 ms.  The 4 x 2 shape (B = 3-8) stays at 0.3 (0.45 and
// 0.6 are flat or slower at B = 4 / 8, profiles/r02s3_lab_dynfrac_b8.log).
constexpr float kScanDynFracB16 = 0.60f;
// The dense B <= 2 one-workgroup-per-CU scan (round 6): a 10 % tail.  Lab,
// same box (profiles/r06/onewg_*): 125k docs 0.597 (0.3) -> 0.591 ms (0.1),
// 100k 0.487 -> 0.484, 1M B=2 4.541 -> 4.538.  (Its static split alone is
// not enough: the odd XCDs stream 17 % behind the even ones at B = 1, and a
// static split waits for them -- profiles/r06/scan_lab_b1_*_split.log.)
constexpr float kScanDynFracOneWg = 0.10f;
constexpr int64_t kMinChunkDocs = 64;

// Fused top-k output of one scan launch: part [B][max_slots][k] keys; the
// launch records how many slots (chunks per query group) it wrote.
struct FusedTopk {
  uint64_t* part = nullptr;
  int k = 0;
  int64_t max_slots = 0;
  int64_t slots = 0;
};

// Work split of one launch: n_chunks static chunks of chunk_docs per query
// group over [0, static_docs), the rest as dynamic tasks on a zeroed counter
// block (the caller's workspace, or a ring slot of the handle).
struct ScanSplit {
  int64_t n_chunks = 1, chunk_docs = 0, static_docs = 0;
  int* ctr = nullptr;
  int task_docs = 0;
  int slices = 1;       // counters per query group (XCD-local tail slices)
  int ring_slot = -1;   // >= 0: the handle's ring slot, released by finish_split
};

// The task-counter block of the scans this host thread issues next (a caller's
// workspace counters, ctr_ws): kCtrDefault zeroes what the launch's tail uses;
// kCtrPrezeroed -- an earlier launch on the stream zeroed the whole block (the
// faithful query split): no memset; kCtrZeroAll -- zero the whole block, tail
// or not (arrival counters of later launches live past the tail's; plan_split
// records in g_ctr_zeroed that it did).  Set with CtrPolicy around the call.
constexpr int kCtrDefault = 0, kCtrPrezeroed = 1, kCtrZeroAll = 2;
// The latency path's host mirror of a search's final ids (cbv2_retrieve_begin
// sets it around its search, retrieve.cpp): the launches that write every
// row's final ids also write them to this device-mapped host buffer and set
// g_ids_mirror_used, so finish needs no D2H copy.
thread_local Mirror g_ids_mirror;
thread_local bool g_ids_mirror_used = false;
// ... and its pre-armed rerank's candidates (cbv2_retrieve_finish sets them
// around its rerank call): a rerank that can take them sets g_cand_tagged_used.
thread_local uint64_t g_wait_ticks = kCandWaitTicks;   // cbv2_set_wait_ticks (lab knob)
thread_local TaggedCand g_cand_tagged;
thread_local bool g_cand_tagged_used = false;
// The final result's host words (cbv2_set_final_mirror, set by retrieve.cpp
// around its rerank call): a rerank whose select writes them sets
// g_final_mirror_used (else the caller copies the result down).
thread_local FinalMirror g_final_mirror;
thread_local bool g_final_mirror_used = false;
// ... and the raw scores of a k = 0 rerank as host words (cbv2_set_raw_mirror,
// around the latency path's stage-1 prescore): a rerank that writes them sets
// g_raw_mirror_used.
thread_local Mirror g_raw_mirror;
thread_local bool g_raw_mirror_used = false;
// The latency path's ready flags (cbv2_set_split_ready_begin around begin's
// search: its first launch publishes this seq to words of the call's mapped
// buffer when the queries / their split are complete; the host launches the
// stage-1 prescore on another stream only after it has seen them -- an
// in-kernel wait on another queue's kernel could starve it of the CUs it
// needs) and the prescore itself (cbv2_set_prescore_ready).
thread_local uint32_t g_split_ready_seq = 0;
thread_local uint32_t g_prescore_ready_seq = 0;   // (only: the prescore must use the search's split)
// where the search just issued wrote its ready flag (row b at
// g_ready_flag[b * g_ready_flag_ld]; nullptr: it wrote none)
thread_local int32_t* g_ready_flag = nullptr;
thread_local int64_t g_ready_flag_ld = 0;
thread_local int32_t* g_split_ready_word = nullptr;   // the bf16 search's flag word (the call's mapped buffer)
// Lab builds (-DCBV2_LAB_STAMPS, tools/chain_lab.py): per-launch phase stamps
// of the latency path's kernels, kind k at g_lab_stamps + k * kLabStride --
// 0 block-max select, 1 phase-1 rescoring, 2 band collect, 3 band rescoring +
// select, 4 rerank + select.  Product builds: no stamps.
#ifdef CBV2_LAB_STAMPS
thread_local uint64_t* g_lab_stamps = nullptr;
#define LAB_STAMPS(kind) (g_lab_stamps != nullptr ? g_lab_stamps + (size_t)(kind) * kLabStride : nullptr)
#else
#define LAB_STAMPS(kind) ((uint64_t*)nullptr)
#endif
// The clock probe the scan launched next passes its workgroups (set by
// scan_maxsim_timed while the handle's probe is on; nullptr otherwise).
thread_local uint64_t* g_clock_probe = nullptr;
thread_local int g_ctr_policy = kCtrDefault;
thread_local bool g_ctr_zeroed = false;
struct CtrPolicy {
  int prev;
  explicit CtrPolicy(int p) : prev(g_ctr_policy) {
    g_ctr_policy = p;
    g_ctr_zeroed = false;
  }
  ~CtrPolicy() { g_ctr_policy = prev; }
};

// (zero_ctr_block below: the memset, or this kernel with the flag)
// The bf16 search's counter block zeroed by a kernel instead of a memset when
// the latency path asked for a ready flag (cbv2_set_split_ready_begin): after
// the zeroing, the flag word = seq (plain stores -> agent release -> relaxed
// flag, as the faithful query split publishes its own) -- the host sees it
// before it launches the stage-1 prescore on another stream (the queries were
// complete when this first launch of the search ran).  The word is the
// call's own (its mapped buffer): no later search can overwrite it.
__global__ __launch_bounds__(256) void ctr_zero_ready_kernel(int* __restrict__ ctr, int n, int* __restrict__ flag,
                                                             uint32_t seq) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) ctr[i] = 0;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, (int)seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

hipError_t zero_ctr_block(int* ctr, hipStream_t st) {
  if (g_split_ready_seq == 0 || g_split_ready_word == nullptr || g_ready_flag != nullptr)
    return hipMemsetAsync(ctr, 0, kCtrBytes, st);
  hipLaunchKernelGGL(ctr_zero_ready_kernel, dim3(1), dim3(256), 0, st, ctr, kRingInts, g_split_ready_word,
                     g_split_ready_seq);
  g_ready_flag = g_split_ready_word;   // one flag for every row
  g_ready_flag_ld = 0;
  return hipGetLastError();
}

int plan_split(cbv2_index* ix, int nq_groups, int64_t target, float dyn_frac, int task_docs, hipStream_t st,
               ScanSplit* sp, int* ctr_ws) {
  int64_t n_chunks = target / nq_groups;   // never more workgroups than resident slots
  if (n_chunks < 1) n_chunks = 1;
  if (n_chunks > ix->n) n_chunks = ix->n;
  sp->task_docs = task_docs > 0 ? std::max(64, task_docs & ~63) : -std::max(4, (-task_docs) & ~3);
  sp->ctr = nullptr;
  sp->ring_slot = -1;
  const int64_t tail_chunk = ((int64_t)((double)ix->n * (1.0 - (double)dyn_frac)) / n_chunks) & ~(int64_t)63;
  const bool have_ctr = ctr_ws != nullptr || ix->task_ring != nullptr;
  sp->slices = ix->dynamic_tail == 2 ? 1 : kTailSlices;
  if (have_ctr && ix->dynamic_tail && dyn_frac > 0.0f && nq_groups * sp->slices <= kRingInts &&
      tail_chunk >= kMinChunkDocs) {
    sp->chunk_docs = tail_chunk;
    sp->static_docs = sp->chunk_docs * n_chunks;
    if (ctr_ws != nullptr) {
      sp->ctr = ctr_ws;
    } else {
      const uint32_t slot = __atomic_fetch_add(&ix->task_seq, 1u, __ATOMIC_RELAXED) % kRingSlots;
      bool wait = false;
      {
        std::lock_guard<std::mutex> lk(ix->mu);
        wait = ix->ring_ev_used[slot];
      }
      // the slot's previous launch (maybe on another stream) must be done with it
      if (wait) CBV2_HIP(hipStreamWaitEvent(st, ix->ring_ev[slot], 0));
      sp->ctr = ix->task_ring + (size_t)slot * kRingInts;
      sp->ring_slot = (int)slot;
    }
    if (ctr_ws == nullptr || g_ctr_policy == kCtrDefault) {
      CBV2_HIP(hipMemsetAsync(sp->ctr, 0, (size_t)nq_groups * sp->slices * sizeof(int), st));
    } else if (g_ctr_policy == kCtrZeroAll) {
      CBV2_HIP(zero_ctr_block(sp->ctr, st));
      g_ctr_zeroed = true;
    }
  } else {
    if (ctr_ws != nullptr && g_ctr_policy == kCtrZeroAll) {
      CBV2_HIP(zero_ctr_block(ctr_ws, st));
      g_ctr_zeroed = true;
    }
    sp->chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
    n_chunks = (ix->n + sp->chunk_docs - 1) / sp->chunk_docs;
    sp->static_docs = ix->n;
  }
  sp->n_chunks = n_chunks;
  if ((int64_t)nq_groups * n_chunks > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  ix->last_plan[0] = (int64_t)nq_groups * n_chunks;
  ix->last_plan[1] = sp->chunk_docs;
  ix->last_plan[2] = sp->static_docs;
  ix->last_plan[3] = sp->ctr != nullptr ? 1 : 0;
  return CBV2_OK;
}

// After the launch: a ring slot's event marks when its counters are free again.
int finish_split(cbv2_index* ix, const ScanSplit& sp, hipStream_t st) {
  if (sp.ring_slot < 0) return CBV2_OK;
  CBV2_HIP(hipEventRecord(ix->ring_ev[sp.ring_slot], st));
  std::lock_guard<std::mutex> lk(ix->mu);
  ix->ring_ev_used[sp.ring_slot] = true;
  return CBV2_OK;
}

// Static chunks per query group of a launch (plan_split's first step): the
// slot count a fused top-k launch writes at most.
int64_t scan_chunks(const cbv2_index* ix, int nq_groups, int64_t target) {
  int64_t n_chunks = target / nq_groups;   // never more workgroups than resident slots
  if (n_chunks < 1) n_chunks = 1;
  if (n_chunks > ix->n) n_chunks = ix->n;
  return n_chunks;
}

template <int WAVES, int QW, int PER_CU, int D, int NBUF, bool STAMPS, int TPI = 32, int OCC = 2, bool SPREAD = false,
          int FK = 0, bool SPLITLOAD = false, bool ARRIVE = false, int PROBE = 0, int LD = kLd, int MORDER = 0,
          int AUX = 0, bool BMK = false>
int launch_scan16x4(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
                    float dyn_frac = kScanDynFrac, int task_docs = kScanTaskDocs, uint64_t* stamps = nullptr,
                    int* ctr_ws = nullptr, FusedTopk* ft = nullptr, uint32_t* bm = nullptr) {
  constexpr int QPB = WAVES * QW;
  const int nq_groups = (B + QPB - 1) / QPB;
  ScanSplit sp;
  int rc = plan_split(ix, nq_groups, (int64_t)PER_CU * cu_count(ix->device), dyn_frac, task_docs, st, &sp, ctr_ws);
  if (rc != CBV2_OK) return rc;
  if (FK > 0) {
    if (ft == nullptr || ft->k < 1 || ft->k > FK - 16 || sp.n_chunks > ft->max_slots)
      return fail(CBV2_EINVAL, "fused top-k: bad k or slot count");
    ft->slots = sp.n_chunks;
  }
  if (BMK && bm == nullptr) return fail(CBV2_EINVAL, "block-key scan without keys");
  hipLaunchKernelGGL((maxsim_scan16x4_kernel<WAVES, QW, D, NBUF, STAMPS, TPI, OCC, SPREAD, FK, SPLITLOAD, ARRIVE, PROBE, LD, MORDER,
                                             AUX, BMK>),
                     dim3((unsigned)(nq_groups * sp.n_chunks)), dim3(WAVES * 64), 0, st, ix->tokens, ix->doclens,
                     ix->n, Q, B, lq, out, ld_out, sp.chunk_docs, sp.static_docs, sp.ctr, sp.task_docs,
                     STAMPS ? stamps : g_clock_probe,
                     ft ? ft->k : 0, ft ? ft->part : nullptr, ft ? (int)ft->max_slots : 0, sp.slices, bm,
                     bm_blocks(ix->n), bm != nullptr ? bm_super_keys(bm, B, ix->n) : nullptr, bm_supers(ix->n));
  if ((rc = launch_check("maxsim_scan16x4_kernel"))) return rc;
  return finish_split(ix, sp, st);
}

// Direct scans (B <= 2): chunks for kDirectOversub x the resident waves (2
// per SIMD), so workgroups that start late balance the XCDs' clock
// differences; lab, same process (profiles/r02s3_lab_direct_oversub.log), B=1:
// 1M docs 5.229 (1x) -> 5.128 (2x) / 5.111 (4x) / 5.169 ms (16x); 100k 0.531
// -> 0.526 (2x) / 0.535 (4x).  The MXFP8 direct scan stays at 1x (1.25M docs
// B=1 3.289 vs 3.314 ms at 2x; B=2 2.636 vs 2.672).
constexpr int kDirectOversub = 2;

template <int QW>
int launch_direct(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st) {
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t target_waves = 8LL * cu_count(ix->device) * kDirectOversub;  // 2 waves per SIMD, oversubscribed
  int64_t n_chunks = target_waves / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  if (n_chunks < 1) n_chunks = 1;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t waves = (int64_t)nq_groups * n_chunks;
  const int64_t grid = (waves + 3) / 4;
  if (grid > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  if (ix->ld != kLd)
    hipLaunchKernelGGL((maxsim_scan_direct_kernel<QW, true>), dim3((unsigned)grid), dim3(256), 0, st, ix->tokens,
                       ix->doclens, ix->n, Q, B, lq, out, ld_out, chunk_docs, (int)ix->ld);
  else
    hipLaunchKernelGGL((maxsim_scan_direct_kernel<QW, false>), dim3((unsigned)grid), dim3(256), 0, st, ix->tokens,
                       ix->doclens, ix->n, Q, B, lq, out, ld_out, chunk_docs, kLd);
  return launch_check("maxsim_scan_direct_kernel");
}

// Streaming scans (variants 14-16; 14 / 15 are the B = 1 / 2 production
// scans of every bf16 index, long documents included): one 4-wave workgroup
// per CU (128 KiB of LDS rings), chunks for kDirectOversub x the resident waves.
// The paired streaming scan (lab variants 22-24): 4 two-wave workgroups per CU
// (2 waves per SIMD), chunks for kDirectOversub x the resident workgroups.
template <int QW>
int launch_pair(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st) {
  if (ix->dtype != CBV2_DTYPE_BF16) return fail(CBV2_EUNSUPPORTED, "pair scan: bf16 index only");
  const int nq_groups = (B + 2 * QW - 1) / (2 * QW);
  const int64_t target_wgs = 4LL * cu_count(ix->device) * kDirectOversub;
  int64_t n_chunks = target_wgs / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  if (n_chunks < 1) n_chunks = 1;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t grid = (int64_t)nq_groups * n_chunks;
  if (grid > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  hipLaunchKernelGGL((maxsim_scan_pair_kernel<QW, 2>), dim3((unsigned)grid), dim3(128), 0, st, ix->tokens,
                     ix->doclens, ix->n, Q, B, lq, out, ld_out, chunk_docs, (int)ix->ld);
  return launch_check("maxsim_scan_pair_kernel");
}

// bm (nullable): fold the block and superblock maxima into the scan (chunks
// rounded up to whole 256-doc superblocks; layout of bm_ws_bytes).
template <int QW, int AUX, int WAVES = 4, int SLOTS = kStreamSlots, bool TW2 = false, bool PF = false>
int launch_stream(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
                  uint32_t* bm = nullptr) {
  if (ix->dtype != CBV2_DTYPE_BF16) return fail(CBV2_EUNSUPPORTED, "stream scan: bf16 index only");
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t target_waves = (int64_t)WAVES * cu_count(ix->device) * kDirectOversub;
  int64_t n_chunks = target_waves / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  if (n_chunks < 1) n_chunks = 1;
  int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  if (bm != nullptr) chunk_docs = (chunk_docs + 255) & ~(int64_t)255;   // whole superblocks
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t grid = ((int64_t)nq_groups * n_chunks + WAVES - 1) / WAVES;
  if (grid > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  hipLaunchKernelGGL((maxsim_scan_stream_kernel<QW, AUX, WAVES, SLOTS, TW2, PF>), dim3((unsigned)grid), dim3(WAVES * 64), 0, st,
                     ix->tokens,
                     ix->doclens, ix->n, Q, B, lq, out, ld_out, chunk_docs, (int)ix->ld, bm, bm_blocks(ix->n),
                     bm ? bm_super_keys(bm, B, ix->n) : nullptr, bm_supers(ix->n));
  return launch_check("maxsim_scan_stream_kernel");
}

// Long documents (index ld = 256 / 512 / 1024): B <= 8 the direct scan in
// 128-token blocks, larger B the production 8-wave doc-interleaved scan with
// its doc group spanning ld / 64 iterations (the row maxima carried across).
int scan_maxsim_long(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
                     int* ctr_ws) {
  // B <= 2: the streaming scan (one query group, so the nt policy costs no L2
  // sharing); B = 3-8 the direct scan, whose query groups share each doc's
  // tiles through L2
  if (B <= kDirectMaxB)
    return B == 1 ? launch_stream<1, 2>(ix, Q, B, lq, out, ld_out, st) : launch_stream<2, 2>(ix, Q, B, lq, out, ld_out, st);
  if (B <= kLongDirectMaxB) return launch_direct<2>(ix, Q, B, lq, out, ld_out, st);
  switch (ix->ld) {
    case 256:
      return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 0, 256>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFrac, kScanTaskDocs, nullptr, ctr_ws);
    case 512:
      return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 0, 512>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFrac, kScanTaskDocs, nullptr, ctr_ws);
    case 1024:
      return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 0, 1024>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFrac, kScanTaskDocs, nullptr, ctr_ws);
    default:
      return fail(CBV2_EUNSUPPORTED, "index ld %d not built", (int)ix->ld);
  }
}

// bm (nullable): the production B <= 2 streaming scans fold the block maxima
// of the block-max top-k into their epilogue (scan_folds_bmax); other scans
// ignore it.
bool scan_folds_bmax(const cbv2_index* ix, int B) {
  return ix->dtype == CBV2_DTYPE_BF16 && ix->ld == kLd && B <= kDirectMaxB && kDefaultScan == kScanAuto &&
         !ix->dense_docs;
}
// ... and the dense-doc 4 x 1 scan (B <= 4) folds them by atomic max into keys
// its caller zeroed (the faithful search's query split does)
bool scan_folds_bmax_zeroed(const cbv2_index* ix, int B) {
  return ix->dtype == CBV2_DTYPE_BF16 && ix->ld == kLd && B <= 4 && kDefaultScan == kScanAuto && ix->dense_docs &&
         ix->fold_keys && pick_shape(kBf16Shapes, B) == kScan16x4W4Q1;
}
int scan_maxsim(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
                int variant = kDefaultScan, int* ctr_ws = nullptr, FusedTopk* ft = nullptr, uint32_t* bm = nullptr) {
  if (ix->n == 0) return CBV2_OK;
  if (ix->ld != kLd) {
    if (ft != nullptr || variant != kScanAuto) return fail(CBV2_EUNSUPPORTED, "long-doc index: automatic scan only");
    return scan_maxsim_long(ix, Q, B, lq, out, ld_out, st, ctr_ws);
  }
  if (ft != nullptr)   // fused top-k: the B > 16 doc-interleaved scan only (fused_eligible)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, kFusedCap, true>(ix, Q, B, lq, nullptr, 0, st,
                                                                               kScanDynFrac, kScanTaskDocs, nullptr,
                                                                               ctr_ws, ft);
  if (variant == kScanAuto) {
    // dense docs: B <= 2 takes the 4 x 1 shape below (bm == nullptr: its
    // caller runs the block maxima, scan_folds_bmax)
    if (B <= kDirectMaxB && !ix->dense_docs)
      return B == 1 ? launch_stream<1, 2>(ix, Q, B, lq, out, ld_out, st, bm)
                    : launch_stream<2, 2>(ix, Q, B, lq, out, ld_out, st, bm);
    variant = pick_shape(kBf16Shapes, B);
  }
  switch (variant) {
    case kScan16x4W4Q1:     // 4 queries per workgroup (1 per wave): B = 3-4 without padded query slots
      // B <= 2 (dense docs: the latency path): ONE workgroup per CU, a 3-deep
      // ring, waves 0-1 issue the LDS-DMA (SPLITLOAD) -- the waves of padded
      // query slots idle, so HBM decides: lab, same box, interleaved
      // (profiles/r06/ringdepth_*): 125k docs B=1 0.634 -> 0.595 ms (6.46 ->
      // 6.88 TB/s), 100k 0.517 -> 0.494 (3-deep, no SPLITLOAD), 1M 4.594 ->
      // 4.522; at B = 4 (every slot live) the two-per-CU form stays (4.70 vs
      // 5.54 ms: one wave per SIMD cannot hide the MFMA latency)
      if (B <= kOneWgMaxB && bm != nullptr)
        return launch_scan16x4<4, 1, 1, 2, 3, false, 32, 1, false, 0, true, false, 0, kLd, 0, 2, true>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracOneWg, kScanTaskDocs, nullptr, ctr_ws, nullptr, bm);
      if (B <= kOneWgMaxB)
        return launch_scan16x4<4, 1, 1, 2, 3, false, 32, 1, false, 0, true, false, 0, kLd, 0, 2>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracOneWg, kScanTaskDocs, nullptr, ctr_ws);
      if (B <= 4 && bm != nullptr)   // the block keys folded in (zeroed by the caller: scan_folds_bmax_zeroed)
        return launch_scan16x4<4, 1, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2, true>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs, nullptr, ctr_ws, nullptr, bm);
      if (B <= 4)           // one query group: every doc byte is read once (non-temporal)
        return launch_scan16x4<4, 1, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs, nullptr, ctr_ws);
      return launch_scan16x4<4, 1, 2, 2, 2, false>(ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs,
                                                   nullptr, ctr_ws);
    case kScan16x4W8:   // SPLITLOAD: lab, same box, 1M / 125k / B=64: 145.25 -> 144.10, 18.14 -> 17.97, 37.98 -> 37.53 ms
      return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true>(ix, Q, B, lq, out, ld_out, st, kScanDynFrac,
                                                                          kScanTaskDocs, nullptr, ctr_ws);
    case kScan16x4W4:
      if (B <= 16)          // one query group: non-temporal doc stream
        return launch_scan16x4<4, 4, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracB16, kScanTaskDocs, nullptr, ctr_ws);
      return launch_scan16x4<4, 4, 2, 2, 2, false>(ix, Q, B, lq, out, ld_out, st, kScanDynFracB16, kScanTaskDocs,
                                                   nullptr, ctr_ws);
    case kScan16x4W4Q2:   // 8 queries per workgroup (2 per wave)
      if (B <= 8)         // one query group: non-temporal doc stream
        return launch_scan16x4<4, 2, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
            ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs, nullptr, ctr_ws);
      return launch_scan16x4<4, 2, 2, 2, 2, false>(ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs,
                                                   nullptr, ctr_ws);
#ifdef CBV2_LAB   // variants tools/scan_lab.hip A/Bs (the product never dispatches them: its library leaves them out)
    case kScanDirectQ1:
      return launch_direct<1>(ix, Q, B, lq, out, ld_out, st);
    case kScanDirectQ2:
      return launch_direct<2>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ1:
      return launch_stream<1, 2>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ2:
      return launch_stream<2, 2>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ1Cached:
      return launch_stream<1, 0>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ1W8:   // lab: 8 waves x 4 tile slots per CU
      return launch_stream<1, 2, 8, 4>(ix, Q, B, lq, out, ld_out, st);
    // lab, 1M docs, same process (profiles/r03z_lab_stream_qg_1m.log): B=4
    // 5.72 ms vs 5.69 for variant 13; B=8 9.95 (18) / 8.58 (19) vs 5.98: not kept
    case kScanStreamQ4:     // lab: B <= 4 in one query group
      return launch_stream<4, 2>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ8:     // lab: B <= 8 in one query group
      return launch_stream<8, 2>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ1Tw2:  // lab: two tiles per wait
      return launch_stream<1, 2, 4, kStreamSlots, true>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ2Tw2:
      return launch_stream<2, 2, 4, kStreamSlots, true>(ix, Q, B, lq, out, ld_out, st);
    case kScanPairQ1:       // lab: two waves sharing one tile ring, 1 / 2 / 4 queries each
      return launch_pair<1>(ix, Q, B, lq, out, ld_out, st);
    case kScanPairQ2:
      return launch_pair<2>(ix, Q, B, lq, out, ld_out, st);
    case kScanPairQ4:
      return launch_pair<4>(ix, Q, B, lq, out, ld_out, st);
    // lab, round 4, 1M docs, same process (profiles/r04l_lab_midbatch.log): the
    // prefetching stream 5.78 vs 5.82 ms at B=4, 4.76 vs 4.78 at B=1 -- not
    // kept; 8 waves x 1 query (30 / 31) 7.1-7.6 ms at B=5-8 vs 4 x 2's 6.1-6.4
    case kScanStreamQ4Pf:   // lab: the next tile's fragments read under this tile's MFMAs
      return launch_stream<4, 2, 4, kStreamSlots, false, true>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ1Pf:
      return launch_stream<1, 2, 4, kStreamSlots, false, true>(ix, Q, B, lq, out, ld_out, st);
    case kScanStreamQ2Pf:
      return launch_stream<2, 2, 4, kStreamSlots, false, true>(ix, Q, B, lq, out, ld_out, st);
    case kScan16x4W4Q1Nt:   // lab: 4 x 1 / 4 x 2 with the non-temporal doc stream (one query group per launch)
      return launch_scan16x4<4, 1, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs, nullptr, ctr_ws);
    case kScan16x4W4Q2Nt:
      return launch_scan16x4<4, 2, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs, nullptr, ctr_ws);
    case kScan16x4W4Nt:     // lab: 4 x 4 with the non-temporal doc stream (B <= 16: one query group)
      return launch_scan16x4<4, 4, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
          ix, Q, B, lq, out, ld_out, st, kScanDynFracB16, kScanTaskDocs, nullptr, ctr_ws);
    case kScan16x4W8Q1:     // lab: 8 queries per workgroup, one per wave (2 waves per SIMD)
      return launch_scan16x4<8, 1, 1, 2, 2, false>(ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB, kScanTaskDocs,
                                                   nullptr, ctr_ws);
    case kScan16x4W8Q1x2:   // lab: the same, two workgroups per CU
      return launch_scan16x4<8, 1, 2, 2, 2, false, 32, 4>(ix, Q, B, lq, out, ld_out, st, kScanDynFracSmallB,
                                                          kScanTaskDocs, nullptr, ctr_ws);
    case kScan32Shfl:
      return launch_scan<4, 4, 2>(maxsim_scan_kernel<4, 4, false>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan_kernel");
    case kScan32Dpp:
      return launch_scan<4, 4, 2>(maxsim_scan_kernel<4, 4, true>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan_kernel");
    case kScan16W4:
      return launch_scan<4, 4, 2>(maxsim_scan16_kernel<4, 4>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
    case kScan16W8:
      return launch_scan<8, 4, 1>(maxsim_scan16_kernel<8, 4>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
    case kScan32DppW8:
      return launch_scan<8, 4, 1>(maxsim_scan_kernel<8, 4, true>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan_kernel");
    case kScan16W4Q8:
      return launch_scan<4, 8, 1>(maxsim_scan16_kernel<4, 8, 1>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
    case kScan16W8Q2:
      return launch_scan<8, 2, 1>(maxsim_scan16_kernel<8, 2>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
    case kScan16W8Q3:
      return launch_scan<8, 3, 1>(maxsim_scan16_kernel<8, 3>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
    case kScan16W4Q2:
      return launch_scan<4, 2, 2>(maxsim_scan16_kernel<4, 2>, ix, Q, B, lq, out, ld_out, st, "maxsim_scan16_kernel");
#endif
    default:
      return fail(CBV2_EINVAL, "unknown scan variant %d", variant);
  }
}

// B <= 2: the direct scan (HBM-bound); 3 <= B <= 8: the doc-interleaved scan
// in 4-wave workgroups x 2 queries, two per CU (lab, r02aa, 1M docs: B=4 3.25
// vs 4.75 ms direct, B=8 3.74 vs 8.93; 125k: B=8 0.46 vs 1.27 ms); larger B
// 8 waves x 8 queries.
constexpr int kF8DirectMaxB = 2;
constexpr int kF8SmallMaxB = 8;
// MXFP8 shapes (scan_f8's shape ids), ms per query group at 1M docs: 9 = 4
// waves x 2 queries, two per CU (3.0; B=8 alone 3.74); 7 = 4 x 4, three per
// CU (5.2; B=16 alone 5.81); 8 = 4 x 8, two per CU (9.5); 5 = 8 x 8, one per
// CU (18.2; B=256 = 4 groups 72.5).  Against the 8 x 8 shape for every B > 8
// (round 1): B=16 17.93 -> 5.81 ms, B=32 18.45 -> 10.77, B=48 19.63 -> 16.88
// (lab r02ad), B=80 35.1 -> 26.2 (r02af).
// round 4: 24 = 4 waves x 1 query, non-temporal (B = 3-4: 3.14 -> 2.49 ms at
// B=4, 2.79 -> 2.38 at B=3, 1M docs; the one-group launches of 9 and 7 stream
// non-temporally and skip padded slots: B=5 3.50 -> 3.40, B=12 5.30 -> 5.08;
// profiles/r04aa_lab_f8_midbatch.log)
constexpr ShapeCost kF8Shapes[] = {{4, 2.45f, 24}, {8, 3.0f, 9}, {16, 5.2f, 7}, {32, 9.5f, 8}, {64, 18.2f, 5}};
constexpr int kF8Waves = 8, kF8QW = 8;
// Fold distance of the doc-interleaved f8 scans: a chain's row max is folded
// 3 MFMAs after it issues (no MFMA -> VALU hazard pads: 122 -> 36 s_nop per
// 128 MFMAs), with the query scale bytes packed four per VGPR (PQS) to pay
// for the two extra accumulators (254 VGPRs, no spill; was 256 + 2 spilled).
// Lab A/B, 1M docs, bit-identical (profiles/r02s3_lab_f8*.log): B=256 72.44
// -> 70.98 ms, B=64 19.19 -> 18.77, B=32 10.26 -> 10.17, B=16 5.73 -> 5.71,
// B=8 3.73 -> 3.65.
constexpr int kF8D = 3;
// ... except the 4-wave shapes 7 and 8 (4 x 4 at three workgroups per CU, 4
// x 8 at two): fold distance 1, where 3 spilled 2 VGPRs (12 B of scratch per
// lane) -- the max is exact, so the bits do not depend on the distance
constexpr int kF8D47 = CBV2_F8_D47;
// Dynamic share of the MXFP8 scans (dyn_frac = kF8DynAuto picks it per shape):
// the 4-wave shapes hand more of the corpus to the ticket tail.  Lab, same
// process, 1M docs (profiles/r02s3_lab_dynfrac_f8.log): B=16 (4 x 4, three
// per CU) 5.99 / 5.61 / 5.55 ms at 0.1 / 0.3 / 0.6; B=32 (4 x 8) 10.39 /
// 10.20 / 9.96; B=8 (4 x 2) 3.80 / 3.68 / 3.70; the 8 x 8 shape is flat (B=64
// 19.28-19.32, B=256 73.35-73.44, 1.25M B=256 91.67-91.81) and keeps 0.1.
constexpr float kF8DynAuto = -1.0f;
constexpr float kF8DynSmall = 0.6f;   // shapes 7 and 8
constexpr float kF8DynB8 = 0.3f;      // shape 9

// QW queries per wave, PER_CU workgroups per CU in the split, OCC the
// launch-bounds occupancy hint (production: 8 waves x 8 queries, one per CU).
template <int TPI, int NBUF, bool PF = false, int QW = kF8QW, int PER_CU = 1, int OCC = 2, int WAVES = kF8Waves,
          int FK = 0, int LD = kLd, int D = 1, bool PQS = false, bool PAIR = false, bool SPREAD2 = false,
          bool SPLIT = false, bool QUAD = false, int PROBE = 0, int AUX = 0>
int launch_f8x4(cbv2_index* ix, const uint8_t* Qb, const uint8_t* Qs, int B, int lq, float* out, int64_t ld_out,
                hipStream_t st, float dyn_frac, int task_docs, int* ctr_ws = nullptr, FusedTopk* ft = nullptr) {
  constexpr int QPB = WAVES * QW;
  const int nq_groups = (B + QPB - 1) / QPB;
  ScanSplit sp;
  int rc = plan_split(ix, nq_groups, (int64_t)PER_CU * cu_count(ix->device), dyn_frac, task_docs, st, &sp, ctr_ws);
  if (rc != CBV2_OK) return rc;
  if (FK > 0) {
    if (ft == nullptr || ft->k < 1 || ft->k > FK - 16 || sp.n_chunks > ft->max_slots)
      return fail(CBV2_EINVAL, "fused top-k: bad k or slot count");
    ft->slots = sp.n_chunks;
  }
  hipLaunchKernelGGL((maxsim_scan_f8x4_kernel<WAVES, QW, D, NBUF, TPI, PF, OCC, FK, LD, PQS, PAIR, SPREAD2, SPLIT, QUAD, PROBE,
                                              AUX>),
                     dim3((unsigned)(nq_groups * sp.n_chunks)), dim3(WAVES * 64), 0, st, ix->tokens, ix->scales,
                     ix->doclens, ix->n, Qb, Qs, B, lq, out, ld_out, sp.chunk_docs, sp.static_docs, sp.ctr,
                     sp.task_docs, ft ? ft->k : 0, ft ? ft->part : nullptr, ft ? (int)ft->max_slots : 0, sp.slices,
                     g_clock_probe);
  if ((rc = launch_check("maxsim_scan_f8x4_kernel"))) return rc;
  return finish_split(ix, sp, st);
}

// MXFP8 long documents (index ld = 256 / 512 / 1024): B <= 2 the direct scan
// in 128-token blocks; larger B the doc-interleaved scan with its doc group
// spanning ld / 32 iterations (the row maxima carried across), B <= 8 in the
// 4-wave x 2-query shape, two per CU, else the production 8 waves x 8 queries.
template <int LD>
int launch_f8_long(cbv2_index* ix, const uint8_t* Qb, const uint8_t* Qs, int B, int lq, float* out, int64_t ld_out,
                   hipStream_t st, int* ctr_ws) {
  if (B <= kF8SmallMaxB)
    return launch_f8x4<32, 3, true, 2, 2, 2, 4, 0, LD, kF8D, true>(ix, Qb, Qs, B, lq, out, ld_out, st, kF8DynB8,
                                                                   kScanTaskDocs, ctr_ws);
  return launch_f8x4<32, 3, true, kF8QW, 1, 2, kF8Waves, 0, LD, kF8D, true>(ix, Qb, Qs, B, lq, out, ld_out, st,
                                                                            kScanDynFrac, kScanTaskDocs, ctr_ws);
}

// The MXFP8 streaming scan (B <= 2, any ld): one 4-wave workgroup per CU,
// chunks for kDirectOversub x the resident waves.
template <int WAVES = 8, int SLOTS = 8, bool TW2 = true>
int launch_f8_stream(cbv2_index* ix, const uint8_t* Qb, const uint8_t* Qs, int B, int lq, float* out, int64_t ld_out,
                     hipStream_t st) {
  constexpr int QW = 2;
  const int nq_groups = (B + QW - 1) / QW;
  int64_t n_chunks = (int64_t)WAVES * cu_count(ix->device) * kDirectOversub / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  if (n_chunks < 1) n_chunks = 1;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t grid = ((int64_t)nq_groups * n_chunks + WAVES - 1) / WAVES;
  if (grid > 0x7fffffff) return fail(CBV2_EUNSUPPORTED, "scan grid too large");
  hipLaunchKernelGGL((maxsim_scan_f8_stream_kernel<QW, 2, WAVES, SLOTS, TW2>), dim3((unsigned)grid), dim3(WAVES * 64), 0, st,
                     ix->tokens,
                     ix->scales, ix->doclens, ix->n, Qb, Qs, B, lq, out, ld_out, chunk_docs, (int)ix->ld);
  return launch_check("maxsim_scan_f8_stream_kernel");
}

int scan_f8_long(cbv2_index* ix, const uint8_t* Qb, const uint8_t* Qs, int B, int lq, float* out, int64_t ld_out,
                 hipStream_t st, int* ctr_ws) {
  if (B <= kF8DirectMaxB) return launch_f8_stream(ix, Qb, Qs, B, lq, out, ld_out, st);
  switch (ix->ld) {
    case 256: return launch_f8_long<256>(ix, Qb, Qs, B, lq, out, ld_out, st, ctr_ws);
    case 512: return launch_f8_long<512>(ix, Qb, Qs, B, lq, out, ld_out, st, ctr_ws);
    case 1024: return launch_f8_long<1024>(ix, Qb, Qs, B, lq, out, ld_out, st, ctr_ws);
    default:
      return fail(CBV2_EUNSUPPORTED, "index ld %d not built", (int)ix->ld);
  }
}

int scan_f8(cbv2_index* ix, const uint8_t* Qb, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
            float dyn_frac = kF8DynAuto, int task_docs = kScanTaskDocs, int shape = 0, int* ctr_ws = nullptr,
            FusedTopk* ft = nullptr) {
  if (ix->n == 0) return CBV2_OK;
  const uint8_t* Qs = Qb + (size_t)B * lq * kDim;
  const bool auto_frac = dyn_frac < 0.0f;
  auto frac = [&](float d) { return auto_frac ? d : dyn_frac; };
  if (ix->ld != kLd) {   // long documents: automatic shape only (B <= 8 direct, else 8 waves x 8 queries)
    if (ft != nullptr || shape != 0) return fail(CBV2_EUNSUPPORTED, "long-doc index: automatic scan only");
    return scan_f8_long(ix, Qb, Qs, B, lq, out, ld_out, st, ctr_ws);
  }
#ifdef CBV2_LAB   // fused top-k on MXFP8 (A/B only: its build spills; fused_slots never picks it in the product)
  if (ft != nullptr)
    return launch_f8x4<32, 3, true, kF8QW, 1, 2, kF8Waves, kFusedCap>(ix, Qb, Qs, B, lq, nullptr, 0, st,
                                                                      frac(kScanDynFrac), task_docs, ctr_ws, ft);
#else
  if (ft != nullptr) return fail(CBV2_EUNSUPPORTED, "fused top-k: not built for MXFP8 indexes");
#endif
  // dense docs (CBV2_OPT_DENSE_DOCS): B <= 2 too on the 4 x 1 shape (every slot streamed)
  if ((B > kF8DirectMaxB || ix->dense_docs) && shape == 0) shape = pick_shape(kF8Shapes, B);
  if (B <= kF8DirectMaxB && shape == 0) return launch_f8_stream(ix, Qb, Qs, B, lq, out, ld_out, st);
#ifdef CBV2_LAB   // shapes tools/scan_lab.hip A/Bs (the product's library leaves them out)
  if (B <= kF8DirectMaxB && shape == 25) return launch_f8_stream(ix, Qb, Qs, B, lq, out, ld_out, st);  // lab
  if (B <= kF8DirectMaxB && shape == 19) return launch_f8_stream<4, 16, false>(ix, Qb, Qs, B, lq, out, ld_out, st);  // lab
  if (B <= kF8DirectMaxB && shape == 21) return launch_f8_stream<16, 4, false>(ix, Qb, Qs, B, lq, out, ld_out, st);  // lab
  // lab: one tile per wait (the production 8 x 8 ring before TW2) / TW2 at 4 x 16
  if (B <= kF8DirectMaxB && shape == 22) return launch_f8_stream<8, 8, false>(ix, Qb, Qs, B, lq, out, ld_out, st);
  if (B <= kF8DirectMaxB && shape == 23) return launch_f8_stream<4, 16, true>(ix, Qb, Qs, B, lq, out, ld_out, st);
  if (B <= kF8DirectMaxB && shape == 20) {   // lab: the direct scan
    constexpr int QW = 2;
    const int nq_groups = (B + QW - 1) / QW;
    const int64_t target_waves = 8LL * cu_count(ix->device);
    int64_t n_chunks = target_waves / nq_groups;
    if (n_chunks > ix->n) n_chunks = ix->n;
    if (n_chunks < 1) n_chunks = 1;
    const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
    n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
    const int64_t grid = ((int64_t)nq_groups * n_chunks + 3) / 4;
    hipLaunchKernelGGL(maxsim_scan_f8_direct_kernel<QW>, dim3((unsigned)grid), dim3(256), 0, st, ix->tokens,
                       ix->scales, ix->doclens, ix->n, Qb, Qs, B, lq, out, ld_out, chunk_docs, kLd);
    return launch_check("maxsim_scan_f8_direct_kernel");
  }
#endif
  // shape: 0 = auto (above); 5 = 8 waves x 8 queries, 32-token iterations,
  // two per barrier (PAIR, round 3: lab, same process, bit-identical, 1M docs
  // B=256 73.95 -> 73.28 ms, 1.25M 92.39 -> 91.75, B=64 19.28 -> 19.20;
  // profiles/r03g_lab_f8_*), with the prefetch after each tile's first MFMA
  // (PF: 75.7 -> 73.5 ms at 1M, B=256); 7 / 8 / 9 = the 4-wave shapes of kF8Shapes.  Lab
  // A/B only: 1 = 5 without PF, 2 = 64 / 2-deep, 3 = 64 / 3-deep, 4 = 128 /
  // 2-deep (2-4 spill at 8 queries per wave), 6 = 2 with PF, 10 = 9 with
  // three workgroups per CU.
  switch (shape) {
    case 5: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 4-wave workgroups (32-token / 3-deep, PF): 7 = 4 queries per wave, three
    // workgroups per CU (3 waves per SIMD); 8 = 8 queries per wave, two per CU
    // (2 waves per SIMD from independent barrier domains); 9 = 2 queries per
    // wave, two per CU
    case 7:
      if (B <= 16)   // one query group: non-temporal doc stream
        return launch_f8x4<32, 3, true, 4, 3, 3, 4, 0, kLd, kF8D47, true, false, false, false, false, 0, 2>(
            ix, Qb, Qs, B, lq, out, ld_out, st, frac(kF8DynSmall), task_docs, ctr_ws);
      return launch_f8x4<32, 3, true, 4, 3, 3, 4, 0, kLd, kF8D47, true>(ix, Qb, Qs, B, lq, out, ld_out, st,
                                                                       frac(kF8DynSmall), task_docs, ctr_ws);
    case 8: return launch_f8x4<32, 3, true, 8, 2, 2, 4, 0, kLd, kF8D47, true>(ix, Qb, Qs, B, lq, out, ld_out, st,
                                                                              frac(kF8DynSmall), task_docs, ctr_ws);
    case 9:
      if (B <= 8)    // one query group: non-temporal doc stream
        return launch_f8x4<32, 3, true, 2, 2, 2, 4, 0, kLd, kF8D, true, false, false, false, false, 0, 2>(
            ix, Qb, Qs, B, lq, out, ld_out, st, frac(kF8DynB8), task_docs, ctr_ws);
      return launch_f8x4<32, 3, true, 2, 2, 2, 4, 0, kLd, kF8D, true>(ix, Qb, Qs, B, lq, out, ld_out, st,
                                                                     frac(kF8DynB8), task_docs, ctr_ws);
    // 24 = 1 query per wave, two per CU (B = 3-4 without padded slots), non-temporal
    case 24: return launch_f8x4<32, 3, true, 1, 2, 2, 4, 0, kLd, 1, true, false, false, false, false, 0, 2>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kF8DynB8), task_docs, ctr_ws);
#ifdef CBV2_LAB
    case 1: return launch_f8x4<32, 3>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 2: return launch_f8x4<64, 2>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 3: return launch_f8x4<64, 3>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 4: return launch_f8x4<128, 2>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 6: return launch_f8x4<64, 2, true>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 12 = shape 5 before PAIR: one 32-token iteration per barrier, 3-deep ring
    case 12: return launch_f8x4<32, 3, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 10: return launch_f8x4<32, 3, true, 2, 3, 3, 4>(ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 11 = shape 5 as it was before the packed scales and D = 3 (round 2)
    case 11: return launch_f8x4<32, 3, true, kF8QW, 1, 2, kF8Waves, 0, kLd, 1, false>(ix, Qb, Qs, B, lq, out, ld_out,
                                                                                     st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 13 / 14 / 15 = shape 5 with SPREAD2 / SPLIT / both
    case 13: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, true, false>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 14: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, false, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 15: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, true, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 16 = QUAD: four 32-token iterations (a whole 128-token doc group) per barrier, 8 ring slots
    case 16: return launch_f8x4<32, 8, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, false, false, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    // 17 / 18 = INVALID probes of shape 5: no per-MFMA fold / no epilogue row sums
    case 17: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, false, false, false, 1>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
    case 18: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true, false, false, false, 2>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
#endif
    default: return launch_f8x4<32, 4, true, kF8QW, 1, 2, kF8Waves, 0, kLd, kF8D, true, true>(
        ix, Qb, Qs, B, lq, out, ld_out, st, frac(kScanDynFrac), task_docs, ctr_ws);
  }
}

// Fused top-k eligibility of a search, and the slot count its workspace
// holds (0 = the unfused path: score matrix + row top-k).  The doc-interleaved
// scans only (bf16 B > 16, MXFP8 B > 8): the small-batch scans write B*n
// scores, a few MB, and the selection over their many per-wave lists would
// cost more than the matrix.
int64_t fused_slots(const cbv2_index* ix, int32_t scorer, int32_t B, int32_t k) {
  if (!ix->fused_topk || scorer != CBV2_SCORER_MAXSIM || ix->n == 0 || k > kFusedMaxK || ix->ld != kLd) return 0;
  // MXFP8: the fused build of the f8 scan spills (its query fragments fill the
  // VGPR file): 78.1 vs 74.1 ms at 1M, B=256 (profiles/r02b_fused_ab.jsonl),
  // so MXFP8 searches stay unfused; CBV2_OPT_FUSED_TOPK = 2 forces it (A/B).
  if (ix->dtype == CBV2_DTYPE_MXFP8) {
#ifndef CBV2_LAB
    return 0;   // (lab builds: CBV2_OPT_FUSED_TOPK = 2 forces it)
#endif
    if (B <= kF8SmallMaxB || ix->fused_topk_mode < 2) return 0;
    return scan_chunks(ix, (B + kF8Waves * kF8QW - 1) / (kF8Waves * kF8QW), cu_count(ix->device));
  }
  if (B <= kSmallLdsMaxB) return 0;
  return scan_chunks(ix, (B + 31) / 32, cu_count(ix->device));
}

// Block-max top-k eligibility of a search (topk_bmax_kernel): the unfused
// MaxSim scan of a 128-slot index, rows long enough for the sampled path
// (shorter ones take the exact row select) and block keys that fit its LDS.
bool bmax_eligible(const cbv2_index* ix, int32_t scorer, int32_t B, int32_t k) {
  return ix->topk_bmax != 0 && scorer == CBV2_SCORER_MAXSIM && ix->ld == kLd && ix->n >= kSampledMinN &&
         bm_blocks(ix->n) <= kBmMaxBlocks && k <= kTopkMax && B <= 65535 && fused_slots(ix, scorer, B, k) == 0;
}
size_t bm_ws_bytes(int32_t B, int64_t n) {
  return ((size_t)B * (size_t)(bm_blocks(n) + bm_supers(n)) * 4 + 255) & ~(size_t)255;
}

// blocks_ready: bm already holds the block maxima (folded into the scan).
// done (nullable; B <= kBmFusedMaxB): zeroed per-row arrival counters -- the
// block maxima and the select then run in ONE launch (bmax_topk_kernel).
constexpr int kBmFusedMaxB = 8;
constexpr int kBmDoneOff = kRingInts - kBmFusedMaxB;   // cbv2_search's arrival counters in its counter block
int topk_bmax(const float* scores, int32_t B, int64_t n, int64_t ld, int32_t k, int64_t id_base, uint32_t* bm,
              float* out_s, int32_t* out_i, hipStream_t st, int dev, bool blocks_ready = false,
              int32_t* done = nullptr, int64_t done_ld = 1) {
  const Mirror mirror = g_ids_mirror;
  if (mirror.w != nullptr) g_ids_mirror_used = true;   // every row's ids written to it below
  static std::atomic<bool> attr_set[64] = {};
  if (dev < 0 || dev >= 64 || !attr_set[dev].load(std::memory_order_relaxed)) {   // once per device
    const int lds_max = (int)(kBmFixedLds + (size_t)kBmMaxBlocks * 4);
    CBV2_HIP(hipFuncSetAttribute((const void*)topk_bmax_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
    CBV2_HIP(hipFuncSetAttribute((const void*)bmax_topk_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_max));
    if (dev >= 0 && dev < 64) attr_set[dev].store(true, std::memory_order_relaxed);
  }
  const int64_t nb = bm_blocks(n), ns = bm_supers(n);
  uint32_t* sb = bm_super_keys(bm, B, n);
  if (!blocks_ready && done != nullptr && B <= kBmFusedMaxB) {
    const size_t lds = bm_select_lds(n, k);
    hipLaunchKernelGGL(bmax_topk_kernel, dim3((unsigned)((nb + kBmFusedBlocksPerWg - 1) / kBmFusedBlocksPerWg),
                                               (unsigned)B),
                       dim3(kTkThreads), lds, st, scores, n, ld, k, id_base, bm, nb, sb, ns, done, done_ld, out_s,
                       out_i, mirror, LAB_STAMPS(0));
    return launch_check("bmax_topk_kernel");
  }
  if (!blocks_ready) {
    hipLaunchKernelGGL(block_max_kernel, dim3((unsigned)((nb + kBmBlocksPerWg - 1) / kBmBlocksPerWg), (unsigned)B),
                       dim3(256), 0, st, scores, n, ld, bm, nb, sb, ns);
    if (int rc = launch_check("block_max_kernel")) return rc;
  }
  const size_t lds = bm_select_lds(n, k);
  hipLaunchKernelGGL(topk_bmax_kernel, dim3((unsigned)B), dim3(kTkThreads), lds, st, scores, n, ld, k, id_base, bm,
                     nb, sb, ns, out_s, out_i, mirror, LAB_STAMPS(0));
  return launch_check("topk_bmax_kernel");
}

int scan_meanpool(cbv2_index* ix, const float* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st) {
  if (ix->n == 0) return CBV2_OK;
  dim3 grid((unsigned)((ix->n + kMpDocs - 1) / kMpDocs), (unsigned)((B + kMpQ - 1) / kMpQ));
  hipLaunchKernelGGL(meanpool_scores_kernel, grid, dim3(256), 0, st, ix->doc_means, ix->n, Q, B, lq, out, ld_out);
  return launch_check("meanpool_scores_kernel");
}

int check_query(cbv2_index* ix, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B, int32_t lq) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  CBV2_REQUIRE(Q != nullptr, "null query pointer");
  CBV2_REQUIRE(B >= 1, "B must be >= 1 (got %d)", B);
  CBV2_REQUIRE(lq >= 1, "lq must be >= 1 (got %d)", lq);
  CBV2_REQUIRE(aligned16(Q), "query pointer must be 16-byte aligned");
  if (scorer == CBV2_SCORER_MAXSIM) {
    if (ix->resid != nullptr && q_dtype == CBV2_DTYPE_F32)
      return fail(CBV2_EINVAL, "f32 queries on an fp32-faithful index go through cbv2_score_f32/_search_f32/_rerank_f32");
    if (ix->dtype == CBV2_DTYPE_MXFP8)
      CBV2_REQUIRE(q_dtype == CBV2_DTYPE_MXFP8, "an MXFP8 index takes MXFP8 queries (cbv2_quantize_mxfp8)");
    else
      CBV2_REQUIRE(q_dtype == CBV2_DTYPE_BF16, "maxsim scorer takes bf16 queries");
    CBV2_REQUIRE(lq <= kLqMax, "maxsim takes at most %d query tokens (got %d)", kLqMax, lq);
  } else if (scorer == CBV2_SCORER_REF_MEANPOOL_COSINE) {
    CBV2_REQUIRE(q_dtype == CBV2_DTYPE_F32, "ref_meanpool_cosine scorer takes f32 queries");
    if (ix->doc_means == nullptr) return fail(CBV2_ESTATE, "doc means not built (cbv2_index_build_means)");
  } else {
    return fail(CBV2_EINVAL, "unknown scorer %d", scorer);
  }
  return CBV2_OK;
}

// Start/stop events of the next timed scan, reserved under the handle's mutex
// (false when timing is off or an event cannot be created: the scan then runs
// untimed).
bool scan_event_pair(cbv2_index* ix, hipEvent_t* e0, hipEvent_t* e1) {
  std::lock_guard<std::mutex> lk(ix->mu);
  if (!ix->time_scans) return false;
  const size_t i = ix->scan_ev_used;
  while (ix->scan_ev.size() < 2 * i + 2) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return false;
    ix->scan_ev.push_back(e);
  }
  *e0 = ix->scan_ev[2 * i];
  *e1 = ix->scan_ev[2 * i + 1];
  ++ix->scan_ev_used;
  return true;
}

int scan_maxsim_timed(cbv2_index* ix, const void* Q, int32_t B, int32_t lq, float* out, int64_t ld_out,
                      hipStream_t st, int* ctr_ws = nullptr, FusedTopk* ft = nullptr, uint32_t* bm = nullptr) {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool timed = scan_event_pair(ix, &e0, &e1);
  if (timed && hipEventRecord(e0, st) != hipSuccess) return fail(CBV2_EHIP, "hipEventRecord failed");
  g_clock_probe = timed && ix->clock_on ? ix->clk : nullptr;
  const int rc = ix->dtype == CBV2_DTYPE_MXFP8
                     ? scan_f8(ix, (const uint8_t*)Q, B, lq, out, ld_out, st, kF8DynAuto, kScanTaskDocs, 0, ctr_ws, ft)
                     : scan_maxsim(ix, (const uint16_t*)Q, B, lq, out, ld_out, st, kDefaultScan, ctr_ws, ft, bm);
  g_clock_probe = nullptr;
  // the stop event is recorded even after a failed launch, so the reserved pair stays readable
  if (timed && hipEventRecord(e1, st) != hipSuccess && rc == CBV2_OK) return fail(CBV2_EHIP, "hipEventRecord failed");
  return rc;
}

// Band timing marks (cbv2_index_band_times): start after the bf16 top-k of a
// faithful search, stop after its band select / fallback.  A stop without a
// recorded start (timing switched on in between) records nothing.
int band_mark(cbv2_index* ix, bool stop, hipStream_t st) {
  std::lock_guard<std::mutex> lk(ix->mu);
  if (!ix->time_scans) return CBV2_OK;
  const size_t i = ix->band_ev_used;
  if (!stop) {
    while (ix->band_ev.size() < 2 * i + 2) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return CBV2_OK;   // untimed, as for the scans
      ix->band_ev.push_back(e);
    }
    CBV2_HIP(hipEventRecord(ix->band_ev[2 * i], st));
    ix->band_open = true;
    return CBV2_OK;
  }
  if (!ix->band_open) return CBV2_OK;
  CBV2_HIP(hipEventRecord(ix->band_ev[2 * i + 1], st));
  ix->band_open = false;
  ++ix->band_ev_used;
  return CBV2_OK;
}

int score_impl(cbv2_index* ix, int32_t scorer, const void* Q, int32_t B, int32_t lq, float* out,
               int64_t ld_out, hipStream_t st, int* ctr_ws = nullptr) {
  if (scorer == CBV2_SCORER_MAXSIM) return scan_maxsim_timed(ix, Q, B, lq, out, ld_out, st, ctr_ws);
  return scan_meanpool(ix, (const float*)Q, B, lq, out, ld_out, st);
}

__global__ void fill_neg_inf_kernel(float* x, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = neg_inf();
}

__global__ void fill_empty_kernel(float* out_s, int32_t* out_i, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < total) {
    out_s[i] = neg_inf();
    out_i[i] = -1;
  }
}

int topk_impl_empty(int32_t B, int32_t k, float* out_s, int32_t* out_i, hipStream_t st) {
  const int64_t total = (int64_t)B * k;
  hipLaunchKernelGGL(fill_empty_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, out_s, out_i, total);
  return launch_check("fill_empty_kernel");
}

size_t topk_ws_bytes(int32_t B, int64_t n) {
  if (n < kSampledMinN) return 0;
  return (size_t)B * kCandCap * sizeof(uint64_t) + (((size_t)B * sizeof(uint32_t) + 255) & ~(size_t)255);
}

int topk_multi(const float* scores, int32_t B, int64_t n, int64_t ld, int32_t k, int64_t id_base,
               const int32_t* ids, int64_t ids_ld, float* out_s, int32_t* out_i, int32_t* out_p, hipStream_t st,
               const int32_t* only_neg = nullptr) {
  hipLaunchKernelGGL(topk_multi_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, scores, n, ld, k, id_base, ids,
                     ids_ld, out_s, out_i, out_p, only_neg);
  return launch_check("topk_multi_kernel");
}

int topk_impl(const float* scores, int32_t B, int64_t n, int64_t ld, int32_t k, int64_t id_base, void* ws,
              size_t ws_bytes, float* out_s, int32_t* out_i, hipStream_t st, int dev) {
  if (k > kTopkMax) return topk_multi(scores, B, n, ld, k, id_base, nullptr, 0, out_s, out_i, nullptr, st);
  const size_t need = topk_ws_bytes(B, n);
  if (need == 0 || ws == nullptr || ws_bytes < need || B > 65535) {  // grid.y of the filter launch
    const Mirror mirror = g_ids_mirror;   // the search's final ids (the latency path's host mirror)
    if (mirror.w != nullptr) g_ids_mirror_used = true;
    hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, scores, n, ld, k, id_base,
                       out_s, out_i, nullptr, mirror);
    return launch_check("topk_rows_kernel");
  }
  uint64_t* cand = (uint64_t*)ws;
  uint32_t* cnt = (uint32_t*)((uint8_t*)ws + (size_t)B * kCandCap * sizeof(uint64_t));
  CBV2_HIP(hipMemsetAsync(cnt, 0, (size_t)B * sizeof(uint32_t), st));
  int64_t splits = (2LL * cu_count(dev) + B - 1) / B;
  const int64_t max_splits = n / 16384;
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  hipLaunchKernelGGL(topk_filter_kernel, dim3((unsigned)splits, (unsigned)B), dim3(256), 0, st, scores, n, ld, k, cnt,
                     cand);
  int rc = launch_check("topk_filter_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(topk_select_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, scores, n, ld, k, id_base, cnt,
                     cand, out_s, out_i);
  return launch_check("topk_select_kernel");
}

// ---------------------------------------------------------------------------
// fp32-faithful path: workspace layout and the three operations.
// ---------------------------------------------------------------------------
struct F32Ws {
  int* ctr = nullptr;
  uint16_t* qhi = nullptr;
  uint16_t* qlo = nullptr;
  float* beta = nullptr;
  float* lb = nullptr;        // SEARCH: the two-pass band's bound, order-preserving bits (atomic min)
  int32_t* count = nullptr;
  int32_t* done = nullptr;    // SEARCH: the fallback's finished-workgroup counter per row (zeroed by the split)
  int32_t* arrive = nullptr;  // [kArriveSlots][B][kArriveInts] row_last_arrival counters (zeroed by the split)
  int32_t* cand = nullptr;
  float* F = nullptr;
  void* tk = nullptr;
  size_t tk_bytes = 0;
  float* T = nullptr;
  // doc-major band rescoring (SEARCH)
  int32_t* dcnt = nullptr;
  int32_t* doff = nullptr;
  int32_t* act = nullptr;
  int32_t* act_off = nullptr;
  int32_t* act_cnt = nullptr;
  int32_t* dctr = nullptr;
  int32_t* pair_b = nullptr;
  int32_t* pair_c = nullptr;
};

// Per-row arrival counters of a faithful workspace (F32Ws::arrive, row b of
// slot j at (j * B + b) * kArriveInts): the launches whose last workgroup per
// row runs the row's selection (row_last_arrival).
constexpr int kArriveSlots = kArriveSlotsK;
constexpr int kArrBmax = 0, kArrBand = 1, kArrRerank = 2, kArrPhase1 = kArrPhase1K;
inline int32_t* arrive_row0(const F32Ws& w, int slot, int B) { return w.arrive + (size_t)slot * B * kArriveInts; }

// op SCORE: split queries; RERANK: + F [B][C]; SEARCH: + band [B][cap] + scan.
size_t f32_ws_layout(const cbv2_index* ix, int op, int B, int lq, int cap, uint8_t* base, F32Ws* w) {
  size_t off = 0;
  auto take = [&](size_t bytes) -> uint8_t* {
    uint8_t* p = base ? base + off : nullptr;
    off += (bytes + 255) & ~(size_t)255;
    return p;
  };
  const size_t qbytes = (size_t)B * lq * kDim * sizeof(uint16_t);
  if (op == CBV2_F32_SEARCH) w->ctr = (int*)take(kCtrBytes);
  w->qhi = (uint16_t*)take(qbytes);
  w->qlo = (uint16_t*)take(qbytes);
  w->beta = (float*)take((size_t)B * sizeof(float));
  if (op == CBV2_F32_SEARCH) w->lb = (float*)take((size_t)B * sizeof(float));
  if (op == CBV2_F32_RERANK) w->F = (float*)take((size_t)B * cap * sizeof(float));
  if (op != CBV2_F32_SCORE) w->arrive = (int32_t*)take((size_t)kArriveSlots * B * kArriveInts * sizeof(int32_t));
  if (op == CBV2_F32_SEARCH) {
    w->count = (int32_t*)take((size_t)B * sizeof(int32_t));
    w->done = (int32_t*)take((size_t)B * sizeof(int32_t));
    w->cand = (int32_t*)take((size_t)B * cap * sizeof(int32_t));
    w->F = (float*)take((size_t)B * cap * sizeof(float));
    w->tk_bytes = std::max(topk_ws_bytes(B, ix->n), bm_ws_bytes(B, ix->n));   // either top-k of T
    w->tk = take(w->tk_bytes);
    w->T = (float*)take((size_t)B * (size_t)(ix->n > 0 ? ix->n : 1) * sizeof(float));
    const size_t nd = (size_t)(ix->n > 0 ? ix->n : 1) * sizeof(int32_t);
    w->dcnt = (int32_t*)take(nd);
    w->doff = (int32_t*)take(nd);
    w->act = (int32_t*)take(nd);
    w->act_off = (int32_t*)take(nd);
    w->act_cnt = (int32_t*)take(nd);
    w->dctr = (int32_t*)take(2 * sizeof(int32_t));
    w->pair_b = (int32_t*)take((size_t)B * cap * sizeof(int32_t));
    w->pair_c = (int32_t*)take((size_t)B * cap * sizeof(int32_t));
  }
  return off;
}

int check_f32(cbv2_index* ix, int op, const float* Q, int32_t B, int32_t lq, int32_t cap, void* ws, size_t wsb,
              F32Ws* w) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  if (ix->resid == nullptr) return fail(CBV2_ESTATE, "index has no fp32 residual (cbv2_index_attach_residual)");
  CBV2_REQUIRE(Q != nullptr && aligned16(Q), "query pointer must be non-null and 16-byte aligned");
  CBV2_REQUIRE(B >= 1 && B <= 65535, "B must be in [1, 65535] (got %d)", B);
  CBV2_REQUIRE(lq >= 1 && lq <= kLqMax, "lq must be in [1, %d] (got %d)", kLqMax, lq);
  const size_t need = f32_ws_layout(ix, op, B, lq, cap, nullptr, w);
  CBV2_REQUIRE(ws != nullptr && wsb >= need && aligned16(ws), "workspace too small or misaligned (%zu < %zu)",
               wsb, need);
  f32_ws_layout(ix, op, B, lq, cap, (uint8_t*)ws, w);
  return CBV2_OK;
}

// (a SEARCH workspace's split also resets the rows' band state: count, lb, done)
// Which queries each workspace's split (qhi / qlo) holds, for
// cbv2_rerank_f32_after_search: the one-trip rerank reuses the split its
// search left in the stage-2 workspace only while the last split enqueued
// into that workspace is that search's (same index, Q pointer, B, lq);
// otherwise it splits Q again.  Keyed by the qhi address; a small ring, so an
// evicted entry only costs the re-split.
struct SplitTag {
  const void* qhi = nullptr;
  const cbv2_index* ix = nullptr;
  const float* Q = nullptr;
  int B = 0, lq = 0;
};
constexpr int kSplitTags = 64;
std::mutex g_split_mu;
SplitTag g_split_tags[kSplitTags];
int g_split_next = 0;

void note_split(const cbv2_index* ix, const float* Q, int B, int lq, const void* qhi) {
  std::lock_guard<std::mutex> lk(g_split_mu);
  int slot = -1;
  for (int i = 0; i < kSplitTags && slot < 0; ++i)
    if (g_split_tags[i].qhi == qhi) slot = i;
  if (slot < 0) slot = g_split_next++ % kSplitTags;
  g_split_tags[slot] = SplitTag{qhi, ix, Q, B, lq};
}

bool split_holds(const cbv2_index* ix, const float* Q, int B, int lq, const void* qhi) {
  std::lock_guard<std::mutex> lk(g_split_mu);
  for (int i = 0; i < kSplitTags; ++i) {
    const SplitTag& t = g_split_tags[i];
    if (t.qhi == qhi) return t.ix == ix && t.Q == Q && t.B == B && t.lq == lq;
  }
  return false;
}

// zero_ctr: the split also zeroes the scan's task-counter block (w->ctr; the
// search's scan then runs under CtrPrezeroed and skips its memset launch).
// zkeys (nullable, 16-B aligned): nz ints zeroed by extra workgroups (the
// block keys the next scan folds in with atomic max)
int split_queries(cbv2_index* ix, const float* Q, int B, int lq, F32Ws* w, hipStream_t st, int count0 = 0,
                  bool zero_ctr = false, uint32_t* zkeys = nullptr, int64_t nz = 0) {
  note_split(ix, Q, B, lq, w->qhi);
  const int64_t extra = zkeys != nullptr ? (nz + kSplitZeroInts - 1) / kSplitZeroInts : 0;
  const bool publish = g_split_ready_seq != 0 && g_split_ready_word != nullptr;
  if (publish) {   // the flags this split publishes: one word per row
    g_ready_flag = g_split_ready_word;
    g_ready_flag_ld = 1;
  }
  hipLaunchKernelGGL(split_query_kernel, dim3((unsigned)(B + extra)), dim3(512), 0, st, Q, lq, w->qhi, w->qlo,
                     ix->resid_max, ix->norm_max, w->beta, w->count, reinterpret_cast<uint32_t*>(w->lb), w->done,
                     count0, w->arrive, kArriveSlots * kArriveInts, zero_ctr ? w->ctr : nullptr,
                     zero_ctr ? kRingInts : 0, publish ? g_split_ready_seq : 0u, B, zkeys, nz,
                     publish ? g_split_ready_word : nullptr);
  return launch_check("split_query_kernel");
}

// pw: candidates per wave step (0 = auto: one per wave for launches of at
// most kRsSmallPairs (query, candidate) pairs, kRsPerWave beyond)
constexpr int64_t kRsSmallPairs = 4096;
constexpr int64_t kRsSplitGrid = 1024;   // workgroups per row of a split rescoring launch (grid-stride beyond)
int launch_rescore(cbv2_index* ix, const F32Ws* w, int B, int lq, const int32_t* cand, const int32_t* count,
                   int64_t limit, int64_t ld_c, float* out, int64_t ld_out, hipStream_t st,
                   const int32_t* only_neg = nullptr, int pw = 0, uint32_t* lb_min = nullptr, int64_t c0 = 0,
                   float* fb_T = nullptr, int32_t* fb_done = nullptr, int fb_k = 0, float* fb_s = nullptr,
                   int32_t* fb_i = nullptr, const RowSelect& rs = RowSelect(), TaggedCand tc = TaggedCand()) {
  if (limit <= c0 && fb_T == nullptr && rs.mode == kSelNone) return CBV2_OK;
  if (ix->rescore_split) {   // one pair per workgroup (its doc split over 4 waves, or 2 for launches past
                             // the chip's resident 4-wave workgroups: one round of 2-wave ones instead of two)
    int64_t span = limit - c0;   // (pairs [c0, min(count, limit)) of a row)
    if (fb_T != nullptr) span = std::max<int64_t>(span, std::min<int64_t>(ix->n, 256));   // the fallback's grid
    if (span < 1) span = 1;      // a row select runs in the row's (last) workgroup even with no pair to score
    // workgroups per row: ~4k per launch, 256..1024 per row -- a row's pairs
    // beyond that grid-stride (band at 1M docs, grid 1024 / 512 / 256: B=256
    // 2.76 / 2.64 / 2.57 ms, B=16 0.247 / 0.238 / 0.225, B=1 39 / 40 / 41 us;
    // profiles/r04w_grid_ab.jsonl)
    const int64_t grid_auto = std::min<int64_t>(kRsSplitGrid, std::max<int64_t>(256, 4096 / std::max(B, 1)));
    const int64_t grid_max = ix->rescore_grid > 0 ? ix->rescore_grid : grid_auto;
    const unsigned gx = (unsigned)(span < grid_max ? span : grid_max);
    // (long documents keep 4 waves: the 2-wave build of the long-doc pair
    // carries its row maxima across blocks and spills; same bits either way)
    const bool two = ix->ld == kLd && (int64_t)gx * B > 3LL * cu_count(ix->device);
    auto kern = ix->ld != kLd ? rescore_split_kernel<true, 4>
                              : (two ? rescore_split_kernel<false, 2> : rescore_split_kernel<false, 4>);
    hipLaunchKernelGGL(kern, dim3(gx, (unsigned)B), dim3(two ? 128 : 256), 0, st, ix->tokens, ix->resid, ix->doclens,
                       ix->n, ix->id_base, w->qhi, w->qlo, lq, cand, count, limit, ld_c, out, ld_out, only_neg,
                       (int)ix->ld, lb_min, c0, fb_T, fb_done, fb_k, fb_s, fb_i, rs, tc);
    return launch_check("rescore_split_kernel");
  }
  if (c0 != 0 || fb_T != nullptr || rs.mode != kSelNone || tc.w != nullptr)
    return fail(CBV2_EUNSUPPORTED, "pair offset / fallback / row select need the split rescoring");
  if (pw <= 0) pw = (int64_t)B * limit <= kRsSmallPairs ? 1 : kRsPerWave;
  const int64_t per_wg = 4LL * pw;
  int64_t gx = (limit + per_wg - 1) / per_wg;
  // at most 1024 workgroups per row (4096 waves: a lone fallback row still
  // streams at full rate), grid-stride beyond; rows that skip exit at once
  gx = gx < 1024 ? gx : 1024;
  hipLaunchKernelGGL(ix->ld != kLd ? rescore_x3_kernel<true> : rescore_x3_kernel<false>, dim3((unsigned)gx, (unsigned)B),
                     dim3(256), 0, st, ix->tokens, ix->resid,
                     ix->doclens, ix->n, ix->id_base, w->qhi, w->qlo, lq, cand, count, limit, ld_c, out, ld_out,
                     only_neg, (int)ix->ld, pw, lb_min);
  return launch_check("rescore_x3_kernel");
}
}  // namespace

extern "C" {

// Internal: lets host_bm25.cpp report errors through cbv2_last_error().
int cbv2_set_error(int code, const char* msg) { return fail(code, "%s", msg); }

int cbv2_abi_version(void) { return CBV2_ABI_VERSION; }

// _build.py passes -DCBV2_BUILD_STAMP="<sha256 prefix of the sources + flags>"; the
// prefix makes the stamp findable in the .so's bytes without loading it.
#ifndef CBV2_BUILD_STAMP
#define CBV2_BUILD_STAMP "unstamped"
#endif
const char* cbv2_build_stamp(void) { return "cbv2-build-stamp:" CBV2_BUILD_STAMP; }

const char* cbv2_last_error(void) { return g_err; }

int cbv2_index_create(int device, const void* tokens, int32_t dtype, int64_t n, int32_t ld, int32_t d,
                      const int32_t* doclens, int64_t id_base, cbv2_index** out) {
  CBV2_REQUIRE(out != nullptr, "null output handle pointer");
  *out = nullptr;
  CBV2_REQUIRE(n >= 0 && n <= 0x7fffffffLL, "n out of range (%lld)", (long long)n);
  CBV2_REQUIRE(id_base >= 0 && id_base + n <= 0x7fffffffLL, "global ids must fit int32");
  if (dtype != CBV2_DTYPE_BF16) return fail(CBV2_EUNSUPPORTED, "index dtype %d not built (bf16 only)", dtype);
  if ((ld != 128 && ld != 256 && ld != 512 && ld != 1024) || d != kDim)
    return fail(CBV2_EUNSUPPORTED, "index geometry ld=%d d=%d not built (ld = 128, 256, 512 or 1024; d = 128)", ld,
                d);
  if (n > 0) {
    CBV2_REQUIRE(tokens != nullptr && doclens != nullptr, "null tokens/doclens");
    CBV2_REQUIRE(aligned16(tokens), "tokens must be 16-byte aligned");
  }
  int ndev = 0;
  CBV2_HIP(hipGetDeviceCount(&ndev));
  CBV2_REQUIRE(device >= 0 && device < ndev, "device %d out of range (%d devices)", device, ndev);
  cbv2_index* ix = new cbv2_index{device, (const uint8_t*)tokens, n, ld, d, doclens, id_base, nullptr,
                                  CBV2_DTYPE_BF16, nullptr};
  alloc_task_ring(ix);
  *out = ix;
  return CBV2_OK;
}

int cbv2_index_create_mxfp8(int device, const void* tokens, const void* scales, int64_t n, int32_t ld, int32_t d,
                            const int32_t* doclens, int64_t id_base, cbv2_index** out) {
  CBV2_REQUIRE(out != nullptr, "null output handle pointer");
  *out = nullptr;
  CBV2_REQUIRE(n >= 0 && n <= 0x7fffffffLL, "n out of range (%lld)", (long long)n);
  CBV2_REQUIRE(id_base >= 0 && id_base + n <= 0x7fffffffLL, "global ids must fit int32");
  if ((ld != 128 && ld != 256 && ld != 512 && ld != 1024) || d != kDim)
    return fail(CBV2_EUNSUPPORTED, "index geometry ld=%d d=%d not built (ld = 128, 256, 512 or 1024; d = 128)", ld,
                d);
  if (n > 0) {
    CBV2_REQUIRE(tokens != nullptr && scales != nullptr && doclens != nullptr, "null tokens/scales/doclens");
    CBV2_REQUIRE(aligned16(tokens), "tokens must be 16-byte aligned");
    CBV2_REQUIRE(((uintptr_t)scales & 3u) == 0, "scales must be 4-byte aligned");
  }
  int ndev = 0;
  CBV2_HIP(hipGetDeviceCount(&ndev));
  CBV2_REQUIRE(device >= 0 && device < ndev, "device %d out of range (%d devices)", device, ndev);
  *out = new cbv2_index{device, (const uint8_t*)tokens, n, ld, d, doclens, id_base, nullptr, CBV2_DTYPE_MXFP8,
                        (const uint8_t*)scales};
  alloc_task_ring(*out);
  return CBV2_OK;
}

int cbv2_quantize_mxfp8(const void* x, int32_t dtype, int64_t rows, void* q, void* scales, void* stream) {
  CBV2_REQUIRE(rows >= 0, "rows must be >= 0");
  if (rows == 0) return CBV2_OK;
  CBV2_REQUIRE(x && q && scales, "null pointer");
  const int64_t want = (rows + 3) / 4;
  const unsigned grid = (unsigned)(want < 65536 ? want : 65536);  // grid-stride beyond 2^24 work-items
  if (dtype == CBV2_DTYPE_F32) {
    hipLaunchKernelGGL(quantize_mxfp8_kernel<float>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const float*)x,
                       rows, (uint8_t*)q, (uint8_t*)scales);
  } else if (dtype == CBV2_DTYPE_BF16) {
    hipLaunchKernelGGL(quantize_mxfp8_kernel<uint16_t>, dim3(grid), dim3(256), 0, (hipStream_t)stream,
                       (const uint16_t*)x, rows, (uint8_t*)q, (uint8_t*)scales);
  } else {
    return fail(CBV2_EINVAL, "quantize takes bf16 or f32 input (got dtype %d)", dtype);
  }
  return launch_check("quantize_mxfp8_kernel");
}

int cbv2_hbm_alloc(int device, size_t bytes, void** out, int32_t* contiguous) {
  CBV2_REQUIRE(out != nullptr, "null output pointer");
  *out = nullptr;
  if (contiguous) *contiguous = 0;
  if (bytes == 0) return CBV2_OK;
  DeviceGuard dg(device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", device);
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocContiguous) == hipSuccess && p != nullptr) {
    *out = p;
    if (contiguous) *contiguous = 1;
    return CBV2_OK;
  }
  (void)hipGetLastError();   // no contiguous range of that size: plain VRAM
  CBV2_HIP(hipMalloc(&p, bytes));
  *out = p;
  return CBV2_OK;
}

int cbv2_hbm_free(int device, void* p) {
  if (p == nullptr) return CBV2_OK;
  DeviceGuard dg(device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", device);
  CBV2_HIP(hipFree(p));
  return CBV2_OK;
}

int cbv2_index_destroy(cbv2_index* index) {
  if (index != nullptr && (index->task_ring != nullptr || !index->scan_ev.empty() || index->clk != nullptr)) {
    int prev = 0;
    if (hipGetDevice(&prev) == hipSuccess && hipSetDevice(index->device) == hipSuccess) {
      if (index->task_ring != nullptr) (void)hipFree(index->task_ring);
      if (index->clk != nullptr) (void)hipFree(index->clk);
      for (hipEvent_t e : index->ring_ev)
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : index->scan_ev) (void)hipEventDestroy(e);
      for (hipEvent_t e : index->band_ev) (void)hipEventDestroy(e);
      (void)hipSetDevice(prev);
    }
  }
  delete index;
  return CBV2_OK;
}

int cbv2_index_time_scans(cbv2_index* ix, int32_t enable) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  CBV2_REQUIRE(enable >= 0 && enable <= 2, "enable must be 0, 1 or 2 (got %d)", enable);
  std::lock_guard<std::mutex> lk(ix->mu);
  if (enable) ix->scan_ev_used = ix->band_ev_used = 0, ix->band_open = false;
  if (enable == 2) {
    DeviceGuard dg(ix->device);
    if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
    if (ix->clk == nullptr) CBV2_HIP(hipMalloc(&ix->clk, 4 * sizeof(uint64_t)));
    CBV2_HIP(hipMemset(ix->clk, 0, 4 * sizeof(uint64_t)));
  }
  ix->time_scans = enable != 0;
  ix->clock_on = enable == 2;
  return CBV2_OK;
}
int cbv2_index_scan_clock(cbv2_index* ix, int64_t* out4, int32_t reset) {
  CBV2_REQUIRE(ix != nullptr && out4 != nullptr, "null index or output");
  std::lock_guard<std::mutex> lk(ix->mu);
  for (int i = 0; i < 4; ++i) out4[i] = 0;
  if (ix->clk == nullptr) return CBV2_OK;
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  CBV2_HIP(hipDeviceSynchronize());
  uint64_t v[4];
  CBV2_HIP(hipMemcpy(v, ix->clk, sizeof(v), hipMemcpyDeviceToHost));
  for (int i = 0; i < 4; ++i) out4[i] = (int64_t)v[i];
  if (reset) CBV2_HIP(hipMemset(ix->clk, 0, 4 * sizeof(uint64_t)));
  return CBV2_OK;
}

int cbv2_index_scan_times(cbv2_index* ix, float* ms, int32_t max, int32_t* count) {
  CBV2_REQUIRE(ix != nullptr && count != nullptr, "null index or count");
  CBV2_REQUIRE(max >= 0 && (max == 0 || ms != nullptr), "bad output buffer");
  std::lock_guard<std::mutex> lk(ix->mu);
  CBV2_REQUIRE(!ix->time_scans, "disable timing (cbv2_index_time_scans(ix, 0)) before reading the times");
  *count = (int32_t)ix->scan_ev_used;
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  for (size_t i = 0; i < ix->scan_ev_used && i < (size_t)max; ++i) {
    if (hipEventSynchronize(ix->scan_ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(ms + i, ix->scan_ev[2 * i], ix->scan_ev[2 * i + 1]) != hipSuccess)
      return fail(CBV2_EHIP, "scan event %zu: %s", i, hipGetErrorString(hipGetLastError()));
  }
  ix->scan_ev_used = 0;  // read once: the record is consumed
  return CBV2_OK;
}

int cbv2_index_band_times(cbv2_index* ix, float* ms, int32_t max, int32_t* count) {
  CBV2_REQUIRE(ix != nullptr && count != nullptr, "null index or count");
  CBV2_REQUIRE(max >= 0 && (max == 0 || ms != nullptr), "bad output buffer");
  std::lock_guard<std::mutex> lk(ix->mu);
  CBV2_REQUIRE(!ix->time_scans, "disable timing (cbv2_index_time_scans(ix, 0)) before reading the times");
  *count = (int32_t)ix->band_ev_used;
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  for (size_t i = 0; i < ix->band_ev_used && i < (size_t)max; ++i) {
    if (hipEventSynchronize(ix->band_ev[2 * i + 1]) != hipSuccess ||
        hipEventElapsedTime(ms + i, ix->band_ev[2 * i], ix->band_ev[2 * i + 1]) != hipSuccess)
      return fail(CBV2_EHIP, "band event %zu: %s", i, hipGetErrorString(hipGetLastError()));
  }
  ix->band_ev_used = 0;
  ix->band_open = false;
  return CBV2_OK;
}

int cbv2_index_build_means(cbv2_index* ix, const float* tokens_f32, int32_t ld_src, float* doc_means,
                           void* stream) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  CBV2_REQUIRE(ld_src >= 1, "ld_src must be >= 1");
  CBV2_REQUIRE(ix->n == 0 || (tokens_f32 && doc_means), "null tokens_f32/doc_means");
  CBV2_REQUIRE(ix->n < (1LL << 25), "build_means: n too large for one dispatch");  // 128 work-items per doc
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  if (ix->n > 0) {
    hipLaunchKernelGGL(meanpool_build_kernel, dim3((unsigned)ix->n), dim3(128), 0, (hipStream_t)stream,
                       tokens_f32, ld_src, ix->doclens, doc_means);
    int rc = launch_check("meanpool_build_kernel");
    if (rc) return rc;
  }
  ix->doc_means = doc_means;
  return CBV2_OK;
}

int cbv2_score(cbv2_index* ix, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
               float* out, int64_t ld_out, void* stream) {
  int rc = check_query(ix, scorer, Q, q_dtype, B, lq);
  if (rc) return rc;
  CBV2_REQUIRE(ix->n == 0 || out != nullptr, "null output");
  CBV2_REQUIRE(ld_out >= ix->n, "ld_out (%lld) < n (%lld)", (long long)ld_out, (long long)ix->n);
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  return score_impl(ix, scorer, Q, B, lq, out, ld_out, (hipStream_t)stream);
}

size_t cbv2_search_workspace_size(const cbv2_index* ix, int32_t B, int32_t k, int32_t scorer) {
  if (!ix || B < 1 || k < 1) return 0;
  const int64_t slots = fused_slots(ix, scorer, B, k);
  if (slots > 0) return kCtrBytes + (size_t)B * slots * k * sizeof(uint64_t);
  const size_t sel = bmax_eligible(ix, scorer, B, k) ? bm_ws_bytes(B, ix->n) : topk_ws_bytes(B, ix->n);
  return kCtrBytes + sel + (size_t)B * (size_t)(ix->n > 0 ? ix->n : 1) * sizeof(float);
}

size_t cbv2_search_workspace_bytes(const cbv2_index* ix, int32_t B) {
  if (!ix || B < 1) return 0;   // enough for any k and scorer (the unfused layouts are the larger)
  return kCtrBytes + std::max(topk_ws_bytes(B, ix->n), bm_ws_bytes(B, ix->n)) +
         (size_t)B * (size_t)(ix->n > 0 ? ix->n : 1) * sizeof(float);
}

int cbv2_search(cbv2_index* ix, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                int32_t k, void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                void* stream) {
  int rc = check_query(ix, scorer, Q, q_dtype, B, lq);
  if (rc) return rc;
  CBV2_REQUIRE(k >= 1, "k must be >= 1 (got %d)", k);
  CBV2_REQUIRE(out_scores && out_ids, "null outputs");
  const size_t need = cbv2_search_workspace_size(ix, B, k, scorer);
  CBV2_REQUIRE(workspace != nullptr && workspace_bytes >= need && aligned16(workspace),
               "workspace too small or misaligned (%zu < %zu)", workspace_bytes, need);
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  hipStream_t st = (hipStream_t)stream;
  if (ix->n == 0) return topk_impl_empty(B, k, out_scores, out_ids, st);
  int* ctr = (int*)workspace;
  uint8_t* rest = (uint8_t*)workspace + kCtrBytes;
  const int64_t slots = fused_slots(ix, scorer, B, k);
  if (slots > 0) {  // fused scan + top-k: per-workgroup lists, then one select per query
    FusedTopk ft{(uint64_t*)rest, k, slots, 0};
    if ((rc = scan_maxsim_timed(ix, Q, B, lq, nullptr, 0, st, ctr, &ft))) return rc;
    hipLaunchKernelGGL(select_keys_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, ft.part, ft.slots * k,
                       slots * k, k, ix->id_base, out_scores, out_ids);
    return launch_check("select_keys_kernel");
  }
  if (bmax_eligible(ix, scorer, B, k)) {   // block maxima, then one select reading only the blocks that can win
    uint32_t* bm = (uint32_t*)rest;
    float* sc = (float*)(rest + bm_ws_bytes(B, ix->n));
    const bool fold = scan_folds_bmax(ix, B);   // the B <= 2 streaming scans write the block maxima themselves
    // small batches select in the block-max launch's last workgroup: its
    // per-row arrival counters sit at the end of the counter block, zeroed
    // with the scan's task counters (no separate launch when the scan zeroes)
    const bool fused = !fold && B <= kBmFusedMaxB;
    int32_t* done = fused ? ctr + kBmDoneOff : nullptr;
    {
      CtrPolicy cp(fused ? kCtrZeroAll : kCtrDefault);
      if ((rc = scan_maxsim_timed(ix, Q, B, lq, sc, ix->n, st, ctr, nullptr, fold ? bm : nullptr))) return rc;
      if (fused && !g_ctr_zeroed) CBV2_HIP(hipMemsetAsync(done, 0, (size_t)B * sizeof(int32_t), st));
    }
    return topk_bmax(sc, B, ix->n, ix->n, k, ix->id_base, bm, out_scores, out_ids, st, ix->device, fold, done);
  }
  const size_t tk = topk_ws_bytes(B, ix->n);
  float* sc = (float*)(rest + tk);
  rc = score_impl(ix, scorer, Q, B, lq, sc, ix->n, st, ctr);
  if (rc) return rc;
  return topk_impl(sc, B, ix->n, ix->n, k, ix->id_base, rest, tk, out_scores, out_ids, st, ix->device);
}

int cbv2_index_set_option(cbv2_index* ix, int32_t option, int64_t value) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  switch (option) {
    case CBV2_OPT_FUSED_TOPK:
      ix->fused_topk = value != 0;
      ix->fused_topk_mode = (int)value;
      return CBV2_OK;
    case CBV2_OPT_DYNAMIC_TAIL:
      ix->dynamic_tail = (int)value;
      return CBV2_OK;
    case CBV2_OPT_BAND_DOC_MAJOR:
      ix->band_doc_major = (int)value;
      return CBV2_OK;
    case CBV2_OPT_BAND_LOWER_BOUND:
      ix->band_lower_bound = value != 0;
      return CBV2_OK;
    case CBV2_OPT_TOPK_BMAX:
      ix->topk_bmax = (int)value;
      return CBV2_OK;
    case CBV2_OPT_BAND_FUSED:
      ix->band_fused = value != 0;
      return CBV2_OK;
    case CBV2_OPT_RESCORE_SPLIT:
      ix->rescore_split = value != 0;
      return CBV2_OK;
    case CBV2_OPT_BAND_REUSE:
      ix->band_reuse = value != 0;
      return CBV2_OK;
    case CBV2_OPT_BAND_BLOCK_SKIP:
      ix->band_block_skip = value != 0;
      return CBV2_OK;
    case CBV2_OPT_DENSE_DOCS:
      ix->dense_docs = value != 0;
      return CBV2_OK;
    case CBV2_OPT_P1_COLLECT_FUSED:
      ix->p1_collect_fused = value != 0;
      return CBV2_OK;
    case CBV2_OPT_FOLD_KEYS:
      ix->fold_keys = value != 0;
      return CBV2_OK;
    case CBV2_OPT_RESCORE_GRID:
      if (value < 0 || value > 65535) return fail(CBV2_EINVAL, "rescore grid must be in [0, 65535]");
      ix->rescore_grid = (int)value;
      return CBV2_OK;
    default:
      return fail(CBV2_EINVAL, "unknown option %d", option);
  }
}

int64_t cbv2_search_fused_slots(const cbv2_index* ix, int32_t B, int32_t k, int32_t scorer) {
  if (!ix || B < 1 || k < 1) return 0;
  return fused_slots(ix, scorer, B, k);
}

int cbv2_index_last_scan_plan(const cbv2_index* ix, int64_t* out4) {
  CBV2_REQUIRE(ix != nullptr && out4 != nullptr, "null index or output");
  for (int i = 0; i < 4; ++i) out4[i] = ix->last_plan[i];
  return CBV2_OK;
}

int cbv2_index_kind(const cbv2_index* ix, int32_t* dtype, int32_t* faithful) {
  CBV2_REQUIRE(ix != nullptr && dtype != nullptr && faithful != nullptr, "null index or output");
  *dtype = ix->dtype;
  *faithful = ix->resid != nullptr ? 1 : 0;
  return CBV2_OK;
}

// Batches up to kRrSplitMaxB take the candidate-parallel raw kernel (+ the
// row select when k > 0, its raw row in the caller's workspace); larger ones
// one workgroup per query (the batch fills the chip by itself).
constexpr int kRrSplitMaxB = 32;

size_t cbv2_rerank_workspace_bytes(int32_t B, int32_t C) {
  if (B < 1 || C < 1) return 0;
  return ((size_t)B * (size_t)C * sizeof(float) + 255) & ~(size_t)255;
}

static int rerank_impl(cbv2_index* ix, const void* Q, int32_t B, int32_t lq, const int32_t* cand, int32_t C,
                       int32_t k, void* ws, size_t ws_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                       void* stream) {
  const int32_t qdt = ix && ix->dtype == CBV2_DTYPE_MXFP8 ? CBV2_DTYPE_MXFP8 : CBV2_DTYPE_BF16;
  int rc = check_query(ix, CBV2_SCORER_MAXSIM, Q, qdt, B, lq);
  if (rc) return rc;
  CBV2_REQUIRE(cand != nullptr, "null candidates");
  CBV2_REQUIRE(C >= 1 && C <= kRerankMaxC, "C must be in [1, %d] (got %d)", kRerankMaxC, C);
  CBV2_REQUIRE(k >= 0, "k must be >= 0 (got %d)", k);
  CBV2_REQUIRE(out_scores != nullptr, "null out_scores");
  CBV2_REQUIRE(k == 0 || out_ids != nullptr, "null out_ids");
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  const hipStream_t st = (hipStream_t)stream;
  const bool big = C > kSmallMax;                 // raw scores in dynamic LDS, multi-pass selection
  const unsigned dyn = big ? (unsigned)C * sizeof(float) : 0u;
  const bool f8 = ix->dtype == CBV2_DTYPE_MXFP8;
  const uint8_t* Qb = (const uint8_t*)Q;
  const uint8_t* Qs = f8 ? Qb + (size_t)B * lq * kDim : nullptr;
  const size_t raw_bytes = (size_t)B * (size_t)C * sizeof(float);
  if (B <= kRrSplitMaxB && (k == 0 || (!big && ws != nullptr && ws_bytes >= raw_bytes))) {
    float* raw = k == 0 ? out_scores : (float*)ws;
    const dim3 grid((unsigned)((C + kRrWaves - 1) / kRrWaves), (unsigned)B);
    TaggedCand tc;
    if (!f8 && ix->rescore_split) {   // one candidate per workgroup, its rows over the 4 waves
      tc = g_cand_tagged;             // the latency path's pre-armed rerank (cand unused then)
      if (tc.w != nullptr) g_cand_tagged_used = true;
      const Mirror rw = k == 0 ? g_raw_mirror : Mirror();
      if (rw.w != nullptr) g_raw_mirror_used = true;
      hipLaunchKernelGGL(rerank_split_kernel, dim3((unsigned)C, (unsigned)B), dim3(256), 0, st, ix->tokens,
                         ix->doclens, ix->n, ix->id_base, (const uint16_t*)Q, lq, cand, C, raw, (int)ix->ld, tc, rw);
      if ((rc = launch_check("rerank_split_kernel"))) return rc;
    } else if (f8)
      hipLaunchKernelGGL(rerank_raw_kernel<true>, grid, dim3(kRrWaves * 64), 0, st, ix->tokens, ix->scales,
                         ix->doclens, ix->n, ix->id_base, Qb, Qs, lq, cand, C, raw, (int)ix->ld);
    else
      hipLaunchKernelGGL(rerank_raw_kernel<false>, grid, dim3(kRrWaves * 64), 0, st, ix->tokens, nullptr,
                         ix->doclens, ix->n, ix->id_base, Qb, nullptr, lq, cand, C, raw, (int)ix->ld);
    if ((rc = launch_check("rerank_raw_kernel"))) return rc;
    if (k == 0) return CBV2_OK;
    const FinalMirror fin = g_final_mirror.k == k ? g_final_mirror : FinalMirror();
    if (fin.w != nullptr) g_final_mirror_used = true;
    hipLaunchKernelGGL(select_small_kernel, dim3((unsigned)B), dim3(256), 0, st, raw, cand, C, k, out_scores, out_ids,
                       out_pos, tc.w, fin);
    return launch_check("select_small_kernel");
  }
  if (f8) {
    if (big) {
      CBV2_HIP(hipFuncSetAttribute((const void*)rerank_f8_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   (int)dyn));
      hipLaunchKernelGGL(rerank_f8_kernel<true>, dim3((unsigned)B), dim3(kRrWaves * 64), dyn, st, ix->tokens,
                         ix->scales, ix->doclens, ix->n, ix->id_base, Qb, Qs, lq, cand, C, k, out_scores, out_ids,
                         out_pos, (int)ix->ld);
    } else {
      hipLaunchKernelGGL(rerank_f8_kernel<false>, dim3((unsigned)B), dim3(kRrWaves * 64), 0, st, ix->tokens,
                         ix->scales, ix->doclens, ix->n, ix->id_base, Qb, Qs, lq, cand, C, k, out_scores, out_ids,
                         out_pos, (int)ix->ld);
    }
    return launch_check("rerank_f8_kernel");
  }
  if (big) {
    CBV2_HIP(hipFuncSetAttribute((const void*)rerank_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)dyn));
    hipLaunchKernelGGL(rerank_kernel<true>, dim3((unsigned)B), dim3(kRrWaves * 64), dyn, st, ix->tokens, ix->doclens,
                       ix->n, ix->id_base, (const uint16_t*)Q, lq, cand, C, k, out_scores, out_ids, out_pos,
                       (int)ix->ld);
  } else {
    hipLaunchKernelGGL(rerank_kernel<false>, dim3((unsigned)B), dim3(kRrWaves * 64), 0, st, ix->tokens, ix->doclens,
                       ix->n, ix->id_base, (const uint16_t*)Q, lq, cand, C, k, out_scores, out_ids, out_pos,
                       (int)ix->ld);
  }
  return launch_check("rerank_kernel");
}

int cbv2_rerank(cbv2_index* ix, const void* Q, int32_t B, int32_t lq, const int32_t* cand, int32_t C, int32_t k,
                float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream) {
  return rerank_impl(ix, Q, B, lq, cand, C, k, nullptr, 0, out_scores, out_ids, out_pos, stream);
}

int cbv2_rerank_ws(cbv2_index* ix, const void* Q, int32_t B, int32_t lq, const int32_t* cand, int32_t C, int32_t k,
                   void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                   void* stream) {
  return rerank_impl(ix, Q, B, lq, cand, C, k, workspace, workspace_bytes, out_scores, out_ids, out_pos, stream);
}

int cbv2_select_topk(const float* scores, const int32_t* ids, int32_t B, int32_t C, int32_t k, float* out_scores,
                     int32_t* out_ids, int32_t* out_pos, void* stream) {
  CBV2_REQUIRE(scores && out_scores, "null scores/out_scores");
  CBV2_REQUIRE(B >= 1, "B must be >= 1");
  CBV2_REQUIRE(C >= 1, "C must be >= 1 (got %d)", C);
  CBV2_REQUIRE(k >= 1, "k must be >= 1 (got %d)", k);
  if (C > kSmallMax)  // long rows: the multi-pass selection (same tie rule)
    return topk_multi(scores, B, C, C, k, 0, ids, C, out_scores, out_ids, out_pos, (hipStream_t)stream);
  hipLaunchKernelGGL(select_small_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, scores, ids, C, k,
                     out_scores, out_ids, out_pos);
  return launch_check("select_small_kernel");
}

// Internal (sharded.cpp): the prescored select of the sharded stage 3
// (prescored_select_kernel; C <= kSmallMax, misses nullable).
int cbv2_prescored_select(const int32_t* recv, int32_t G, int64_t blk, int32_t B, int32_t k, int32_t kb,
                          const int32_t* cand, int32_t C, int32_t fk, float* out_s, int32_t* out_i, int32_t* out_p,
                          int32_t* misses, void* stream) {
  CBV2_REQUIRE(recv && cand && out_s && out_i, "null blocks / candidates / outputs");
  CBV2_REQUIRE(G >= 1 && B >= 1 && k >= 1 && kb >= 0 && fk >= 1, "bad sizes (G %d, B %d, k %d, kb %d, k %d)", G, B,
               k, kb, fk);
  CBV2_REQUIRE(C >= 1 && C <= kSmallMax, "prescored select: C must be in [1, %d] (got %d)", kSmallMax, C);
  hipLaunchKernelGGL(prescored_select_kernel, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, recv, G, blk, B,
                     k, kb, cand, C, fk, out_s, out_i, out_p, misses);
  return launch_check("prescored_select_kernel");
}

int cbv2_split_f32(const float* x, int64_t rows, int32_t ld, const int32_t* doclens, void* hi, void* lo,
                   float* bounds, void* stream) {
  CBV2_REQUIRE(rows >= 0, "rows must be >= 0");
  CBV2_REQUIRE(doclens == nullptr || (ld >= 1 && rows % ld == 0), "with doclens, rows must be docs of ld rows");
  if (rows == 0) return CBV2_OK;
  CBV2_REQUIRE(x && hi && lo && bounds, "null pointer");
  CBV2_REQUIRE(aligned16(x) && aligned16(hi) && aligned16(lo), "x, hi and lo must be 16-byte aligned");
  const int64_t want = (rows * 16 + 255) / 256;
  const unsigned grid = (unsigned)(want < 65536 ? want : 65536);  // grid-stride beyond
  hipLaunchKernelGGL(split_f32_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, x, rows, ld, doclens,
                     (uint16_t*)hi,
                     (uint16_t*)lo, bounds);
  return launch_check("split_f32_kernel");
}

int cbv2_index_attach_residual(cbv2_index* ix, const void* lo, float resid_max, float norm_max) {
  CBV2_REQUIRE(ix != nullptr, "null index");
  CBV2_REQUIRE(ix->dtype == CBV2_DTYPE_BF16, "a residual attaches to a bf16 index");
  CBV2_REQUIRE(ix->n == 0 || (lo != nullptr && aligned16(lo)), "residual must be non-null and 16-byte aligned");
  CBV2_REQUIRE(resid_max >= 0.0f && norm_max >= 0.0f && resid_max < 3.0e38f && norm_max < 3.0e38f,
               "bounds must be finite and >= 0");
  ix->resid = (const uint8_t*)lo;
  ix->resid_max = resid_max;
  ix->norm_max = norm_max;
  return CBV2_OK;
}

size_t cbv2_f32_workspace_bytes(const cbv2_index* ix, int32_t op, int32_t B, int32_t lq, int32_t cap) {
  if (!ix || B < 1 || lq < 1 || cap < 0 || op < CBV2_F32_SCORE || op > CBV2_F32_RERANK) return 0;
  F32Ws w;
  return f32_ws_layout(ix, op, B, lq, cap, nullptr, &w);
}

int cbv2_score_f32(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, void* ws, size_t wsb, float* out,
                   int64_t ld_out, void* stream) {
  F32Ws w;
  int rc = check_f32(ix, CBV2_F32_SCORE, Q, B, lq, 0, ws, wsb, &w);
  if (rc) return rc;
  CBV2_REQUIRE(ix->n == 0 || out != nullptr, "null output");
  CBV2_REQUIRE(ld_out >= ix->n, "ld_out (%lld) < n (%lld)", (long long)ld_out, (long long)ix->n);
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  hipStream_t st = (hipStream_t)stream;
  if (ix->n == 0) return CBV2_OK;
  rc = split_queries(ix, Q, B, lq, &w, st);
  if (rc) return rc;
  return launch_rescore(ix, &w, B, lq, nullptr, nullptr, ix->n, 0, out, ld_out, st);
}

namespace {
// Faithful search, phase 1: split the queries, bf16 scan of hi (T), its top-k
// (out), and -- with the two-pass band (want_lb) -- the exact lower bound of
// each row's k-th faithful score (the minimum faithful score of the bf16
// top-k, atomic-min'ed into w.lb as order-preserving bits by the rescoring
// itself); fk_out (nullable): those k faithful scores themselves, [B][k].
// Returns 1 when the whole search is already done (k beyond any band: the
// full faithful scan ran, status -1 everywhere).
// The two-pass band (lbu) reuses phase 1's faithful scores of the bf16 top-k
// as its first k slots instead of rescoring those docs again (they are always
// in the band): the split rescoring, not the fused latency launch, n >= k.
bool band_reuses_topk(const cbv2_index* ix, int32_t B, int32_t k) {
  return ix->band_reuse && ix->rescore_split && ix->n >= k && !(B <= kBandPairMaxB && ix->ld == kLd && ix->band_fused);
}
// The two-pass band's phase 1 and band collect in one launch
// (phase1_collect_kernel): small batches whose band reuses the bf16 top-k, on
// the block keys of the block-max select, pair by pair with the row select
// and the fallback in the rescoring launch.
bool phase1_collect_fused(const cbv2_index* ix, int32_t B, int32_t k) {
  return ix->p1_collect_fused && B <= kBandPairMaxB && k <= kTopkMax && band_reuses_topk(ix, B, k) &&
         bmax_eligible(ix, CBV2_SCORER_MAXSIM, B, k) && ix->band_block_skip && !ix->band_doc_major;
}

int search_f32_phase1(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap, F32Ws& w,
                      float* out_scores, int32_t* out_ids, int32_t* out_status, bool want_lb, hipStream_t st,
                      float* fk_out = nullptr) {
  int rc;
  if (ix->n == 0) {
    CBV2_HIP(hipMemsetAsync(out_status, 0, (size_t)B * sizeof(int32_t), st));
    if ((rc = topk_impl_empty(B, k, out_scores, out_ids, st))) return rc;
    return 1;
  }
  // the block-max select's keys: folded into the scan -- by the streaming
  // scans directly, by the dense 4 x 1 scan with atomic max into keys the
  // query split zeroes
  const bool bmax = k <= kBandCapMax && bmax_eligible(ix, CBV2_SCORER_MAXSIM, B, k);
  const bool fold0 = bmax && !scan_folds_bmax(ix, B) && scan_folds_bmax_zeroed(ix, B);
  if ((rc = split_queries(ix, Q, B, lq, &w, st, want_lb && band_reuses_topk(ix, B, k) ? k : 0, true,
                          fold0 ? (uint32_t*)w.tk : nullptr,
                          fold0 ? (int64_t)B * (bm_blocks(ix->n) + bm_supers(ix->n)) : 0)))
    return rc;
  if (k > kBandCapMax) {   // no band can hold k: every row takes the full faithful scan (status -1)
    CBV2_HIP(hipMemsetAsync(out_status, 0xff, (size_t)B * sizeof(int32_t), st));
    if ((rc = launch_rescore(ix, &w, B, lq, nullptr, nullptr, ix->n, 0, w.T, ix->n, st))) return rc;
    if ((rc = topk_multi(w.T, B, ix->n, ix->n, k, ix->id_base, nullptr, 0, out_scores, out_ids, nullptr, st)))
      return rc;
    return 1;
  }
  // 1. bf16 scan of hi, top-k of T (its k-th score anchors the band)
  const bool fold = bmax && (scan_folds_bmax(ix, B) || fold0);
  {
    CtrPolicy cp(kCtrPrezeroed);   // the split zeroed the scan's counters
    if ((rc = scan_maxsim_timed(ix, w.qhi, B, lq, w.T, ix->n, st, w.ctr, nullptr, fold ? (uint32_t*)w.tk : nullptr)))
      return rc;
  }
  const Mirror mirror = g_ids_mirror;   // the bf16 top-k is not the search's answer: no host mirror here
  g_ids_mirror = Mirror();
  rc = bmax ? topk_bmax(w.T, B, ix->n, ix->n, k, ix->id_base, (uint32_t*)w.tk, out_scores, out_ids, st, ix->device,
                        fold, arrive_row0(w, kArrBmax, B), kArriveInts)
            : topk_impl(w.T, B, ix->n, ix->n, k, ix->id_base, w.tk, w.tk_bytes, out_scores, out_ids, st, ix->device);
  g_ids_mirror = mirror;
  if (rc) return rc;
  if ((rc = band_mark(ix, false, st))) return rc;
  if (fk_out != nullptr)     // the bf16 top-k's own faithful scores, for the caller's cross-shard bound
    return launch_rescore(ix, &w, B, lq, out_ids, nullptr, k, k, fk_out, k, st);
  if (want_lb && phase1_collect_fused(ix, B, k))   // in phase 2's first launch (phase1_collect_kernel)
    return CBV2_OK;
  if (want_lb) {   // the bf16 top-k's own faithful scores: k docs score at least their minimum
    RowSelect lab;
    lab.stamps = LAB_STAMPS(1);
    return launch_rescore(ix, &w, B, lq, out_ids, nullptr, k, k, w.F, cap, st, nullptr, 0,
                          reinterpret_cast<uint32_t*>(w.lb), 0, nullptr, nullptr, 0, nullptr, nullptr, lab);
  }
  return CBV2_OK;
}

// Phase 2: the band (every doc with T >= lb - beta; lb == nullptr: T_k - 2
// beta, the one-pass band), its faithful rescoring, the exact top-k of the
// band, and the full faithful scan for rows whose band overflowed cap.
int search_f32_phase2_impl(cbv2_index* ix, int32_t B, int32_t lq, int32_t k, int32_t cap, F32Ws& w,
                           const float* lb, const uint32_t* lbu, float* out_scores, int32_t* out_ids,
                           int32_t* out_status, hipStream_t st) {
  int rc;
  // (count[b] was reset by the query split of phase 1: to k with the reuse)
  const bool reuse = lbu != nullptr && band_reuses_topk(ix, B, k);
  const int c0 = reuse ? k : 0;
  // the band goes pair by pair (not fused with the collect, not doc-major):
  // its rescoring launch also runs the overflow fallback (no separate launch)
  const bool pair_path = !(B <= kBandPairMaxB && ix->ld == kLd && ix->band_fused) &&
                         !(ix->band_doc_major && B > kBandPairMaxB);
  const bool fb_fused = pair_path && ix->rescore_split && k <= kTopkMax;
  int64_t splits = (8LL * cu_count(ix->device) + B - 1) / B;    // ~8 workgroups per CU
  const int64_t max_splits = (ix->n + 8191) / 8192;
  splits = splits < max_splits ? splits : max_splits;
  splits = splits < 1 ? 1 : splits;
  if (lbu != nullptr && phase1_collect_fused(ix, B, k)) {
    // phase 1 + the collect in one launch (phase 1 was left out of phase1)
    const int64_t groups = (bm_blocks(ix->n) + 63) / 64;
    hipLaunchKernelGGL(phase1_collect_kernel, dim3((unsigned)(k + groups), (unsigned)B), dim3(256), 0, st,
                       ix->tokens, ix->resid, ix->doclens, ix->n, ix->id_base, w.qhi, w.qlo, lq, out_ids, out_scores,
                       k, w.F, (int64_t)cap, const_cast<uint32_t*>(lbu), arrive_row0(w, kArrPhase1, B),
                       (int64_t)kArriveInts, w.T, w.beta, reinterpret_cast<const uint32_t*>(w.tk), cap, w.cand,
                       w.count, g_wait_ticks, LAB_STAMPS(1));
    if ((rc = launch_check("phase1_collect_kernel"))) return rc;
  } else if (B <= kBandPairMaxB && ix->ld == kLd && ix->band_fused) {
    // the latency path: collect + rescore in one launch, one band doc per wave
    const int64_t gx = (ix->n + kBcrDocs - 1) / kBcrDocs;
    hipLaunchKernelGGL(band_collect_rescore_kernel, dim3((unsigned)gx, (unsigned)B), dim3(256), 0, st, w.T, ix->n,
                       out_scores, k, w.beta, lb, lbu, ix->tokens, ix->resid, ix->doclens, ix->id_base, w.qhi, w.qlo,
                       lq, cap, w.cand, w.F, w.count);
    if ((rc = launch_check("band_collect_rescore_kernel"))) return rc;
  } else {
    // phase 1's block-max select left the rows' 64-doc block keys in w.tk
    const bool bkeys = bmax_eligible(ix, CBV2_SCORER_MAXSIM, B, k) && ix->band_block_skip;
    if (bkeys) {   // 64 block keys per workgroup, as many workgroups as that takes up to ~8 per CU
      const int64_t per_row = (8LL * cu_count(ix->device) + B - 1) / B;
      const int64_t groups = (bm_blocks(ix->n) + 63) / 64;
      splits = std::max<int64_t>(1, std::min(per_row, groups));
    }
    hipLaunchKernelGGL(band_collect_kernel, dim3((unsigned)splits, (unsigned)B), dim3(256), 0, st, w.T, ix->n,
                       out_scores, k, w.beta, ix->id_base, cap, w.cand, w.count, lb, lbu,
                       reuse ? out_ids : nullptr, bkeys ? reinterpret_cast<const uint32_t*>(w.tk) : nullptr,
                       LAB_STAMPS(2));
    if ((rc = launch_check("band_collect_kernel"))) return rc;
  }
  // pairs grouped by doc (each band doc's tiles read once per batch) pay when
  // the queries' bands overlap; a batch of at most kBandPairMaxB queries
  // rescores pair by pair, one band doc per wave, without the doc-major
  // passes over all n docs (count memset, offsets)
  if (B <= kBandPairMaxB && ix->ld == kLd && ix->band_fused) {
    // rescored above
  } else if (ix->band_doc_major && B > kBandPairMaxB) {
    CBV2_HIP(hipMemsetAsync(w.dcnt, 0, (size_t)ix->n * sizeof(int32_t), st));
    CBV2_HIP(hipMemsetAsync(w.dctr, 0, 2 * sizeof(int32_t), st));
    const unsigned gc = (unsigned)std::min<int64_t>((cap + 255) / 256, 16);
    hipLaunchKernelGGL(band_count_kernel, dim3(gc, (unsigned)B), dim3(256), 0, st, w.cand, w.count, cap, ix->id_base,
                       ix->n, w.dcnt, c0);
    if ((rc = launch_check("band_count_kernel"))) return rc;
    const unsigned go = (unsigned)std::min<int64_t>((ix->n + 255) / 256, 1024);
    hipLaunchKernelGGL(band_offsets_kernel, dim3(go), dim3(256), 0, st, w.dcnt, ix->n, w.doff, w.act, w.act_off,
                       w.act_cnt, w.dctr);
    if ((rc = launch_check("band_offsets_kernel"))) return rc;
    hipLaunchKernelGGL(band_scatter_kernel, dim3(gc, (unsigned)B), dim3(256), 0, st, w.cand, w.count, cap,
                       ix->id_base, ix->n, w.dcnt, w.doff, w.pair_b, w.pair_c, c0);
    if ((rc = launch_check("band_scatter_kernel"))) return rc;
    if ((ix->band_doc_major == 3 || ix->band_doc_major == 4) && ix->ld == kLd) {   // the doc split over the workgroup
      const bool two = ix->band_doc_major == 4;
      // resident workgroups per CU (2 waves per SIMD), x4; grid-stride beyond
      const unsigned gs = (unsigned)((two ? 4 : 3) * cu_count(ix->device) * 4);
      hipLaunchKernelGGL(two ? rescore_docs_split_kernel<2> : rescore_docs_split_kernel<4>, dim3(gs),
                         dim3(two ? 128 : 256), 0, st, ix->tokens, ix->resid, ix->doclens, w.qhi, w.qlo, B, lq, w.act,
                         w.act_off, w.act_cnt, w.dctr, w.pair_b, w.pair_c, w.F, cap);
      if ((rc = launch_check("rescore_docs_split_kernel"))) return rc;
    } else {
      const unsigned gr = (unsigned)(2 * cu_count(ix->device) * 4);   // 4 waves each; grid-stride over docs
      auto kern = ix->band_doc_major == 2 ? (ix->ld != kLd ? rescore_docs_kernel<true, true> : rescore_docs_kernel<true>)
                                          : (ix->ld != kLd ? rescore_docs_kernel<false, true> : rescore_docs_kernel<false>);
      hipLaunchKernelGGL(kern, dim3(gr), dim3(256), 0, st, ix->tokens, ix->resid, ix->doclens, w.qhi, w.qlo, B, lq,
                         w.act, w.act_off, w.act_cnt, w.dctr, w.pair_b, w.pair_c, w.F, cap, (int)ix->ld);
      if ((rc = launch_check("rescore_docs_kernel"))) return rc;
    }
  } else {
    // small batches (the latency path): the band select runs in the rescoring
    // launch's last workgroup per row (select_band_row), no select launch
    RowSelect rs;
    if (fb_fused && B <= kBandPairMaxB) {
      rs.mode = kSelBand;
      rs.arrive = arrive_row0(w, kArrBand, B);
      rs.k = k;
      rs.out_s = out_scores;
      rs.out_i = out_ids;
      rs.lb = lb;
      rs.lbu = lbu;
      rs.status = out_status;
      rs.ids_mirror = g_ids_mirror;
      if (g_ids_mirror.w != nullptr) g_ids_mirror_used = true;   // selected or fallen back, every row writes it
      rs.stamps = LAB_STAMPS(3);
    }
    if ((rc = launch_rescore(ix, &w, B, lq, w.cand, w.count, cap, cap, w.F, cap, st, nullptr,
                             B <= kBandPairMaxB ? 1 : 0, nullptr, c0, fb_fused ? w.T : nullptr,
                             fb_fused ? w.done : nullptr, k, out_scores, out_ids, rs)))
      return rc;
    if (rs.mode != kSelNone) return CBV2_OK;   // selected (and the fallback run) in that launch
  }
  hipLaunchKernelGGL(band_select_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, w.F, w.cand, w.count, cap, k,
                     ix->id_base, out_scores, out_ids, out_status, lb, lbu);
  if ((rc = launch_check("band_select_kernel"))) return rc;
  // rows whose band overflowed cap (status -1): the full faithful scan over
  // every doc and an exact top-k, on the device (other rows exit at once);
  // pair-by-pair bands did it inside their rescoring launch already
  if (fb_fused) return CBV2_OK;
  if (ix->rescore_split && k <= kTopkMax) {   // scan + top-k in one launch (last workgroup per row)
    // (a grid of this size is dispatched whether or not a row overflowed: it
    // stays small -- an overflowing row then takes a few ms)
    const int64_t fb = std::max<int64_t>(64, 256 / B);
    const unsigned gx = (unsigned)(ix->n < fb ? ix->n : fb);
    hipLaunchKernelGGL(ix->ld != kLd ? fallback_split_kernel<true> : fallback_split_kernel<false>, dim3(gx, (unsigned)B),
                       dim3(256), 0, st, ix->tokens, ix->resid, ix->doclens, ix->n, ix->id_base, w.qhi, w.qlo, lq,
                       w.T, out_status, (int)ix->ld, w.done, k, out_scores, out_ids);
    return launch_check("fallback_split_kernel");
  }
  if ((rc = launch_rescore(ix, &w, B, lq, nullptr, nullptr, ix->n, 0, w.T, ix->n, st, out_status))) return rc;
  if (k > kTopkMax)
    return topk_multi(w.T, B, ix->n, ix->n, k, ix->id_base, nullptr, 0, out_scores, out_ids, nullptr, st, out_status);
  hipLaunchKernelGGL(topk_rows_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, st, w.T, ix->n, ix->n, k, ix->id_base,
                     out_scores, out_ids, out_status);
  return launch_check("topk_rows_kernel");
}

int search_f32_phase2(cbv2_index* ix, int32_t B, int32_t lq, int32_t k, int32_t cap, F32Ws& w, const float* lb,
                      const uint32_t* lbu, float* out_scores, int32_t* out_ids, int32_t* out_status,
                      hipStream_t st) {
  const int rc = search_f32_phase2_impl(ix, B, lq, k, cap, w, lb, lbu, out_scores, out_ids, out_status, st);
  if (rc) return rc;
  return band_mark(ix, true, st);
}

// The faithful rerank after its query split: rescoring of the C candidates
// (raw scores), then the top-k select (k == 0: the raw scores themselves).
// arrive (nullable): the rerank slot's zeroed arrival counters -- the select
// then runs in the rescoring launch's last workgroup per row (C <= kSmallMax).
int rerank_f32_split(cbv2_index* ix, F32Ws& w, int32_t B, int32_t lq, const int32_t* cand, int32_t C, int32_t k,
                     float* out_scores, int32_t* out_ids, int32_t* out_pos, hipStream_t st,
                     int32_t* arrive = nullptr) {
  int rc;
  float* raw = k == 0 ? out_scores : w.F;
  if (k > 0 && C <= kSmallMax && arrive != nullptr && ix->rescore_split) {
    RowSelect rs;
    rs.mode = kSelCand;
    rs.arrive = arrive;
    rs.k = k;
    rs.out_s = out_scores;
    rs.out_i = out_ids;
    rs.out_p = out_pos;
    const TaggedCand tc = g_cand_tagged;   // the latency path's pre-armed rerank (cand unused then)
    if (tc.w != nullptr) g_cand_tagged_used = true;
    if (g_final_mirror.w != nullptr && g_final_mirror.k == k) {
      rs.fin = g_final_mirror;
      g_final_mirror_used = true;
    }
    rs.stamps = LAB_STAMPS(4);
    return launch_rescore(ix, &w, B, lq, cand, nullptr, C, C, raw, C, st, nullptr, 0, nullptr, 0, nullptr, nullptr, 0,
                          nullptr, nullptr, rs, tc);
  }
  RowSelect rw;
  if (k == 0 && g_raw_mirror.w != nullptr) {   // the raw scores also as host words
    rw.raw = g_raw_mirror;
    g_raw_mirror_used = true;
  }

  if ((rc = launch_rescore(ix, &w, B, lq, cand, nullptr, C, C, raw, C, st, nullptr, 0, nullptr, 0, nullptr, nullptr, 0,
                           nullptr, nullptr, rw)))
    return rc;
  if (k == 0) return CBV2_OK;
  if (C > kSmallMax) return topk_multi(raw, B, C, C, k, 0, cand, C, out_scores, out_ids, out_pos, st);
  const FinalMirror fin = g_final_mirror.k == k ? g_final_mirror : FinalMirror();
  if (fin.w != nullptr) g_final_mirror_used = true;
  hipLaunchKernelGGL(select_small_kernel, dim3((unsigned)B), dim3(256), 0, st, raw, cand, C, k, out_scores, out_ids,
                     out_pos, nullptr, fin);
  return launch_check("select_small_kernel");
}

int check_search_f32(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap, void* ws,
                     size_t wsb, F32Ws* w) {
  CBV2_REQUIRE(k >= 1, "k must be >= 1 (got %d)", k);
  CBV2_REQUIRE(k > kBandCapMax || (cap >= k && cap <= kBandCapMax), "cap must be in [k, %d] (got %d)", kBandCapMax,
               cap);
  return check_f32(ix, CBV2_F32_SEARCH, Q, B, lq, cap, ws, wsb, w);
}
}  // namespace

int cbv2_search_f32(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap, void* ws,
                    size_t wsb, float* out_scores, int32_t* out_ids, int32_t* out_status, void* stream) {
  F32Ws w;
  int rc = check_search_f32(ix, Q, B, lq, k, cap, ws, wsb, &w);
  if (rc) return rc;
  CBV2_REQUIRE(out_scores && out_ids && out_status, "null outputs");
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  hipStream_t st = (hipStream_t)stream;
  // 2. the band: every doc with T >= lb - beta, lb = an exact lower bound of
  //    the k-th faithful score (the bf16 top-k's own faithful scores: the
  //    minimum of k of them), or T_k - 2 beta without that pass (A/B);
  // 3. faithful rescoring of the band, 4. exact top-k of the band
  const bool two_pass = ix->band_lower_bound;
  rc = search_f32_phase1(ix, Q, B, lq, k, cap, w, out_scores, out_ids, out_status, two_pass, st);
  if (rc) return rc < 0 ? rc : CBV2_OK;
  return search_f32_phase2(ix, B, lq, k, cap, w, nullptr, two_pass ? reinterpret_cast<const uint32_t*>(w.lb) : nullptr,
                           out_scores, out_ids, out_status, st);
}

int cbv2_search_f32_begin(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap, void* ws,
                          size_t wsb, float* fk, float* out_scores, int32_t* out_ids, int32_t* out_status,
                          void* stream) {
  F32Ws w;
  int rc = check_search_f32(ix, Q, B, lq, k, cap, ws, wsb, &w);
  if (rc) return rc;
  CBV2_REQUIRE(fk && out_scores && out_ids && out_status, "null outputs");
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  hipStream_t st = (hipStream_t)stream;
  // fk = -inf unless phase 1 writes it (an empty shard, k beyond any band)
  hipLaunchKernelGGL(fill_neg_inf_kernel, dim3((unsigned)(((int64_t)B * k + 255) / 256)), dim3(256), 0, st, fk,
                     (int64_t)B * k);
  if ((rc = launch_check("fill_neg_inf_kernel"))) return rc;
  rc = search_f32_phase1(ix, Q, B, lq, k, cap, w, out_scores, out_ids, out_status, false, st, fk);
  return rc < 0 ? rc : CBV2_OK;
}

int cbv2_search_f32_finish(cbv2_index* ix, int32_t B, int32_t lq, int32_t k, int32_t cap, void* ws, size_t wsb,
                           const float* lb, float* out_scores, int32_t* out_ids, int32_t* out_status, void* stream) {
  F32Ws w;
  CBV2_REQUIRE(ix != nullptr, "null index");
  if (ix->resid == nullptr) return fail(CBV2_ESTATE, "index has no fp32 residual (cbv2_index_attach_residual)");
  CBV2_REQUIRE(B >= 1 && B <= 65535 && lq >= 1 && lq <= kLqMax, "bad B / lq");
  CBV2_REQUIRE(k >= 1, "k must be >= 1 (got %d)", k);
  CBV2_REQUIRE(k > kBandCapMax || (cap >= k && cap <= kBandCapMax), "cap must be in [k, %d] (got %d)", kBandCapMax,
               cap);
  const size_t need = f32_ws_layout(ix, CBV2_F32_SEARCH, B, lq, cap, nullptr, &w);
  CBV2_REQUIRE(ws != nullptr && wsb >= need && aligned16(ws), "workspace too small or misaligned");
  f32_ws_layout(ix, CBV2_F32_SEARCH, B, lq, cap, (uint8_t*)ws, &w);
  CBV2_REQUIRE(lb && out_scores && out_ids && out_status, "null inputs/outputs");
  if (ix->n == 0 || k > kBandCapMax) return CBV2_OK;   // phase 1 already finished these
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  return search_f32_phase2(ix, B, lq, k, cap, w, lb, nullptr, out_scores, out_ids, out_status, (hipStream_t)stream);
}

int cbv2_rerank_f32(cbv2_index* ix, const float* Q, int32_t B, int32_t lq, const int32_t* cand, int32_t C,
                    int32_t k, void* ws, size_t wsb, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                    void* stream) {
  CBV2_REQUIRE(cand != nullptr, "null candidates");
  CBV2_REQUIRE(C >= 1, "C must be >= 1 (got %d)", C);
  CBV2_REQUIRE(k >= 0, "k must be >= 0 (got %d)", k);
  CBV2_REQUIRE(out_scores != nullptr, "null out_scores");
  CBV2_REQUIRE(k == 0 || out_ids != nullptr, "null out_ids");
  F32Ws w;
  int rc = check_f32(ix, CBV2_F32_RERANK, Q, B, lq, C, ws, wsb, &w);
  if (rc) return rc;
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  hipStream_t st = (hipStream_t)stream;
  if ((rc = split_queries(ix, Q, B, lq, &w, st))) return rc;
  return rerank_f32_split(ix, w, B, lq, cand, C, k, out_scores, out_ids, out_pos, st, arrive_row0(w, kArrRerank, B));
}

// Internal (retrieve.cpp): cbv2_rerank_f32 for the queries a cbv2_search_f32
// with the same (B, lq) and band capacity `cap` split into `search_ws` before
// on the same stream: while that split is still the last one enqueued into
// the workspace (split_holds: same index, Q, B, lq), the rerank reads it (qhi
// / qlo) instead of launching the query split again; otherwise it splits Q
// into its own workspace, as cbv2_rerank_f32 does.  Same arithmetic, same
// results either way.
int cbv2_rerank_f32_after_search(cbv2_index* ix, const void* search_ws, size_t search_wsb, int32_t cap, int32_t B,
                                 int32_t lq, const int32_t* cand, int32_t C, int32_t k, void* ws, size_t wsb,
                                 float* out_scores, int32_t* out_ids, int32_t* out_pos, const float* Q, void* stream) {
  CBV2_REQUIRE(cand != nullptr && C >= 1 && k >= 0 && out_scores != nullptr && (k == 0 || out_ids != nullptr),
               "bad candidates / outputs");
  CBV2_REQUIRE(ix != nullptr && ix->resid != nullptr, "not an fp32-faithful index");
  CBV2_REQUIRE(B >= 1 && B <= 65535 && lq >= 1 && lq <= kLqMax, "bad B / lq");
  F32Ws sw, w;
  const size_t sneed = f32_ws_layout(ix, CBV2_F32_SEARCH, B, lq, cap, nullptr, &sw);
  CBV2_REQUIRE(search_ws != nullptr && search_wsb >= sneed && aligned16(search_ws), "search workspace too small");
  f32_ws_layout(ix, CBV2_F32_SEARCH, B, lq, cap, (uint8_t*)search_ws, &sw);
  const size_t need = f32_ws_layout(ix, CBV2_F32_RERANK, B, lq, C, nullptr, &w);
  CBV2_REQUIRE(ws != nullptr && wsb >= need && aligned16(ws), "workspace too small or misaligned (%zu < %zu)", wsb,
               need);
  f32_ws_layout(ix, CBV2_F32_RERANK, B, lq, C, (uint8_t*)ws, &w);
  DeviceGuard dg(ix->device);
  if (!dg.ok) return fail(CBV2_EHIP, "cannot select device %d", ix->device);
  const hipStream_t st = (hipStream_t)stream;
  int32_t* arrive;   // zeroed by the split the rerank reads
  if (split_holds(ix, Q, B, lq, sw.qhi)) {
    w.qhi = sw.qhi;
    w.qlo = sw.qlo;
    arrive = arrive_row0(sw, kArrRerank, B);
  } else if (g_prescore_ready_seq != 0) {
    return fail(CBV2_ESTATE, "stage-1 prescore: the search's query split is not in the workspace");
  } else {
    CBV2_REQUIRE(Q != nullptr, "null queries");
    int rc = split_queries(ix, Q, B, lq, &w, st);
    if (rc) return rc;
    arrive = arrive_row0(w, kArrRerank, B);
  }
  return rerank_f32_split(ix, w, B, lq, cand, C, k, out_scores, out_ids, out_pos, st, arrive);
}

// Internal (retrieve.cpp): the host mirror of the next search's final ids on
// this thread (nullptr: none); cbv2_ids_mirror_used: whether the search just
// issued writes it (then it holds every row's ids once the stream gets there).
void cbv2_set_ids_mirror(void* p, uint32_t seq, int64_t score_off) {
  g_ids_mirror = Mirror{(uint64_t*)p, seq, p != nullptr ? score_off : 0};
  g_ids_mirror_used = false;
}
int cbv2_ids_mirror_used(void) { return g_ids_mirror_used ? 1 : 0; }
void cbv2_set_cand_tagged(const void* p, uint32_t seq, void* gate) {
  g_cand_tagged = TaggedCand{(const uint64_t*)p, seq, (uint64_t*)gate, g_wait_ticks};
  g_cand_tagged_used = false;
}
// Lab knob (retrieve.cpp's cbv2_set_wait_lab, this thread): the bound of the
// in-kernel waits on host words and on phase 1 (s_memrealtime ticks; < 0:
// the default 1 s, 0: give up at once).
void cbv2_set_wait_ticks(int64_t ticks) { g_wait_ticks = ticks < 0 ? kCandWaitTicks : (uint64_t)ticks; }
int cbv2_cand_tagged_used(void) { return g_cand_tagged_used ? 1 : 0; }
void cbv2_set_final_mirror(void* p, uint32_t seq, int32_t k) {
  g_final_mirror = p != nullptr ? FinalMirror{(uint64_t*)p, seq, (int)k} : FinalMirror();
  g_final_mirror_used = false;
}
int cbv2_final_mirror_used(void) { return g_final_mirror_used ? 1 : 0; }
int cbv2_host_result_copy(const void* words, uint32_t seq, int32_t B, int32_t k, float* out_s, int32_t* out_i,
                          int32_t* out_p, void* gate, void* stream) {
  hipLaunchKernelGGL(host_result_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, (const uint64_t*)words, seq, B, k,
                     out_s, out_i, out_p, (uint64_t*)gate, g_wait_ticks);
  return launch_check("host_result_kernel");
}
void cbv2_set_split_ready(uint32_t seq) {
  g_split_ready_seq = seq;
  if (seq == 0) g_split_ready_word = nullptr;
}
// around the stage-1 prescore (its queries' split must still be the search's)
void cbv2_set_prescore_ready(uint32_t seq) { g_prescore_ready_seq = seq; }
// before a search: publish seq to words (device pointer into the call's
// mapped buffer: the faithful split one per row, a bf16 search word 0),
// record where (cbv2_last_ready_flag)
void cbv2_set_split_ready_begin(uint32_t seq, void* word) {
  g_split_ready_seq = seq;
  g_split_ready_word = (int32_t*)word;
  g_ready_flag = nullptr;
  g_ready_flag_ld = 0;
}
const void* cbv2_last_ready_flag(int64_t* ld) {
  if (ld != nullptr) *ld = g_ready_flag_ld;
  return g_ready_flag;
}
void cbv2_set_raw_mirror(void* p, uint32_t seq) {
  g_raw_mirror = Mirror{(uint64_t*)p, seq, 0};
  g_raw_mirror_used = false;
}
int cbv2_raw_mirror_used(void) { return g_raw_mirror_used ? 1 : 0; }
#ifdef CBV2_LAB_STAMPS
void cbv2_lab_set_stamps(void* p) { g_lab_stamps = (uint64_t*)p; }
#endif

// Internal (retrieve.cpp): the device an index lives on (-1: null index).
int cbv2_index_device(const cbv2_index* ix) { return ix ? ix->device : -1; }

size_t cbv2_topk_workspace_bytes(int32_t B, int64_t n) { return B >= 1 && n >= 1 ? topk_ws_bytes(B, n) : 0; }

int cbv2_topk_rows(const float* scores, int32_t B, int64_t n, int64_t ld, int32_t k, int64_t id_base,
                   void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids, void* stream) {
  CBV2_REQUIRE(scores && out_scores && out_ids, "null pointer");
  CBV2_REQUIRE(B >= 1, "B must be >= 1");
  CBV2_REQUIRE(n >= 1 && n <= 0x7fffffffLL, "n out of range");
  CBV2_REQUIRE(ld >= n, "ld < n");
  CBV2_REQUIRE(k >= 1, "k must be >= 1 (got %d)", k);
  CBV2_REQUIRE(id_base >= 0 && id_base + n <= 0x7fffffffLL, "ids must fit int32");
  int dev = 0;
  CBV2_HIP(hipGetDevice(&dev));
  return topk_impl(scores, B, n, ld, k, id_base, workspace, workspace_bytes, out_scores, out_ids,
                   (hipStream_t)stream, dev);
}

int cbv2_merge_topk_strided(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B, int32_t k,
                            size_t g_stride, float* out_scores, int32_t* out_ids, void* stream);

int cbv2_merge_topk(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B, int32_t k,
                    float* out_scores, int32_t* out_ids, void* stream) {
  return cbv2_merge_topk_strided(in_scores, in_ids, G, B, k, (size_t)B * k, out_scores, out_ids, stream);
}

// Internal (sharded.cpp): lb[b] = the k-th largest of the G lists of row b
// (union_kth_kernel), shard g's lists at g * g_stride.
int cbv2_union_kth(const float* fk, int32_t G, int32_t B, int32_t k, size_t g_stride, float* lb, void* stream) {
  CBV2_REQUIRE(fk && lb, "null pointer");
  CBV2_REQUIRE(G >= 1 && G <= 64 && B >= 1 && k >= 1, "bad sizes (G %d, B %d, k %d)", G, B, k);
  CBV2_REQUIRE((int64_t)G * k <= 0x7fffffffLL && g_stride >= (size_t)B * k, "bad list layout");
  hipLaunchKernelGGL(union_kth_kernel, dim3((unsigned)B), dim3(kTkThreads), 0, (hipStream_t)stream, fk, G, k, g_stride,
                     lb);
  return launch_check("union_kth_kernel");
}

// Internal (sharded.cpp): the same merge with shard g's lists at g * g_stride.
int cbv2_merge_topk_strided(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B, int32_t k,
                            size_t g_stride, float* out_scores, int32_t* out_ids, void* stream) {
  CBV2_REQUIRE(in_scores && in_ids && out_scores && out_ids, "null pointer");
  CBV2_REQUIRE(G >= 1 && G <= 64, "G must be in [1, 64]");
  CBV2_REQUIRE(B >= 1, "B must be >= 1");
  CBV2_REQUIRE(k >= 1, "k must be >= 1");
  if ((int64_t)G * k <= kMergeMax)
    hipLaunchKernelGGL(merge_topk_kernel<true>, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, in_scores,
                       in_ids, G, B, k, g_stride, out_scores, out_ids);
  else
    hipLaunchKernelGGL(merge_topk_kernel<false>, dim3((unsigned)B), dim3(256), 0, (hipStream_t)stream, in_scores,
                       in_ids, G, B, k, g_stride, out_scores, out_ids);
  return launch_check("merge_topk_kernel");
}

}  // extern "C"

// Test-only (sharded.cpp's loopback communicator): out[i] = max over g of srcs[g][i].
struct LoopbackSrcs {
  const float* p[64];
};
__global__ void __launch_bounds__(256) loopback_max_kernel(LoopbackSrcs s, int32_t G, int64_t n, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float m = s.p[0][i];
    for (int32_t g = 1; g < G; ++g) m = fmaxf(m, s.p[g][i]);
    out[i] = m;
  }
}

extern "C" int cbv2_loopback_max(const float* const* srcs, int32_t G, int64_t n, float* out, void* stream) {
  CBV2_REQUIRE(srcs && out, "null pointer");
  CBV2_REQUIRE(G >= 1 && G <= 64, "G must be in [1, 64]");
  CBV2_REQUIRE(n >= 1, "n must be >= 1");
  LoopbackSrcs s{};
  for (int32_t g = 0; g < G; ++g) {
    CBV2_REQUIRE(srcs[g], "null source %d", g);
    s.p[g] = srcs[g];
  }
  const unsigned grid = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(loopback_max_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, s, G, n, out);
  return launch_check("loopback_max_kernel");
}
