// Scan-kernel A/B lab (development tool, not part of the product ABI).
// Includes the product source so every variant is the exact production code,
// and exports one entry point that launches a chosen scan variant.
// Variants >= 100 are experimental copies of maxsim_scan16_kernel<8,4>:
//   100: same code path (sanity)        101: epilogue reduced to one add (INVALID scores: timing only)
//   102: one max per MFMA chain (INVALID) 103: waves 4-7 defer each doc's epilogue to mid-next-doc
//   104: full docs as a software-pipelined chain stream (doc16_pipe) with sched_barriers;  105: same, no barriers
//   106: doc16_pipe with sched_group_barrier (MFMA x2, VALU x3, MFMA x2) per chain
//   107 / 108: 2 / 4 independent chains interleaved by k-step (tile16_il)
//   111 / 112 / 113: doc16_deep, chain k's max after chains k+1..k+D (D = 1 / 2 / 3)
// The doc-interleaved kernel these experiments led to is in the product
// (maxsim_scan16x4_kernel, variants 11/12); its lab history: pipeline depth
// D=1/2/3 70.8/74.2/74.1 %, 3-deep LDS ring +0.4 %, without doc streaming 76.0 %.
//   109: no doc streaming and no barrier (doc 0's LDS image reused; INVALID)  110: same with the per-doc barrier
#define CBV2_LAB 1
#include "../hybrid-rag-colbertv2_amd/csrc/colbert_mi355x.hip"

namespace {

template <int QW>
__device__ __forceinline__ void tile16_cheap(const bf16x8 (&a)[4], const bf16x8 (&qf)[QW][2][4], float (&m)[QW][2]) {
#pragma unroll
  for (int q = 0; q < QW; ++q) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      f32x4 acc = f32x4{};
#pragma unroll
      for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], qf[q][ct][s], acc, 0, 0, 0);
      m[q][ct] = fmaxf(m[q][ct], acc[0] + acc[3]);
    }
  }
}

// Row tile with NI independent MFMA chains interleaved by k-step (chains of
// the same tile share the A fragment), so one wave keeps several MFMAs in
// flight instead of waiting on each chain's dependent accumulation.
template <int QW, int NI>
__device__ __forceinline__ void tile16_il(const bf16x8 (&a)[4], const bf16x8 (&qf)[QW][2][4], float (&m)[QW][2]) {
  constexpr int NC = 2 * QW;
#pragma unroll
  for (int c0 = 0; c0 < NC; c0 += NI) {
    f32x4 acc[NI];
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[j] = f32x4{};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int c = c0 + j;
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[s], qf[c >> 1][c & 1][s], acc[j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NI; ++j) {
      const int c = c0 + j;
      float& mm = m[c >> 1][c & 1];
      mm = __builtin_fmaxf(__builtin_fmaxf(mm, __builtin_fmaxf(acc[j][0], acc[j][1])),
                           __builtin_fmaxf(acc[j][2], acc[j][3]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Deeper pipeline: chain k's max runs after chains k+1 .. k+D have issued
// (D+1 accumulators), so the MFMA->VALU read hazard is covered by MFMAs
// instead of s_nop; the max is two v_max3 (exact, any association).
template <int QW, int D, typename Frag>
__device__ __forceinline__ void doc16_deep(Frag frag, const bf16x8 (&qf)[QW][2][4], float (&m)[QW][2]) {
  constexpr int NC = 2 * QW;
  constexpr int NK = kLd / 16 * NC;
#pragma unroll
  for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
  bf16x8 a[2][4];
  f32x4 acc[D + 1];
  frag(0, a[0]);
#pragma unroll
  for (int k = 0; k < NK + D; ++k) {
    if (k < NK) {
      const int rt = k / NC, c = k % NC;
      if (c == 0 && rt + 1 < kLd / 16) frag(rt + 1, a[(rt + 1) & 1]);
      const int q = c >> 1, ct = c & 1;
      f32x4 x = f32x4{};
#pragma unroll
      for (int s = 0; s < 4; ++s) x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt & 1][s], qf[q][ct][s], x, 0, 0, 0);
      acc[k % (D + 1)] = x;
    }
    if (k >= D) {
      const int kk = k - D;
      const int pc = kk % NC;
      const f32x4& y = acc[kk % (D + 1)];
      float& mm = m[pc >> 1][pc & 1];
      mm = __builtin_fmaxf(__builtin_fmaxf(mm, __builtin_fmaxf(y[0], y[1])), __builtin_fmaxf(y[2], y[3]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Full doc as one software-pipelined stream of 8 tiles x 2*QW MFMA chains:
// chain k's 4 MFMAs are issued while chain k-1's max runs (2 accumulators);
// sched_barrier keeps hipcc from re-serialising the chains.
template <int QW, int SB, typename Frag>
__device__ __forceinline__ void doc16_pipe(Frag frag, const bf16x8 (&qf)[QW][2][4], float (&m)[QW][2]) {
  constexpr int NC = 2 * QW;
#pragma unroll
  for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
  bf16x8 a[2][4];
  f32x4 acc[2];
  frag(0, a[0]);
#pragma unroll
  for (int rt = 0; rt < kLd / 16; ++rt) {
    if (rt + 1 < kLd / 16) frag(rt + 1, a[(rt + 1) & 1]);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const int k = rt * NC + c;
      const int q = c >> 1, ct = c & 1;
      f32x4 x = f32x4{};
#pragma unroll
      for (int s = 0; s < 4; ++s) x = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[rt & 1][s], qf[q][ct][s], x, 0, 0, 0);
      acc[k & 1] = x;
      if (k > 0) {
        const int pc = (k - 1) % NC;
        const f32x4& y = acc[(k - 1) & 1];
        float& mm = m[pc >> 1][pc & 1];
        mm = __builtin_fmaxf(__builtin_fmaxf(mm, __builtin_fmaxf(y[0], y[1])), __builtin_fmaxf(y[2], y[3]));
      }
      if (SB == 1) __builtin_amdgcn_sched_barrier(0);
      if (SB == 2) {   // 2 MFMA, the previous chain's max (<= 3 VALU), 2 MFMA
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  {
    const int pc = NC - 1;
    const f32x4& y = acc[(kLd / 16 * NC - 1) & 1];
    float& mm = m[pc >> 1][pc & 1];
    mm = __builtin_fmaxf(__builtin_fmaxf(mm, __builtin_fmaxf(y[0], y[1])), __builtin_fmaxf(y[2], y[3]));
  }
}

template <int WAVES, int QW, int MODE>
__global__ __launch_bounds__(WAVES * 64, 2) void scan16x_kernel(
    const uint8_t* __restrict__ tokens, const int32_t* __restrict__ doclens, int64_t n,
    const uint16_t* __restrict__ Q, int B, int lq, float* __restrict__ out, int64_t ld_out,
    int64_t chunk_docs) {
  constexpr int QPB = WAVES * QW;
  constexpr int kPieces = kDocBytes / 1024;
  constexpr int kPiecesPerWave = kPieces / WAVES;
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

  auto epilogue = [&](int j, float (&m)[QW][2]) {
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const float v = MODE == 101 ? m[q][0] + m[q][1] : reduce16(m[q][0], m[q][1], lane, lq);
      sc[q] = (lane == (j & 63)) ? v : sc[q];
    }
    if ((j & 63) == 63 || j == nd - 1) {
      const int i0 = j & ~63;
      const int cnt = j - i0 + 1;
#pragma unroll
      for (int q = 0; q < QW; ++q) {
        const int qi = g * QPB + wave * QW + q;
        if (qi < B && lane < cnt) out[(size_t)qi * ld_out + d_begin + i0 + lane] = sc[q];
      }
    }
  };

  const bool defer = MODE == 103 && wave >= 4;
  float mp[QW][2];
  int jp = -1;

  issue(0, 0);
  if (MODE == 109 || MODE == 110) {      // timing probes: doc 0's image only (INVALID scores)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  for (int i = 0; i < nd; ++i) {
    if (MODE != 109 && MODE != 110) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (i + 1 < nd) issue(i + 1, (i + 1) & 1);
    } else if (MODE == 110) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    const uint8_t* buf = smem + ((MODE == 109 || MODE == 110) ? 0 : (i & 1) * kDocBytes);
    int dl = doclens[d_begin + i];
    dl = dl < 0 ? 0 : (dl > kLd ? kLd : dl);
    float m[QW][2];
    auto frag = [&](int rt, bf16x8 (&a)[4]) { lds_afrag16(buf, rt, lane, a); };
    if ((MODE == 104 || MODE == 105 || MODE == 106) && dl >= kLd) {
      doc16_pipe<QW, MODE == 104 ? 1 : (MODE == 106 ? 2 : 0)>(frag, qf, m);
      epilogue(i, m);
    } else if ((MODE == 111 || MODE == 112 || MODE == 113) && dl >= kLd) {
      doc16_deep<QW, (MODE >= 111 && MODE <= 113) ? MODE - 110 : 1>(frag, qf, m);
      epilogue(i, m);
    } else if ((MODE == 107 || MODE == 108) && dl >= kLd) {
      constexpr int NI = MODE == 107 ? 2 : 4;
#pragma unroll
      for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
      bf16x8 a0[4], a1[4];
      frag(0, a0);
#pragma unroll
      for (int rt = 0; rt < kLd / 16; rt += 2) {
        frag(rt + 1, a1);
        tile16_il<QW, NI>(a0, qf, m);
        if (rt + 2 < kLd / 16) frag(rt + 2, a0);
        tile16_il<QW, NI>(a1, qf, m);
      }
      epilogue(i, m);
    } else if (MODE == 102 && dl >= kLd) {
#pragma unroll
      for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
      bf16x8 a0[4], a1[4];
      frag(0, a0);
#pragma unroll
      for (int rt = 0; rt < kLd / 16; rt += 2) {
        frag(rt + 1, a1);
        tile16_cheap<QW>(a0, qf, m);
        if (rt + 2 < kLd / 16) frag(rt + 2, a0);
        tile16_cheap<QW>(a1, qf, m);
      }
      epilogue(i, m);
    } else if (MODE == 103 && dl >= kLd) {
#pragma unroll
      for (int q = 0; q < QW; ++q) m[q][0] = m[q][1] = neg_inf();
      bf16x8 a0[4], a1[4];
      frag(0, a0);
#pragma unroll
      for (int rt = 0; rt < kLd / 16; rt += 2) {
        frag(rt + 1, a1);
        tile16<QW>(a0, qf, f32x4{}, m);
        if (rt + 2 < kLd / 16) frag(rt + 2, a0);
        tile16<QW>(a1, qf, f32x4{}, m);
        if (rt == 2 && defer && jp >= 0) {       // mid-doc: the previous doc's epilogue
          epilogue(jp, mp);
          jp = -1;
        }
      }
      if (defer) {
#pragma unroll
        for (int q = 0; q < QW; ++q) mp[q][0] = m[q][0], mp[q][1] = m[q][1];
        jp = i;
      } else {
        epilogue(i, m);
      }
    } else {
      if (defer && jp >= 0) {
        epilogue(jp, mp);
        jp = -1;
      }
      doc16<QW>(frag, qf, dl, lane, m);
      epilogue(i, m);
    }
  }
  if (defer && jp >= 0) epilogue(jp, mp);
}

template <int MODE>
int launch_x(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld, hipStream_t st) {
  return launch_scan<8, 4, 1>(scan16x_kernel<8, 4, MODE>, ix, Q, B, lq, out, ld, st, "scan16x_kernel");
}
}  // namespace

// The production B > 16 scan with an explicit work split: dyn_frac of the
// corpus as dynamic tasks of task_docs (0 = the static split); stamps != null
// runs the STAMPS build (per-workgroup s_memrealtime / s_memtime, 4 x u64).
extern "C" int lab_scan16x4(cbv2_index* ix, const void* Q, int B, int lq, float* out, int64_t ld, void* stream,
                            float dyn_frac, int task_docs, void* stamps, int kind) {
  const uint16_t* q = (const uint16_t*)Q;
  hipStream_t st = (hipStream_t)stream;
  // kind: lab-only kernel builds (round 1: max placement one MFMA later,
  // D = 1/2/3 -> 73.3 / 76.3 / 76.1 % vs product 76.3 %; removed)
  //   kind 0 = production (64-token iterations, 2-deep ring: 142.5 -> 139.1 ms
  //   at 1M vs 32-token iterations with a 3-deep ring, which is kind 1)
  if (kind == 1) return launch_scan16x4<8, 4, 1, 2, 3, false, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  // (kinds 2-5, round 1: one wave per SIMD, 4 waves x 8 queries, 163 vs 142 ms: removed)
  // mid-batch shapes (B = 16 / 64): 6 = production 4-wave x 4 queries (2 WGs/CU, 32-token ring),
  // 7 = 8 waves x 2 queries (one WG/CU, 64-token ring), 8 = 4 x 4 with 64-token iterations,
  // 9 = 8 waves x 2 queries, 32-token 3-deep ring
  if (kind == 6) return launch_scan16x4<4, 4, 2, 2, 2, false, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  if (kind == 7) return launch_scan16x4<8, 2, 1, 2, 2, false, 64>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  if (kind == 8) return launch_scan16x4<4, 4, 2, 2, 2, false, 64>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  if (kind == 9) return launch_scan16x4<8, 2, 1, 2, 3, false, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  // kind 10: production shape with the spread DMA issue (SPREAD); kind 11: its
  // phase-stamped build (STAMPS + SPREAD; the stamps buffer is required)
  if (kind == 10) return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, true>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  if (kind == 11 && stamps != nullptr)
    return launch_scan16x4<8, 4, 1, 2, 2, true, 64, 2, true>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs,
                                                             (uint64_t*)stamps);
  // kind 12: the B <= 16 production shape (kind 6) phase-stamped
  if (kind == 12 && stamps != nullptr)
    return launch_scan16x4<4, 4, 2, 2, 2, true, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps);
  // kind 13: production shape (round 2: SPLITLOAD, waves 0-3 issue all LDS-DMA
  // pieces; kind 0 is the round-1 shape, every wave issuing its own); kind 14:
  // its phase-stamped build; kind 15 / 16: the fused top-k build (k = 100,
  // keys into `out`) without / with SPLITLOAD (16 = what cbv2_search runs).
  // Round 2, one box, 1M docs B=256: k0 145.25, k13 144.10, k15 146.33, k16
  // 145.58 ms; phase stamps per iteration (cycles, waves 0-3 | 4-7): k0 wait
  // 4288 | 111, issue 762 | 1599, compute 13211 | 16548; k14 wait 3919 | 116,
  // issue 1405 | 398, compute 12642 | 17459 (r02c)
  if (kind == 13)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                        task_docs);
  if (kind == 14 && stamps != nullptr)
    return launch_scan16x4<8, 4, 1, 2, 2, true, 64, 2, false, 0, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                       task_docs, (uint64_t*)stamps);
  if (kind == 15 || kind == 16) {
    FusedTopk ft{(uint64_t*)out, 100, scan_chunks(ix, (B + 31) / 32, cu_count(ix->device)), 0};
    if ((int64_t)B * ft.max_slots * 100 * 8 > ld * (int64_t)B * 4) return -1;   // keys must fit the buffer
    if (kind == 15)
      return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, kFusedCap, false>(
          ix, q, B, lq, nullptr, 0, st, dyn_frac, task_docs, nullptr, nullptr, &ft);
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, kFusedCap, true>(
        ix, q, B, lq, nullptr, 0, st, dyn_frac, task_docs, nullptr, nullptr, &ft);
  }
  // kinds 17-22 (round 2): ARRIVE -- LDS landed/done counters instead of the
  // per-iteration barrier.  17: 32-token iterations, 4-deep ring; 18: 64-token,
  // 2-deep; 19: 32-token, 3-deep; 20: kind 17 phase-stamped; 21 / 22: the fused
  // top-k builds of 17 / 18 (k = 100, keys into `out`).
  if (kind == 17)
    return launch_scan16x4<8, 4, 1, 2, 4, false, 32, 2, false, 0, true, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                             task_docs);
  if (kind == 18)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                             task_docs);
  if (kind == 19)
    return launch_scan16x4<8, 4, 1, 2, 3, false, 32, 2, false, 0, true, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                             task_docs);
  if (kind == 20 && stamps != nullptr)
    return launch_scan16x4<8, 4, 1, 2, 4, true, 32, 2, false, 0, true, true>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                            task_docs, (uint64_t*)stamps);
  if (kind == 21 || kind == 22) {
    FusedTopk ft{(uint64_t*)out, 100, scan_chunks(ix, (B + 31) / 32, cu_count(ix->device)), 0};
    if ((int64_t)B * ft.max_slots * 100 * 8 > ld * (int64_t)B * 4) return -1;
    if (kind == 21)
      return launch_scan16x4<8, 4, 1, 2, 4, false, 32, 2, false, kFusedCap, true, true>(
          ix, q, B, lq, nullptr, 0, st, dyn_frac, task_docs, nullptr, nullptr, &ft);
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, kFusedCap, true, true>(
        ix, q, B, lq, nullptr, 0, st, dyn_frac, task_docs, nullptr, nullptr, &ft);
  }
  // kind 23: energy probe (INVALID scores) -- kind 13 with half the LDS read
  // bytes (odd tiles reuse the even tile's fragments), same MFMA stream
  if (kind == 23)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 1>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                                 task_docs);
  // kind 24: energy probe (INVALID) -- kind 13 without doc streaming after the first fill
  if (kind == 24)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 2>(ix, q, B, lq, out, ld, st, dyn_frac,
                                                                                 task_docs);
  // kind 25: kind 13 with the k-step-major MFMA order (iter4_full_kmajor: 8 live
  // accumulators, consecutive MFMAs share the doc fragment); bit-identical
  if (kind == 25)
    return launch_scan16x4<8, 4, 1, 2, 2, false, 64, 2, false, 0, true, false, 0, kLd, 1>(ix, q, B, lq, out, ld, st,
                                                                                         dyn_frac, task_docs);
  // kind 26: the B <= 16 shape (kind 6) with the k-step-major MFMA order
  if (kind == 26)
    return launch_scan16x4<4, 4, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 1>(ix, q, B, lq, out, ld, st,
                                                                                          dyn_frac, task_docs);
  // kind 27 / 28: the 4-wave shape with 2 queries per wave (8 per workgroup:
  // production kScan16x4W4Q2) / its phase-stamped build
  if (kind == 27)
    return launch_scan16x4<4, 2, 2, 2, 2, false, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs);
  if (kind == 28 && stamps != nullptr)
    return launch_scan16x4<4, 2, 2, 2, 2, true, 32>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps);
  // kinds 29-32 (round 5, power probe): the one-group non-temporal mid-batch
  // shapes -- 29: 4 x 4 (B = 9-16, production kScan16x4W4Nt), 30: the same
  // with PROBE 3 (INVALID: the FLOPs on v_mfma_f32_32x32x16_bf16); 31 / 32:
  // 4 x 2 (B = 5-8) and its PROBE 3 build
  // stamps != null: the STAMPS build of the same shape (per-workgroup clock)
#define LAB_MID(W, QW_, D_, PR)                                                                                  \
  return stamps ? launch_scan16x4<W, QW_, 2, D_, 2, true, 32, 2, false, 0, false, false, PR, kLd, 0, 2>(            \
                      ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)                   \
                : launch_scan16x4<W, QW_, 2, D_, 2, false, 32, 2, false, 0, false, false, PR, kLd, 0, 2>(           \
                      ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr)
  if (kind == 29) LAB_MID(4, 4, 2, 0);
  if (kind == 30) LAB_MID(4, 4, 0, 3);
  if (kind == 31) LAB_MID(4, 2, 2, 0);
  if (kind == 32) LAB_MID(4, 2, 1, 3);
#undef LAB_MID
  // kind 33 (round 6): the B <= 4 dense-doc production shape, 4 waves x 1
  // query, two per CU, non-temporal (kScan16x4W4Q1 without the folded keys);
  // stamps != null: its STAMPS build (per-workgroup clock, start skew, tail)
  if (kind == 33)
    return stamps ? launch_scan16x4<4, 1, 2, 2, 2, true, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  // kinds 34-36 (round 6): the B <= 4 shape with more doc bytes in flight per
  // CU -- 34: one workgroup per CU, 3-deep 32-token ring (96 KiB of LDS);
  // 35: one per CU, 64-token iterations, 2-deep (128 KiB); 36: one per CU,
  // ARRIVE (no per-iteration barrier, waves 0-1 load), 4-deep 32-token ring
  if (kind == 34)
    return stamps ? launch_scan16x4<4, 1, 1, 2, 3, true, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 1, 2, 3, false, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  if (kind == 35)
    return stamps ? launch_scan16x4<4, 1, 1, 2, 2, true, 64, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 1, 2, 2, false, 64, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  if (kind == 36)
    return stamps ? launch_scan16x4<4, 1, 1, 2, 4, true, 32, 1, false, 0, true, true, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 1, 2, 4, false, 32, 1, false, 0, true, true, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  // kinds 37 / 38: kind 34 with SPLITLOAD (waves 0-1 issue every DMA piece) /
  // with a 4-deep ring (128 KiB of LDS, three iterations in flight)
  if (kind == 37)
    return stamps ? launch_scan16x4<4, 1, 1, 2, 3, true, 32, 1, false, 0, true, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 1, 2, 3, false, 32, 1, false, 0, true, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  if (kind == 38)
    return stamps ? launch_scan16x4<4, 1, 1, 2, 4, true, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, (uint64_t*)stamps, nullptr)
                  : launch_scan16x4<4, 1, 1, 2, 4, false, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
                        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  // kinds 39 / 40: the B = 5-8 shape (4 x 2) at one workgroup per CU, 3- / 4-deep
  if (kind == 39)
    return launch_scan16x4<4, 2, 1, 2, 3, false, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  if (kind == 40)
    return launch_scan16x4<4, 2, 1, 2, 4, false, 32, 1, false, 0, false, false, 0, kLd, 0, 2>(
        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  // kind 41: the production B = 5-8 shape (4 x 2, two per CU, nt)
  if (kind == 41)
    return launch_scan16x4<4, 2, 2, 2, 2, false, 32, 2, false, 0, false, false, 0, kLd, 0, 2>(
        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr);
  // kind 42: the production dense B <= 2 scan WITH the block-max keys folded
  // in (the latency path's form; kind 37 is the same without them): the keys
  // zeroed by a memset inside the timed region (as the query split does in
  // the product)
  if (kind == 42) {
    static uint32_t* bm = nullptr;
    static size_t bm_bytes = 0;
    const size_t need = (size_t)B * (bm_blocks(ix->n) + bm_supers(ix->n)) * 4;
    if (need > bm_bytes) {
      if (bm) (void)hipFree(bm);
      if (hipMalloc(&bm, need) != hipSuccess) return -2;
      bm_bytes = need;
    }
    if (hipMemsetAsync(bm, 0, need, st) != hipSuccess) return -3;
    return launch_scan16x4<4, 1, 1, 2, 3, false, 32, 1, false, 0, true, false, 0, kLd, 0, 2, true>(
        ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr, nullptr, nullptr, bm);
  }
  if (kind != 0) return -1;
  if (stamps != nullptr)
    return launch_scan16x4<8, 4, 1, 2, 2, true, 64>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs,
                                                    (uint64_t*)stamps);
  return launch_scan16x4<8, 4, 1, 2, 2, false, 64>(ix, q, B, lq, out, ld, st, dyn_frac, task_docs, nullptr);
}

// The B <= 2 direct scan with mult x the production chunk count (smaller
// per-wave chunks: the dispatcher balances late workgroups over the XCDs).
namespace {
template <int QW>
int lab_direct(cbv2_index* ix, const uint16_t* Q, int B, int lq, float* out, int64_t ld_out, hipStream_t st,
               int mult) {
  const int nq_groups = (B + QW - 1) / QW;
  const int64_t target_waves = 8LL * cu_count(ix->device) * mult;
  int64_t n_chunks = target_waves / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  if (n_chunks < 1) n_chunks = 1;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  const int64_t grid = ((int64_t)nq_groups * n_chunks + 3) / 4;
  hipLaunchKernelGGL((maxsim_scan_direct_kernel<QW, false>), dim3((unsigned)grid), dim3(256), 0, st, ix->tokens,
                     ix->doclens, ix->n, Q, B, lq, out, ld_out, chunk_docs, kLd);
  return launch_check("maxsim_scan_direct_kernel");
}
}  // namespace

extern "C" int lab_scan(cbv2_index* ix, int variant, const void* Q, int B, int lq, float* out, int64_t ld,
                        void* stream) {
  if (variant >= 200 && variant < 300)   // 200 + mult: the direct scan (one query per wave) oversubscribed
    return lab_direct<1>(ix, (const uint16_t*)Q, B, lq, out, ld, (hipStream_t)stream, variant - 200);
  const uint16_t* q = (const uint16_t*)Q;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 100: return launch_x<100>(ix, q, B, lq, out, ld, st);
    case 101: return launch_x<101>(ix, q, B, lq, out, ld, st);
    case 102: return launch_x<102>(ix, q, B, lq, out, ld, st);
    case 103: return launch_x<103>(ix, q, B, lq, out, ld, st);
    case 104: return launch_x<104>(ix, q, B, lq, out, ld, st);
    case 105: return launch_x<105>(ix, q, B, lq, out, ld, st);
    case 106: return launch_x<106>(ix, q, B, lq, out, ld, st);
    case 107: return launch_x<107>(ix, q, B, lq, out, ld, st);
    case 108: return launch_x<108>(ix, q, B, lq, out, ld, st);
    case 109: return launch_x<109>(ix, q, B, lq, out, ld, st);
    case 110: return launch_x<110>(ix, q, B, lq, out, ld, st);
    case 111: return launch_x<111>(ix, q, B, lq, out, ld, st);
    case 112: return launch_x<112>(ix, q, B, lq, out, ld, st);
    case 113: return launch_x<113>(ix, q, B, lq, out, ld, st);
    default: return scan_maxsim(ix, q, B, lq, out, ld, st, variant);
  }
}

// MXFP8 scans: variant 0 = the per-doc maxsim_scan_f8_kernel (round-1
// production), 1 = the doc-interleaved maxsim_scan_f8x4_kernel (production:
// guided dynamic tail), 2 = the same with the static split only.
extern "C" int lab_scan_f8(cbv2_index* ix, int variant, const void* Qbuf, int B, int lq, float* out, int64_t ld,
                           void* stream) {
  const uint8_t* Qb = (const uint8_t*)Qbuf;
  const uint8_t* Qs = Qb + (size_t)B * lq * kDim;
  hipStream_t st = (hipStream_t)stream;
  // 300 / 301 (round 6): the dense B <= 2 shape (24: 4 waves x 1 query, 3-deep
  // ring, nt) at ONE workgroup per CU, without / with SPLIT (waves 0-1 load);
  // 302: the production shape 24 (two per CU) at a 10 % tail
  if (variant == 300)
    return launch_f8x4<32, 3, true, 1, 1, 1, 4, 0, kLd, 1, true, false, false, false, false, 0, 2>(
        ix, Qb, Qs, B, lq, out, ld, st, kF8DynB8, kScanTaskDocs, nullptr);
  if (variant == 301)
    return launch_f8x4<32, 3, true, 1, 1, 1, 4, 0, kLd, 1, true, false, false, true, false, 0, 2>(
        ix, Qb, Qs, B, lq, out, ld, st, kF8DynB8, kScanTaskDocs, nullptr);
  if (variant == 302)
    return launch_f8x4<32, 3, true, 1, 2, 2, 4, 0, kLd, 1, true, false, false, false, false, 0, 2>(
        ix, Qb, Qs, B, lq, out, ld, st, 0.1f, kScanTaskDocs, nullptr);
  if (variant == 303)
    return launch_f8x4<32, 3, true, 1, 1, 1, 4, 0, kLd, 1, true, false, false, true, false, 0, 2>(
        ix, Qb, Qs, B, lq, out, ld, st, 0.1f, kScanTaskDocs, nullptr);
  if (variant >= 200 && variant < 300) {   // 200 + mult: the f8 direct scan (QW = 2) with mult x the resident waves
    constexpr int QW = 2;
    const int nq_groups = (B + QW - 1) / QW;
    int64_t n_chunks = 8LL * cu_count(ix->device) * (variant - 200) / nq_groups;
    if (n_chunks > ix->n) n_chunks = ix->n;
    if (n_chunks < 1) n_chunks = 1;
    const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
    n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
    const int64_t grid = ((int64_t)nq_groups * n_chunks + 3) / 4;
    hipLaunchKernelGGL(maxsim_scan_f8_direct_kernel<QW>, dim3((unsigned)grid), dim3(256), 0, st, ix->tokens,
                       ix->scales, ix->doclens, ix->n, Qb, Qs, B, lq, out, ld, chunk_docs);
    return launch_check("maxsim_scan_f8_direct_kernel");
  }
  // variant 100 * j + shape (j = 1, 2, 3): that shape with a dynamic share of 0.3 j
  if (variant >= 100) return scan_f8(ix, Qb, B, lq, out, ld, st, 0.3f * (float)(variant / 100), kScanTaskDocs,
                                     variant % 100);
  if (variant == 1 || (B <= kF8SmallMaxB && variant < 10)) return scan_f8(ix, Qb, B, lq, out, ld, st);
  if (variant == 2) return scan_f8(ix, Qb, B, lq, out, ld, st, 0.0f);  // doc-interleaved, static split only
  if (variant >= 10 && variant <= 40) return scan_f8(ix, Qb, B, lq, out, ld, st, kScanDynFrac, kScanTaskDocs,
                                                     variant - 10);  // iteration shapes, see scan_f8
  constexpr int QPB = kF8Waves * kF8QW;
  const int nq_groups = (B + QPB - 1) / QPB;
  int64_t n_chunks = cu_count(ix->device) / nq_groups;
  if (n_chunks > ix->n) n_chunks = ix->n;
  const int64_t chunk_docs = (ix->n + n_chunks - 1) / n_chunks;
  n_chunks = (ix->n + chunk_docs - 1) / chunk_docs;
  hipLaunchKernelGGL((maxsim_scan_f8_kernel<kF8Waves, kF8QW>), dim3((unsigned)(nq_groups * n_chunks)),
                     dim3(kF8Waves * 64), 0, st, ix->tokens, ix->scales, ix->doclens, ix->n, Qb, Qs, B, lq, out, ld,
                     chunk_docs);
  return launch_check("maxsim_scan_f8_kernel");
}
