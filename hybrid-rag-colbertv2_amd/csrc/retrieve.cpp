// retrieve.cpp — HybridRetriever.retrieve (local_rag_complete.py:894-935) for one
// query batch with ONE host round trip and no Python between the stages:
//
//   begin   stage 2: scan + top-k of this shard (sharded: into the send block of
//           the exchange), enqueued on the caller's stream; returns at once so
//           the caller runs stage 1 (host BM25, LRC:937-950) while the GPU scans.
//   finish  (sharded: the stage-2 + stage-1 all-gather and merges) -> D2H of the
//           ColBERT top-k (and of the merged BM25 lists) -> wait -> host RRF +
//           [:C] cut (cbv2_rrf_fuse, LRC:960-978, :916) -> H2D of the fused
//           candidates -> stage 3 rerank (sharded: all-reduce MAX) + top-k select.
//
// Results are those of the separate calls (cbv2_search / _f32 / _sharded_*,
// cbv2_rrf_fuse, cbv2_rerank_ws / _f32 / _sharded) bit for bit: this file only
// sequences them, so the arithmetic and the tie rules live in one place.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);
extern "C" int cbv2_rerank_f32_after_search(cbv2_index* ix, const void* search_ws, size_t search_wsb, int32_t cap,
                                            int32_t B, int32_t lq, const int32_t* cand, int32_t C, int32_t k, void* ws,
                                            size_t wsb, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                                            const float* Q, void* stream);
extern "C" int cbv2_index_device(const cbv2_index* ix);

namespace {
int err(int code, const char* fmt, ...) {
  char buf[384];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return cbv2_set_error(code, buf);
}

#define RT_HIP(call)                                                          \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) return err(CBV2_EHIP, "%s (%d)", #call, (int)e_); \
  } while (0)

size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

// The round trip's wait: an event recorded after the D2H copy.  A blocking
// wait wakes the host tens of microseconds after the copy lands (measured:
// 26-39 us from the D2H copy's end to the next H2D copy's start), a poll
// (hipEventQuery) within about a microsecond -- but a poll holds a core for
// as long as the stream work ahead of the copy runs.  So only small batches
// poll flat out: B <= kSpinMaxB (one scan of <= 8 queries: ~5-7 ms at 1M
// docs, where a wake-up would be ~0.5 % of the latency), for at most kSpinNs,
// then as below.
// Larger batches (one B=256 scan: ~140 ms, whose host side runs the BM25
// threads meanwhile) poll between sleeps of 1/32 of the time waited so far
// (20 us .. 500 us): the thread wakes at most ~3 % (and 0.5 ms) after the
// copy and is asleep otherwise.  (hipEventSynchronize is no substitute:
// measured on the GPU box, a B=256 call over 200k docs burned its whole
// 28 ms wait on a core even with a hipEventBlockingSync event.)
//
// Events come from a process-wide pool per device: taken for one wait and
// returned after it, so the pool holds at most as many events as threads
// ever waited at once (cbv2_retrieve_wait_events counts them), none leaks per
// thread, and an event is always created on the device of the index whose
// stream it is recorded on (the caller's current device may differ).
constexpr long long kSpinNs = 50LL * 1000 * 1000;
constexpr int32_t kSpinMaxB = 8;
constexpr int kMaxDev = 64;

struct EventPool {
  std::mutex mu;
  std::vector<hipEvent_t> free_ev[kMaxDev];
  int64_t created = 0;
};
EventPool& pool() {
  static EventPool* p = new EventPool;   // never destroyed: no teardown-order issue at exit
  return *p;
}

int take_event(int dev, hipEvent_t* ev) {
  EventPool& P = pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto& v = P.free_ev[dev];
    if (!v.empty()) {
      *ev = v.back();
      v.pop_back();
      return CBV2_OK;
    }
  }
  RT_HIP(hipEventCreateWithFlags(ev, hipEventDisableTiming));
  std::lock_guard<std::mutex> lk(P.mu);
  ++P.created;
  return CBV2_OK;
}

void give_event(int dev, hipEvent_t ev) {
  EventPool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.free_ev[dev].push_back(ev);
}

// The caller has selected the index's device (DevSel below).
int wait_copy(hipStream_t st, int dev, int32_t B) {
  if (dev < 0 || dev >= kMaxDev) return hipStreamSynchronize(st) == hipSuccess ? CBV2_OK : err(CBV2_EHIP, "sync failed");
  hipEvent_t ev = nullptr;
  if (int rc = take_event(dev, &ev)) return rc;
  hipError_t e = hipEventRecord(ev, st);
  const auto t0 = std::chrono::steady_clock::now();
  while (e == hipSuccess) {
    e = hipEventQuery(ev);
    if (e != hipErrorNotReady) break;
    e = hipSuccess;
    const long long waited =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (B > kSpinMaxB || waited > kSpinNs)   // a long wait: sleep between polls
      std::this_thread::sleep_for(std::chrono::nanoseconds(std::min(500000LL, std::max(20000LL, waited / 32))));
  }
  give_event(dev, ev);
  return e == hipSuccess ? CBV2_OK : err(CBV2_EHIP, "round-trip wait (%d)", (int)e);
}

// The fused candidates the one-shard rerank reads straight from host memory:
// coherent, device-mapped pinned buffers (hipHostMallocMapped | Coherent; the
// caller's host stage may be pageable or non-coherent pinned memory, so it is
// never handed to a kernel).  The host RRF writes the [B][C] candidate ids
// into one, and the rerank's workgroups read their candidate id through the
// mapped pointer (one 4-byte PCIe read each): no H2D copy launch between the
// host fusion and the rerank -- the latency path's host -> GPU hop is one
// kernel launch.  A buffer goes back to the per-device pool with an event
// recorded after the rerank that reads it; it is handed out again only once
// that event completed, so a later call (any thread, any stream) never
// overwrites candidates a queued rerank has still to read.
struct MappedBuf {
  void* h = nullptr;
  void* d = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;
  bool recorded = false;
};
struct MappedPool {
  std::mutex mu;
  std::vector<MappedBuf> free_buf[kMaxDev];
};
MappedPool& mapped_pool() {
  static MappedPool* p = new MappedPool;   // never destroyed (buffers live for the process)
  return *p;
}

// A buffer of >= bytes whose last reader finished; false: none could be made
// (the caller falls back to the copy through its own host stage).
bool take_mapped(int dev, size_t bytes, MappedBuf* out) {
  MappedPool& P = mapped_pool();
  {
    std::lock_guard<std::mutex> lk(P.mu);
    auto& v = P.free_buf[dev];
    for (size_t i = 0; i < v.size(); ++i) {
      if (v[i].bytes < bytes) continue;
      if (v[i].recorded && hipEventQuery(v[i].ev) != hipSuccess) continue;   // still read by a queued rerank
      *out = v[i];
      v.erase(v.begin() + (long)i);
      return true;
    }
  }
  MappedBuf b;
  b.bytes = std::max<size_t>(bytes, 64 * 1024);
  if (hipHostMalloc(&b.h, b.bytes, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable) != hipSuccess)
    return false;
  if (hipHostGetDevicePointer(&b.d, b.h, 0) != hipSuccess ||
      hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipHostFree(b.h);
    return false;
  }
  *out = b;
  return true;
}

void give_mapped(int dev, MappedBuf b, hipStream_t st) {
  b.recorded = hipEventRecord(b.ev, st) == hipSuccess;
  if (!b.recorded) (void)hipStreamSynchronize(st);   // cannot mark the reader: wait for it instead
  MappedPool& P = mapped_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.free_buf[dev].push_back(b);
}

// Selects the index's device for one call and restores the caller's.
struct DevSel {
  int prev = -1, dev = -1;
  bool ok = false;
  explicit DevSel(const cbv2_index* ix) {
    dev = cbv2_index_device(ix);
    if (dev < 0 || hipGetDevice(&prev) != hipSuccess) return;
    ok = prev == dev || hipSetDevice(dev) == hipSuccess;
  }
  ~DevSel() {
    if (ok && prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
};

struct Kind {
  int32_t dtype = 0, faithful = 0;
};

// Device workspace: [stage-2 part | s B*k | ids B*k | lex ids B*kb | cand B*C | status B | rerank part]
struct Layout {
  size_t stage2 = 0, rerank = 0, total = 0;
  uint8_t* base = nullptr;
  float* s = nullptr;
  int32_t *ids = nullptr, *lex_ids = nullptr, *cand = nullptr, *status = nullptr;
  uint8_t* rr = nullptr;
};

Layout layout(const cbv2_index* ix, const cbv2_comm* c, Kind kd, int32_t B, int32_t lq, int32_t k, int32_t kb,
              int32_t C, void* ws) {
  Layout L;
  if (c)
    L.stage2 = a256(cbv2_sharded_workspace_bytes(ix, c, B, k, kb, 0));
  else if (kd.faithful)
    L.stage2 = a256(cbv2_f32_workspace_bytes(ix, CBV2_F32_SEARCH, B, lq, k > CBV2_RETRIEVE_BAND_CAP ? k
                                                                                               : CBV2_RETRIEVE_BAND_CAP));
  else
    L.stage2 = a256(cbv2_search_workspace_size(ix, B, k, CBV2_SCORER_MAXSIM));
  if (c)        // cbv2_rerank_sharded: raw [B][C] (+ a faithful shard's rerank workspace after it)
    L.rerank = a256((size_t)B * C * 4) +
               (kd.faithful ? a256(cbv2_f32_workspace_bytes(ix, CBV2_F32_RERANK, B, lq, C)) : 0);
  else if (kd.faithful)
    L.rerank = a256(cbv2_f32_workspace_bytes(ix, CBV2_F32_RERANK, B, lq, C));
  else
    L.rerank = a256(cbv2_rerank_workspace_bytes(B, C));
  const size_t bk = a256((size_t)B * k * 4), bkb = a256((size_t)B * (kb > 0 ? kb : 1) * 4),
               bc = a256((size_t)B * C * 4), bs = a256((size_t)B * 4);
  L.total = L.stage2 + 2 * bk + bkb + bc + bs + L.rerank;
  if (ws) {
    uint8_t* p = (uint8_t*)ws;
    L.base = p;
    p += L.stage2;
    L.s = (float*)p;
    p += bk;
    L.ids = (int32_t*)p;
    p += bk;
    L.lex_ids = (int32_t*)p;
    p += bkb;
    L.cand = (int32_t*)p;
    p += bc;
    L.status = (int32_t*)p;
    p += bs;
    L.rr = p;
  }
  return L;
}

// Host stage: [ids B*k | merged lex ids B*kb | cand B*C | lex ids B*kb | lex scores B*kb] (4-byte words)
struct HostLayout {
  int32_t *ids, *lex_merged, *cand, *lex_ids, *lex_scores;
};
size_t host_words(int32_t B, int32_t k, int32_t kb, int32_t C) {
  return (size_t)B * k + (size_t)3 * B * kb + (size_t)B * C;
}
HostLayout host_layout(void* h, int32_t B, int32_t k, int32_t kb, int32_t C) {
  HostLayout H;
  int32_t* p = (int32_t*)h;
  H.ids = p;
  H.lex_merged = H.ids + (size_t)B * k;
  H.cand = H.lex_merged + (size_t)B * kb;
  H.lex_ids = H.cand + (size_t)B * C;
  H.lex_scores = H.lex_ids + (size_t)B * kb;
  return H;
}

int check_common(const cbv2_index* ix, Kind* kd, const cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B,
                 int32_t lq, int32_t k, int32_t kb) {
  if (!ix) return err(CBV2_EINVAL, "null index");
  if (int rc = cbv2_index_kind(ix, &kd->dtype, &kd->faithful)) return rc;
  if (!Q) return err(CBV2_EINVAL, "null queries");
  if (B < 1 || k < 1 || kb < 0) return err(CBV2_EINVAL, "bad sizes (B %d, k %d, kb %d)", B, k, kb);
  if (lq < 1 || lq > 32) return err(CBV2_EINVAL, "lq must be in [1, 32] (got %d); longer queries go by blocks", lq);
  const int32_t want = kd->faithful ? CBV2_DTYPE_F32 : kd->dtype;
  if (q_dtype != want) return err(CBV2_EINVAL, "query dtype %d does not match the index (needs %d)", q_dtype, want);
  return CBV2_OK;
}
}  // namespace

extern "C" {

size_t cbv2_retrieve_workspace_bytes(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t lq, int32_t k,
                                     int32_t kb, int32_t C) {
  Kind kd;
  if (!ix || B < 1 || k < 1 || kb < 0 || C < 1 || lq < 1 || cbv2_index_kind(ix, &kd.dtype, &kd.faithful)) return 0;
  return layout(ix, c, kd, B, lq, k, kb, C, nullptr).total;
}

int64_t cbv2_retrieve_wait_events(void) {
  EventPool& P = pool();
  std::lock_guard<std::mutex> lk(P.mu);
  return P.created;
}

size_t cbv2_retrieve_host_bytes(int32_t B, int32_t k, int32_t kb, int32_t C) {
  if (B < 1 || k < 1 || kb < 0 || C < 1) return 0;
  return host_words(B, k, kb, C) * 4;
}

int cbv2_retrieve_begin(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                        int32_t k, int32_t kb, int32_t C, void* workspace, size_t workspace_bytes, void* stream) {
  Kind kd;
  if (int rc = check_common(ix, &kd, c, Q, q_dtype, B, lq, k, kb)) return rc;
  if (C < 1) return err(CBV2_EINVAL, "C must be >= 1 (got %d)", C);
  const Layout L = layout(ix, c, kd, B, lq, k, kb, C, workspace);
  if (!workspace || workspace_bytes < L.total || ((uintptr_t)workspace & 255))
    return err(CBV2_EINVAL, "workspace too small or not 256-B aligned (%zu bytes needed)", L.total);
  DevSel ds(ix);
  if (!ds.ok) return err(CBV2_EHIP, "cannot select the index's device %d", ds.dev);
  if (c)
    return cbv2_search_sharded_local(ix, c, CBV2_SCORER_MAXSIM, Q, q_dtype, B, lq, k, kb, L.base, L.stage2, stream);
  if (kd.faithful)
    return cbv2_search_f32(ix, (const float*)Q, B, lq, k, k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP,
                           L.base, L.stage2, L.s, L.ids, L.status, stream);
  return cbv2_search(ix, CBV2_SCORER_MAXSIM, Q, q_dtype, B, lq, k, L.base, L.stage2, L.s, L.ids, stream);
}

int cbv2_retrieve_finish(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                         int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb, int32_t rrf_k,
                         int32_t C, int32_t final_k, void* workspace, size_t workspace_bytes, void* host_stage,
                         size_t host_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream) {
  Kind kd;
  if (int rc = check_common(ix, &kd, c, Q, q_dtype, B, lq, k, kb)) return rc;
  if (C < 1 || final_k < 1) return err(CBV2_EINVAL, "C and final_k must be >= 1 (got %d, %d)", C, final_k);
  if (kb > 0 && (!lex_ids || (c && !lex_scores))) return err(CBV2_EINVAL, "null stage-1 lists");
  if (!out_scores || !out_ids || !out_pos) return err(CBV2_EINVAL, "null outputs");
  const Layout L = layout(ix, c, kd, B, lq, k, kb, C, workspace);
  if (!workspace || workspace_bytes < L.total || ((uintptr_t)workspace & 255))
    return err(CBV2_EINVAL, "workspace too small or not 256-B aligned (%zu bytes needed)", L.total);
  if (!host_stage || host_bytes < host_words(B, k, kb, C) * 4)
    return err(CBV2_EINVAL, "host stage too small (%zu bytes needed)", host_words(B, k, kb, C) * 4);
  DevSel ds(ix);
  if (!ds.ok) return err(CBV2_EHIP, "cannot select the index's device %d", ds.dev);
  hipStream_t st = (hipStream_t)stream;
  const HostLayout H = host_layout(host_stage, B, k, kb, C);
  const int32_t* bm = lex_ids;   // the stage-1 lists the RRF reads (host)
  int rc;
  if (c) {
    // this rank's BM25 lists ride the stage-2 all-gather (staged in the pinned
    // host buffer, so their H2D is asynchronous); merged lists come back
    if (kb > 0) {
      std::memcpy(H.lex_ids, lex_ids, (size_t)B * kb * 4);
      std::memcpy(H.lex_scores, lex_scores, (size_t)B * kb * 4);
    }
    rc = cbv2_search_sharded_exchange(ix, c, B, k, kb > 0 ? H.lex_ids : nullptr,
                                      kb > 0 ? (const float*)H.lex_scores : nullptr, kb, L.base, L.stage2, L.s,
                                      L.ids, kb > 0 ? L.lex_ids : nullptr, st);
    if (rc) return rc;
    if (kb > 0) RT_HIP(hipMemcpyAsync(H.lex_merged, L.lex_ids, (size_t)B * kb * 4, hipMemcpyDeviceToHost, st));
    bm = H.lex_merged;
  }
  RT_HIP(hipMemcpyAsync(H.ids, L.ids, (size_t)B * k * 4, hipMemcpyDeviceToHost, st));
  // one shard: the fused candidates go to a mapped buffer the rerank reads
  // in place (no H2D launch); sharded: through the device workspace (the
  // exchange's collectives read device memory)
  MappedBuf mb;
  const bool mapped = !c && ds.dev >= 0 && ds.dev < kMaxDev && take_mapped(ds.dev, (size_t)B * C * 4, &mb);
  int32_t* cand_h = mapped ? (int32_t*)mb.h : H.cand;
  const int32_t* cand_d = mapped ? (const int32_t*)mb.d : L.cand;
  rc = wait_copy(st, ds.dev, B);   // the one host round trip: the ColBERT (and merged BM25) top-k are here
  if (!rc) rc = cbv2_rrf_fuse(bm, kb, H.ids, k, B, rrf_k, C, cand_h, nullptr, nullptr);
  if (!rc && !mapped && hipMemcpyAsync(L.cand, H.cand, (size_t)B * C * 4, hipMemcpyHostToDevice, st) != hipSuccess)
    rc = err(CBV2_EHIP, "candidate upload failed");
  if (!rc) {
    if (c)
      rc = cbv2_rerank_sharded(ix, c, Q, B, lq, L.cand, C, final_k, L.rr, L.rerank, out_scores, out_ids, out_pos, st);
    else if (kd.faithful)   // the search's query split (begin, same stream) serves the rerank when it is still there
      rc = cbv2_rerank_f32_after_search(ix, L.base, L.stage2, k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP,
                                        B, lq, cand_d, C, final_k, L.rr, L.rerank, out_scores, out_ids, out_pos,
                                        (const float*)Q, st);
    else
      rc = cbv2_rerank_ws(ix, Q, B, lq, cand_d, C, final_k, L.rr, L.rerank, out_scores, out_ids, out_pos, st);
  }
  if (mapped) give_mapped(ds.dev, mb, st);   // free again once the rerank that reads it ran
  return rc;
}

}  // extern "C"
