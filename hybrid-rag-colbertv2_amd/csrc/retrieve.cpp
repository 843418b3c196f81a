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
#include <climits>
#include <cstring>
#include <algorithm>
#include <limits>
#include <atomic>
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
extern "C" void cbv2_set_ids_mirror(void* p, uint32_t seq, int64_t score_off);
extern "C" int cbv2_ids_mirror_used(void);
extern "C" void cbv2_set_cand_tagged(const void* p, uint32_t seq, void* gate);
extern "C" void cbv2_set_wait_ticks(int64_t ticks);
extern "C" int cbv2_cand_tagged_used(void);
extern "C" void cbv2_set_final_mirror(void* p, uint32_t seq, int32_t k);
extern "C" int cbv2_final_mirror_used(void);
extern "C" void cbv2_set_raw_mirror(void* p, uint32_t seq);
extern "C" void cbv2_set_split_ready(uint32_t seq);
extern "C" void cbv2_set_split_ready_begin(uint32_t seq, void* word);
extern "C" const void* cbv2_last_ready_flag(int64_t* ld);
extern "C" void cbv2_set_prescore_ready(uint32_t seq);
extern "C" int cbv2_raw_mirror_used(void);
extern "C" int cbv2_host_result_copy(const void* words, uint32_t seq, int32_t B, int32_t k, float* out_s, int32_t* out_i,
                                     int32_t* out_p, void* gate, void* stream);

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

// The round trip's wait: poll the stream until the work enqueued on it -- the
// search and the D2H copy (or the ids' host mirror) -- has completed
// (hipStreamQuery), small batches flat out, larger ones sleeping between
// polls.  A blocking hipStreamSynchronize wakes the host tens of microseconds
// after the work lands (measured: 26-39 us from the D2H copy's end to the
// next H2D copy's start); a poll sees it within about a microsecond.  But a
// poll holds a core for as long as the stream runs, so only B <= kSpinMaxB
// (one scan of <= 8 queries: ~5-7 ms at 1M docs, where a wake-up would be
// ~0.5 % of the latency) polls flat out, for at most kSpinNs, then as below;
// larger batches (one B=256 scan: ~140 ms, whose host side runs the BM25
// threads meanwhile) sleep between polls for 1/32 of the time waited so far
// (20 us .. 500 us): the thread wakes at most ~3 % (and 0.5 ms) after the
// work and is asleep otherwise (hipEventSynchronize is no substitute:
// measured on the GPU box, a B=256 call over 200k docs burned its whole 28 ms
// wait on a core even with a hipEventBlockingSync event).
// Small batches poll the stream rather than an event recorded after the copy
// (round 5 lab, profiles/r05/latency_wait_ab.jsonl, same process,
// interleaved): B=1 p50 at a 125k-doc faithful shard 726.1 -> 719.5 us, 1M
// 4713.9 -> 4709.5 -- the event record is a marker packet of its own.  The
// stream must not be shared with other threads' work while finish waits (it
// would wait for theirs too).  Large batches keep the event (below).
constexpr long long kSpinNs = 50LL * 1000 * 1000;
constexpr int32_t kSpinMaxB = 8;
constexpr int kMaxDev = 64;

// Lab knob (cbv2_set_wait_mode, internal): 1 = poll hipStreamQuery (default),
// 0 = record an event after the copy and poll hipEventQuery (round 4's wait).
int g_wait_mode = 1;

int wait_copy(hipStream_t st, int32_t B) {
  hipEvent_t ev = nullptr;
  // large batches poll an event between sleeps: a hipStreamQuery call held
  // the core for the whole wait (measured: a B=256 call over 200k docs used
  // 29 ms of CPU for its 29 ms wait even sleeping between queries)
  if (g_wait_mode == 0 || B > kSpinMaxB) {
    RT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    if (hipEventRecord(ev, st) != hipSuccess) {
      (void)hipEventDestroy(ev);
      return err(CBV2_EHIP, "hipEventRecord failed");
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t q;
  for (;;) {
    q = ev ? hipEventQuery(ev) : hipStreamQuery(st);
    if (q != hipErrorNotReady) break;
    const long long waited =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (B > kSpinMaxB || waited > kSpinNs)   // a long wait: sleep between polls
      std::this_thread::sleep_for(std::chrono::nanoseconds(std::min(500000LL, std::max(20000LL, waited / 32))));
  }
  if (ev) (void)hipEventDestroy(ev);
  return q == hipSuccess ? CBV2_OK : err(CBV2_EHIP, "round-trip wait (%d)", (int)q);
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
  uint32_t seq = 0;   // this buffer's call counter (next_tag: words of older calls carry older tags)
};

// A call's tag in its buffer's words (high half): the buffer's call counter
// with the top bit set.  The calls also leave plain 32-bit data in a pooled
// buffer -- the GPU rerank's candidate ids and the stage-1 ids (int32 >= -1,
// two per word), the raw prescores (floats) -- and a later call with another
// layout may poll words where such data lies: a small counter as the tag
// could equal a stale doc id in a word's high half and pass the check with
// the other id as its value (round-6 soak, tools/stress_onetrip.py: 3-5 in
// 120k calls).  No id, position or MaxSim score has the top bit set with the
// rest below 2^31 - 1 (-0.0 is counter 0, never used; -inf and -1 sit at
// counters no process reaches), so a stale word never passes for a call's.
uint32_t next_tag(MappedBuf& b) {
  b.seq = (b.seq + 1) & 0x7fffffffu;
  if (b.seq == 0) b.seq = 1;
  return 0x80000000u | b.seq;
}
struct MappedPool {
  std::mutex mu;
  std::vector<MappedBuf> free_buf[kMaxDev];
  int64_t created = 0;
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
  std::memset(b.h, 0, b.bytes);   // tag 0 is never a call's
  if (hipHostGetDevicePointer(&b.d, b.h, 0) != hipSuccess ||
      hipEventCreateWithFlags(&b.ev, hipEventDisableTiming) != hipSuccess) {
    (void)hipHostFree(b.h);
    return false;
  }
  {
    std::lock_guard<std::mutex> lk(P.mu);
    ++P.created;
  }
  *out = b;
  return true;
}

// Marks the buffer's last reader (an event after it on st) ...
void mark_mapped(MappedBuf& b, hipStream_t st) {
  b.recorded = hipEventRecord(b.ev, st) == hipSuccess;
  if (!b.recorded) (void)hipStreamSynchronize(st);   // cannot mark the reader: wait for it instead
}
// ... and puts it back in the pool (reusable once that event completed).
void pool_mapped(int dev, const MappedBuf& b) {
  MappedPool& P = mapped_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  P.free_buf[dev].push_back(b);
}
void give_mapped(int dev, MappedBuf b, hipStream_t st) {
  mark_mapped(b, st);
  pool_mapped(dev, b);
}

// begin -> finish: the mapped buffer a one-shard begin took for its call
// ([B][k] ids mirrored by the search's final select | [B][C] fused
// candidates), keyed by the workspace (begin and finish share it).
struct Pending {
  MappedBuf mb;
  bool ids_mirrored = false;
  uint32_t seq = 0;
  uint32_t ready_seq = 0;   // the search's ready-flag value (0: none) ...
  const int32_t* ready = nullptr;   // ... and the host words it wrote it to (ready[0 .. ready_n))
  int32_t ready_n = 0;
};

// Process-wide call tags of the ready flags (never 0): a pooled buffer's flag
// words keep an earlier call's tag, which never equals a later call's.
std::atomic<uint32_t> g_ready_seq{0};
uint32_t next_ready_seq() {
  uint32_t v = g_ready_seq.fetch_add(1, std::memory_order_relaxed) + 1;
  if (v == 0) v = g_ready_seq.fetch_add(1, std::memory_order_relaxed) + 1;
  return v;
}

// The host rerank's second stream (per host thread and device; never
// destroyed, like the mapped buffers): the stage-1 prescore runs on it
// concurrently with stage 2's scan instead of after it.
// High priority: its queue's workgroups are dispatched ahead of the scan's
// (lab: at normal priority they waited for the scan's own to retire).
hipStream_t side_stream(int dev) {
  thread_local hipStream_t s[kMaxDev] = {};
  if (dev < 0 || dev >= kMaxDev) return nullptr;
  if (s[dev] == nullptr) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&s[dev], hipStreamNonBlocking, greatest) != hipSuccess)
      s[dev] = nullptr;
  }
  return s[dev];
}
std::mutex g_pending_mu;
std::vector<std::pair<const void*, Pending>> g_pending;

void put_pending(const void* ws, const Pending& p, int dev, hipStream_t st) {
  Pending old;
  bool had = false;
  {
    std::lock_guard<std::mutex> lk(g_pending_mu);
    for (auto& e : g_pending)
      if (e.first == ws) {
        old = e.second;
        e.second = p;
        had = true;
        break;
      }
    if (!had) g_pending.emplace_back(ws, p);
  }
  if (had) give_mapped(dev, old.mb, st);   // a begin without its finish: the buffer goes back
}

bool take_pending(const void* ws, Pending* out) {
  std::lock_guard<std::mutex> lk(g_pending_mu);
  for (size_t i = 0; i < g_pending.size(); ++i)
    if (g_pending[i].first == ws) {
      *out = g_pending[i].second;
      g_pending.erase(g_pending.begin() + (long)i);
      return true;
    }
  return false;
}

// Host marks of this thread's last cbv2_retrieve_finish (steady_clock ns,
// CLOCK_MONOTONIC on Linux): [0] enter, [1] D2H issued, [2] wait done, [3]
// fusion done, [4] rerank enqueued, [5] exit (cbv2_retrieve_host_marks; the
// latency lab lines them up with a kernel trace).
thread_local int64_t t_marks[6] = {};
inline int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
inline void mark(int i) { t_marks[i] = now_ns(); }

// Lab probe of begin (cbv2_set_begin_probe / cbv2_retrieve_begin_marks,
// internal; off by default): [0] begin entered, [1] the search returned
// (every launch enqueued), [2] the host saw the search's ready flags (the
// first kernel's last store: an upper bound, with no profiler attached, on
// when the first kernel ran), 0 where not taken.  On, begin polls for the
// flags before it returns -- a latency lab's knob, never the product's.
thread_local int32_t t_begin_probe = 0;
thread_local int64_t t_begin_marks[3] = {};

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
  else if (kd.faithful)   // (C or kb: the host rerank's stage-1 prescore rescores kb per row in it)
    L.rerank = a256(cbv2_f32_workspace_bytes(ix, CBV2_F32_RERANK, B, lq, kb > C ? kb : C));
  else
    L.rerank = a256(cbv2_rerank_workspace_bytes(B, kb > C ? kb : C));
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

// Stage 3 of one call: the sharded one (the fused candidates' scores looked
// up in the exchange's gathered blocks: no collective; kb = this call's
// stage-1 width, as the exchange laid out the workspace), the faithful
// rerank on begin's query split, or the bf16 / MXFP8 one.
int rerank_call(cbv2_index* ix, cbv2_comm* c, Kind kd, const void* Q, int32_t B, int32_t lq, int32_t k,
                int32_t kb, const Layout& L, const int32_t* cand, int32_t C, int32_t final_k, float* out_scores,
                int32_t* out_ids, int32_t* out_pos, hipStream_t st) {
  if (c)
    return C <= 1024 ? cbv2_rerank_sharded_prescored(ix, c, B, k, kb, cand, C, final_k, L.base, L.stage2, out_scores,
                                                     out_ids, out_pos, nullptr, st)
                     : cbv2_rerank_sharded(ix, c, Q, B, lq, cand, C, final_k, L.rr, L.rerank, out_scores, out_ids,
                                           out_pos, st);
  if (kd.faithful)   // the search's query split (begin, same stream) serves the rerank when it is still there
    return cbv2_rerank_f32_after_search(ix, L.base, L.stage2, k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP,
                                        B, lq, cand, C, final_k, L.rr, L.rerank, out_scores, out_ids, out_pos,
                                        (const float*)Q, st);
  return cbv2_rerank_ws(ix, Q, B, lq, cand, C, final_k, L.rr, L.rerank, out_scores, out_ids, out_pos, st);
}

// finish_host calls whose results came from the final select's host words
// (cbv2_retrieve_pool_stats [2]: the tests check that path is the one taken)
std::atomic<int64_t> g_final_words_calls{0};
// ... and finish calls that took the host rerank (cbv2_retrieve_pool_stats [3])
std::atomic<int64_t> g_host_rerank_calls{0};

// Lab knob (cbv2_set_prearm, internal): 0 = the rerank is launched after the
// fusion (no tagged candidates), 1 = pre-armed (default).
int g_prearm = 1;

// Polls the call's tagged words until every one carries seq (a kernel on
// stream st writes them; written whole, in any order).  No wall-clock
// deadline (a call queued behind other work, or on a shared GPU, is slow,
// not failed): flat out for kSpinNs, then sleeping between polls (1/32 of the
// time waited, 20-500 us) and asking the stream -- an error on it fails the
// call, and a stream that completed without writing every word too.
int wait_words(const uint64_t* w, size_t n, uint32_t seq, hipStream_t st, const char* what = "stage-2 results") {
  const volatile uint64_t* vw = w;
  const auto t0 = std::chrono::steady_clock::now();
  bool drained = false;   // the stream had completed at the last query
  for (size_t i = 0; i < n;) {
    if ((uint32_t)(vw[i] >> 32) == seq) {
      ++i;
      continue;
    }
    if (drained) return err(CBV2_EHIP, "%s: the stream completed without writing them", what);
    const long long waited =
        std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    if (waited <= kSpinNs) continue;
    std::this_thread::sleep_for(std::chrono::nanoseconds(std::min(500000LL, std::max(20000LL, waited / 32))));
    const hipError_t q = hipStreamQuery(st);
    if (q == hipSuccess) {
      std::atomic_thread_fence(std::memory_order_acquire);
      drained = true;   // every word must be there now: one more pass decides
    } else if (q != hipErrorNotReady) {
      return err(CBV2_EHIP, "%s: stream error while waiting (%d)", what, (int)q);
    }
  }
  return CBV2_OK;
}

// The host's side of the wait gate of the in-kernel waits on host words
// (colbert_mi355x.hip, TaggedCand): the host's word, a seq_cst fence, the
// kernels' word.  true = no kernel gave up before this commit, so every
// waiting kernel takes the words the host publishes next; false = one gave
// up (its outputs are -inf / -1): the call must fail.
bool gate_commit(uint64_t* gate, uint32_t seq) {
  const uint64_t t = ((uint64_t)seq << 32) | 1u;
  __atomic_store_n(gate + 1, t, __ATOMIC_SEQ_CST);
  __atomic_thread_fence(__ATOMIC_SEQ_CST);
  return __atomic_load_n(gate, __ATOMIC_SEQ_CST) != t;
}

// Lab knob (cbv2_set_wait_lab, this thread): the host sleeps this long before
// it commits and publishes the words a kernel waits for (with a short
// in-kernel bound, the tests force each device-side timeout once).
thread_local int32_t t_lab_publish_delay_us = 0;
void lab_publish_delay() {
  if (t_lab_publish_delay_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(t_lab_publish_delay_us));
}

// A one-shard call's mapped buffer, in 8-byte words: [B][k] stage-2 id words
// | [B][k] their score words | [B][C] fused candidate words | [B][3 fk] final
// words | [B][kb] stage-1 prescore words | [B][kb] stage-1 ids (int32) +
// [B][kb] raw prescores (float), one word per pair | ... | the wait gate (2
// words) | the search's ready flags (int32, row b's at the last B words'
// first int) at the buffer's end.
size_t mapped_words(int32_t B, int32_t k, int32_t C, int32_t fk, int32_t kb) {
  return (size_t)B * (2 * (size_t)k + (size_t)C + 3 * (size_t)fk + 2 * (size_t)kb + 1) + 2;
}
size_t ready_word_off(const MappedBuf& b, int32_t B) { return b.bytes / 8 - (size_t)B; }   // in 8-byte words
size_t gate_word_off(const MappedBuf& b, int32_t B) { return ready_word_off(b, B) - 2; }

// Whether the search has published its ready flags (every one reads seq),
// polled for at most bound: the stage-1 prescore may then run on the second
// stream (what it reads is complete) with no wait of its own in the kernel.
bool flags_seen(const int32_t* f, int32_t n, uint32_t seq, std::chrono::microseconds bound) {
  const volatile int32_t* vf = f;
  const auto t0 = std::chrono::steady_clock::now();
  for (int32_t i = 0; i < n;) {
    if ((uint32_t)vf[i] == seq) {
      ++i;
      continue;
    }
    if (std::chrono::steady_clock::now() - t0 > bound) return false;
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return true;
}

constexpr int kHostRerankDeclined = 1;   // host_rerank: not taken, nothing enqueued

// Lab knob (cbv2_set_host_rerank, internal): 1 = the host rerank (default),
// 0 = the GPU rerank after the fusion (pre-armed or launched), 2 = the host
// rerank with its prescore behind the search on the call's stream (the path
// a late ready flag takes; the tests pin it).
int g_host_rerank = 1;

// The host rerank's select of one row: the C fused candidates' scores (stage
// 2's for its own ids, stage 1's prescore for the others), the best fk by
// (score desc, position asc) -- select_from_lds's keys and tie rule.
inline uint32_t key_bits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
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

int cbv2_retrieve_host_marks(int64_t* out, int32_t max) {
  if (!out || max < 0) return err(CBV2_EINVAL, "null output");
  for (int i = 0; i < 6 && i < max; ++i) out[i] = t_marks[i];
  return CBV2_OK;
}

void cbv2_set_wait_mode(int32_t mode) { g_wait_mode = mode; }
// Lab knob (tests): this thread's in-kernel wait bound (ticks of 10 ns; < 0
// the default 1 s, 0 give up at once) and the host's delay before it
// publishes what those kernels wait for.
void cbv2_set_wait_lab(int64_t ticks, int32_t publish_delay_us) {
  cbv2_set_wait_ticks(ticks);
  t_lab_publish_delay_us = publish_delay_us;
}
void cbv2_set_host_rerank(int32_t on) { g_host_rerank = on; }
void cbv2_set_prearm(int32_t on) { g_prearm = on; }
void cbv2_set_begin_probe(int32_t on) { t_begin_probe = on; }
int cbv2_retrieve_begin_marks(int64_t* out, int32_t max) {
  if (!out || max < 0) return err(CBV2_EINVAL, "null output");
  for (int i = 0; i < 3 && i < max; ++i) out[i] = t_begin_marks[i];
  return CBV2_OK;
}

int cbv2_retrieve_cancel(cbv2_index* ix, void* workspace, void* stream) {
  if (!ix) return err(CBV2_EINVAL, "null index");
  Pending pd;
  if (!take_pending(workspace, &pd)) return CBV2_OK;   // nothing outstanding (sharded, or finished)
  DevSel ds(ix);
  if (!ds.ok) return err(CBV2_EHIP, "cannot select the index's device %d", ds.dev);
  give_mapped(ds.dev, pd.mb, (hipStream_t)stream);      // reusable once begin's search has run
  return CBV2_OK;
}

int cbv2_retrieve_pool_stats(int64_t* out, int32_t max) {
  if (!out || max < 0) return err(CBV2_EINVAL, "null output");
  MappedPool& P = mapped_pool();
  std::lock_guard<std::mutex> lk(P.mu);
  if (max > 0) out[0] = P.created;
  if (max > 1) {
    int64_t idle = 0;
    for (int d = 0; d < kMaxDev; ++d) idle += (int64_t)P.free_buf[d].size();
    out[1] = idle;
  }
  if (max > 2) out[2] = g_final_words_calls.load(std::memory_order_relaxed);
  if (max > 3) out[3] = g_host_rerank_calls.load(std::memory_order_relaxed);
  return CBV2_OK;
}

size_t cbv2_retrieve_host_bytes(int32_t B, int32_t k, int32_t kb, int32_t C) {
  if (B < 1 || k < 1 || kb < 0 || C < 1) return 0;
  return host_words(B, k, kb, C) * 4;
}

int cbv2_retrieve_begin(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                        int32_t k, int32_t kb, int32_t C, void* workspace, size_t workspace_bytes, void* stream) {
  if (t_begin_probe) t_begin_marks[0] = now_ns(), t_begin_marks[1] = t_begin_marks[2] = 0;
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
  // one shard: a mapped host buffer for this call -- the search's final select
  // mirrors the ids into it (no D2H copy in finish) and the fusion writes the
  // candidates the rerank reads from it
  Pending pd;
  const bool mapped =
      ds.dev >= 0 && ds.dev < kMaxDev && take_mapped(ds.dev, mapped_words(B, k, C, C, kb) * 8, &pd.mb);
  if (mapped) {
    pd.seq = next_tag(pd.mb);
  }
  // small batches on bf16 / faithful shards (the host rerank's candidates):
  // the stage-2 ids and, B * k words further, their scores; the search's
  // first launch publishes ready flags to the buffer's end (once the host has
  // seen them, the stage-1 prescore can read the queries from another stream)
  const bool host_rr = mapped && B <= kSpinMaxB && (kd.faithful || kd.dtype == CBV2_DTYPE_BF16);
  if (host_rr) {   // a pooled buffer's flag slots may hold any earlier call's words: cleared before the search
    volatile uint64_t* fl = (uint64_t*)pd.mb.h + ready_word_off(pd.mb, B);
    for (int32_t b = 0; b < B; ++b) fl[b] = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
  }
  cbv2_set_ids_mirror(mapped ? pd.mb.d : nullptr, pd.seq, host_rr ? (int64_t)B * k : 0);
  pd.ready_seq = host_rr ? next_ready_seq() : 0;
  cbv2_set_split_ready_begin(pd.ready_seq, host_rr ? (uint64_t*)pd.mb.d + ready_word_off(pd.mb, B) : nullptr);
  int rc;
  if (kd.faithful)
    rc = cbv2_search_f32(ix, (const float*)Q, B, lq, k, k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP,
                         L.base, L.stage2, L.s, L.ids, L.status, stream);
  else
    rc = cbv2_search(ix, CBV2_SCORER_MAXSIM, Q, q_dtype, B, lq, k, L.base, L.stage2, L.s, L.ids, stream);
  if (t_begin_probe) t_begin_marks[1] = now_ns();
  int64_t ld = 0;
  if (cbv2_last_ready_flag(&ld) != nullptr) {   // one flag per row (ld 1) or one for all (ld 0)
    pd.ready = (const int32_t*)((const uint64_t*)pd.mb.h + ready_word_off(pd.mb, B));
    pd.ready_n = ld != 0 ? B : 1;
    if (t_begin_probe && rc == CBV2_OK &&
        flags_seen(pd.ready, pd.ready_n, pd.ready_seq, std::chrono::microseconds(2000)))
      t_begin_marks[2] = now_ns();
  } else {
    pd.ready_seq = 0;   // this search's path wrote no flag: the GPU rerank
  }
  cbv2_set_split_ready(0);
  pd.ids_mirrored = mapped && cbv2_ids_mirror_used() != 0;
  cbv2_set_ids_mirror(nullptr, 0, 0);
  if (mapped) {
    if (rc == CBV2_OK)
      put_pending(workspace, pd, ds.dev, (hipStream_t)stream);
    else
      give_mapped(ds.dev, pd.mb, (hipStream_t)stream);
  }
  return rc;
}

}  // extern "C"

namespace {
// The host rerank of one-shard small batches (finish_impl): the stage-1
// prescore and the device outputs' copy enqueued first (the copy polls the
// final words the host writes at the end), then the round trip's wait (the
// stage-2 id and score words, the prescore words), the RRF, and per row the
// select over the candidates' known scores.  Marks the mapped buffer after
// its last reader; the caller pools it.
int host_rerank(cbv2_index* ix, Kind kd, const void* Q, int32_t B, int32_t lq, int32_t k, const int32_t* lex_ids,
                int32_t kb, int32_t rrf_k, int32_t C, int32_t fk, const Layout& L, Pending& pd, float* out_scores,
                int32_t* out_ids, int32_t* out_pos, hipStream_t st, float* host_s, int32_t* host_i, int32_t* host_p) {
  const size_t Bk = (size_t)B * k, Bkb = (size_t)B * kb;
  uint64_t* const idw = (uint64_t*)pd.mb.h;
  uint64_t* const sw = idw + Bk;
  uint64_t* const fw = sw + Bk + (size_t)B * C;
  uint64_t* const lxw = fw + (size_t)3 * B * fk;
  int32_t* const lxi = (int32_t*)(lxw + Bkb);
  auto dev = [&](const void* h) { return (uint8_t*)pd.mb.d + ((const uint8_t*)h - (const uint8_t*)pd.mb.h); };
  uint64_t* const gate = (uint64_t*)pd.mb.h + gate_word_off(pd.mb, B);
  int rc = CBV2_OK;
  hipStream_t pre = st;   // the stream the stage-1 prescore went to
  // 1. stage 1's prescore: the rerank's raw scores of the whole stage-1 list
  if (kb > 0) {
    std::memcpy(lxi, lex_ids, Bkb * 4);
    cbv2_set_raw_mirror(dev(lxw), pd.seq);
    const int32_t* lxi_d = (const int32_t*)dev(lxi);
    float* lxf_d = (float*)dev(lxi + Bkb);
    // on the second stream once the host has seen the search's ready flags
    // (the search is then past its first launch: the queries and their split
    // are complete), so it runs while stage 2 scans; else after the search on
    // its own stream.  No kernel waits for another stream's (an in-kernel
    // wait there can hold the CUs the awaited kernel needs).  Everything it
    // reads or writes is done when the host has seen its last word (each
    // workgroup's word is its last store), so neither stream waits for the
    // other.  The bound costs no latency: a flag still missing means stage
    // 2's scan has not started, and the host waits for its results anyway.
    const bool seen =
        g_host_rerank != 2 && flags_seen(pd.ready, pd.ready_n, pd.ready_seq, std::chrono::microseconds(2000));
    cbv2_set_prescore_ready(pd.ready_seq);
    hipStream_t side = seen ? side_stream(cbv2_index_device(ix)) : st;
    pre = side;
    rc = kd.faithful ? cbv2_rerank_f32_after_search(ix, L.base, L.stage2,
                                                    k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP, B, lq,
                                                    lxi_d, kb, 0, L.rr, L.rerank, lxf_d, nullptr, nullptr,
                                                    (const float*)Q, side)
                     : cbv2_rerank_ws(ix, Q, B, lq, lxi_d, kb, 0, L.rr, L.rerank, lxf_d, nullptr, nullptr, side);
    cbv2_set_prescore_ready(0);
    const bool used = cbv2_raw_mirror_used() != 0;
    cbv2_set_raw_mirror(nullptr, 0);
    // refused before anything was enqueued (the workspace holds another
    // split: the stage-1 callable searched into it): the caller takes the
    // GPU rerank instead
    if (rc == CBV2_ESTATE) return kHostRerankDeclined;
    if (!rc && !used) rc = err(CBV2_ESTATE, "stage-1 prescore without host words");
  }
  // 2. the device outputs: a copy launched now, polling the final words
  if (!rc) rc = cbv2_host_result_copy(dev(fw), pd.seq, B, fk, out_scores, out_ids, out_pos, dev(gate), st);
  const bool copy_armed = rc == CBV2_OK;
  mark_mapped(pd.mb, st);   // every reader of the buffer is enqueued
  mark(1);
  // 3. the round trip: stage 2's ids and scores, stage 1's prescores
  if (!rc) rc = wait_words(idw, 2 * Bk, pd.seq, st);
  if (!rc && kb > 0) rc = wait_words(lxw, Bkb, pd.seq, pre, "stage-1 prescores");
  mark(2);
  thread_local std::vector<int32_t> ids_s, cand_s;
  ids_s.resize(Bk);
  cand_s.resize((size_t)B * C);
  if (!rc) {
    for (size_t i = 0; i < Bk; ++i) ids_s[i] = (int32_t)(uint32_t)idw[i];
    rc = cbv2_rrf_fuse(lex_ids, kb, ids_s.data(), k, B, rrf_k, C, cand_s.data(), nullptr, nullptr);
  }
  mark(3);
  // 4. per row: the candidates' scores (id -> score by open addressing over
  //    the row's stage-2 and stage-1 lists), the best fk of them
  const uint64_t tag = (uint64_t)pd.seq << 32;
  volatile uint64_t* const vf = fw;
  const float ninf = -std::numeric_limits<float>::infinity();
  uint32_t ninf_bits;
  std::memcpy(&ninf_bits, &ninf, 4);
  // a failed call: the prescore on the second stream may still read the
  // buffer (and Q): the call's stream waits for it before the buffer is
  // marked free again
  auto fence_side = [&]() {
    if (kb <= 0 || pre == st) return;
    thread_local hipEvent_t ev[kMaxDev] = {};
    const int d = cbv2_index_device(ix);
    if (d < 0 || d >= kMaxDev) return;
    if ((ev[d] == nullptr && hipEventCreateWithFlags(&ev[d], hipEventDisableTiming) != hipSuccess) ||
        hipEventRecord(ev[d], pre) != hipSuccess || hipStreamWaitEvent(st, ev[d], 0) != hipSuccess)
      (void)hipStreamSynchronize(pre);
    mark_mapped(pd.mb, st);
  };
  if (rc) {   // the armed copy must not wait for its timeout: publish -inf / -1
    if (copy_armed)
      for (size_t i = 0; i < (size_t)3 * B * fk; ++i)
        vf[i] = tag | ((i / fk) % 3 == 0 ? ninf_bits : 0xffffffffu);
    fence_side();
    return rc;
  }
  lab_publish_delay();
  // the copy kernel's wait gate: committed before the first final word (below)
  const bool gate_ok = gate_commit(gate, pd.seq);
  int bits = 4;
  while ((1 << bits) < 2 * (k + kb)) ++bits;
  const uint32_t hmask = (1u << bits) - 1;
  thread_local std::vector<int32_t> tab_id;
  thread_local std::vector<float> tab_sc;
  thread_local std::vector<uint32_t> used;
  thread_local std::vector<uint64_t> keys;
  thread_local std::vector<int> order;
  tab_id.assign((size_t)hmask + 1, INT32_MIN);
  tab_sc.resize((size_t)hmask + 1);
  keys.resize((size_t)C);
  order.resize((size_t)C);
  for (int32_t b = 0; b < B && !rc; ++b) {
    for (uint32_t h : used) tab_id[h] = INT32_MIN;
    used.clear();
    auto put = [&](int32_t id, uint64_t word) {
      if (id < 0) return;
      uint32_t h = ((uint32_t)id * 2654435761u) >> (32 - bits);
      for (; tab_id[h] != INT32_MIN; h = (h + 1) & hmask)
        if (tab_id[h] == id) return;   // already there (the same score: the same doc's MaxSim)
      tab_id[h] = id;
      const uint32_t sb = (uint32_t)word;
      std::memcpy(&tab_sc[h], &sb, 4);
      used.push_back(h);
    };
    for (int32_t j = 0; j < k; ++j) put(ids_s[(size_t)b * k + j], sw[(size_t)b * k + j]);
    for (int32_t j = 0; j < kb; ++j) put(lex_ids[(size_t)b * kb + j], lxw[(size_t)b * kb + j]);
    for (int32_t t = 0; t < C; ++t) {
      const int32_t id = cand_s[(size_t)b * C + t];
      float v = ninf;
      if (id >= 0) {
        uint32_t h = ((uint32_t)id * 2654435761u) >> (32 - bits);
        while (tab_id[h] != INT32_MIN && tab_id[h] != id) h = (h + 1) & hmask;
        if (tab_id[h] != id) {
          rc = err(CBV2_ESTATE, "fused candidate %d is in neither list", id);
          break;
        }
        v = tab_sc[h];
      }
      keys[t] = ((uint64_t)key_bits(v) << 32) | (uint32_t)~(uint32_t)t;
      order[t] = t;
    }
    if (rc) break;
    const int m = fk < C ? fk : C;
    std::partial_sort(order.begin(), order.begin() + m, order.end(), [&](int x, int y) { return keys[x] > keys[y]; });
    volatile uint64_t* row = vf + (size_t)b * 3 * fk;
    for (int32_t r = 0; r < fk; ++r) {
      const int t = r < m ? order[r] : -1;
      const uint32_t sb = t >= 0 ? (uint32_t)(keys[t] >> 32) : key_bits(ninf);
      const uint32_t vb = (sb & 0x80000000u) ? (sb & 0x7fffffffu) : ~sb;   // back from the key to the float bits
      const int32_t id = t >= 0 ? cand_s[(size_t)b * C + t] : -1;
      if (host_s) {
        std::memcpy(host_s + (size_t)b * fk + r, &vb, 4);
        host_i[(size_t)b * fk + r] = id;
        host_p[(size_t)b * fk + r] = t;
      }
      row[r] = tag | vb;
      row[fk + r] = tag | (uint32_t)id;
      row[2 * (size_t)fk + r] = tag | (uint32_t)t;
    }
  }
  if (rc)   // (a row failed: every word still gets published)
    for (size_t i = 0; i < (size_t)3 * B * fk; ++i) vf[i] = tag | ((i / fk) % 3 == 0 ? ninf_bits : 0xffffffffu);
  else if (!gate_ok)
    rc = err(CBV2_EHIP, "the device copy of the results gave up its wait before the host published them "
                        "(device outputs are -inf / -1)");
  else
    g_host_rerank_calls.fetch_add(1, std::memory_order_relaxed);
  mark(4);   // (the GPU rerank's "rerank enqueued" slot: the host select published)
  return rc;
}

// finish; host_s (nullable): the final top-k also to the host arrays host_s /
// host_i / host_p ([B][final_k]) before the call returns -- read from the
// final select's tagged words when it wrote them (one-shard calls), else
// copied down and waited for
int finish_impl(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq, int32_t k,
                const int32_t* lex_ids, const float* lex_scores, int32_t kb, int32_t rrf_k, int32_t C,
                int32_t final_k, void* workspace, size_t workspace_bytes, void* host_stage, size_t host_bytes,
                float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream, float* host_s,
                int32_t* host_i, int32_t* host_p) {
  mark(0);
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
    // (with Q: this rank's BM25 top-kb prescored before the all-gather, so
    // stage 3 needs no collective -- cbv2_rerank_sharded_prescored)
    rc = cbv2_search_sharded_exchange(ix, c, Q, q_dtype, lq, B, k, kb > 0 ? H.lex_ids : nullptr,
                                      kb > 0 ? (const float*)H.lex_scores : nullptr, kb, L.base, L.stage2, L.s,
                                      L.ids, kb > 0 ? L.lex_ids : nullptr, st);
    if (rc) return rc;
    if (kb > 0) RT_HIP(hipMemcpyAsync(H.lex_merged, L.lex_ids, (size_t)B * kb * 4, hipMemcpyDeviceToHost, st));
    bm = H.lex_merged;
  }
  // one shard: the mapped buffer begin took -- the ids are already mirrored
  // into it by the search's select (else copied down as for the sharded
  // path), the fused candidates go into it and the rerank reads them in place
  // (no H2D launch); sharded: through the device workspace (the exchange's
  // collectives read device memory)
  Pending pd;
  const bool mapped = !c && take_pending(workspace, &pd);
  // the call's tagged words in the mapped buffer (mapped_words): [B][k]
  // stage-2 ids and [B][k] their scores (the search's select wrote them,
  // ids_mirrored) | [B][C] fused candidates | [B][3 final_k] final result | ...
  uint64_t* const idw = mapped ? (uint64_t*)pd.mb.h : nullptr;
  uint64_t* const cw = mapped ? idw + 2 * (size_t)B * k : nullptr;
  const uint64_t* const cwd = mapped ? (const uint64_t*)pd.mb.d + 2 * (size_t)B * k : nullptr;
  const bool mirrored = mapped && pd.ids_mirrored;
  // small batches on bf16 / faithful shards: the host rerank -- every fused
  // candidate's rerank score is stage 2's own (the same MaxSim of the same
  // doc, bit for bit) or, for stage-1-only candidates, the prescore of the
  // whole stage-1 list enqueued now (it runs right after stage 2 on the
  // stream, while the host waits and fuses), so the top final_k is picked
  // on the host: no rerank launch after the fusion, no round trip back
  if (mirrored && g_host_rerank && B <= kSpinMaxB && (kd.faithful || kd.dtype == CBV2_DTYPE_BF16) &&
      pd.ready_seq != 0 &&
      mapped_words(B, k, C, final_k, kb) * 8 <= pd.mb.bytes && side_stream(ds.dev) != nullptr) {
    rc = host_rerank(ix, kd, Q, B, lq, k, lex_ids, kb, rrf_k, C, final_k, L, pd, out_scores, out_ids, out_pos, st,
                     host_s, host_i, host_p);
    if (rc != kHostRerankDeclined) {
      pool_mapped(ds.dev, pd.mb);   // (marked by host_rerank after its last reader)
      mark(5);
      return rc;
    }
    rc = CBV2_OK;
  }
  // small batches pre-arm the rerank: it is launched now, before the wait,
  // and polls its candidates' words (the host writes them after the fusion),
  // so the host -> GPU hop after the fusion is a PCIe read, not a launch
  const bool prearm = mirrored && g_prearm && B <= kSpinMaxB && (kd.faithful || kd.dtype == CBV2_DTYPE_BF16);
  // host results: the final select's words after the candidate words, when the
  // buffer holds them (pool buffers are >= 64 KiB)
  const size_t fin_words = (size_t)3 * B * final_k;
  uint64_t* const fw = mapped && host_s && ((size_t)B * (2 * (size_t)k + C) + fin_words) * 8 <= pd.mb.bytes
                           ? cw + (size_t)B * C : nullptr;
  uint64_t* const fwd = fw ? (uint64_t*)pd.mb.d + (size_t)B * (2 * (size_t)k + C) : nullptr;
  bool fin_used = false;
  rc = CBV2_OK;
  if (!mirrored && hipMemcpyAsync(H.ids, L.ids, (size_t)B * k * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
    rc = err(CBV2_EHIP, "stage-2 ids copy failed");
  mark(1);
  bool armed = false;
  uint64_t* const gate = mapped ? (uint64_t*)pd.mb.h + gate_word_off(pd.mb, B) : nullptr;
  if (!rc && prearm) {
    cbv2_set_cand_tagged(cwd, pd.seq, (uint64_t*)pd.mb.d + gate_word_off(pd.mb, B));
    if (fwd) cbv2_set_final_mirror(fwd, pd.seq, final_k);
    rc = rerank_call(ix, c, kd, Q, B, lq, k, kb, L, L.cand, C, final_k, out_scores, out_ids, out_pos, st);
    armed = cbv2_cand_tagged_used() != 0;   // else it read L.cand (any ids are range-checked): rerun below
    fin_used = armed && fwd && cbv2_final_mirror_used() != 0;
    cbv2_set_cand_tagged(nullptr, 0, nullptr);
    cbv2_set_final_mirror(nullptr, 0, 0);
  }
  // the one host round trip: the ColBERT (and merged BM25) top-k are here
  if (!rc) rc = mirrored && B <= kSpinMaxB ? wait_words(idw, (size_t)B * k, pd.seq, st) : wait_copy(st, B);
  mark(2);
  thread_local std::vector<int32_t> ids_s, cand_s;
  const int32_t* ids_h = H.ids;
  if (mirrored && !rc) {   // the ids out of their words (complete: polled, or the stream has run)
    ids_s.resize((size_t)B * k);
    for (size_t i = 0; i < ids_s.size(); ++i) ids_s[i] = (int32_t)(uint32_t)idw[i];
    ids_h = ids_s.data();
  }
  int32_t* cand_h = H.cand;
  if (mapped) {
    cand_s.resize((size_t)B * C);
    cand_h = cand_s.data();
  }
  if (!rc) rc = cbv2_rrf_fuse(bm, kb, ids_h, k, B, rrf_k, C, cand_h, nullptr, nullptr);
  mark(3);
  if (armed) {   // always publish, failed or not: the armed rerank must not wait for its timeout
    if (!rc) {
      lab_publish_delay();
      if (!gate_commit(gate, pd.seq))
        rc = err(CBV2_EHIP, "the pre-armed rerank gave up its wait before the host published the candidates "
                            "(device outputs are invalid)");
    }
    const uint64_t tag = (uint64_t)pd.seq << 32;
    volatile uint64_t* vw = cw;
    for (size_t i = 0; i < (size_t)B * C; ++i) vw[i] = tag | (uint32_t)(rc ? -1 : cand_h[i]);
  } else if (!rc) {
    const int32_t* cand_d = L.cand;
    if (mapped) {   // plain ids in the buffer's candidate words, read in place by the rerank
      int32_t* ci = (int32_t*)cw;
      std::memcpy(ci, cand_h, (size_t)B * C * 4);
      cand_d = (const int32_t*)cwd;
    } else if (hipMemcpyAsync(L.cand, H.cand, (size_t)B * C * 4, hipMemcpyHostToDevice, st) != hipSuccess) {
      rc = err(CBV2_EHIP, "candidate upload failed");
    }
    if (!rc) {
      if (fwd) cbv2_set_final_mirror(fwd, pd.seq, final_k);
      rc = rerank_call(ix, c, kd, Q, B, lq, k, kb, L, cand_d, C, final_k, out_scores, out_ids, out_pos, st);
      fin_used = fwd && cbv2_final_mirror_used() != 0;
      cbv2_set_final_mirror(nullptr, 0, 0);
    }
  }
  mark(4);
  if (mapped) mark_mapped(pd.mb, st);   // free again once the rerank that reads it ran ...
  if (!rc && host_s) {
    const size_t n = (size_t)B * final_k;
    if (fin_used) {   // the final select's words, row by row: [k] scores | [k] ids | [k] positions
      rc = wait_words(fw, fin_words, pd.seq, st, "final results");
      if (!rc) g_final_words_calls.fetch_add(1, std::memory_order_relaxed);
      for (size_t i = 0; !rc && i < n; ++i) {
        const uint64_t* row = fw + (i / final_k) * 3 * final_k;
        const size_t r = i % final_k;
        const uint32_t sb = (uint32_t)row[r];
        std::memcpy(host_s + i, &sb, 4);
        host_i[i] = (int32_t)(uint32_t)row[final_k + r];
        host_p[i] = (int32_t)(uint32_t)row[2 * final_k + r];
      }
    } else if (hipMemcpyAsync(host_s, out_scores, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(host_i, out_ids, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipMemcpyAsync(host_p, out_pos, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess) {
      rc = err(CBV2_EHIP, "final results copy failed");
    } else {
      rc = wait_copy(st, B);
    }
  }
  if (mapped) pool_mapped(ds.dev, pd.mb);   // ... and not before its host words were read
  mark(5);
  return rc;
}
}  // namespace

extern "C" {

int cbv2_retrieve_finish(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                         int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb, int32_t rrf_k,
                         int32_t C, int32_t final_k, void* workspace, size_t workspace_bytes, void* host_stage,
                         size_t host_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream) {
  return finish_impl(ix, c, Q, q_dtype, B, lq, k, lex_ids, lex_scores, kb, rrf_k, C, final_k, workspace,
                     workspace_bytes, host_stage, host_bytes, out_scores, out_ids, out_pos, stream, nullptr, nullptr,
                     nullptr);
}

int cbv2_retrieve_finish_host(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                              int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb, int32_t rrf_k,
                              int32_t C, int32_t final_k, void* workspace, size_t workspace_bytes, void* host_stage,
                              size_t host_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                              float* host_scores, int32_t* host_ids, int32_t* host_pos, void* stream) {
  if (!host_scores || !host_ids || !host_pos) return err(CBV2_EINVAL, "null host outputs");
  return finish_impl(ix, c, Q, q_dtype, B, lq, k, lex_ids, lex_scores, kb, rrf_k, C, final_k, workspace,
                     workspace_bytes, host_stage, host_bytes, out_scores, out_ids, out_pos, stream, host_scores,
                     host_ids, host_pos);
}

}  // extern "C"
