// sharded.cpp — the multi-GPU exchange behind the C ABI (SURVEY.md §8(b),(e)):
// cbv2_comm_init borrows an initialised RCCL communicator (e.g. the one
// torch.distributed's "nccl" backend created: ProcessGroupNCCL._comm_ptr()),
// and the stages run with ONE collective in all, everything enqueued on the
// caller's stream:
//
//   search:  local scan + top-k written straight into this rank's send block
//            [scores B*k | ids B*k | bm25 scores B*kb | bm25 ids B*kb |
//             bm25 prescores B*kb]  (the prescores: the rerank's raw scores
//            of the rank's own BM25 top-kb, scored before the all-gather)
//            -> ncclAllGather of the blocks -> HIP merge (score desc, id asc)
//            of the G stage-2 lists and of the G stage-1 lists.
//   rerank:  cbv2_rerank_sharded_prescored (no collective): every fused
//            candidate is in a stage-2 list or a stage-1 list, so its rerank
//            score is in the gathered blocks already (the owner's top-k score
//            -- the rerank's bits -- or its prescore); a HIP lookup + select.
//            cbv2_rerank_sharded keeps the collective form for candidates
//            from anywhere: raw candidate scores (-inf for ids this shard
//            does not own) -> ncclAllReduce(MAX) -> HIP top-k select.
//
// An fp32-faithful shard bounds its band by the GLOBAL k-th
// faithful score: the local call runs the bf16 scan + top-k and the exact
// faithful scores fk [B][k] of that top-k (cbv2_search_f32_begin), ONE
// ncclAllGather of fk, the k-th largest of the union (union_kth_kernel) as
// the lower bound lb, then the band rescoring of only the docs that can reach
// the global top-k (cbv2_search_f32_finish) into the send block; the rerank
// scores the owned candidates faithfully (cbv2_rerank_f32).  Results equal
// the unsharded faithful search and rerank bit for bit (the merge completes
// the exact global top-k; any lower bound of the k-th score keeps it exact).
//
// No reference counterpart: the reference is single-process.
// RCCL is resolved with dlsym from the library that created the communicator
// (passed by path; NULL = "librccl.so"), so the borrowed ncclComm_t and the
// calls made on it always come from the same RCCL build.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);
extern "C" int cbv2_merge_topk_strided(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B, int32_t k,
                                       size_t g_stride, float* out_scores, int32_t* out_ids, void* stream);
extern "C" int cbv2_union_kth(const float* fk, int32_t G, int32_t B, int32_t k, size_t g_stride, float* lb,
                              void* stream);
extern "C" int cbv2_prescored_select(const int32_t* recv, int32_t G, int64_t blk, int32_t B, int32_t k, int32_t kb,
                                     const int32_t* cand, int32_t C, int32_t fk, float* out_s, int32_t* out_i,
                                     int32_t* out_p, int32_t* misses, void* stream);
extern "C" int cbv2_rerank_f32_after_search(cbv2_index* ix, const void* search_ws, size_t search_wsb, int32_t cap,
                                            int32_t B, int32_t lq, const int32_t* cand, int32_t C, int32_t k, void* ws,
                                            size_t wsb, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                                            const float* Q, void* stream);

namespace {
// The RCCL entry points used here (rccl.h: ncclResult_t is an int enum,
// ncclInt32 = 2, ncclFloat32 = 7, ncclMax = 2).
using AllGatherFn = int (*)(const void*, void*, size_t, int, void*, hipStream_t);
using AllReduceFn = int (*)(const void*, void*, size_t, int, int, void*, hipStream_t);
using CountFn = int (*)(const void*, int*);
using ErrStrFn = const char* (*)(int);
constexpr int kNcclInt32 = 2, kNcclFloat32 = 7, kNcclMax = 2;

int err(int code, const char* fmt, ...) {
  char buf[384];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return cbv2_set_error(code, buf);
}

#define SH_HIP(call)                                                          \
  do {                                                                        \
    hipError_t e_ = (call);                                                   \
    if (e_ != hipSuccess) return err(CBV2_EHIP, "%s (%d)", #call, (int)e_); \
  } while (0)

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

struct cbv2_comm {
  void* nccl = nullptr;  // borrowed ncclComm_t (loopback: this comm's LoopRank)
  void* lib = nullptr;
  AllGatherFn all_gather = nullptr;
  AllReduceFn all_reduce = nullptr;
  ErrStrFn err_str = nullptr;
  int nranks = 0, rank = 0;
  bool loopback = false;
  int64_t gathers = 0, reduces = 0;   // collectives issued on this handle (cbv2_comm_stats)
};

namespace {
int nccl_check(const cbv2_comm* c, int rc, const char* what) {
  if (rc == 0) return CBV2_OK;
  return err(CBV2_EHIP, "%s failed (%d): %s", what, rc, c->err_str ? c->err_str(rc) : "rccl error");
}

// ---------------------------------------------------------------------------
// Test-only loopback communicator (cbv2_comm_loopback_init): G "ranks" in ONE
// process and on ONE device, each driven by its own host thread and stream,
// with collectives that have RCCL's semantics -- every rank must call, the
// call returns once every rank has enqueued, and no rank's stream runs past
// the collective before every peer's data is in.  all-gather = G device
// copies; all-reduce(MAX) = one max kernel over the G send buffers into a
// scratch, then a copy into the (possibly in-place) receive buffer.  It lets
// one GPU run cbv2_search_sharded_* / cbv2_rerank_sharded at G = 2..64 on real
// per-shard data; production code never creates one.
constexpr int kLoopRcTimeout = 1001, kLoopRcType = 1002, kLoopRcHip = 1003;
const char* loop_err_str(int rc) {
  switch (rc) {
    case kLoopRcTimeout: return "loopback: a peer rank did not reach the collective within 60 s";
    case kLoopRcType: return "loopback: unsupported datatype / reduction";
    case kLoopRcHip: return "loopback: HIP call failed";
    default: return "loopback error";
  }
}

struct LoopGroup {
  int G = 0, refs = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> send;
  std::vector<hipEvent_t> ready, done;
  bool broken = false;

  // generation barrier; false on timeout (the group is then broken for good,
  // so peers fail fast instead of waiting out the timeout one by one)
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t gen = generation;
    if (++arrived == G) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return true;
    }
    if (!cv.wait_for(lk, std::chrono::seconds(60), [&] { return generation != gen || broken; }) || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

struct LoopRank {
  LoopGroup* g = nullptr;
  int rank = 0;
  float* scratch = nullptr;
  size_t scratch_bytes = 0;
};

extern "C" int cbv2_loopback_max(const float* const* srcs, int32_t G, int64_t n, float* out, void* stream);

#define LOOP_HIP(call)                      \
  do {                                      \
    if ((call) != hipSuccess) return kLoopRcHip; \
  } while (0)

// phase 1 (every rank): this rank's send buffer is ready on its stream
int loop_enter(LoopRank* r, const void* send, hipStream_t st) {
  LoopGroup* g = r->g;
  LOOP_HIP(hipEventRecord(g->ready[r->rank], st));
  g->send[r->rank] = send;
  return g->barrier() ? 0 : kLoopRcTimeout;
}

// phase 2 (every rank): this rank's reads of the peers are enqueued; no stream
// passes the collective until every rank's reads are done (so no rank can
// overwrite a send buffer a peer is still reading)
int loop_leave(LoopRank* r, hipStream_t st) {
  LoopGroup* g = r->g;
  LOOP_HIP(hipEventRecord(g->done[r->rank], st));
  if (!g->barrier()) return kLoopRcTimeout;
  for (int p = 0; p < g->G; ++p) LOOP_HIP(hipStreamWaitEvent(st, g->done[p], 0));
  return 0;
}

int loop_all_gather(const void* send, void* recv, size_t count, int dtype, void* comm, hipStream_t st) {
  auto* r = (LoopRank*)comm;
  if (dtype != kNcclInt32 && dtype != kNcclFloat32) return kLoopRcType;
  if (int rc = loop_enter(r, send, st)) return rc;
  for (int p = 0; p < r->g->G; ++p) {
    LOOP_HIP(hipStreamWaitEvent(st, r->g->ready[p], 0));
    LOOP_HIP(hipMemcpyAsync((uint8_t*)recv + (size_t)p * count * 4, r->g->send[p], count * 4,
                            hipMemcpyDeviceToDevice, st));
  }
  return loop_leave(r, st);
}

int loop_all_reduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm, hipStream_t st) {
  auto* r = (LoopRank*)comm;
  if (dtype != kNcclFloat32 || op != kNcclMax) return kLoopRcType;
  if (count * 4 > r->scratch_bytes) {  // test-only code: allocation outside the collective is fine
    LOOP_HIP(hipStreamSynchronize(st));
    if (r->scratch) LOOP_HIP(hipFree(r->scratch));
    r->scratch = nullptr;
    r->scratch_bytes = 0;
    LOOP_HIP(hipMalloc(&r->scratch, count * 4));
    r->scratch_bytes = count * 4;
  }
  if (int rc = loop_enter(r, send, st)) return rc;
  std::vector<const float*> srcs(r->g->G);
  for (int p = 0; p < r->g->G; ++p) {
    LOOP_HIP(hipStreamWaitEvent(st, r->g->ready[p], 0));
    srcs[p] = (const float*)r->g->send[p];
  }
  if (cbv2_loopback_max(srcs.data(), r->g->G, (int64_t)count, r->scratch, st)) return kLoopRcHip;
  if (int rc = loop_leave(r, st)) return rc;
  LOOP_HIP(hipMemcpyAsync(recv, r->scratch, count * 4, hipMemcpyDeviceToDevice, st));
  return 0;
}

void loop_release(LoopRank* r) {
  LoopGroup* g = r->g;
  if (r->scratch) (void)hipFree(r->scratch);
  delete r;
  bool last;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    last = --g->refs == 0;
  }
  if (last) {
    for (auto e : g->ready) (void)hipEventDestroy(e);
    for (auto e : g->done) (void)hipEventDestroy(e);
    delete g;
  }
}
}  // namespace

extern "C" {

int cbv2_comm_init(void* nccl_comm, const char* rccl_library, cbv2_comm** out) {
  if (!out) return err(CBV2_EINVAL, "null output handle pointer");
  *out = nullptr;
  if (!nccl_comm) return err(CBV2_EINVAL, "null ncclComm_t");
  const char* path = rccl_library ? rccl_library : "librccl.so";
  void* lib = dlopen(path, RTLD_NOW | RTLD_NOLOAD);  // prefer the already-loaded copy
  if (!lib) lib = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!lib) return err(CBV2_EUNSUPPORTED, "cannot load RCCL (%s)", path);
  auto* c = new cbv2_comm;
  c->nccl = nccl_comm;
  c->lib = lib;
  c->all_gather = (AllGatherFn)dlsym(lib, "ncclAllGather");
  c->all_reduce = (AllReduceFn)dlsym(lib, "ncclAllReduce");
  c->err_str = (ErrStrFn)dlsym(lib, "ncclGetErrorString");
  auto count = (CountFn)dlsym(lib, "ncclCommCount");
  auto user_rank = (CountFn)dlsym(lib, "ncclCommUserRank");
  if (!c->all_gather || !c->all_reduce || !count || !user_rank) {
    dlclose(lib);
    delete c;
    return err(CBV2_EUNSUPPORTED, "RCCL library %s lacks the collectives", path);
  }
  int rc = count(nccl_comm, &c->nranks);
  if (!rc) rc = user_rank(nccl_comm, &c->rank);
  if (rc || c->nranks < 1 || c->nranks > 64 || c->rank < 0 || c->rank >= c->nranks) {
    dlclose(lib);
    delete c;
    return err(CBV2_EINVAL, "ncclCommCount/ncclCommUserRank failed (rc %d)", rc);
  }
  *out = c;
  return CBV2_OK;
}

int cbv2_comm_loopback_init(int32_t nranks, cbv2_comm** out) {
  if (!out) return err(CBV2_EINVAL, "null output array");
  if (nranks < 1 || nranks > 64) return err(CBV2_EINVAL, "nranks must be in [1, 64] (got %d)", nranks);
  for (int r = 0; r < nranks; ++r) out[r] = nullptr;
  auto* g = new LoopGroup;
  g->G = nranks;
  g->refs = nranks;
  g->send.assign(nranks, nullptr);
  g->ready.assign(nranks, nullptr);
  g->done.assign(nranks, nullptr);
  for (int r = 0; r < nranks; ++r) {
    if (hipEventCreateWithFlags(&g->ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->done[r], hipEventDisableTiming) != hipSuccess) {
      for (auto e : g->ready) if (e) (void)hipEventDestroy(e);
      for (auto e : g->done) if (e) (void)hipEventDestroy(e);
      delete g;
      return err(CBV2_EHIP, "hipEventCreate failed");
    }
  }
  for (int r = 0; r < nranks; ++r) {
    auto* lr = new LoopRank;
    lr->g = g;
    lr->rank = r;
    auto* c = new cbv2_comm;
    c->nccl = lr;
    c->all_gather = loop_all_gather;
    c->all_reduce = loop_all_reduce;
    c->err_str = loop_err_str;
    c->nranks = nranks;
    c->rank = r;
    c->loopback = true;
    out[r] = c;
  }
  return CBV2_OK;
}

int cbv2_comm_size(const cbv2_comm* c) { return c ? c->nranks : -1; }
int cbv2_comm_rank(const cbv2_comm* c) { return c ? c->rank : -1; }

int cbv2_comm_destroy(cbv2_comm* c) {
  if (c) {
    if (c->loopback) loop_release((LoopRank*)c->nccl);
    if (c->lib) dlclose(c->lib);
    delete c;  // the ncclComm_t is borrowed: its owner destroys it
  }
  return CBV2_OK;
}

namespace {
// The band capacity of a faithful shard's search (as cbv2_retrieve_* use) and
// its workspaces, sized for lq = 32 (the most a MaxSim call takes; a call
// with fewer query tokens needs less).
int32_t band_cap(int32_t k) { return k > CBV2_RETRIEVE_BAND_CAP ? k : CBV2_RETRIEVE_BAND_CAP; }
bool is_faithful(const cbv2_index* ix) {
  int32_t dt = 0, f = 0;
  return ix && cbv2_index_kind(ix, &dt, &f) == CBV2_OK && f != 0;
}
size_t f32_search_bytes(const cbv2_index* ix, int32_t B, int32_t k) {
  return align256(cbv2_f32_workspace_bytes(ix, CBV2_F32_SEARCH, B, 32, band_cap(k)));
}
// rerank part: raw [B][C] at the head of the workspace (+ a faithful shard's
// rerank workspace after it, for queries of lq tokens)
size_t rerank_bytes(const cbv2_index* ix, int32_t B, int32_t C, int32_t lq = 32) {
  const size_t raw = align256((size_t)B * (C > 0 ? C : 1) * 4);
  return raw + (is_faithful(ix) && C > 0 ? align256(cbv2_f32_workspace_bytes(ix, CBV2_F32_RERANK, B, lq, C)) : 0);
}

// [local search part | send block | recv blocks | merged BM25 scores | rerank part]
// (send block, words: [scores B*k | ids B*k | bm25 scores B*kb | bm25 ids B*kb | bm25 prescores B*kb])
// local search part: bf16 / MXFP8: the cbv2_search workspace; fp32-faithful:
// [f32 search workspace | fk B*k | fk of every rank G*B*k | lb B | status B].
struct Layout {
  size_t search_ws, blk, f32_ws;
  int32_t *send, *recv;
  float* lex_s_out;
  float *fk, *fk_all, *lb;
  int32_t* status;
  uint8_t* rr;   // the rerank part (the exchange's stage-1 prescore: a faithful shard's rerank workspace)
};
Layout layout(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t k, int32_t kb, void* ws) {
  Layout L{};
  uint8_t* base = (uint8_t*)ws;
  if (is_faithful(ix)) {
    L.f32_ws = f32_search_bytes(ix, B, k);
    const size_t bk = align256((size_t)B * k * 4), gbk = align256((size_t)c->nranks * B * k * 4),
                 b4 = align256((size_t)B * 4);
    L.search_ws = L.f32_ws + bk + gbk + 2 * b4;
    if (base) {
      L.fk = (float*)(base + L.f32_ws);
      L.fk_all = (float*)(base + L.f32_ws + bk);
      L.lb = (float*)(base + L.f32_ws + bk + gbk);
      L.status = (int32_t*)(base + L.f32_ws + bk + gbk + b4);
    }
  } else {
    L.search_ws = align256(cbv2_search_workspace_size(ix, B, k, CBV2_SCORER_MAXSIM));
  }
  L.blk = (size_t)B * (2 * (size_t)k + 3 * (size_t)kb);
  if (base) {
    uint8_t* p = base + L.search_ws;
    L.send = (int32_t*)p;
    L.recv = (int32_t*)(p + align256(L.blk * 4));
    L.lex_s_out = (float*)(p + align256(L.blk * 4) + align256(L.blk * 4 * c->nranks));
    L.rr = (uint8_t*)L.lex_s_out + align256((size_t)B * (kb > 0 ? kb : 1) * 4);
  }
  return L;
}
}  // namespace

size_t cbv2_sharded_workspace_bytes(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t k, int32_t kb,
                                    int32_t C) {
  if (!ix || !c || B < 1 || k < 1 || kb < 0 || C < 0) return 0;
  const Layout L = layout(ix, c, B, k, kb, nullptr);
  const size_t gather = align256(L.blk * 4) + align256(L.blk * 4 * c->nranks);
  const size_t lex_out = align256((size_t)B * (kb > 0 ? kb : 1) * 4);
  // the local search's part is sized for MaxSim (the sharded exchange's scorer;
  // cbv2_search rejects another scorer's larger need with CBV2_EINVAL); the
  // rerank part serves the exchange's stage-1 prescore (kb candidates) too
  return L.search_ws + gather + lex_out + rerank_bytes(ix, B, C > kb ? C : kb);
}

namespace {
int check_sizes(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t k, int32_t kb, void* ws, size_t ws_bytes) {
  if (!ix || !c) return err(CBV2_EINVAL, "null index/comm");
  if (B < 1 || k < 1 || kb < 0) return err(CBV2_EINVAL, "bad sizes (B %d, k %d, kb %d)", B, k, kb);
  const size_t need = cbv2_sharded_workspace_bytes(ix, c, B, k, kb, 0);
  if (!ws || ws_bytes < need) return err(CBV2_EINVAL, "workspace too small (%zu bytes needed)", need);
  return CBV2_OK;
}
}  // namespace

int cbv2_search_sharded_local(cbv2_index* ix, cbv2_comm* c, int32_t scorer, const void* Q, int32_t q_dtype,
                              int32_t B, int32_t lq, int32_t k, int32_t kb, void* workspace, size_t workspace_bytes,
                              void* stream) {
  if (int rc = check_sizes(ix, c, B, k, kb, workspace, workspace_bytes)) return rc;
  const Layout L = layout(ix, c, B, k, kb, workspace);
  hipStream_t st = (hipStream_t)stream;
  float* send_s = (float*)L.send;
  int32_t* send_i = L.send + (size_t)B * k;
  if (!is_faithful(ix))   // local stage 2 straight into this rank's send block
    return cbv2_search(ix, scorer, Q, q_dtype, B, lq, k, workspace, L.search_ws, send_s, send_i, st);
  if (scorer != CBV2_SCORER_MAXSIM || q_dtype != CBV2_DTYPE_F32)
    return err(CBV2_EINVAL, "an fp32-faithful shard takes MaxSim with f32 queries");
  const int32_t cap = band_cap(k);
  int rc = cbv2_search_f32_begin(ix, (const float*)Q, B, lq, k, cap, workspace, L.f32_ws, L.fk, send_s, send_i,
                                 L.status, st);
  if (rc) return rc;
  // the global bound: every rank's fk, the k-th largest of their union
  rc = nccl_check(c, c->all_gather(L.fk, L.fk_all, (size_t)B * k, kNcclFloat32, c->nccl, st), "ncclAllGather");
  if (rc) return rc;
  ++c->gathers;
  if ((rc = cbv2_union_kth(L.fk_all, c->nranks, B, k, (size_t)B * k, L.lb, st))) return rc;
  return cbv2_search_f32_finish(ix, B, lq, k, cap, workspace, L.f32_ws, L.lb, send_s, send_i, L.status, st);
}

int cbv2_search_sharded_exchange(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t q_dtype, int32_t lq,
                                 int32_t B, int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb,
                                 void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                                 int32_t* out_lex_ids, void* stream) {
  if (int rc = check_sizes(ix, c, B, k, kb, workspace, workspace_bytes)) return rc;
  if (kb > 0 && (!lex_ids || !lex_scores || !out_lex_ids)) return err(CBV2_EINVAL, "null bm25 lists/output");
  if (!out_scores || !out_ids) return err(CBV2_EINVAL, "null outputs");
  if (Q && (lq < 1 || lq > 32)) return err(CBV2_EINVAL, "lq must be in [1, 32] (got %d)", lq);
  hipStream_t st = (hipStream_t)stream;
  const Layout L = layout(ix, c, B, k, kb, workspace);
  int rc;
  if (kb > 0) {
    int32_t* ls = L.send + (size_t)2 * B * k;
    SH_HIP(hipMemcpyAsync(ls, lex_scores, (size_t)B * kb * 4, hipMemcpyDefault, st));
    SH_HIP(hipMemcpyAsync(ls + (size_t)B * kb, lex_ids, (size_t)B * kb * 4, hipMemcpyDefault, st));
    if (Q) {   // the stage-1 prescore: the rerank's raw scores of this rank's own BM25 top-kb
      const int32_t* ids_d = ls + (size_t)B * kb;
      float* pre = (float*)(ls + (size_t)2 * B * kb);
      const size_t rrb = workspace_bytes - (size_t)(L.rr - (uint8_t*)workspace);
      if (is_faithful(ix)) {   // on the local search's query split (re-split from Q if it is gone)
        if (q_dtype != CBV2_DTYPE_F32) return err(CBV2_EINVAL, "an fp32-faithful shard takes f32 queries");
        rc = cbv2_rerank_f32_after_search(ix, workspace, L.f32_ws, band_cap(k), B, lq, ids_d, kb, 0, L.rr, rrb, pre,
                                          nullptr, nullptr, (const float*)Q, st);
      } else {
        rc = cbv2_rerank_ws(ix, Q, B, lq, ids_d, kb, 0, L.rr, rrb, pre, nullptr, nullptr, st);
      }
      if (rc) return rc;
    }
  }
  // one all-gather of the blocks, then the merges (shard g's block at g * blk words)
  rc = nccl_check(c, c->all_gather(L.send, L.recv, L.blk, kNcclInt32, c->nccl, st), "ncclAllGather");
  if (rc) return rc;
  ++c->gathers;
  rc = cbv2_merge_topk_strided((const float*)L.recv, L.recv + (size_t)B * k, c->nranks, B, k, L.blk, out_scores,
                               out_ids, st);
  if (rc || kb == 0) return rc;
  const int32_t* lr = L.recv + (size_t)2 * B * k;
  return cbv2_merge_topk_strided((const float*)lr, lr + (size_t)B * kb, c->nranks, B, kb, L.blk, L.lex_s_out,
                                 out_lex_ids, st);
}

int cbv2_search_sharded(cbv2_index* ix, cbv2_comm* c, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B,
                        int32_t lq, int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb,
                        void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                        int32_t* out_lex_ids, void* stream) {
  int rc = cbv2_search_sharded_local(ix, c, scorer, Q, q_dtype, B, lq, k, kb, workspace, workspace_bytes, stream);
  if (rc) return rc;
  return cbv2_search_sharded_exchange(ix, c, Q, q_dtype, lq, B, k, lex_ids, lex_scores, kb, workspace,
                                      workspace_bytes, out_scores, out_ids, out_lex_ids, stream);
}

int cbv2_rerank_sharded(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t B, int32_t lq, const int32_t* cand,
                        int32_t C, int32_t k, void* workspace, size_t workspace_bytes, float* out_scores,
                        int32_t* out_ids, int32_t* out_pos, void* stream) {
  if (!ix || !c) return err(CBV2_EINVAL, "null index/comm");
  if (B < 1 || C < 1 || k < 1 || lq < 1) return err(CBV2_EINVAL, "bad sizes (B, C, k, lq)");
  if (!workspace || workspace_bytes < rerank_bytes(ix, B, C, lq))
    return err(CBV2_EINVAL, "workspace too small (%zu bytes needed)", rerank_bytes(ix, B, C, lq));
  hipStream_t st = (hipStream_t)stream;
  float* raw = (float*)workspace;
  int rc;
  if (is_faithful(ix)) {   // faithful scores of the owned candidates (f32 queries)
    const size_t off = align256((size_t)B * C * 4);
    rc = cbv2_rerank_f32(ix, (const float*)Q, B, lq, cand, C, 0, (uint8_t*)workspace + off, workspace_bytes - off,
                         raw, nullptr, nullptr, st);
  } else {
    rc = cbv2_rerank(ix, Q, B, lq, cand, C, 0, raw, nullptr, nullptr, st);
  }
  if (rc) return rc;
  rc = nccl_check(c, c->all_reduce(raw, raw, (size_t)B * C, kNcclFloat32, kNcclMax, c->nccl, st), "ncclAllReduce");
  if (rc) return rc;
  ++c->reduces;
  return cbv2_select_topk(raw, cand, B, C, k, out_scores, out_ids, out_pos, st);
}

int cbv2_rerank_sharded_prescored(cbv2_index* ix, cbv2_comm* c, int32_t B, int32_t k, int32_t kb,
                                  const int32_t* cand, int32_t C, int32_t final_k, void* workspace,
                                  size_t workspace_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                                  int32_t* misses, void* stream) {
  if (int rc = check_sizes(ix, c, B, k, kb, workspace, workspace_bytes)) return rc;
  if (!cand || !out_scores || !out_ids) return err(CBV2_EINVAL, "null candidates/outputs");
  if (C < 1 || C > 1024 || final_k < 1) return err(CBV2_EINVAL, "C must be in [1, 1024], final_k >= 1 (C %d, k %d)", C,
                                                   final_k);
  const Layout L = layout(ix, c, B, k, kb, workspace);
  return cbv2_prescored_select(L.recv, c->nranks, (int64_t)L.blk, B, k, kb, cand, C, final_k, out_scores, out_ids,
                               out_pos, misses, stream);
}

int cbv2_comm_stats(const cbv2_comm* c, int64_t* out2) {
  if (!c || !out2) return err(CBV2_EINVAL, "null comm/output");
  out2[0] = c->gathers;
  out2[1] = c->reduces;
  return CBV2_OK;
}

}  // extern "C"
