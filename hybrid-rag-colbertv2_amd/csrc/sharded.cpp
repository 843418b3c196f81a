// sharded.cpp — the multi-GPU exchange behind the C ABI (SURVEY.md §8(b),(e)):
// cbv2_comm_init borrows an initialised RCCL communicator (e.g. the one
// torch.distributed's "nccl" backend created: ProcessGroupNCCL._comm_ptr()),
// and cbv2_search_sharded / cbv2_rerank_sharded run one stage each with ONE
// collective, everything enqueued on the caller's stream:
//
//   search:  local scan + top-k written straight into this rank's send block
//            [scores B*k | ids B*k | bm25 scores B*kb | bm25 ids B*kb]
//            -> ncclAllGather of the blocks -> HIP merge (score desc, id asc)
//            of the G stage-2 lists and of the G stage-1 lists.
//   rerank:  raw candidate scores (-inf for ids this shard does not own)
//            -> ncclAllReduce(MAX) -> HIP top-k select.
//
// No reference counterpart: the reference is single-process.
// RCCL is resolved with dlsym from the library that created the communicator
// (passed by path; NULL = "librccl.so"), so the borrowed ncclComm_t and the
// calls made on it always come from the same RCCL build.
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);
extern "C" int cbv2_merge_topk_strided(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B, int32_t k,
                                       size_t g_stride, float* out_scores, int32_t* out_ids, void* stream);

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
  void* nccl = nullptr;  // borrowed ncclComm_t
  void* lib = nullptr;
  AllGatherFn all_gather = nullptr;
  AllReduceFn all_reduce = nullptr;
  ErrStrFn err_str = nullptr;
  int nranks = 0, rank = 0;
};

namespace {
int nccl_check(const cbv2_comm* c, int rc, const char* what) {
  if (rc == 0) return CBV2_OK;
  return err(CBV2_EHIP, "%s failed (%d): %s", what, rc, c->err_str ? c->err_str(rc) : "rccl error");
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

int cbv2_comm_size(const cbv2_comm* c) { return c ? c->nranks : -1; }
int cbv2_comm_rank(const cbv2_comm* c) { return c ? c->rank : -1; }

int cbv2_comm_destroy(cbv2_comm* c) {
  if (c) {
    if (c->lib) dlclose(c->lib);
    delete c;  // the ncclComm_t is borrowed: its owner destroys it
  }
  return CBV2_OK;
}

size_t cbv2_sharded_workspace_bytes(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t k, int32_t kb,
                                    int32_t C) {
  if (!ix || !c || B < 1 || k < 1 || kb < 0 || C < 0) return 0;
  const size_t blk = (size_t)2 * B * (k + kb);  // 4-byte words per rank
  const size_t gather = align256(blk * 4) + align256(blk * 4 * c->nranks);
  const size_t lex_out = align256((size_t)B * (kb > 0 ? kb : 1) * 4);
  const size_t raw = align256((size_t)B * (C > 0 ? C : 1) * 4);
  // the local search's part is sized for MaxSim (the sharded exchange's scorer;
  // cbv2_search rejects another scorer's larger need with CBV2_EINVAL)
  return align256(cbv2_search_workspace_size(ix, B, k, CBV2_SCORER_MAXSIM)) + gather + lex_out + raw;
}

namespace {
struct Layout {
  size_t search_ws, blk;
  int32_t *send, *recv;
  float* lex_s_out;
};
Layout layout(const cbv2_index* ix, const cbv2_comm* c, int32_t B, int32_t k, int32_t kb, void* ws) {
  Layout L;
  L.search_ws = align256(cbv2_search_workspace_size(ix, B, k, CBV2_SCORER_MAXSIM));
  L.blk = (size_t)2 * B * (k + kb);
  uint8_t* p = (uint8_t*)ws + L.search_ws;
  L.send = (int32_t*)p;
  L.recv = (int32_t*)(p + align256(L.blk * 4));
  L.lex_s_out = (float*)(p + align256(L.blk * 4) + align256(L.blk * 4 * c->nranks));
  return L;
}
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
  // local stage 2 straight into this rank's send block
  return cbv2_search(ix, scorer, Q, q_dtype, B, lq, k, workspace, L.search_ws, (float*)L.send,
                     L.send + (size_t)B * k, (hipStream_t)stream);
}

int cbv2_search_sharded_exchange(cbv2_index* ix, cbv2_comm* c, int32_t B, int32_t k, const int32_t* lex_ids,
                                 const float* lex_scores, int32_t kb, void* workspace, size_t workspace_bytes,
                                 float* out_scores, int32_t* out_ids, int32_t* out_lex_ids, void* stream) {
  if (int rc = check_sizes(ix, c, B, k, kb, workspace, workspace_bytes)) return rc;
  if (kb > 0 && (!lex_ids || !lex_scores || !out_lex_ids)) return err(CBV2_EINVAL, "null bm25 lists/output");
  if (!out_scores || !out_ids) return err(CBV2_EINVAL, "null outputs");
  hipStream_t st = (hipStream_t)stream;
  const Layout L = layout(ix, c, B, k, kb, workspace);
  if (kb > 0) {
    int32_t* ls = L.send + (size_t)2 * B * k;
    SH_HIP(hipMemcpyAsync(ls, lex_scores, (size_t)B * kb * 4, hipMemcpyDefault, st));
    SH_HIP(hipMemcpyAsync(ls + (size_t)B * kb, lex_ids, (size_t)B * kb * 4, hipMemcpyDefault, st));
  }
  // one all-gather of the blocks, then the merges (shard g's block at g * blk words)
  int rc = nccl_check(c, c->all_gather(L.send, L.recv, L.blk, kNcclInt32, c->nccl, st), "ncclAllGather");
  if (rc) return rc;
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
  return cbv2_search_sharded_exchange(ix, c, B, k, lex_ids, lex_scores, kb, workspace, workspace_bytes, out_scores,
                                      out_ids, out_lex_ids, stream);
}

int cbv2_rerank_sharded(cbv2_index* ix, cbv2_comm* c, const void* Q, int32_t B, int32_t lq, const int32_t* cand,
                        int32_t C, int32_t k, void* workspace, size_t workspace_bytes, float* out_scores,
                        int32_t* out_ids, int32_t* out_pos, void* stream) {
  if (!ix || !c) return err(CBV2_EINVAL, "null index/comm");
  if (B < 1 || C < 1 || k < 1) return err(CBV2_EINVAL, "bad sizes (B, C, k)");
  if (!workspace || workspace_bytes < (size_t)B * C * 4) return err(CBV2_EINVAL, "workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* raw = (float*)workspace;
  int rc = cbv2_rerank(ix, Q, B, lq, cand, C, 0, raw, nullptr, nullptr, st);
  if (rc) return rc;
  rc = nccl_check(c, c->all_reduce(raw, raw, (size_t)B * C, kNcclFloat32, kNcclMax, c->nccl, st), "ncclAllReduce");
  if (rc) return rc;
  return cbv2_select_topk(raw, cand, B, C, k, out_scores, out_ids, out_pos, st);
}

}  // extern "C"
