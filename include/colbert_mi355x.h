/*
 * colbert_mi355x.h — C ABI of libcolbert_mi355x.so, the MI355X (gfx950) ColBERT
 * late-interaction scoring path.
 *
 * The reference (techmum21p/hybrid-rag-ColBERTv2) has no FFI: its seam is the
 * Python object `DualIndexer.colbert_retriever` (local_rag_complete.py:844)
 * called as `.search(query=, k=)` (:954) and `.rerank(query=, documents=, k=)`
 * (:999).  Each entry point below replaces one piece of arithmetic behind that
 * seam; the Python package (hybrid-rag-colbertv2_amd/) binds them with ctypes
 * and keeps the reference's method names and result dicts.
 *
 * Conventions
 *  - Every pointer argument except `cbv2_index*` is a DEVICE pointer owned by
 *    the caller (torch tensors in the Python layer), except where a
 *    declaration says HOST: the host-only helpers (cbv2_rrf_fuse, BM25, the
 *    index file, the stemmer) and the stage-1 lists / host stage of
 *    cbv2_retrieve_finish.  Nothing is allocated or freed inside a compute
 *    call; every call but cbv2_retrieve_finish (which waits for its round
 *    trip) is asynchronous and hipGraph-capturable.
 *  - Calls are asynchronous on `stream` (a hipStream_t; NULL = legacy default
 *    stream).  One index handle belongs to one device.
 *  - Return 0 on success, a negative CBV2_E* code on error; the message is in
 *    the thread-local `cbv2_last_error()`.  Arguments are validated on the host
 *    BEFORE any launch: a call that returns an error has launched nothing.
 *  - Ranking ties are broken deterministically: score descending, then the
 *    lower index in the scored list (doc id for search, candidate position for
 *    rerank).  The reference's torch.topk / argsort (local_rag_complete.py:767,
 *    :789) leave tie order unspecified; this is the defined refinement.
 *
 * Index layout in HBM (see DESIGN.md "Data layout"):
 *    tokens   bf16 [n][ld][d = 128], row-major, 16-byte aligned; ld = 128
 *             token slots (every path), or 256 / 512 / 1024 for long
 *             documents (bf16 and MXFP8 MaxSim scan, search and rerank, the
 *             fp32-faithful index and the native file; scales of an MXFP8
 *             index are [n][ld][2]);
 *             rows t >= doclens[i] of doc i are padding and never score.
 *    doclens  int32 [n], 0 <= doclens[i] <= ld.
 *    Local doc i has global id  id_base + i  (contiguous shard of the corpus).
 */
#ifndef COLBERT_MI355X_H
#define COLBERT_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CBV2_ABI_VERSION 2

/* dtypes */
#define CBV2_DTYPE_BF16 1
#define CBV2_DTYPE_F32 2
#define CBV2_DTYPE_MXFP8 3 /* e4m3 bytes + one E8M0 scale per token per 64 dims */

/* scorers */
#define CBV2_SCORER_MAXSIM 0              /* sum_i max_j <q_i, d_j>            */
#define CBV2_SCORER_REF_MEANPOOL_COSINE 1 /* cos(mean_i q_i, mean_j d_j)       */

/* error codes */
#define CBV2_OK 0
#define CBV2_EINVAL -1       /* bad argument (shape, null pointer, range)       */
#define CBV2_EUNSUPPORTED -2 /* valid but not built (e.g. ld != 128)             */
#define CBV2_EHIP -3         /* a HIP runtime call failed                        */
#define CBV2_ESTATE -4       /* handle not ready (e.g. meanpool means not built) */

typedef struct cbv2_index cbv2_index;

/* Library / error reporting ------------------------------------------------ */
int cbv2_abi_version(void);
const char* cbv2_last_error(void);
/* "cbv2-build-stamp:<hex>": a content hash of the sources and compiler flags
 * the library was built from (build provenance; the Python loader refuses a
 * library whose stamp differs from the tree's sources).                     */
const char* cbv2_build_stamp(void);

/* Index handle --------------------------------------------------------------
 * Replaces the tensor the reference keeps in `self.corpus_embeddings`
 * (local_rag_complete.py:735-739 index(), :751-752 load()).  The handle
 * BORROWS `tokens`, `doclens` (and later `doc_means`): the caller keeps them
 * alive until cbv2_index_destroy.  `device` is the HIP device ordinal.      */
int cbv2_index_create(int device, const void* tokens, int32_t dtype, int64_t n, int32_t ld,
                      int32_t d, const int32_t* doclens, int64_t id_base, cbv2_index** out);
int cbv2_index_destroy(cbv2_index* index);

/* Index memory placement (no reference counterpart).  cbv2_hbm_alloc: `bytes`
 * of device memory on `device`, PHYSICALLY CONTIGUOUS when the driver can
 * provide it (hipExtMallocWithFlags(hipDeviceMallocContiguous); *contiguous =
 * 1), else plain hipMalloc (0).  Large index buffers (the token arrays every
 * scan streams) belong there: the B = 1 streaming scan over 1M docs (32.8 GB)
 * ran 4.63-4.67 ms from contiguous allocations and 4.75-4.99 ms from plain
 * hipMalloc ones of the same process (tools/probes/alloc_probe.cpp) -- the
 * translation of a streamed range is cheaper when it is one contiguous
 * physical range.  Free with cbv2_hbm_free (synchronous, like hipFree).    */
int cbv2_hbm_alloc(int device, size_t bytes, void** out, int32_t* contiguous);
int cbv2_hbm_free(int device, void* p);

/* Scan timing (measurement only; no reference counterpart -- the reference
 * prints wall-clock stage timings, local_rag_complete.py:905-933).  While
 * enabled, every MaxSim scan launch of this handle (cbv2_score / cbv2_search /
 * cbv2_search_f32) is bracketed by HIP events recorded on the launch's own
 * stream, so a benchmark can time the dominant kernel inside its timed region
 * without a side launch.  enable=1 clears the previous record.
 * cbv2_index_scan_times (timing disabled first) waits for the recorded launches
 * and writes min(count, max) durations in ms; *count = launches recorded;
 * the record is then cleared.
 * cbv2_index_band_times: the same for the fp32-faithful searches' band work
 * (cbv2_search_f32 / _begin + _finish), each bracketed from the end of the
 * bf16 top-k of its scan to the end of its band select and full-scan fallback:
 * the time the faithful arithmetic adds to a bf16 search (the query split
 * before the scan, one small kernel, is outside the bracket).
 * enable=2: the events, plus the clock probe of the doc-interleaved scans
 * (bf16 maxsim_scan16x4_kernel, MXFP8 maxsim_scan_f8x4_kernel): each of their
 * workgroups adds its run time in shader cycles (s_memtime) and in 10-ns ticks
 * (s_memrealtime) to the handle's sums.  cbv2_index_scan_clock (after the
 * launches completed) writes out4 = {sum of cycles, sum of ticks, workgroups
 * started, workgroups ended} since enable=2 or the last reset (reset != 0
 * zeroes them after the read): the clock the scans held in THIS run is
 * out4[0] / out4[1] x 0.1 GHz.  */
int cbv2_index_time_scans(cbv2_index* index, int32_t enable);
int cbv2_index_scan_times(cbv2_index* index, float* ms, int32_t max, int32_t* count);
int cbv2_index_band_times(cbv2_index* index, float* ms, int32_t max, int32_t* count);
int cbv2_index_scan_clock(cbv2_index* index, int64_t* out4, int32_t reset);

/* Handle options (A/B and tests; defaults = production):
 *  CBV2_OPT_FUSED_TOPK   1: cbv2_search fuses the top-k into eligible scans
 *                        (the bf16 doc-interleaved scan; 2 the same -- the
 *                        fused MXFP8 scan spills and is built in lab builds
 *                        only).  Default 0: on MI355X the fused scan runs
 *                        ~1 % longer than the scan + radix top-k.
 *  CBV2_OPT_DYNAMIC_TAIL 1: large scans hand the last part of the corpus out
 *                        as dynamic tasks, in 8 XCD-local slices (2: one
 *                        shared tail; 0: static chunks only).
 *  CBV2_OPT_BAND_DOC_MAJOR 0 (default): cbv2_search_f32 rescores the band
 *                        pair by pair (one (query, doc) pair per workgroup);
 *                        1-4: a batch of more than 8 queries grouped by doc
 *                        (each band doc read once per batch) -- 1 one wave
 *                        per doc, its halves in turn; 2 the same, pair-outer;
 *                        3 / 4 one doc per workgroup of 4 / 2 waves (128-slot
 *                        docs; others take 1).  Identical results either way.
 *  CBV2_OPT_BAND_LOWER_BOUND 1: cbv2_search_f32 first rescores the bf16
 *                        top-k, whose minimum faithful score lb bounds the
 *                        k-th from below, and bands T >= lb - beta (0: the
 *                        wider T >= T_k - 2 beta).  Identical results.
 *  CBV2_OPT_BAND_FUSED   1: cbv2_search_f32 on at most 8 queries (128-slot
 *                        docs) collects the band and rescores it in ONE
 *                        launch (0: a collect launch, then a rescoring
 *                        launch).  Identical results.
 *  CBV2_OPT_RESCORE_SPLIT 1: the fp32-faithful rescorings (the bf16 top-k, the
 *                        band of <= 8 queries, rerank candidates, the
 *                        full-scan fallback) score one (query, doc) pair per
 *                        workgroup, the doc's rows split over its 4 waves (0:
 *                        one pair per wave).  Identical results.
 *  CBV2_OPT_BAND_REUSE   1: the two-pass band of cbv2_search_f32 keeps the
 *                        faithful scores phase 1 computed for the bf16 top-k
 *                        (its lower bound) as its first k entries and rescores
 *                        only the rest (0: the whole band).  Needs
 *                        CBV2_OPT_RESCORE_SPLIT.  Identical results.
 *  CBV2_OPT_BAND_BLOCK_SKIP 1: the band collect of cbv2_search_f32 reads only
 *                        the 64-doc blocks whose maximum (left by the
 *                        block-max top-k) reaches the band threshold (0: the
 *                        whole score row).  Identical results.
 *  CBV2_OPT_RESCORE_GRID  workgroups per row of a split rescoring launch (0:
 *                        automatic, 4096 / B within [256, 1024]; rows with
 *                        more pairs grid-stride).
 *                        Identical results.
 *  CBV2_OPT_DENSE_DOCS    1: the docs fill (nearly) all 128 token slots, so
 *                        searches of B <= 2 stream every slot on the 4-wave
 *                        x 1-query scan (non-temporal) instead of the
 *                        streaming scan that skips empty 16-token tiles
 *                        (0, the default; the Python ColbertIndex sets it
 *                        when >= 98 % of the tiles hold tokens).  Identical
 *                        results.
 *  CBV2_OPT_TOPK_BMAX    1: cbv2_search's unfused MaxSim scan (rows of >= 65,536
 *                        and <= 1,572,864 docs, k <= 1024) also folds the max of
 *                        every 64-doc block, and ONE select launch reads only
 *                        the blocks that can reach the top-k (0: the sampled
 *                        filter + select).  Identical results.
 *  CBV2_OPT_P1_COLLECT_FUSED 1: the two-pass band of cbv2_search_f32 on at
 *                        most 8 queries runs its phase 1 (the bf16 top-k's
 *                        faithful scores) and the band collect in ONE launch
 *                        (the collect's loads overlap phase 1; 0: two
 *                        launches).  Identical results.
 *  CBV2_OPT_FOLD_KEYS     1: cbv2_search_f32 on at most 4 queries of a
 *                        dense-doc index folds the block-max select's block
 *                        keys into its 4 x 1 scan (atomic max into keys the
 *                        query split zeroes; 0: a pass over the scores).
 *                        Identical results.
 * cbv2_index_last_scan_plan: the work split of this handle's latest scan
 * launch: {workgroups, static chunk docs, static docs, dynamic tail 0/1}.
 * Thread safety: one handle may be used from several host threads and
 * streams; the options and the last plan are plain fields (set options
 * before sharing the handle).                                               */
#define CBV2_OPT_FUSED_TOPK 1
#define CBV2_OPT_DYNAMIC_TAIL 2
#define CBV2_OPT_BAND_DOC_MAJOR 3
#define CBV2_OPT_BAND_LOWER_BOUND 4
#define CBV2_OPT_TOPK_BMAX 5
#define CBV2_OPT_BAND_FUSED 6
#define CBV2_OPT_RESCORE_SPLIT 7
#define CBV2_OPT_BAND_REUSE 8
#define CBV2_OPT_BAND_BLOCK_SKIP 9
#define CBV2_OPT_RESCORE_GRID 10
#define CBV2_OPT_DENSE_DOCS 11
#define CBV2_OPT_P1_COLLECT_FUSED 12
#define CBV2_OPT_FOLD_KEYS 13
int cbv2_index_set_option(cbv2_index* index, int32_t option, int64_t value);
int cbv2_index_last_scan_plan(const cbv2_index* index, int64_t* out4);
/* Per-query workgroup lists a cbv2_search of (B, k, scorer) keeps with the
 * top-k fused into the scan; 0 = that search runs unfused.                  */
int64_t cbv2_search_fused_slots(const cbv2_index* index, int32_t B, int32_t k, int32_t scorer);

/* MXFP8 index (config 5: half the HBM bytes of bf16, scored on the
 * block-scaled fp8 MFMA): tokens e4m3 [n][128][128] (16-B aligned), scales
 * E8M0 [n][128][2] (byte h scales dims 64h .. 64h+63 by 2^(byte-127)).
 * Queries for such an index are MXFP8 too (q_dtype CBV2_DTYPE_MXFP8): one
 * buffer holding B*lq*128 e4m3 bytes followed by B*lq*2 scale bytes, as
 * written by cbv2_quantize_mxfp8 (rows = B*lq, scales = q + rows*128).     */
int cbv2_index_create_mxfp8(int device, const void* tokens, const void* scales, int64_t n, int32_t ld,
                            int32_t d, const int32_t* doclens, int64_t id_base, cbv2_index** out);

/* cbv2_quantize_mxfp8 — rows of 128 values (dtype BF16 or F32) -> e4m3 bytes
 * q [rows][128] (round-to-nearest-even) and E8M0 scales [rows][2], with
 * scale = the smallest power of two that keeps each 64-value half <= 448.   */
int cbv2_quantize_mxfp8(const void* x, int32_t dtype, int64_t rows, void* q, void* scales, void* stream);

/* Literal-reference scorer support: build the L2-normalised per-doc token means
 * the reference recomputes on every call (local_rag_complete.py:822,825-829)
 * ONCE, from the fp32 encoder output `tokens_f32` [n][ld_src][d].
 * `doc_means` is a caller-owned f32 [n][d] buffer the handle borrows.        */
int cbv2_index_build_means(cbv2_index* index, const float* tokens_f32, int32_t ld_src,
                           float* doc_means, void* stream);

/* Scoring -------------------------------------------------------------------
 * cbv2_score — JinaColBERTRetriever._maxsim_score (local_rag_complete.py:802-831)
 * for a batch of B queries against every doc of the index:
 *    out[b * ld_out + i] = score(Q[b], doc i)     (i = local index)
 *  scorer MAXSIM:              Q bf16 [B][lq][128], 1 <= lq <= 32.
 *  scorer REF_MEANPOOL_COSINE: Q f32  [B][lq][128], any lq >= 1 (means must
 *                              be built).                                    */
int cbv2_score(cbv2_index* index, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B,
               int32_t lq, float* out, int64_t ld_out, void* stream);

/* cbv2_search — JinaColBERTRetriever.search (local_rag_complete.py:755-777):
 * score every doc, then top-k (torch.topk at :767) with the deterministic tie
 * rule.  Writes out_scores f32 [B][k] and out_ids int32 [B][k] (GLOBAL ids =
 * id_base + local index), best first; slots past min(k, n) hold -inf / -1.
 * `workspace` (16-B aligned, caller-owned, also holds the scan's work-split
 * counters, so concurrent calls on distinct streams need distinct workspaces)
 * must hold cbv2_search_workspace_size(index, B, k, scorer) bytes;
 * cbv2_search_workspace_bytes(index, B) is enough for any k and scorer.
 * With CBV2_OPT_FUSED_TOPK on, MaxSim with k <= 104 on the bf16
 * doc-interleaved scan (B > 16) fuses the top-k into the scan (no [B][n]
 * score matrix: each workgroup keeps its best k per query in LDS, then one
 * selection per query); results are those of the unfused path bit for bit.
 * Any k >= 1 (torch.topk takes any k): k > 1024 selects in passes of 4096
 * keys, each bounded below the previous pass's last key (same tie rule).
 * Extends §8(b)'s prototype with scorer / q_dtype / workspace.  */
size_t cbv2_search_workspace_size(const cbv2_index* index, int32_t B, int32_t k, int32_t scorer);
size_t cbv2_search_workspace_bytes(const cbv2_index* index, int32_t B);
int cbv2_search(cbv2_index* index, int32_t scorer, const void* Q, int32_t q_dtype, int32_t B,
                int32_t lq, int32_t k, void* workspace, size_t workspace_bytes,
                float* out_scores, int32_t* out_ids, void* stream);

/* cbv2_rerank — JinaColBERTRetriever.rerank (local_rag_complete.py:779-800)
 * without re-encoding: the C candidate docs of each query are GATHERED from
 * the HBM index by global id (cand int32 [B][C]; ids outside this shard or < 0
 * score -inf) and MaxSim-scored against Q (bf16 [B][lq][128]).
 *  k > 0:  out_scores [B][k], out_ids [B][k] (global ids), out_pos [B][k]
 *          (candidate position = the reference's `result_index`), best first;
 *          slots past C hold -inf / -1 / -1.
 *  1 <= C <= 32768 (the reference's argsort takes any C, :789): C > 1024
 *  keeps the raw scores in dynamic LDS and selects in multiple passes.
 *  k == 0: out_scores [B][C] receives the raw candidate scores (for the
 *          sharded path: all-reduce(max) across shards, then cbv2_select_topk). */
int cbv2_rerank(cbv2_index* index, const void* Q, int32_t B, int32_t lq, const int32_t* cand,
                int32_t C, int32_t k, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                void* stream);

/* cbv2_rerank_ws — cbv2_rerank with a caller workspace of
 * cbv2_rerank_workspace_bytes(B, C) bytes: batches of up to 32 queries then
 * score one (query, candidate) per wave across the chip (the raw row in the
 * workspace) and select the top-k in a second kernel — the same scores, ids
 * and positions, bit for bit, as the one-workgroup-per-query kernel
 * cbv2_rerank uses (a B=1 rerank of 50 candidates otherwise runs 7 docs per
 * wave in sequence on one CU).  A null or short workspace, C > 1024 or
 * B > 32 take cbv2_rerank's path.  (cbv2_rerank with k == 0 and B <= 32 uses
 * the candidate-parallel kernel directly into out_scores.) */
size_t cbv2_rerank_workspace_bytes(int32_t B, int32_t C);
int cbv2_rerank_ws(cbv2_index* index, const void* Q, int32_t B, int32_t lq, const int32_t* cand,
                   int32_t C, int32_t k, void* workspace, size_t workspace_bytes, float* out_scores,
                   int32_t* out_ids, int32_t* out_pos, void* stream);

/* fp32-faithful index ---------------------------------------------------------
 * The reference keeps fp32 embeddings (local_rag_complete.py:735-746: the
 * encode output, torch.save'd as is) and scores them in fp32 (:802-831).  A
 * bf16 index alone is within ~5e-3 of those scores; this mode returns scores
 * within ~1e-5 and the top-k of those scores over the WHOLE corpus.
 *  - cbv2_split_f32: x f32 [rows][128] -> hi = bf16(x) (RNE; the index
 *    tokens) and lo = bf16(x - hi) (the residual), both bf16 [rows][128];
 *    bounds f32[2] (DEVICE, zeroed by the caller) receive max ||x - hi||_2 and
 *    max ||hi||_2 over the rows, rounded up (atomic max).  doclens (nullable,
 *    device int32 [rows / ld]): rows are docs of ld rows and padding rows
 *    (t >= doclens[doc]) are split but left out of the bounds.
 *  - cbv2_index_attach_residual: a bf16 index built on hi borrows lo and
 *    keeps the two bounds (host floats read back from cbv2_split_f32).
 * Queries are f32 [B][lq][128] (lq <= 32); every call needs a workspace of
 * cbv2_f32_workspace_bytes(index, op, B, lq, cap) bytes (16-B aligned), with
 * cap = the band capacity (SEARCH) or C (RERANK), 0 for SCORE.
 *  - cbv2_score_f32: faithful scores of every doc, out[b * ld_out + i]
 *    (lo.qhi + hi.qlo + hi.qhi on the bf16 MFMA, fp32 accumulate).
 *  - cbv2_search_f32: bf16 scan of hi (T), its top-k, whose faithful scores'
 *    minimum lb bounds the k-th faithful score from below; then every doc
 *    with T >= lb - beta(q) is rescored faithfully and the exact top-k of
 *    that band is returned.  beta(q) bounds |T - S| for every doc
 *    (Cauchy-Schwarz on the residuals of docs and query, plus accumulation
 *    slack), so the band holds the faithful top-k of the whole corpus.
 *    out_status int32 [B]: the band size, or -1 when the band exceeded `cap`
 *    (k <= cap <= 16384): that row was then recomputed on the device by the
 *    full faithful scan (cbv2_score_f32's arithmetic) and an exact top-k.
 *    k > 16384 (no band can hold it): every row takes the full scan (-1).
 *    Either way the result is the faithful top-k of the whole corpus; the
 *    call stays asynchronous (no host round trip).
 *  - cbv2_search_f32_begin / _finish: the same search in two calls, for a
 *    sharded corpus.  begin runs the scan and top-k and writes fk (DEVICE f32
 *    [B][k]): the exact faithful scores of the shard's bf16 top-k (-inf
 *    padded; all -inf for an empty shard).  The caller derives lb (DEVICE f32
 *    [B]) from them: the k-th largest of the fk of ALL shards (one all-gather)
 *    -- k docs of the corpus score at least that, so it is <= the global k-th
 *    faithful score; any such lower bound keeps the result exact (one shard:
 *    the minimum of its fk).  finish rescores only the docs with T >= lb -
 *    beta(q) and returns this shard's part of the global top-k (-inf / -1
 *    padded where fewer of its docs can reach it), which the cross-shard merge
 *    completes.  Same workspace between the two calls.
 *  - cbv2_rerank_f32: cbv2_rerank with faithful scores.                      */
#define CBV2_F32_SCORE 0
#define CBV2_F32_SEARCH 1
#define CBV2_F32_RERANK 2
int cbv2_split_f32(const float* x, int64_t rows, int32_t ld, const int32_t* doclens, void* hi, void* lo,
                   float* bounds, void* stream);
int cbv2_index_attach_residual(cbv2_index* index, const void* lo, float resid_max, float norm_max);
size_t cbv2_f32_workspace_bytes(const cbv2_index* index, int32_t op, int32_t B, int32_t lq, int32_t cap);
int cbv2_score_f32(cbv2_index* index, const float* Q, int32_t B, int32_t lq, void* workspace,
                   size_t workspace_bytes, float* out, int64_t ld_out, void* stream);
int cbv2_search_f32(cbv2_index* index, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap,
                    void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                    int32_t* out_status, void* stream);
int cbv2_search_f32_begin(cbv2_index* index, const float* Q, int32_t B, int32_t lq, int32_t k, int32_t cap,
                          void* workspace, size_t workspace_bytes, float* fk, float* out_scores, int32_t* out_ids,
                          int32_t* out_status, void* stream);
int cbv2_search_f32_finish(cbv2_index* index, int32_t B, int32_t lq, int32_t k, int32_t cap, void* workspace,
                           size_t workspace_bytes, const float* lb, float* out_scores, int32_t* out_ids,
                           int32_t* out_status, void* stream);
int cbv2_rerank_f32(cbv2_index* index, const float* Q, int32_t B, int32_t lq, const int32_t* cand,
                    int32_t C, int32_t k, void* workspace, size_t workspace_bytes, float* out_scores,
                    int32_t* out_ids, int32_t* out_pos, void* stream);

/* Selection -----------------------------------------------------------------
 * cbv2_select_topk — top-k of each row of a score matrix [B][C] (rerank after
 * the cross-shard all-reduce): rank counting in LDS for C <= 1024, the
 * multi-pass selection beyond (any C, any k).  ids (nullable) [B][C] maps
 * positions to doc ids (NULL: id = position).  Ties: lower position first.
 * out_pos (nullable) receives positions.                                    */
int cbv2_select_topk(const float* scores, const int32_t* ids, int32_t B, int32_t C, int32_t k,
                     float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream);

/* cbv2_topk_rows — top-k of each row of a large score matrix scores[b*ld + i],
 * i < n; ids written = id_base + i.  With a workspace of
 * cbv2_topk_workspace_bytes(B, n) bytes (0 for short rows) long rows use the
 * sampled-threshold filter + candidate sort; with workspace NULL, or on a
 * candidate overflow, the exact single-pass-per-digit radix select; k > 1024
 * selects in bounded passes (no workspace needed).  The result is identical
 * either way.                                                               */
size_t cbv2_topk_workspace_bytes(int32_t B, int64_t n);
int cbv2_topk_rows(const float* scores, int32_t B, int64_t n, int64_t ld, int32_t k,
                   int64_t id_base, void* workspace, size_t workspace_bytes,
                   float* out_scores, int32_t* out_ids, void* stream);

/* cbv2_merge_topk — merge G per-shard sorted top-k lists ([G][B][k] scores and
 * global ids, e.g. after an RCCL all-gather) into the global top-k [B][k].
 * Entries with id < 0 are padding (a suffix of each list).  Any k: lists of
 * G*k <= 8192 keys are staged in LDS, longer ones searched in place.        */
int cbv2_merge_topk(const float* in_scores, const int32_t* in_ids, int32_t G, int32_t B,
                    int32_t k, float* out_scores, int32_t* out_ids, void* stream);

/* Host fusion (HOST pointers, no GPU) --------------------------------------
 * cbv2_rrf_fuse — HybridRetriever._reciprocal_rank_fusion
 * (local_rag_complete.py:960-978) for B queries at once, followed by the
 * `[:50]` cut of :916 (C = 50): float64 1/(rrf_k + rank) sums in the
 * reference's order and a stable sort, so results and tie order are identical
 * to the Python.  bm25_ids [B][kb], colbert_ids [B][kc] (ids < 0 = padding);
 * out_ids [B][C] (-1 padded), out_scores [B][C] (nullable), out_count [B]
 * (nullable) = distinct ids per query.                                     */
int cbv2_rrf_fuse(const int32_t* bm25_ids, int32_t kb, const int32_t* colbert_ids, int32_t kc, int32_t B,
                  int32_t rrf_k, int32_t C, int32_t* out_ids, double* out_scores, int32_t* out_count);

/* Host BM25 (HOST pointers, no GPU) ---------------------------------------
 * Stage 1 of HybridRetriever.retrieve (local_rag_complete.py:937-950; the
 * reference uses bm25s: LRC:851-858, 939-945) over term ids (tokenisation
 * and stopwords stay in the caller).  Lucene BM25:
 *   idf = ln(1 + (N - df + 0.5) / (df + 0.5)),
 *   w   = idf * tf * (k1 + 1) / (tf + k1 * (1 - b + b * |d| / avgdl)),
 * summed over the query's term ids in query order, repeats included (bm25s
 * sums the postings of every query token).  Corpus as CSR: doc i's term ids are
 * doc_terms[doc_offsets[i] .. doc_offsets[i+1]).  Search: queries as CSR,
 * out_ids [B][k] (score desc, then doc id asc; padded with the lowest-id
 * zero-score docs, then -1), out_scores [B][k] (nullable).  n_threads <= 0:
 * min(16, hardware threads).  Parity with bm25s itself: unpinned.          */
typedef struct cbv2_bm25 cbv2_bm25;
int cbv2_bm25_build(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int32_t vocab,
                    float k1, float b, cbv2_bm25** out);
int cbv2_bm25_search(const cbv2_bm25* index, const int32_t* q_terms, const int64_t* q_offsets, int32_t B,
                     int32_t k, int32_t n_threads, int32_t* out_ids, float* out_scores);
/* Sharded BM25 (no reference counterpart): a rank indexes
 * only its doc range [id_base, id_base + n_docs) but with the GLOBAL
 * statistics (n_global docs, total_global tokens, df_global [vocab] from an
 * all-reduce of cbv2_bm25_doc_freq), so every weight equals the unsharded
 * index's; search then returns global ids (local + id_base), and merging the
 * ranks' lists by (score desc, id asc) reproduces the unsharded top-k.      */
int cbv2_bm25_doc_freq(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int32_t vocab,
                       int64_t* df_out);
int cbv2_bm25_build_shard(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int32_t vocab,
                          float k1, float b, int64_t id_base, int64_t n_global, int64_t total_global,
                          const int64_t* df_global, cbv2_bm25** out);
int64_t cbv2_bm25_num_docs(const cbv2_bm25* index);
int cbv2_bm25_destroy(cbv2_bm25* index);

/* English stemmer (HOST pointers, no GPU): the Snowball English ("Porter2")
 * algorithm PyStemmer's Stemmer("english") implements, which the reference
 * passes to bm25s.tokenize (local_rag_complete.py:851-855, 939-943).  Words
 * are UTF-8, lower-cased by the caller; word i = words[offsets[i] ..
 * offsets[i+1]).  Stems go to out (out_cap >= offsets[n] - offsets[0]
 * suffices: no stem is longer than its word), out_offsets [n + 1].        */
int cbv2_stem_en(const char* words, const int64_t* offsets, int64_t n, char* out, int64_t out_cap,
                 int64_t* out_offsets);

/* Native index file (replaces the torch.save/torch.load of
 * indexes/colbert/index.pt at local_rag_complete.py:743-746, 751 for large
 * corpora — the index.pt reader stays in Python).  One flat file: a 4 KiB
 * header, int32 doclens [n], tokens [n][ld][128] (bf16, or e4m3 bytes) and,
 * for MXFP8, E8M0 scales [n][ld][2]; each section 4 KiB-aligned.  ld = 128
 * token slots (the functions without _ld), or 256 / 512 / 1024 for a bf16
 * long-document index (the _ld variants); readers take ld from the header.
 * cbv2_index_file_write  — DEVICE pointers (an HBM-resident index), D2H in
 *                          64 MiB pinned chunks overlapped with pwrite.
 * cbv2_index_file_read   — docs [begin, end) into DEVICE buffers (tokens
 *                          (end-begin)*ld*128*elem bytes, scales, doclens):
 *                          pread (O_DIRECT where aligned) into two pinned
 *                          buffers overlapped with H2D copies on `stream`;
 *                          returns when the data is in HBM.
 * cbv2_index_file_info   — dtype, doc count and id_base of a file
 *                          (cbv2_index_file_info_ld: and its ld).
 * *_host variants: HOST pointers, no GPU involved.                          */
int cbv2_index_file_info(const char* path, int32_t* dtype, int64_t* n, int64_t* id_base);
int cbv2_index_file_info_ld(const char* path, int32_t* dtype, int64_t* n, int64_t* id_base, int32_t* ld);
int cbv2_index_file_write_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, const void* tokens,
                             const void* scales, const int32_t* doclens, int64_t id_base, void* stream);
int cbv2_index_file_write_host_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, const void* tokens,
                                  const void* scales, const int32_t* doclens, int64_t id_base);
int cbv2_index_file_write(const char* path, int32_t dtype, int64_t n, const void* tokens, const void* scales,
                          const int32_t* doclens, int64_t id_base, void* stream);
int cbv2_index_file_read(const char* path, int64_t begin, int64_t end, void* tokens, void* scales, int32_t* doclens,
                         void* stream);
int cbv2_index_file_write_host(const char* path, int32_t dtype, int64_t n, const void* tokens, const void* scales,
                               const int32_t* doclens, int64_t id_base);
int cbv2_index_file_read_host(const char* path, int64_t begin, int64_t end, void* tokens, void* scales,
                              int32_t* doclens);

/* Streaming index writer (bounded-memory ingest): declare the
 * doc count, append contiguous batches (DEVICE pointers with on_device = 1 --
 * D2H through 64 MiB pinned buffers on `stream` -- or HOST pointers), close.
 * The header is written by close() only when every declared doc was
 * appended; close() after an incomplete ingest (or a failed header write)
 * deletes the file and returns CBV2_EINVAL, so an interrupted ingest never
 * leaves a file behind, valid-looking or not.
 * Host memory is two staging buffers whatever the corpus size.             */
typedef struct cbv2_index_writer cbv2_index_writer;
int cbv2_index_writer_open(const char* path, int32_t dtype, int64_t n, int64_t id_base, cbv2_index_writer** out);
int cbv2_index_writer_open_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, int64_t id_base,
                              cbv2_index_writer** out);
int cbv2_index_writer_append(cbv2_index_writer* w, int64_t count, const void* tokens, const void* scales,
                             const int32_t* doclens, int32_t on_device, void* stream);
int64_t cbv2_index_writer_count(const cbv2_index_writer* w);
int cbv2_index_writer_close(cbv2_index_writer* w);

/* Multi-GPU exchange (SURVEY.md §8(b) "cbv2_comm_init(ncclComm_t) +
 * cbv2_search_sharded", §8(e)).  No reference counterpart: the reference is
 * single-process.  One process per GPU, each holding the shard
 * [id_base, id_base + n) of the corpus as a cbv2_index.
 *
 * cbv2_comm_init — borrow an initialised RCCL communicator (ncclComm_t; e.g.
 *   torch's ProcessGroupNCCL._comm_ptr()).  rccl_library: path of the RCCL
 *   library that created it (NULL: "librccl.so"); the collectives are
 *   resolved from that library.  cbv2_comm_destroy does not free the comm.
 * cbv2_search_sharded — every rank: local scan + top-k, plus (kb > 0) this
 *   rank's stage-1 BM25 top-kb over its doc shard (global ids; host or device
 *   pointers), -> ONE ncclAllGather -> merged global top-k [B][k] and merged
 *   BM25 ids [B][kb] (out_lex_ids, device), identical on every rank.
 *   Workspace: cbv2_sharded_workspace_bytes(ix, comm, B, k, kb, 0).
 *   The same in two calls, so a host stage-1 can run while the GPU scans:
 *   cbv2_search_sharded_local (enqueue the local scan) then
 *   cbv2_search_sharded_exchange (lists in, all-gather, merges) with the SAME
 *   workspace, sized for the exchange's kb (the local call writes only the
 *   head of the send block; its kb just sizes its workspace check).
 *   Q (nullable; the local call's queries, q_dtype, lq): with kb > 0 the
 *   exchange first scores this rank's own BM25 top-kb with the rerank's
 *   arithmetic (raw MaxSim; faithful shards on the local call's query split)
 *   and those prescores ride the same all-gather.
 * cbv2_rerank_sharded_prescored — stage 3 with NO collective, after an
 *   exchange with Q (or kb = 0) on the same workspace with the same B, k, kb:
 *   the fused candidates (RRF of the exchange's merged lists, as
 *   cbv2_retrieve_finish builds them) all sit in the gathered blocks -- in
 *   their owner's stage-2 top-k (whose scores are the rerank's bits) or its
 *   BM25 top-kb (prescored) -- so every rank looks their scores up and selects
 *   the top final_k (score desc, position asc), as cbv2_rerank_sharded would.
 *   cand [B][C] device, C <= 1024.  A candidate found in no list scores -inf
 *   and is counted into *misses (device int32, nullable; the caller zeroes
 *   it): candidates from elsewhere take cbv2_rerank_sharded.
 * cbv2_rerank_sharded — every rank scores the candidates it owns (-inf
 *   otherwise) -> ncclAllReduce(MAX) -> top-k select; cand [B][C] global ids
 *   (device).  Workspace: the size above with C (a bf16 / MXFP8 shard needs
 *   only B*C*4 bytes).
 * cbv2_comm_stats (diagnostic): out2 = {all-gathers, all-reduces} issued on
 *   the handle so far.
 * fp32-faithful shards (cbv2_index_attach_residual; Q f32, q_dtype
 *   CBV2_DTYPE_F32): the local call runs the faithful search against the
 *   GLOBAL k-th bound -- bf16 scan + top-k + the exact faithful scores of that
 *   top-k (cbv2_search_f32_begin), ONE ncclAllGather of those [B][k] scores,
 *   their union's k-th largest as lb, the band rescoring (cbv2_search_f32_finish,
 *   band capacity CBV2_RETRIEVE_BAND_CAP) -- so the local call is itself a
 *   collective; the rerank scores the owned candidates faithfully
 *   (cbv2_rerank_f32).  Results equal the unsharded faithful search / rerank
 *   bit for bit.
 * Collectives are enqueued on `stream`; every rank must call in the same
 * order (as with any RCCL program).                                        */
typedef struct cbv2_comm cbv2_comm;
int cbv2_comm_init(void* nccl_comm, const char* rccl_library, cbv2_comm** out);
int cbv2_comm_size(const cbv2_comm* comm);
int cbv2_comm_rank(const cbv2_comm* comm);
int cbv2_comm_destroy(cbv2_comm* comm);
size_t cbv2_sharded_workspace_bytes(const cbv2_index* index, const cbv2_comm* comm, int32_t B, int32_t k,
                                    int32_t kb, int32_t C);
int cbv2_search_sharded(cbv2_index* index, cbv2_comm* comm, int32_t scorer, const void* Q, int32_t q_dtype,
                        int32_t B, int32_t lq, int32_t k, const int32_t* lex_ids, const float* lex_scores,
                        int32_t kb, void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                        int32_t* out_lex_ids, void* stream);
int cbv2_search_sharded_local(cbv2_index* index, cbv2_comm* comm, int32_t scorer, const void* Q, int32_t q_dtype,
                              int32_t B, int32_t lq, int32_t k, int32_t kb, void* workspace, size_t workspace_bytes,
                              void* stream);
int cbv2_search_sharded_exchange(cbv2_index* index, cbv2_comm* comm, const void* Q, int32_t q_dtype, int32_t lq,
                                 int32_t B, int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb,
                                 void* workspace, size_t workspace_bytes, float* out_scores, int32_t* out_ids,
                                 int32_t* out_lex_ids, void* stream);
int cbv2_rerank_sharded_prescored(cbv2_index* index, cbv2_comm* comm, int32_t B, int32_t k, int32_t kb,
                                  const int32_t* cand, int32_t C, int32_t final_k, void* workspace,
                                  size_t workspace_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos,
                                  int32_t* misses, void* stream);
int cbv2_rerank_sharded(cbv2_index* index, cbv2_comm* comm, const void* Q, int32_t B, int32_t lq,
                        const int32_t* cand, int32_t C, int32_t k, void* workspace, size_t workspace_bytes,
                        float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream);
int cbv2_comm_stats(const cbv2_comm* comm, int64_t* out2);

/* TEST-ONLY -- not for production use.  cbv2_comm_loopback_init writes
 * `nranks` (1..64) communicator handles out[0..nranks) that form ONE group
 * inside this process, on the current device: rank r is driven by its own
 * host thread and stream, and the collectives the calls above use keep RCCL's
 * semantics (every rank calls; a call returns once every rank has enqueued;
 * no rank's stream passes the collective before all peers' data is in):
 * all-gather = device copies of the G send blocks, all-reduce(MAX) = a max
 * kernel over them.  It exercises the sharded exchange at G > 1 on one GPU.
 * A rank that does not reach a collective within 60 s fails the group.
 * Free each handle with cbv2_comm_destroy.                                  */
int cbv2_comm_loopback_init(int32_t nranks, cbv2_comm** out);

/* One query batch through HybridRetriever.retrieve's stages 2 -> RRF -> 3
 * (local_rag_complete.py:894-935) with ONE host round trip and no caller code
 * between the stages (the latency path: no D2H / RRF / H2D / launch hops in the
 * host language).  Replaces the sequence _colbert_search (:952-958) ->
 * _reciprocal_rank_fusion (:960-978) -> [:C] (:916) -> _colbert_rerank
 * (:996-1014) for the caller; results equal those of the separate calls
 * (cbv2_search[_f32] / cbv2_search_sharded_*, cbv2_rrf_fuse, cbv2_rerank_ws /
 * _f32 / cbv2_rerank_sharded) bit for bit.
 *  comm: NULL for one shard; else a cbv2_comm (the exchange above, for
 *        bf16, MXFP8 and fp32-faithful shards alike).
 *  Q:    the index's query type: bf16 [B][lq][128] (bf16 index), the
 *        cbv2_quantize_mxfp8 buffer (MXFP8), f32 (fp32-faithful); lq <= 32.
 *  cbv2_retrieve_begin enqueues stage 2 (this shard's scan + top-k; the band
 *    capacity of a faithful search is CBV2_RETRIEVE_BAND_CAP) and returns:
 *    the caller runs stage 1 (host BM25) meanwhile.  Its kb is an upper
 *    bound of the kb finish will pass (the stage-1 list width is known only
 *    after stage 1 ran); B, lq, k, C and the workspace must be the same.
 *  cbv2_retrieve_finish takes the stage-1 lists (HOST pointers: lex_ids
 *    [B][kb] global ids, -1 padded; lex_scores [B][kb], read only with a
 *    comm; kb = 0: no stage 1), (comm: all-gather + merges), copies the
 *    ColBERT top-k to host_stage, WAITS for it (the round trip), fuses on the
 *    host (cbv2_rrf_fuse with rrf_k, first C), uploads the candidates and
 *    enqueues the rerank + select: out_scores f32 [B][final_k], out_ids
 *    int32 [B][final_k] (global ids), out_pos int32 [B][final_k] (position
 *    in the fused list), device, best first, -inf / -1 padded.  One shard,
 *    B <= 8, bf16 / fp32-faithful: the rerank's scores are already known
 *    (stage 2's own for its ids; a stage-1 prescore of the kb lists, launched
 *    at finish entry on a second stream of the calling thread), so the host
 *    picks the top final_k itself and a one-workgroup kernel copies it into
 *    the device outputs (same results, bit for bit).
 *  workspace: device, 256-B aligned, cbv2_retrieve_workspace_bytes(index,
 *    comm, B, lq, k, kb, C) bytes, the same one for begin and finish;
 *    host_stage: host (pinned for asynchronous copies),
 *    cbv2_retrieve_host_bytes(B, k, kb, C) bytes, one per stream.
 *  Q at finish: the same buffer and contents as at begin.  For a single
 *    fp32-faithful shard finish reuses the query split begin left in the
 *    workspace while it is still the last split enqueued there (same index,
 *    Q pointer, B, lq); if anything split other queries into that workspace
 *    in between, finish splits Q again (same results either way).
 *  Both calls select the index's device themselves (the caller's current
 *    device may differ) and restore the caller's.  finish's wait polls the
 *    stream (hipStreamQuery) -- flat out for B <= 8, sleeping between polls
 *    for larger batches, so it never holds a core for a whole batch scan;
 *    the stream must carry no other thread's work meanwhile.  A one-shard
 *    call takes a device-mapped host buffer from a per-device pool at begin
 *    (the search's final select writes the ids into it, the fused candidates
 *    go into it and the rerank reads them in place) and returns it at finish,
 *    reusable once that rerank has run.
 * cbv2_retrieve_finish_host: finish, and the final top-k also in the HOST
 *    arrays host_scores / host_ids / host_pos ([B][final_k], any host memory)
 *    when it returns (the reference's retrieve returns host results,
 *    LRC:935).  One shard: the final select writes them into the call's
 *    mapped buffer as tagged words and the host polls them (no D2H copy, no
 *    stream wait); otherwise they are copied down and waited for.  The
 *    device outputs are written as by finish.
 * cbv2_retrieve_cancel: a begin that will not be finished (the caller's
 *    stage 1 failed): returns its host buffer to the pool (no-op otherwise).
 * cbv2_retrieve_host_marks (diagnostic): host timestamps (steady_clock ns) of
 *    this thread's last finish: enter, D2H issued, wait done, fusion done,
 *    rerank enqueued (the host rerank: its select done), exit (max entries
 *    written, up to 6).
 * cbv2_retrieve_pool_stats (diagnostic): [0] mapped buffers created in this
 *    process, [1] buffers idle in the pools (at most the number of calls that
 *    ever ran at once), [2] finish_host calls whose results were read from the
 *    final select's host words, [3] finish calls that picked the final top-k
 *    on the host (one shard, B <= 8, bf16 / fp32-faithful: every fused
 *    candidate's score is stage 2's own or stage 1's prescore).
 * cbv2_index_kind: the index's dtype (CBV2_DTYPE_*) and whether a residual is
 *    attached (fp32-faithful, 1) or not (0).                                */
#define CBV2_RETRIEVE_BAND_CAP 16384
int cbv2_index_kind(const cbv2_index* index, int32_t* dtype, int32_t* faithful);
size_t cbv2_retrieve_workspace_bytes(const cbv2_index* index, const cbv2_comm* comm, int32_t B, int32_t lq,
                                     int32_t k, int32_t kb, int32_t C);
size_t cbv2_retrieve_host_bytes(int32_t B, int32_t k, int32_t kb, int32_t C);
int cbv2_retrieve_cancel(cbv2_index* index, void* workspace, void* stream);
int cbv2_retrieve_host_marks(int64_t* out, int32_t max);
int cbv2_retrieve_pool_stats(int64_t* out, int32_t max);
int cbv2_retrieve_begin(cbv2_index* index, cbv2_comm* comm, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                        int32_t k, int32_t kb, int32_t C, void* workspace, size_t workspace_bytes, void* stream);
int cbv2_retrieve_finish(cbv2_index* index, cbv2_comm* comm, const void* Q, int32_t q_dtype, int32_t B, int32_t lq,
                         int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb, int32_t rrf_k,
                         int32_t C, int32_t final_k, void* workspace, size_t workspace_bytes, void* host_stage,
                         size_t host_bytes, float* out_scores, int32_t* out_ids, int32_t* out_pos, void* stream);
int cbv2_retrieve_finish_host(cbv2_index* index, cbv2_comm* comm, const void* Q, int32_t q_dtype, int32_t B,
                              int32_t lq, int32_t k, const int32_t* lex_ids, const float* lex_scores, int32_t kb,
                              int32_t rrf_k, int32_t C, int32_t final_k, void* workspace, size_t workspace_bytes,
                              void* host_stage, size_t host_bytes, float* out_scores, int32_t* out_ids,
                              int32_t* out_pos, float* host_scores, int32_t* host_ids, int32_t* host_pos,
                              void* stream);

#ifdef __cplusplus
}
#endif
#endif /* COLBERT_MI355X_H */
