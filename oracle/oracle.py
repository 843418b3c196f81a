"""CPU ORACLE for the ColBERT retrieval hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / the timed CPU baseline.  The product
(hybrid-rag-colbertv2_amd/) never calls it: it has no CPU fallback.

Each function restates the reference's arithmetic in numpy, citing the
reference line it follows (LRC = /root/reference/local_rag_complete.py):

  meanpool_cosine   LRC:814-831  _maxsim_score as written (mean-pool + cosine,
                                 torch's x/max(||x||,eps) form of cosine_similarity)
  maxsim            the north-star contract the reference's docstring describes
                    (LRC:807-812): S = sum_q max_t <q, d_t>, padded rows excluded
  topk              LRC:767 torch.topk, with the tie rule made explicit:
                    score desc, then lower index
  rerank_select     LRC:789-798 argsort(desc)[:k] + 1-based rank, same tie rule
  rrf               LRC:960-978 reciprocal rank fusion, float64, stable sort
  merge_topk        cross-shard merge (no reference counterpart; exact by the
                    same tie rule)
  split_f32 /       the fp32-faithful index (LRC:735-746 keeps fp32 embeddings):
  band_beta         hi/lo split and the bound |T - S| <= beta(q) the faithful
                    search's band rests on
  codebook_*        maxsim + topk for corpora whose tokens are rows of a small
                    codebook: max_t <q, d_t> is the max over the doc's code SET,
                    so a 1M-doc corpus is scored exactly in seconds (checked
                    against maxsim itself in tests/test_oracle_golden.py)

Pinning: meanpool_cosine, rrf and the search/rerank
dict pipeline are checked against golden vectors produced by the reference's
own functions (tests/golden/gen_golden.py, AST-extracted from LRC).  maxsim is
pinned (a) at one doc token, where the reference's ranking equals MaxSim's
(tests/golden/single_token.npz), and (b) by exact-rational known answers on
the k/16 grid (tests/golden/exact_grid.npz).
"""
from __future__ import annotations

import ctypes
import os
from typing import List, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


# ------------------------------------------------------------------ bf16 helpers
def to_bf16_bits(x: np.ndarray) -> np.ndarray:
    """float32 -> bf16 bit patterns, round-to-nearest-even (torch's .to(bfloat16))."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = (u + 0x7FFF + ((u >> 16) & 1)) >> 16
    return r.astype(np.uint16)


def from_bf16_bits(b: np.ndarray) -> np.ndarray:
    return (np.asarray(b, dtype=np.uint16).astype(np.uint32) << 16).view(np.float32)


def bf16_round(x: np.ndarray) -> np.ndarray:
    return from_bf16_bits(to_bf16_bits(x))


# ------------------------------------------------------------------ MXFP8 helpers
def _e4m3_table() -> np.ndarray:
    """OCP e4m3fn decode of all 256 byte values (0x7F / 0xFF are NaN)."""
    t = np.empty(256, np.float64)
    for v in range(256):
        s, e, m = v >> 7, (v >> 3) & 15, v & 7
        x = (m / 8.0) * 2.0 ** -6 if e == 0 else (1 + m / 8.0) * 2.0 ** (e - 7)
        t[v] = -x if s else x
    t[0x7F] = t[0xFF] = np.nan
    return t


E4M3 = _e4m3_table()


def mxfp8_dequant(q: np.ndarray, scales: np.ndarray) -> np.ndarray:
    """e4m3 bytes [..., 128] + E8M0 scales [..., 2] (one per 64 dims) -> float64 values."""
    vals = E4M3[np.asarray(q, np.uint8)]
    mult = np.exp2(np.asarray(scales, np.float64) - 127.0)
    return vals * np.repeat(mult, 64, axis=-1)


def mxfp8_quantize(x: np.ndarray):
    """Restatement of cbv2_quantize_mxfp8: per 64-value half, e = the smallest integer
    with max|x| <= 448 * 2^e (0 for an all-zero half), bytes = RNE(x / 2^e) in e4m3."""
    x = np.asarray(x, np.float32).astype(np.float64)
    h = x.reshape(*x.shape[:-1], 2, 64)
    m = np.abs(h).max(axis=-1)
    f, p = np.frexp(m)                                   # m = f * 2^p, f in [0.5, 1)
    e = np.where(f <= 0.875, p - 9, p - 8)
    e = np.where(m > 0, np.clip(e, -127, 127), 0)
    y = h / np.exp2(e)[..., None]
    a = np.abs(y)
    E = np.floor(np.log2(np.where(a > 0, a, 1.0)))
    E = np.maximum(E, -6.0)                              # subnormals share the 2^-6 binade's quantum
    quantum = np.exp2(E - 3)
    r = np.round(a / quantum) * quantum                  # numpy rounds half to even
    pos = {float(E4M3[v]): v for v in range(0x7F)}
    code = np.vectorize(lambda z: pos[float(z)])(r).astype(np.uint8)
    code = np.where(np.signbit(y), code | 0x80, code).astype(np.uint8)   # sign kept, also for -0 (as the hardware)
    return code.reshape(x.shape), (e + 127).astype(np.uint8)


# ------------------------------------------------------------------ scorers
def maxsim(Q: np.ndarray, docs: np.ndarray, doclens: np.ndarray | None = None,
           dtype=np.float64) -> np.ndarray:
    """True MaxSim: Q [B, lq, D], docs [N, L, D] -> [B, N] (float64 by default;
    dtype=np.float32 is the reference's own CPU arithmetic, used as the timed baseline).

    Rows t >= doclens[n] never score; an empty doc scores -inf.
    """
    Q = np.asarray(Q, dtype=dtype)
    if Q.ndim == 2:
        Q = Q[None]
    docs = np.asarray(docs, dtype=dtype)
    N, L, _ = docs.shape
    if doclens is None:
        doclens = np.full(N, L, np.int64)
    valid = np.arange(L)[None, :] < np.asarray(doclens)[:, None]            # [N, L]
    out = np.empty((Q.shape[0], N), dtype)
    for b in range(Q.shape[0]):
        sim = np.einsum("nld,qd->nlq", docs, Q[b], optimize=True)           # [N, L, lq]
        sim = np.where(valid[:, :, None], sim, -np.inf)
        out[b] = sim.max(axis=1).sum(axis=1)
    return out


def meanpool_cosine(Q: np.ndarray, docs: np.ndarray, doclens: np.ndarray | None = None,
                    eps: float = 1e-8) -> np.ndarray:
    """LRC:814-831: cosine(mean_t q_t, mean_t d_t) -> [B, N] (float64).

    The reference averages every stored row; with doclens, the first doclens[n]
    rows are the stored rows.  Cosine as torch computes it: each vector divided
    by max(||v||, eps), then the sum of products.
    """
    Q = np.asarray(Q, dtype=np.float64)
    if Q.ndim == 2:
        Q = Q[None]
    docs = np.asarray(docs, dtype=np.float64)
    N, L, _ = docs.shape
    if doclens is None:
        doclens = np.full(N, L, np.int64)
    doclens = np.asarray(doclens)
    valid = (np.arange(L)[None, :] < doclens[:, None]).astype(np.float64)
    dsum = np.einsum("nld,nl->nd", docs, valid)
    dmean = dsum / np.maximum(doclens, 1)[:, None]
    dmean[doclens == 0] = 0.0
    qmean = Q.mean(axis=1)
    dn = dmean / np.maximum(np.linalg.norm(dmean, axis=1, keepdims=True), eps)
    qn = qmean / np.maximum(np.linalg.norm(qmean, axis=1, keepdims=True), eps)
    return qn @ dn.T


# ------------------------------------------------------------------ fp32-faithful index
def split_f32(x: np.ndarray, doclens: np.ndarray | None = None):
    """cbv2_split_f32: fp32 [N, L, D] -> (hi = bf16(x), lo = bf16(x - hi), (max ||x - hi||, max ||hi||)),
    the maxima over the scoring rows (t < doclens[n])."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    hi = bf16_round(x)
    r = x - hi                                      # exact in fp32
    lo = bf16_round(r)
    rn = np.linalg.norm(r.astype(np.float64), axis=-1)
    hn = np.linalg.norm(hi.astype(np.float64), axis=-1)
    if doclens is not None:
        valid = np.arange(x.shape[1])[None, :] < np.asarray(doclens)[:, None]
        rn, hn = rn[valid], hn[valid]
    return hi, lo, (float(rn.max(initial=0.0)), float(hn.max(initial=0.0)))


def band_beta(Q: np.ndarray, resid_max: float, norm_max: float, slack: float = 2.0 ** -12) -> np.ndarray:
    """split_query_kernel's beta(q) (without its fp32 round-up):
    sum_i ||q_i|| E + ||q_i - bf16(q_i)|| M + slack (||q_i|| + ||q_i - bf16(q_i)||) M.

    For every doc, |maxsim(bf16 Q, hi) - maxsim(Q, x)| <= beta (Cauchy-Schwarz on
    <q, x - hi> and <q - bf16(q), hi>; slack covers fp32/MFMA accumulation)."""
    Q = np.asarray(Q, np.float32)
    if Q.ndim == 2:
        Q = Q[None]
    q = Q.astype(np.float64)
    nq = np.linalg.norm(q, axis=-1)
    eq = np.linalg.norm(q - bf16_round(Q).astype(np.float64), axis=-1)
    return (nq * resid_max + eq * norm_max + slack * (nq + eq) * norm_max).sum(axis=-1)


# ------------------------------------------------------------------ selection
def topk(scores: np.ndarray, k: int, id_base: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """LRC:767 with ties -> lower index.  [B, N] -> (scores [B, k], ids [B, k]); pads -inf / -1."""
    s = np.atleast_2d(np.asarray(scores))
    B, N = s.shape
    kk = min(k, N)
    out_s = np.full((B, k), -np.inf, np.float64)
    out_i = np.full((B, k), -1, np.int64)
    idx = np.arange(N)
    for b in range(B):
        order = np.lexsort((idx, -s[b].astype(np.float64)))[:kk]
        out_s[b, :kk] = s[b, order]
        out_i[b, :kk] = order + id_base
    return out_s, out_i


def rerank_select(scores: np.ndarray, k: int):
    """LRC:789-798: positions sorted by score desc (ties: lower position), [:k], 1-based ranks."""
    s = np.asarray(scores, dtype=np.float64)
    order = np.lexsort((np.arange(len(s)), -s))[:k]
    return [(int(p), float(s[p]), r + 1) for r, p in enumerate(order)]


def rerank(Q: np.ndarray, docs: np.ndarray, doclens: np.ndarray, cand: np.ndarray, k: int, id_base: int = 0):
    """MaxSim of each query's candidate ids (global), then top-k by (score desc, position asc).

    Returns (scores [B, k], ids [B, k], positions [B, k]); out-of-shard / negative ids score -inf.
    """
    Q = np.asarray(Q, np.float64)
    cand = np.atleast_2d(np.asarray(cand, np.int64))
    B, C = cand.shape
    N = docs.shape[0]
    out_s = np.full((B, k), -np.inf)
    out_i = np.full((B, k), -1, np.int64)
    out_p = np.full((B, k), -1, np.int64)
    for b in range(B):
        sc = np.full(C, -np.inf)
        for c in range(C):
            loc = cand[b, c] - id_base
            if cand[b, c] >= 0 and 0 <= loc < N:
                sc[c] = maxsim(Q[b:b + 1], docs[loc:loc + 1], doclens[loc:loc + 1])[0, 0]
        order = np.lexsort((np.arange(C), -sc))[:k]
        m = len(order)
        out_s[b, :m] = sc[order]
        out_i[b, :m] = cand[b, order]
        out_p[b, :m] = order
    return out_s, out_i, out_p


def merge_topk(scores: np.ndarray, ids: np.ndarray, k: int):
    """[G, B, k] per-shard lists -> global [B, k]; padding ids < 0 ignored."""
    G, B, _ = scores.shape
    out_s = np.full((B, k), -np.inf)
    out_i = np.full((B, k), -1, np.int64)
    for b in range(B):
        s = scores[:, b].reshape(-1).astype(np.float64)
        i = ids[:, b].reshape(-1).astype(np.int64)
        keep = i >= 0
        s, i = s[keep], i[keep]
        order = np.lexsort((i, -s))[:k]
        out_s[b, :len(order)] = s[order]
        out_i[b, :len(order)] = i[order]
    return out_s, out_i


# ------------------------------------------------------------------ BM25 (stage 1)
def bm25_topk(doc_terms, doc_offsets, q_terms, q_offsets, vocab: int, k: int, k1: float = 1.5, b: float = 0.75):
    """Lucene BM25 as bm25s scores it (LRC:851-858, 939-945; bm25s absent here, so
    its published formula), restated with the C++ index's exact operation order
    so every float matches: weights in float64 -> float32, the query's term ids in
    query order with repeats (bm25s sums the postings of every query token),
    float32 accumulation in doc order, ties -> lower doc id, all docs ranked."""
    import math
    k1, b = float(np.float32(k1)), float(np.float32(b))      # the C ABI takes them as float
    doc_terms = np.asarray(doc_terms, np.int64)
    doc_offsets = np.asarray(doc_offsets, np.int64)
    N = len(doc_offsets) - 1
    avgdl = float(int(doc_offsets[-1])) / N if N else 1.0
    per_doc = []
    df = np.zeros(vocab, np.int64)
    for d in range(N):
        t, tf = np.unique(doc_terms[doc_offsets[d]:doc_offsets[d + 1]], return_counts=True)
        per_doc.append((t, tf, int(doc_offsets[d + 1] - doc_offsets[d])))
        df[t] += 1
    idf = [math.log(1.0 + (N - int(df[t]) + 0.5) / (int(df[t]) + 0.5)) for t in range(vocab)]
    post = [[] for _ in range(vocab)]
    for d, (ts, tfs, dl) in enumerate(per_doc):
        for t, tf in zip(ts.tolist(), tfs.tolist()):
            norm = tf + k1 * (1.0 - b + b * dl / avgdl)
            post[t].append((d, np.float32(idf[t] * tf * (k1 + 1.0) / norm)))
    B = len(q_offsets) - 1
    out_i = np.full((B, k), -1, np.int64)
    out_s = np.zeros((B, k), np.float32)
    for qb in range(B):
        acc = np.zeros(N, np.float32)
        for t in (int(x) for x in q_terms[q_offsets[qb]:q_offsets[qb + 1]]):
            if 0 <= t < vocab:
                for d, w in post[t]:
                    acc[d] = np.float32(acc[d] + w)
        order = np.lexsort((np.arange(N), -acc))[:k]
        out_i[qb, :len(order)] = order
        out_s[qb, :len(order)] = acc[order]
    return out_i, out_s


# ------------------------------------------------------------------ fusion
def rrf(bm25_ids: Sequence[int], colbert_ids: Sequence[int], k: int = 60) -> List[Tuple[int, float]]:
    """LRC:960-978: score[id] += 1/(k + rank) over the BM25 list, then the ColBERT
    list (rank 1-based); Python float64; sorted(..., reverse=True) is stable, so
    equal scores keep first-insertion order."""
    scores = {}
    for rank, cid in enumerate(bm25_ids, 1):
        scores[cid] = scores.get(cid, 0) + (1 / (k + rank))
    for rank, cid in enumerate(colbert_ids, 1):
        scores[cid] = scores.get(cid, 0) + (1 / (k + rank))
    return sorted(scores.items(), key=lambda x: x[1], reverse=True)


# ------------------------------------------------------------------ C restatement
_CLIB = None
C_LIB_PATH = os.path.join(HERE, "_build", "libcbv2_oracle.so")


def c_lib():
    """ctypes handle to oracle/cbv2_oracle.c (built by __graft_entry__.build())."""
    global _CLIB
    if _CLIB is None:
        if not os.path.exists(C_LIB_PATH):
            raise RuntimeError(f"{C_LIB_PATH} missing: build it with `make -C oracle`")
        L = ctypes.CDLL(C_LIB_PATH)
        L.oracle_maxsim_bf16.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
        L.oracle_topk.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_codebook_topk.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p]
        _CLIB = L
    return _CLIB


def c_maxsim_bf16(q_bits: np.ndarray, doc_bits: np.ndarray, doclens: np.ndarray) -> np.ndarray:
    """C restatement of maxsim on bf16 bit patterns: q [B, lq, 128], docs [N, L, 128] -> f64 [B, N]."""
    q_bits = np.ascontiguousarray(q_bits, np.uint16)
    doc_bits = np.ascontiguousarray(doc_bits, np.uint16)
    doclens = np.ascontiguousarray(doclens, np.int32)
    B, lq, D = q_bits.shape
    N, L, _ = doc_bits.shape
    assert D == 128
    out = np.empty((B, N), np.float64)
    c_lib().oracle_maxsim_bf16(q_bits.ctypes.data, B, lq, doc_bits.ctypes.data, doclens.ctypes.data, N, L,
                               out.ctypes.data)
    return out


def c_topk(scores_row: np.ndarray, k: int) -> np.ndarray:
    s = np.ascontiguousarray(scores_row, np.float64)
    ids = np.empty(k, np.int64)
    vals = np.empty(k, np.float64)
    c_lib().oracle_topk(s.ctypes.data, len(s), k, vals.ctypes.data, ids.ctypes.data)
    return ids


# ------------------------------------------------------------------ codebook corpora (exact 1M-doc parity)
def codebook_masks(codes: np.ndarray, doclens: np.ndarray, chunk: int = 65536) -> np.ndarray:
    """codes uint8 [n, L] (codebook row of every token slot), doclens [n] -> uint32 [n]:
    bit c set when code c fills one of doc n's scoring rows (t < doclens[n])."""
    codes = np.asarray(codes)
    doclens = np.asarray(doclens)
    n, L = codes.shape
    out = np.empty(n, np.uint32)
    t = np.arange(L)[None, :]
    for a in range(0, n, chunk):
        c = codes[a:a + chunk].astype(np.uint32)
        bits = np.where(t < doclens[a:a + chunk, None], np.left_shift(np.uint32(1), c), np.uint32(0))
        out[a:a + chunk] = np.bitwise_or.reduce(bits, axis=1)
    return out


def codebook_table(Q: np.ndarray, codebook: np.ndarray) -> np.ndarray:
    """T[b, q, c] = <Q[b, q], code_c> in float64: [B, lq, K]."""
    return np.einsum("bqd,cd->bqc", np.asarray(Q, np.float64), np.asarray(codebook, np.float64))


def codebook_maxsim(T: np.ndarray, masks: np.ndarray) -> np.ndarray:
    """maxsim() for codebook docs given by their code sets: [B, n] float64
    (sum over q of the max over the doc's codes; an empty set scores -inf)."""
    T = np.asarray(T, np.float64)
    K = T.shape[2]
    bits = ((np.asarray(masks, np.uint64)[:, None] >> np.arange(K, dtype=np.uint64)) & 1).astype(bool)   # [n, K]
    v = np.where(bits[None, None], T[:, :, None, :], -np.inf).max(axis=3)                               # [B, lq, n]
    return v.sum(axis=1)


def codebook_topk(T: np.ndarray, masks: np.ndarray, k: int, over_ids=None, over_scores=None):
    """Top-k (score desc, id asc) of maxsim over a codebook corpus of n = len(masks)
    docs (C: oracle_codebook_topk).  over_ids [P] / over_scores [B, P]: docs whose
    scores the caller computed itself (planted docs with non-codebook tokens).
    -> (scores float64 [B, k], ids int64 [B, k])."""
    T = np.ascontiguousarray(T, np.float64)
    B, lq, K = T.shape
    assert K <= 32
    umask, inv = np.unique(np.asarray(masks, np.uint32), return_inverse=True)
    umask = np.ascontiguousarray(umask, np.uint32)
    inv = np.ascontiguousarray(inv.reshape(-1), np.int32)
    n = len(inv)
    over_idx = np.full(n, -1, np.int32)
    if over_ids is not None and len(over_ids):
        over_idx[np.asarray(over_ids, np.int64)] = np.arange(len(over_ids), dtype=np.int32)
        over = np.ascontiguousarray(over_scores, np.float64).reshape(B, len(over_ids))
    else:
        over = np.zeros((B, 1), np.float64)
    vals = np.empty((B, k), np.float64)
    ids = np.empty((B, k), np.int64)
    c_lib().oracle_codebook_topk(T.ctypes.data, B, lq, K, umask.ctypes.data, len(umask), inv.ctypes.data,
                                 over_idx.ctypes.data, over.ctypes.data, over.shape[1], n, int(k),
                                 vals.ctypes.data, ids.ctypes.data)
    return vals, ids
