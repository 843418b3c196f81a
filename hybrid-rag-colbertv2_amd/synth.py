"""Synthetic ColBERT corpora for benchmarks and size-independent checks.

SURVEY.md §8(d): doc and query tokens are L2-normalised N(0, I_128) vectors
(bf16 in HBM); each query has ``planted`` docs whose first ``lq`` tokens are
noisy copies of its tokens (noise norm ``sigma``), so the true top-10 is known
and well separated.  Generation is keyed by GLOBAL doc id ranges (fixed
chunks of ``CHUNK`` ids, one RNG seed per chunk), so any shard can build its
own range on its own GPU and every rank sees the same corpus.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

CHUNK = 16384
DIM = 128
LD = 128


def _unit(x: torch.Tensor) -> torch.Tensor:
    return x / x.norm(dim=-1, keepdim=True).clamp_min(1e-12)


def make_queries(B: int, lq: int = 32, seed: int = 1) -> torch.Tensor:
    """fp32 [B, lq, 128] unit tokens, generated on the host (identical on every rank)."""
    g = torch.Generator().manual_seed(seed)
    return _unit(torch.randn(B, lq, DIM, generator=g))


def planted_ids(B: int, n_total: int, per_query: int = 10, seed: int = 2) -> np.ndarray:
    """[B, per_query] distinct global doc ids that carry each query's planted positives."""
    rng = np.random.default_rng(seed)
    need = B * per_query
    if need > n_total:
        raise ValueError("corpus too small for the planted positives")
    return rng.choice(n_total, size=need, replace=False).reshape(B, per_query).astype(np.int64)


def bm25_lists(B: int, n_total: int, planted: np.ndarray, k: int = 100, hits: int = 5, seed: int = 3):
    """Stand-in stage-1 output [B, k] int32: ``hits`` planted ids + random ids, shuffled."""
    rng = np.random.default_rng(seed)
    out = np.empty((B, k), np.int32)
    for b in range(B):
        ids = list(planted[b, :hits])
        ids += list(rng.choice(n_total, size=k - hits, replace=False))
        rng.shuffle(ids)
        out[b] = ids[:k]
    return out


def iter_shard(begin: int, end: int, Q: torch.Tensor, planted: np.ndarray, device, seed: int = 0,
               sigma: float = 0.1, dtype: torch.dtype = torch.bfloat16):
    """Docs [begin, end) of the synthetic corpus, one generator chunk at a time:
    yields (lo, hi, tokens ``dtype`` [hi - lo, 128, 128] on ``device``) with the
    planted positives already in place, so a corpus larger than HBM in fp32 /
    bf16 (10M docs = 328 GB of bf16) can be quantised or indexed chunk by chunk
    with bounded memory.  Concatenating the chunks gives ``make_shard``'s tokens."""
    lq = Q.shape[1]
    flat = planted.reshape(-1)
    owner = np.repeat(np.arange(planted.shape[0]), planted.shape[1])
    gen = torch.Generator().manual_seed(seed + 17)
    noise_all = torch.randn(len(flat), lq, DIM, generator=gen)          # same draws whatever the shard
    c0, c1 = begin // CHUNK, (end + CHUNK - 1) // CHUNK
    for c in range(c0, c1):
        g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + c)
        x = _unit(torch.randn((CHUNK, LD, DIM), generator=g, device=device, dtype=torch.float32))
        lo, hi = max(begin, c * CHUNK), min(end, (c + 1) * CHUNK)
        t = x[lo - c * CHUNK: hi - c * CHUNK].to(dtype)
        del x
        mine = (flat >= lo) & (flat < hi)
        if mine.any():
            docs = _unit(Q[torch.from_numpy(owner[mine])] + sigma * _unit(noise_all[torch.from_numpy(mine)]))
            t[torch.from_numpy(flat[mine] - lo).to(device), :lq] = docs.to(device=device, dtype=dtype)
        yield lo, hi, t


def make_shard(begin: int, end: int, Q: torch.Tensor, planted: np.ndarray, device, seed: int = 0,
               sigma: float = 0.1, dtype: torch.dtype = torch.bfloat16) -> Tuple[torch.Tensor, torch.Tensor]:
    """Docs [begin, end) of the synthetic corpus: (``dtype`` [n, 128, 128], int32 doclens [n]) on ``device``
    (bf16 = the fp32 draw rounded, so both dtypes describe the same corpus)."""
    from .index import hbm_empty
    n = end - begin
    # the index array (bf16 / MXFP8) in contiguous HBM like every index build;
    # an fp32 source (split into an fp32-faithful index) in torch's allocator
    tokens = (torch.empty((n, LD, DIM), dtype=dtype, device=device) if dtype == torch.float32
              else hbm_empty((n, LD, DIM), dtype, device))
    doclens = torch.full((n,), LD, dtype=torch.int32, device=device)
    for lo, hi, t in iter_shard(begin, end, Q, planted, device, seed, sigma, dtype):
        tokens[lo - begin: hi - begin] = t
    return tokens, doclens


def make_shard_mxfp8(begin: int, end: int, Q: torch.Tensor, planted: np.ndarray, device, seed: int = 0,
                     sigma: float = 0.1):
    """Docs [begin, end) quantised to MXFP8 chunk by chunk (HIP quantizer on the
    bf16 tokens, exactly as ``ColbertIndex.mxfp8(make_shard(...))`` would):
    (e4m3 uint8 [n, 128, 128], E8M0 uint8 [n, 128, 2], int32 doclens [n]).
    Peak extra memory is one generator chunk, so 10M docs (167 GB) fit one HBM."""
    from .index import hbm_empty, quantize_mxfp8
    n = end - begin
    q = hbm_empty((n, LD, DIM), torch.uint8, device)
    sc = hbm_empty((n, LD, 2), torch.uint8, device)
    doclens = torch.full((n,), LD, dtype=torch.int32, device=device)
    for lo, hi, t in iter_shard(begin, end, Q, planted, device, seed, sigma, torch.bfloat16):
        qq, ss = quantize_mxfp8(t)
        q[lo - begin: hi - begin] = qq
        sc[lo - begin: hi - begin] = ss
        del t, qq, ss
    return q, sc, doclens


BM25_VOCAB = 30000


def bm25_queries(B: int, q_len: int = 6, seed: int = 4):
    """Stage-1 queries as term-id CSR: ``q_len`` mid-frequency terms each."""
    rng = np.random.default_rng([seed, 1 << 20])
    q = rng.integers(100, 5000, size=(B, q_len)).astype(np.int32)
    return q.reshape(-1), np.arange(B + 1, dtype=np.int64) * q_len


def bm25_shard(begin: int, end: int, planted: np.ndarray, q_len: int = 6, vocab: int = BM25_VOCAB, seed: int = 4):
    """Docs [begin, end) of the synthetic stage-1 corpus as term ids (CSR with
    offsets from 0): lengths U[40, 120], Zipf-like term frequencies
    (p ~ 1/(rank + 10)), one RNG per CHUNK of global ids so any rank can build
    its own range.  Planted docs get their query's terms appended, so the
    lexical and late-interaction stages agree on the positives as they would
    on a relevant chunk.  Returns (doc_terms int32, doc_offsets int64, vocab)."""
    q_terms, _ = bm25_queries(planted.shape[0], q_len, seed)
    q_terms = q_terms.reshape(-1, q_len)
    flat = planted.reshape(-1)
    owner = dict(zip(flat.tolist(), np.repeat(np.arange(planted.shape[0]), planted.shape[1]).tolist()))
    p = 1.0 / (np.arange(vocab, dtype=np.float64) + 10.0)
    cdf = np.cumsum(p / p.sum())
    rows_t, rows_l = [], []
    for c in range(begin // CHUNK, (end + CHUNK - 1) // CHUNK):
        rng = np.random.default_rng([seed, c])
        lens = rng.integers(40, 121, size=CHUNK)
        terms = np.minimum(np.searchsorted(cdf, rng.random(int(lens.sum()))), vocab - 1).astype(np.int32)
        off = np.zeros(CHUNK + 1, np.int64)
        off[1:] = np.cumsum(lens)
        lo, hi = max(begin, c * CHUNK) - c * CHUNK, min(end, (c + 1) * CHUNK) - c * CHUNK
        mine = [d for d in owner if c * CHUNK + lo <= d < c * CHUNK + hi]
        if not mine:
            rows_t.append(terms[off[lo]:off[hi]])
            rows_l.append(lens[lo:hi])
            continue
        prev = lo
        for d in sorted(mine):
            dl = d - c * CHUNK
            rows_t.append(terms[off[prev]:off[dl + 1]])
            rows_t.append(q_terms[owner[d]])
            ln = lens[prev:dl + 1].copy()
            ln[-1] += q_len
            rows_l.append(ln)
            prev = dl + 1
        rows_t.append(terms[off[prev]:off[hi]])
        rows_l.append(lens[prev:hi])
    lens = np.concatenate(rows_l) if rows_l else np.zeros(0, np.int64)
    offsets = np.zeros(len(lens) + 1, np.int64)
    offsets[1:] = np.cumsum(lens)
    terms = np.concatenate(rows_t).astype(np.int32) if rows_t else np.zeros(0, np.int32)
    return terms, offsets, vocab


class SyntheticDocEncoder:
    """Encoder stand-in for ingest at scale: ``encode(texts)`` for texts
    ``"synthetic doc <id>"`` returns the synthetic corpus's tokens of those
    global ids (bf16 [m, 128, 128] on ``device``, generated by ``make_shard``),
    so a 1M-doc ingest needs no real model and no host-side embeddings.  The
    ids of one call must be consecutive (ingest batches are)."""

    def __init__(self, Q: torch.Tensor, planted: np.ndarray, device, seed: int = 0):
        self.Q, self.planted, self.device, self.seed = Q, planted, torch.device(device), seed

    @staticmethod
    def texts(begin: int, end: int):
        return [f"synthetic doc {i}" for i in range(begin, end)]

    def encode(self, texts, convert_to_tensor: bool = True, **_unused):
        texts = [texts] if isinstance(texts, str) else list(texts)
        ids = [int(t.rsplit(" ", 1)[1]) for t in texts]
        if not ids:
            return torch.zeros((0, LD, DIM), dtype=torch.bfloat16, device=self.device)
        a, b = ids[0], ids[-1] + 1
        if ids != list(range(a, b)):
            raise ValueError("SyntheticDocEncoder encodes consecutive doc ids only")
        tokens, _ = make_shard(a, b, self.Q, self.planted, self.device, seed=self.seed)
        return tokens
