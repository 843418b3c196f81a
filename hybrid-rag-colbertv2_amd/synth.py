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


def make_shard(begin: int, end: int, Q: torch.Tensor, planted: np.ndarray, device, seed: int = 0,
               sigma: float = 0.1) -> Tuple[torch.Tensor, torch.Tensor]:
    """Docs [begin, end) of the synthetic corpus: (bf16 [n, 128, 128], int32 doclens [n]) on ``device``."""
    n = end - begin
    tokens = torch.empty((n, LD, DIM), dtype=torch.bfloat16, device=device)
    doclens = torch.full((n,), LD, dtype=torch.int32, device=device)
    c0, c1 = begin // CHUNK, (end + CHUNK - 1) // CHUNK
    for c in range(c0, c1):
        g = torch.Generator(device=device).manual_seed(seed * 1_000_003 + c)
        x = _unit(torch.randn((CHUNK, LD, DIM), generator=g, device=device, dtype=torch.float32))
        lo, hi = max(begin, c * CHUNK), min(end, (c + 1) * CHUNK)
        tokens[lo - begin: hi - begin] = x[lo - c * CHUNK: hi - c * CHUNK].to(torch.bfloat16)
        del x
    lq = Q.shape[1]
    flat = planted.reshape(-1)
    owner = np.repeat(np.arange(planted.shape[0]), planted.shape[1])
    mine = (flat >= begin) & (flat < end)
    if mine.any():
        ids = flat[mine]
        qb = owner[mine]
        gen = torch.Generator().manual_seed(seed + 17)
        noise = torch.randn(len(flat), lq, DIM, generator=gen)[torch.from_numpy(mine)]
        docs = _unit(Q[torch.from_numpy(qb)] + sigma * _unit(noise))
        tokens[torch.from_numpy(ids - begin).to(device), :lq] = docs.to(device=device, dtype=torch.bfloat16)
    return tokens, doclens
