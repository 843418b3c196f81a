"""Exact-arithmetic codebook corpora on the k/16 grid (test infrastructure).

Every token value is k/16 with |k| <= 16, so
  * bf16 represents it exactly, so does e4m3 under the MXFP8 quantizer's
    power-of-two half scales (every value has <= 4 significant bits and a
    half's smallest non-zero value is >= max/16), and the fp32-faithful split
    has lo = 0;
  * every product is a multiple of 1/256 and every partial dot product, max
    and sum over 32 query tokens stays far below 2^24 / 256 in magnitude, so
    fp32 accumulation in ANY order is exact.
The GPU's scores must therefore equal the oracle's exact scores bit for bit,
and ids, order and ties (score desc, id asc) are defined exactly -- at any
corpus size, including the 1M-doc headline corpus of BASELINE config 3.

Corpus: ``K`` content codes.  Doc n draws m_n in [1, 6] distinct codes; each
of its doclens[n] scoring rows is one of them (ragged doclens, ~0.1 % empty
docs), and its padding rows hold codes it does NOT use (any read of padding
changes the score).  ``copies`` rows of each planted doc (10 per query) are
its query's tokens with j grid steps of perturbation (j = planted rank), so
the planted docs lead every ranking with scores 1/256 apart or tied; the last
planted doc of each query is a token-for-token copy of the one before it (an
exact tie: lower id first).
"""
import numpy as np
import torch

from oracle import oracle as orc

K = 24
LD = 128
DIM = 128
CHUNK = 65536


def grid_values(rng, shape):
    return (rng.integers(-16, 17, size=shape) / 16.0).astype(np.float32)


class GridCorpus:
    def __init__(self, N: int, B: int, seed: int = 123, lq: int = 32, n_planted: int = 10, copies: int = 8):
        self.N, self.B, self.lq = N, B, lq
        rng = np.random.default_rng([seed, 0])
        self.codebook = grid_values(rng, (K, DIM))
        self.Q = grid_values(rng, (B, lq, DIM))
        self.codes = np.empty((N, LD), np.uint8)
        self.doclens = np.empty(N, np.int32)
        for a in range(0, N, CHUNK):
            n = min(CHUNK, N - a)
            r = np.random.default_rng([seed, 1 + a // CHUNK])
            perm = np.argsort(r.random((n, K), dtype=np.float32), axis=1).astype(np.uint8)
            m = r.integers(1, 7, size=n)
            dl = r.integers(m, LD + 1).astype(np.int32)
            dl[r.random(n) < 1e-3] = 0
            t = np.arange(LD)[None, :]
            use = (r.random((n, LD), dtype=np.float32) * m[:, None]).astype(np.int64)
            pad = m[:, None] + (r.random((n, LD), dtype=np.float32) * (K - m)[:, None]).astype(np.int64)
            sel = np.where(t < dl[:, None], use, pad)
            self.codes[a:a + n] = np.take_along_axis(perm, sel, axis=1)
            self.doclens[a:a + n] = dl
        # planted docs: [B, n_planted] distinct ids
        self.planted = rng.choice(N, size=B * n_planted, replace=False).reshape(B, n_planted).astype(np.int64)
        flat = self.planted.reshape(-1)
        P = len(flat)
        self.copy_slots = np.empty((P, copies), np.int64)
        self.copy_vals = np.empty((P, copies, DIM), np.float32)
        for b in range(B):
            for j in range(n_planted):
                p = b * n_planted + j
                d = flat[p]
                if j == n_planted - 1 and j > 0:            # exact copy of the previous planted doc
                    prev = flat[p - 1]
                    self.codes[d] = self.codes[prev]
                    self.doclens[d] = self.doclens[prev]
                    self.copy_slots[p] = self.copy_slots[p - 1]
                    self.copy_vals[p] = self.copy_vals[p - 1]
                    continue
                self.doclens[d] = max(int(self.doclens[d]), 40)        # former padding rows now score
                self.copy_slots[p] = rng.choice(int(self.doclens[d]), size=copies, replace=False)
                v = self.Q[b, rng.choice(lq, size=copies, replace=False)].copy()
                for _ in range(j):                           # j grid steps, kept inside [-1, 1]
                    c, e = rng.integers(copies), rng.integers(DIM)
                    v[c, e] += -1 / 16 if v[c, e] > 0 else 1 / 16
                self.copy_vals[p] = v
        self.planted_flat = flat
        self.masks = orc.codebook_masks(self.codes, self.doclens)
        self.T = orc.codebook_table(self.Q, self.codebook)               # [B, lq, K] float64, exact
        self.planted_scores = self._planted_scores()                     # [B, P] float64, exact
        self._planted_pos = {int(d): p for p, d in enumerate(flat)}

    # ------------------------------------------------------------------ oracle side
    def _planted_masks(self):
        """Code sets of the planted docs' NON-copy scoring rows."""
        out = np.zeros(len(self.planted_flat), np.uint32)
        for p, d in enumerate(self.planted_flat):
            keep = np.ones(int(self.doclens[d]), bool)
            keep[self.copy_slots[p]] = False
            for c in np.unique(self.codes[d, : self.doclens[d]][keep]):
                out[p] |= np.uint32(1) << np.uint32(c)
        return out

    def _planted_scores(self, chunk: int = 64):
        """maxsim of every planted doc for every query: max over the copy rows
        (float64 dot products) and over the doc's other codes, summed over q."""
        masks = self._planted_masks()
        Qf = self.Q.reshape(-1, DIM).astype(np.float64)
        P = len(self.planted_flat)
        out = np.empty((self.B, P), np.float64)
        bits_all = ((masks[:, None].astype(np.uint64) >> np.arange(K, dtype=np.uint64)) & 1).astype(bool)
        for a in range(0, P, chunk):
            cv = self.copy_vals[a:a + chunk].astype(np.float64)                           # [c, copies, D]
            c = cv.shape[0]
            cd = (Qf @ cv.reshape(-1, DIM).T).reshape(self.B, self.lq, c, -1).max(axis=3)  # [B, lq, c]
            bits = bits_all[a:a + chunk]
            cm = np.where(bits[None, None], self.T[:, :, None, :], -np.inf).max(axis=3)    # [B, lq, c]
            out[:, a:a + chunk] = np.maximum(cd, cm).sum(axis=1)
        return out

    def topk(self, k: int):
        """Oracle top-k of every query over the whole corpus: (float64 [B, k], int64 [B, k])."""
        return orc.codebook_topk(self.T, self.masks, k, over_ids=self.planted_flat, over_scores=self.planted_scores)

    def exact_scores(self, rows, ids: np.ndarray) -> np.ndarray:
        """Exact maxsim of query ``rows[r]`` with doc ``ids[r, j]`` ([R, C] float64; id < 0 -> -inf)."""
        ids = np.asarray(ids, np.int64)
        out = np.full(ids.shape, -np.inf)
        for r, b in enumerate(rows):
            for j, d in enumerate(ids[r]):
                if d < 0 or d >= self.N:
                    continue
                p = self._planted_pos.get(int(d))
                out[r, j] = self.planted_scores[b, p] if p is not None else \
                    orc.codebook_maxsim(self.T[b:b + 1], self.masks[d:d + 1])[0, 0]
        return out

    # ------------------------------------------------------------------ token rows
    def rows_f32(self, a: int, b: int) -> np.ndarray:
        """Host float32 token rows of docs [a, b) (planted copies in place)."""
        x = self.codebook[self.codes[a:b]]
        sel = (self.planted_flat >= a) & (self.planted_flat < b)
        for p in np.nonzero(sel)[0]:
            x[self.planted_flat[p] - a, self.copy_slots[p]] = self.copy_vals[p]
        return x

    def tokens_on(self, device, dtype=torch.bfloat16, chunk: int = 16384) -> torch.Tensor:
        """The whole corpus's token rows as ``dtype`` [N, 128, 128] on ``device``
        (gathered from the codebook on the device, planted rows patched in)."""
        cb = torch.from_numpy(self.codebook).to(device=device, dtype=dtype)
        out = torch.empty((self.N, LD, DIM), dtype=dtype, device=device)
        for a in range(0, self.N, chunk):
            b = min(self.N, a + chunk)
            out[a:b] = cb[torch.from_numpy(self.codes[a:b]).to(device).long()]
        pos = torch.from_numpy(self.planted_flat).to(device)
        slots = torch.from_numpy(self.copy_slots).to(device)
        vals = torch.from_numpy(self.copy_vals).to(device=device, dtype=dtype)
        out[pos[:, None], slots] = vals
        return out

    def doclens_on(self, device) -> torch.Tensor:
        return torch.from_numpy(self.doclens).to(device)
