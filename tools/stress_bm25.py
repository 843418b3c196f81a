#!/usr/bin/env python3
"""CPU soak of the doc-sharded BM25 (bm25.NativeBM25 shards with global
statistics, merged by (score desc, id asc)) against the unsharded index:
random corpora (tiny vocabularies: many ties; empty docs; shards of empty
docs), 1-8 shards at random cut points, repeated query terms, k up to 5,000.
Padding differs only in its score -- (0.0, -1) unsharded, (-inf, -1) from the
merge -- so ids are compared everywhere and scores where an id is real (the
RRF reads the ids).  Runs in the container (no GPU).
usage: stress_bm25.py [--seconds S]"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25  # noqa: E402


def merge(lists_i, lists_s, k):
    """The (score desc, id asc) merge of the shards' lists, -1 entries skipped."""
    I, S = np.concatenate(lists_i, 1), np.concatenate(lists_s, 1)
    B = I.shape[0]
    mi = np.full((B, k), -1, np.int32)
    ms = np.full((B, k), -np.inf, np.float32)
    for r in range(B):
        valid = I[r] >= 0
        ii, ss = I[r][valid], S[r][valid]
        o = np.lexsort((ii, -ss.astype(np.float64)))[:k]
        mi[r, :len(o)] = ii[o]
        ms[r, :len(o)] = ss[o]
    return mi, ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    a = ap.parse_args()
    rng = np.random.default_rng(0)
    t0 = time.time()
    cases = bad = 0
    while time.time() - t0 < a.seconds:
        N, V = int(rng.integers(1, 3000)), int(rng.integers(2, 60))
        lens = rng.integers(0, int(rng.integers(1, 40)), size=N)
        off = np.zeros(N + 1, np.int64)
        off[1:] = np.cumsum(lens)
        terms = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
        B, ql = int(rng.integers(1, 6)), int(rng.integers(1, 6))
        qt = (rng.integers(0, V + 2, size=B * ql) % V).astype(np.int32)   # repeated terms allowed
        qo = np.arange(B + 1, dtype=np.int64) * ql
        k = int(rng.choice([1, 5, 50, 100, 5000]))
        fi, fs = NativeBM25(terms, off, V).search(qt, qo, k)
        G = int(rng.integers(1, 9))
        cuts = np.concatenate([[0], np.sort(rng.integers(0, N + 1, size=G - 1)), [N]])
        stats = (N, int(off[-1]), NativeBM25.doc_freq(terms, off, V))
        lists_i, lists_s = [], []
        for g in range(G):
            lo, hi = int(cuts[g]), int(cuts[g + 1])
            i, s = NativeBM25(terms[off[lo]:off[hi]], off[lo:hi + 1] - off[lo], V, id_base=lo,
                              stats=stats).search(qt, qo, k)
            lists_i.append(i)
            lists_s.append(s)
        mi, ms = merge(lists_i, lists_s, k)
        real = fi >= 0
        ok = np.array_equal(mi, fi) and np.array_equal(ms[real].view(np.int32), fs[real].view(np.int32))
        cases += 1
        if not ok:
            bad += 1
            if bad <= 3:
                print(f"MISMATCH: N {N} V {V} G {G} k {k}", flush=True)
    print({"cases": cases, "mismatches": bad}, flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
