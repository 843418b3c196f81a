#!/usr/bin/env python3
"""CPU soak of the doc-sharded BM25 (bm25.NativeBM25 shards with global
statistics, merged by (score desc, id asc)) against the unsharded index:
random corpora (tiny vocabularies: many ties; empty docs; shards of empty
docs), 1-8 shards at random cut points, repeated query terms, k up to 5,000.
Runs in the container (no GPU).  usage: python3 tools/stress_bm25.py"""
import sys, time, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
rng = np.random.default_rng(0)
t0 = time.time(); cases = bad = 0
while time.time() - t0 < 120:
    N = int(rng.integers(1, 3000)); V = int(rng.integers(2, 60))
    lens = rng.integers(0, int(rng.integers(1, 40)), size=N)
    off = np.zeros(N + 1, np.int64); off[1:] = np.cumsum(lens)
    terms = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    B = int(rng.integers(1, 6)); ql = int(rng.integers(1, 6))
    qt = rng.integers(0, V + 2, size=B * ql).astype(np.int32) % V   # repeated terms allowed
    qo = np.arange(B + 1, dtype=np.int64) * ql
    k = int(rng.choice([1, 5, 50, 100, 5000]))
    full = NativeBM25(terms, off, V)
    fi, fs = full.search(qt, qo, k)
    G = int(rng.integers(1, 9))
    cuts = np.sort(rng.integers(0, N + 1, size=G - 1)); cuts = np.concatenate([[0], cuts, [N]])
    df = NativeBM25.doc_freq(terms, off, V); stats = (N, int(off[-1]), df)
    lists_i, lists_s = [], []
    for g in range(G):
        a, b = int(cuts[g]), int(cuts[g + 1])
        sh = NativeBM25(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a, stats=stats)
        i, s = sh.search(qt, qo, k)
        lists_i.append(i); lists_s.append(s)
    I = np.concatenate(lists_i, 1); S = np.concatenate(lists_s, 1)
    mi = np.full((B, k), -1, np.int32); ms = np.full((B, k), -np.inf, np.float32)
    for r in range(B):
        valid = I[r] >= 0
        ii, ss = I[r][valid], S[r][valid]
        o = np.lexsort((ii, -ss.astype(np.float64)))[:k]
        mi[r, :len(o)] = ii[o]; ms[r, :len(o)] = ss[o]
    valid = fi >= 0   # padding: (0.0, -1) unsharded, (-inf, -1) merged -- the ids are what the RRF reads
    ok = np.array_equal(mi, fi) and np.array_equal(ms[valid].view(np.int32), fs[valid].view(np.int32))
    cases += 1
    if not ok:
        bad += 1
        if bad <= 3:
            r = int(np.nonzero((mi != fi).any(1) | (ms != fs).any(1))[0][0])
            print("MISMATCH N", N, "V", V, "G", G, "k", k, "row", r, mi[r][:10], fi[r][:10], ms[r][:5], fs[r][:5])
print({"cases": cases, "mismatches": bad})
