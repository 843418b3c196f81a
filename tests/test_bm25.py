"""CPU: the native host BM25 (csrc/host_bm25.cpp, stage 1 of
HybridRetriever.retrieve, local_rag_complete.py:937-950) against the oracle's
restatement (oracle/oracle.py:bm25_topk), bit-for-bit: ids and float32 score
bits.  Parity with bm25s itself is unpinned (bm25s is not installed; see
DESIGN.md); the formula is bm25s' published Lucene variant.
"""
import numpy as np
import pytest

from oracle import oracle as orc


def _corpus(rng, N, V, maxlen=30, dup=0.0):
    lens = rng.integers(0, maxlen, size=N)
    rows = [rng.integers(0, V, size=int(n)).astype(np.int32) for n in lens]
    for d in range(1, N):                 # duplicated docs -> exactly tied scores
        if rng.random() < dup:
            rows[d] = rows[int(rng.integers(0, d))].copy()
    off = np.zeros(N + 1, np.int64)
    off[1:] = np.cumsum([len(r) for r in rows])
    terms = np.concatenate(rows) if N else np.zeros(0, np.int32)
    return terms.astype(np.int32), off


def _queries(rng, B, V, maxq=6):
    ql = rng.integers(0, maxq, size=B)
    qo = np.zeros(B + 1, np.int64)
    qo[1:] = np.cumsum(ql)
    return rng.integers(-1, V + 2, size=int(qo[-1])).astype(np.int32), qo


def _same(a_ids, a_sc, b_ids, b_sc):
    assert np.array_equal(a_ids.astype(np.int64), b_ids.astype(np.int64))
    assert np.array_equal(np.asarray(a_sc, np.float32).view(np.uint32), np.asarray(b_sc, np.float32).view(np.uint32))


@pytest.mark.parametrize("seed", range(6))
def test_native_bm25_matches_oracle(seed):
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    rng = np.random.default_rng(seed)
    N = int(rng.integers(1, 400))
    V = int(rng.integers(1, 60))
    terms, off = _corpus(rng, N, V, dup=0.2)
    qt, qo = _queries(rng, 9, V)
    for k in (1, 10, N, N + 7):              # k > N: -1 padding after every doc
        ids, sc = NativeBM25(terms, off, V).search(qt, qo, k, n_threads=3)
        oi, os_ = orc.bm25_topk(terms, off, qt, qo, V, k)
        _same(ids, sc, oi, os_)


def test_native_bm25_k1_b_and_threads():
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    rng = np.random.default_rng(11)
    terms, off = _corpus(rng, 500, 40, maxlen=60)
    qt, qo = _queries(rng, 33, 40)
    ix = NativeBM25(terms, off, 40, k1=0.9, b=0.4)
    ref = orc.bm25_topk(terms, off, qt, qo, 40, 20, k1=0.9, b=0.4)
    for th in (1, 2, 8, 64):
        _same(*ix.search(qt, qo, 20, n_threads=th), *ref)


@pytest.mark.parametrize("G", [2, 3, 5])
def test_sharded_bm25_merge_equals_unsharded(G):
    """Doc-sharded index with global statistics: the (score desc, id asc)
    merge of the shards' top-k lists is the unsharded top-k, ties included."""
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    from hybrid_rag_colbertv2_amd.distributed import shard_range
    rng = np.random.default_rng(G)
    N, V, k = 257, 25, 30
    terms, off = _corpus(rng, N, V, dup=0.3)
    qt, qo = _queries(rng, 12, V)
    parts = []
    for r in range(G):
        a, b = shard_range(N, r, G)
        parts.append((a, terms[off[a]:off[b]], off[a:b + 1] - off[a]))
    df = sum(NativeBM25.doc_freq(t, o, V) for _, t, o in parts)
    stats = (N, int(off[-1]), df)
    res = [NativeBM25(t, o, V, id_base=a, stats=stats).search(qt, qo, k) for a, t, o in parts]
    S = np.stack([r[1] for r in res])
    I = np.stack([r[0] for r in res])
    ms, mi = orc.merge_topk(S, I, k)
    oi, os_ = orc.bm25_topk(terms, off, qt, qo, V, k)
    _same(mi, ms, oi, os_)


def test_bm25_validation():
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    with pytest.raises(ValueError):
        NativeBM25(np.array([0, 5], np.int32), np.array([0, 2], np.int64), 3)        # term >= vocab
    with pytest.raises(ValueError):
        NativeBM25(np.array([0, 1], np.int32), np.array([2, 0], np.int64), 3)        # offsets descending
    with pytest.raises(ValueError):
        NativeBM25(np.array([0], np.int32), np.array([0, 1], np.int64), 3, id_base=5,
                   stats=(2, 1, np.ones(3, np.int64)))                               # shard beyond n_global
    ix = NativeBM25(np.array([0, 1], np.int32), np.array([0, 1, 2], np.int64), 2)
    with pytest.raises(ValueError):
        ix.search(np.zeros(0, np.int32), np.zeros(2, np.int64), 0)                   # k < 1
    ids, sc = ix.search(np.zeros(0, np.int32), np.zeros(2, np.int64), 3)           # empty query
    assert ids.tolist() == [[0, 1, -1]] and sc.tolist() == [[0, 0, 0]]


def test_synth_bm25_shards_compose_and_plant():
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    n, B = 40000, 8
    pl = synth.planted_ids(B, n, 10)
    terms, off, V = synth.bm25_shard(0, n, pl)
    assert len(off) == n + 1 and terms.min() >= 0 and terms.max() < V
    a, b = 12345, 30001
    t2, o2, _ = synth.bm25_shard(a, b, pl)
    assert np.array_equal(t2, terms[off[a]:off[b]]) and np.array_equal(o2, off[a:b + 1] - off[a])
    qt, qo = synth.bm25_queries(B)
    ids, _ = NativeBM25(terms, off, V).search(qt, qo, 100)
    assert all(set(pl[q]) <= set(ids[q].tolist()) for q in range(B))


def test_hostbm25_text_roundtrip(tmp_path):
    from hybrid_rag_colbertv2_amd.bm25 import HostBM25, to_csr
    corpus = ["The quick brown fox", "jumps over the lazy dog", "quick quick dog", "", "fox and dog"]
    bm = HostBM25()
    bm.index(bm.tokenize(corpus))
    ids, sc = bm.retrieve(bm.tokenize("quick dog"), k=5)
    # oracle over the same term ids
    rows = [bm._ids(t, grow=False) for t in bm._rows(bm.tokenize(corpus))]
    terms, off = to_csr(rows)
    q, qo = to_csr([bm._ids(t, grow=False) for t in bm._rows(bm.tokenize("quick dog"))])
    oi, os_ = orc.bm25_topk(terms, off, q, qo, len(bm.vocab), 5)
    _same(ids, sc, oi, os_)
    assert ids[0][0] == 2
    bm.save(str(tmp_path))
    bm2 = HostBM25.load(str(tmp_path))
    assert bm2.stemmer.algorithm == "english"
    ids2, sc2 = bm2.retrieve(bm2.tokenize("quick dog"), k=5)
    assert np.array_equal(ids, ids2) and np.array_equal(sc, sc2)
    # a bm25.json of the earlier, unstemmed tokenizer (no format / stemmer record) is refused
    import json
    meta = json.load(open(tmp_path / "bm25.json"))
    for drop in ("format", "stemmer"):
        old = {k: v for k, v in meta.items() if k != drop}
        json.dump(old, open(tmp_path / "bm25.json", "w"))
        with pytest.raises(ValueError, match="rebuild the BM25 index"):
            HostBM25.load(str(tmp_path))
    # a custom stemmer is recorded as such and must be passed back in
    bm3 = HostBM25(stemmer=type("S", (), {"stemWords": lambda self, w: [x[:4] for x in w]})())
    bm3.index(bm3.tokenize(corpus))
    bm3.save(str(tmp_path / "c"))
    with pytest.raises(ValueError, match="custom stemmer"):
        HostBM25.load(str(tmp_path / "c"))
    bm4 = HostBM25.load(str(tmp_path / "c"), stemmer=bm3.stemmer)
    assert np.array_equal(bm4.retrieve(bm4.tokenize("quick dog"), 3)[0], bm3.retrieve(bm3.tokenize("quick dog"), 3)[0])


def test_native_bm25_repeated_query_terms():
    """A repeated query term counts once per occurrence (bm25s sums the
    postings of every query token), in query order."""
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    rng = np.random.default_rng(7)
    terms, off = _corpus(rng, 300, 40)
    ix = NativeBM25(terms, off, 40)
    rep = np.array([3, 5, 3, 3, 9], np.int32)
    ids, sc = ix.search(rep, np.array([0, 5], np.int64), 20)
    oi, os_ = orc.bm25_topk(terms, off, rep, np.array([0, 5], np.int64), 40, 20)
    _same(ids, sc, oi, os_)
    # a doc holding term 3 but not 5 or 9 scores exactly 3 x its term-3 weight
    holds3 = [d for d in range(300) if set(terms[off[d]:off[d + 1]].tolist()) & {3, 5, 9} == {3}]
    assert holds3
    i3, s3 = ix.search(np.array([3], np.int32), np.array([0, 1], np.int64), 300)
    ir, sr = ix.search(rep, np.array([0, 5], np.int64), 300)
    w3 = dict(zip(i3[0].tolist(), s3[0].tolist()))
    wr = dict(zip(ir[0].tolist(), sr[0].tolist()))
    for d in holds3:
        assert wr[d] == np.float32(np.float32(w3[d] + w3[d]) + w3[d])


def test_bm25_shard_of_empty_docs():
    """A shard whose docs hold no token at all (empty chunks) builds -- no
    terms pointer to pass -- and the merge of every shard's list still equals
    the unsharded top-k (round-6 soak: the build used to refuse it, so one
    rank of a sharded index would fail)."""
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    V = 7
    empty = NativeBM25(np.zeros(0, np.int32), np.zeros(5, np.int64), V)               # 4 empty docs
    ids, sc = empty.search(np.array([1, 2], np.int32), np.array([0, 2], np.int64), 6)
    assert ids.tolist() == [[0, 1, 2, 3, -1, -1]] and sc.tolist() == [[0.0] * 6]
    assert NativeBM25.doc_freq(np.zeros(0, np.int32), np.zeros(5, np.int64), V).tolist() == [0] * V
    rng = np.random.default_rng(11)
    N = 60
    lens = rng.integers(1, 6, size=N)
    lens[20:35] = 0                                                                    # shard 1: all empty
    off = np.zeros(N + 1, np.int64)
    off[1:] = np.cumsum(lens)
    terms = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    qt, qo = np.array([1, 3, 3, 5], np.int32), np.array([0, 2, 4], np.int64)
    cuts = [0, 20, 35, N]
    stats = (N, int(off[-1]), NativeBM25.doc_freq(terms, off, V))
    res = [NativeBM25(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a, stats=stats).search(qt, qo, 40)
           for a, b in zip(cuts[:-1], cuts[1:])]
    ms, mi = orc.merge_topk(np.stack([r[1] for r in res]), np.stack([r[0] for r in res]), 40)
    oi, os_ = orc.bm25_topk(terms, off, qt, qo, V, 40)
    _same(mi, ms, oi, os_)
