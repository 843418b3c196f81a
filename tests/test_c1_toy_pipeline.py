"""CPU, config 1: the 50-chunk toy corpus through the reference's pipeline,
restated with the oracle (FakeEncoder -> literal scorer -> top-k -> RRF ->
[:50] -> rerank -> dicts), must reproduce the reference's own outputs
recorded in tests/golden/toy_c1.json (search, rerank, RRF and retrieve).
"""
import json
import os

import numpy as np

from conftest import GOLDEN
from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
from oracle import oracle as orc

TOY = json.load(open(os.path.join(GOLDEN, "toy_c1.json")))


def _setup():
    enc = FakeEncoder(**TOY["encoder"])
    docs = enc.encode(TOY["corpus"], convert_to_tensor=False)
    return enc, docs


def test_fake_encoder_is_stable():
    enc = FakeEncoder(maxlen=8)
    a = enc.encode("alpha beta", convert_to_tensor=False)
    b = FakeEncoder(maxlen=8).encode("alpha beta", convert_to_tensor=False)
    assert a.shape == (8, 128) and np.array_equal(a, b)
    np.testing.assert_allclose(np.linalg.norm(a, axis=1), 1.0, atol=1e-6)


def test_search_matches_reference():
    enc, docs = _setup()
    for q, ref in zip(TOY["queries"], TOY["search"]):
        s = orc.meanpool_cosine(enc.encode(q, convert_to_tensor=False), docs)
        vs, ids = orc.topk(s, 10)
        assert [r["document_id"] for r in ref] == list(ids[0])
        np.testing.assert_allclose([r["score"] for r in ref], vs[0], atol=1e-6)


def test_rerank_matches_reference():
    enc, docs = _setup()
    sub = docs[0:50:3]
    for q, ref in zip(TOY["queries"], TOY["rerank"]):
        s = orc.meanpool_cosine(enc.encode(q, convert_to_tensor=False), sub)[0]
        got = orc.rerank_select(s, 5)
        assert [(r["result_index"], r["rank"]) for r in ref["results"]] == [(p, rk) for p, _, rk in got]
        np.testing.assert_allclose([r["score"] for r in ref["results"]], [x for _, x, _ in got], atol=1e-6)


def test_rrf_matches_reference():
    enc, docs = _setup()
    for q, bm, ref in zip(TOY["queries"], TOY["bm25"], TOY["rrf"]):
        s = orc.meanpool_cosine(enc.encode(q, convert_to_tensor=False), docs)
        _, ids = orc.topk(s, 100)
        cb = [int(i) for i in ids[0] if i >= 0]
        got = orc.rrf(bm["ids"], cb)
        assert [(r["chunk_id"], r["rrf_score"]) for r in ref] == got


def test_retrieve_matches_reference():
    enc, docs = _setup()
    chunks = {c["id"]: c for c in TOY["chunks"]}
    for q, bm, ref in zip(TOY["queries"], TOY["bm25"], TOY["retrieve"]):
        qe = enc.encode(q, convert_to_tensor=False)
        _, ids = orc.topk(orc.meanpool_cosine(qe, docs), 100)
        fused = orc.rrf(bm["ids"], [int(i) for i in ids[0] if i >= 0])[:50]
        cand = [cid for cid, _ in fused]
        s = orc.meanpool_cosine(qe, docs[cand])[0]
        got = []
        for pos, score, rank in orc.rerank_select(s, 10):
            c = chunks[cand[pos]]
            got.append({"chunk_id": c["id"], "document_id": c["document_id"], "heading_path": c["heading_path"],
                        "has_images": c["has_images"],
                        "metadata": json.loads(c["metadata"]) if c["metadata"] else {},
                        "score": score, "rank": rank})
        assert [g["chunk_id"] for g in got] == [r["chunk_id"] for r in ref]
        for g, r in zip(got, ref):
            assert {k: v for k, v in g.items() if k != "score"} == {k: v for k, v in r.items() if k != "score"}
            assert abs(g["score"] - r["score"]) < 1e-6


def test_native_rrf_random_lists_match_reference():
    """cbv2_rrf_fuse (host C++) against the reference's RRF restated in
    oracle.rrf (LRC:960-978: float64 1/(k + rank) sums, BM25 list first,
    stable descending sort -> equal sums keep first-insertion order) + [:C],
    over random overlapping lists: small id ranges (many shared ids and exact
    ties), empty lists, trailing -1 padding (as the searches pad), several
    rrf_k and C."""
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    rng = np.random.default_rng(17)
    for case in range(300):
        m = int(rng.integers(1, 200))
        B = int(rng.integers(1, 4))
        kb, kc = int(rng.integers(0, 121)), int(rng.integers(0, 121))
        C = int(rng.choice([1, 10, 50, 250]))
        rk = int(rng.choice([60, 1, 7]))
        bm = np.full((B, kb), -1, np.int32)
        cb = np.full((B, kc), -1, np.int32)
        for b in range(B):
            nb, nc = min(kb, int(rng.integers(0, m + 1))), min(kc, int(rng.integers(0, m + 1)))
            bm[b, :nb] = rng.permutation(m)[:nb]
            cb[b, :nc] = rng.permutation(m)[:nc]
        got, sc, cnt = rrf_fuse(bm, cb, rrf_k=rk, C=C, return_scores=True)
        for b in range(B):
            full = orc.rrf([int(x) for x in bm[b] if x >= 0], [int(x) for x in cb[b] if x >= 0], k=rk)
            want = full[:C]
            ids = [cid for cid, _ in want]
            assert got[b, :len(ids)].tolist() == ids, (case, b)
            assert (got[b, len(ids):] == -1).all() and int(cnt[b]) == len(full), (case, b)   # count: distinct ids (before [:C], the header)
            assert sc[b, :len(ids)].tolist() == [s for _, s in want], (case, b)
