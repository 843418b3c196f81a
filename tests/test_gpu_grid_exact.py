"""GPU: rank-order parity at the headline config, bit for bit.

BASELINE config 3 / north_star: "top-10 ranks identical to the CPU reference"
on a 1M-chunk x 128-token corpus; the reference ranks with torch.topk /
argsort (local_rag_complete.py:767, 789), the tie rule made explicit here as
(score desc, id asc) / (score desc, position asc).

The corpus (tests/_grid.py) is 1M ragged docs on the k/16 grid, where every
score is exact in fp32 whatever the accumulation order, so the kernels'
results must EQUAL the oracle's: the stage-2 top-100 and the final top-10 of
the whole pipelined path (scan top-100 -> RRF with a stage-1 list -> rerank of
the fused 50 -> top-10) are compared for ids, ORDER and float32 score bits for
all 256 queries, ties included (~11 % of adjacent top-100 pairs are exact
ties), for the bf16 index, the fp32-faithful index and the MXFP8 index, and at
the batch shapes of the other kernels (B = 1 direct scan, B = 16).  The
oracle scores the 1M docs through their code sets (oracle.codebook_topk),
which tests/test_grid_oracle.py checks against the plain maxsim oracle.
"""
import numpy as np
import pytest
import torch

from _grid import GridCorpus
from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever
from hybrid_rag_colbertv2_amd.index import ColbertIndex
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
N, B, K2, C, KF = 1_000_000, 256, 100, 50, 10


def _bits(x):
    return np.ascontiguousarray(np.asarray(x, np.float32)).view(np.int32)


@pytest.fixture(scope="module")
def grid():
    g = GridCorpus(N, B, seed=123)
    es, ei = g.topk(K2)
    bm = synth.bm25_lists(B, N, g.planted, k=K2, hits=5, seed=31)
    fin_s = np.full((B, KF), -np.inf)
    fin_i = np.full((B, KF), -1, np.int64)
    for b in range(B):
        fused = [cid for cid, _ in orc.rrf(bm[b].tolist(), ei[b].tolist(), k=60)[:C]]
        sc = g.exact_scores([b], np.array([fused]))[0]
        for r, (p, s, _) in enumerate(orc.rerank_select(sc, KF)):
            fin_s[b, r], fin_i[b, r] = s, fused[p]
    return g, es, ei, bm, fin_s, fin_i


def _index(g, kind, dev):
    torch.cuda.empty_cache()
    dl = g.doclens_on(dev)
    if kind == "fp32":
        x = g.tokens_on(dev, torch.float32)
        ix = ColbertIndex.faithful_f32(x, dl)
        del x
        return ix, torch.from_numpy(g.Q).to(dev)
    t = g.tokens_on(dev)
    ix = ColbertIndex.mxfp8(t, dl) if kind == "mxfp8" else ColbertIndex(t, dl)
    del t
    return ix, torch.from_numpy(g.Q).to(dev, torch.bfloat16)


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("kind", ["bf16", "fp32", "mxfp8"])
def test_grid_1m_pipeline_ranks_and_scores_exact(dev, grid, kind):
    g, es, ei, bm, fin_s, fin_i = grid
    ix, Q = _index(g, kind, dev)
    if kind == "mxfp8":
        assert ix.fp8
    if kind == "fp32":
        assert ix.faithful
    # stage 2 at the headline batch: ids, order and score bits of the whole top-100
    s, i = ix.search(Q, K2)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    bad = np.nonzero((i != ei).any(axis=1))[0]
    assert len(bad) == 0, f"{kind}: {len(bad)} of {B} rows differ from the oracle, first {bad[:5]}"
    assert np.array_equal(_bits(s), _bits(es)), f"{kind}: top-100 score bits differ"
    # the other scan kernels: direct (B = 1) and mid-batch (B = 16)
    for lo, hi in ((0, 1), (37, 38), (64, 80)):
        s1, i1 = ix.search(Q[lo:hi], K2)
        assert np.array_equal(i1.cpu().numpy(), ei[lo:hi]), (kind, lo, hi)
        assert np.array_equal(_bits(s1.cpu().numpy()), _bits(es[lo:hi])), (kind, lo, hi)
    # the full pipelined path (two batches in flight): final top-10 ids, order, score bits
    outs = PipelinedRetriever(ix, dev, colbert_k=K2, fused=C, final_k=KF).run([(Q, bm), (Q, bm)])
    for fs, fi in outs:
        fs, fi = fs.cpu().numpy(), fi.cpu().numpy()
        assert np.array_equal(fi, fin_i), f"{kind}: final top-10 ids/order differ"
        assert np.array_equal(_bits(fs), _bits(fin_s)), f"{kind}: final top-10 score bits differ"
    # rank 1..10 of every query are its planted docs, the exact tie in id order
    for b in range(B):
        assert set(fin_i[b].tolist()) == set(g.planted[b].tolist())
    del ix
