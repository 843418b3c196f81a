"""GPU parity at BASELINE.json's full sizes (config 3: 1M chunks x 128 tokens
x 128-d, B=256, k=100), through size-independent properties the oracle can
check without scoring the whole corpus:

* every query's top-10 are exactly its 10 planted positives;
* the top-100 lists are sorted, ids unique and in range;
* scores of the returned docs equal the oracle's MaxSim of those docs
  (float64 on the stored values; 1e-3 bf16 / 2e-3 fp8 / 1e-4 fp32-faithful);
* the B=256 LDS scan and the B=1 streaming scan give bit-identical rows;
* two half-corpus shards + the HIP merge == the unsharded search, bit for bit;
* the fp32-faithful search certifies every row (no band overflow).
"""
import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex, merge_topk
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
N, B, K = 1_000_000, 256, 100


@pytest.fixture(scope="module")
def corpus(dev):
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    return Qf, planted


def _check_lists(s, i, planted, n):
    s, i = s.cpu(), i.cpu().numpy()
    assert (torch.diff(s, dim=1) <= 0).all()
    assert ((i >= 0) & (i < n)).all()
    assert all(len(set(row)) == len(row) for row in i)
    assert all(set(i[b, :10]) == set(planted[b]) for b in range(len(planted)))


def _spot(Qd, docs_fn, s, i, tol, rows=(0, 77, 255)):
    for b in rows:
        ids = i[b, :12].cpu()
        ref = orc.maxsim(Qd[b:b + 1], docs_fn(ids))[0]
        np.testing.assert_allclose(s[b, :12].cpu().numpy(), ref, atol=tol, rtol=0)


def test_fullsize_bf16_search(dev, corpus):
    torch.cuda.empty_cache()
    Qf, planted = corpus
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, seed=0)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    s, i = ix.search(Q, K)
    _check_lists(s, i, planted, N)
    _spot(Q.float().cpu().numpy(), lambda ids: tokens[ids.to(dev)].float().cpu().numpy(), s, i, 1e-3)
    # B=256 (LDS scan) vs B=1 (streaming scan): the same bits for query 0
    row_b = ix.score(Q)[0]
    row_1 = ix.score(Q[:1])[0]
    assert torch.equal(row_b, row_1)
    # two shards + merge == unsharded
    h = N // 2
    parts = [ColbertIndex(tokens[a:b], doclens[a:b], id_base=a).search(Q, K) for a, b in ((0, h), (h, N))]
    ms, mi = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), K)
    assert torch.equal(mi, i) and torch.equal(ms, s)


def test_fullsize_fp8_search(dev, corpus):
    torch.cuda.empty_cache()
    Qf, planted = corpus
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, seed=0)
    ix = ColbertIndex.mxfp8(tokens, doclens)
    del tokens
    Q = Qf.to(dev, torch.bfloat16)
    s, i = ix.search(Q, K)
    _check_lists(s, i, planted, N)
    from hybrid_rag_colbertv2_amd.index import quantize_mxfp8
    qq, qs = quantize_mxfp8(Q)
    Qd = orc.mxfp8_dequant(qq.cpu().numpy(), qs.cpu().numpy())
    _spot(Qd, lambda ids: orc.mxfp8_dequant(ix.tokens[ids.to(dev)].cpu().numpy(),
                                            ix.scales[ids.to(dev)].cpu().numpy()), s, i, 2e-3)


def test_fullsize_fp32_faithful_search(dev, corpus):
    torch.cuda.empty_cache()
    Qf, planted = corpus
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, seed=0, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(tokens, doclens)
    Q = Qf.to(dev)
    s, i = ix.search(Q, K)
    assert (ix.last_band >= K).all()                       # every row certified
    _check_lists(s, i, planted, N)
    _spot(Q.cpu().numpy(), lambda ids: tokens[ids.to(dev)].cpu().numpy(), s, i, 1e-4)
