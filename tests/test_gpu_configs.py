"""GPU tests of BASELINE.json's configs on one MI355X.

* C2 -- 100k chunks x 128 tokens, MaxSim-only top-100 at B = 1, 16, 64, 256:
  every query's top-10 = its planted positives; the top-100 is exactly the
  oracle's selection of the GPU's score matrix (bit for bit); the returned
  docs' scores equal the oracle's float64 MaxSim within 1e-3 and rank as the
  oracle ranks them; every batch size gives the same score bits.
* C4 -- 10M bf16 chunks as eight 1.25M-doc shards (the 8-GPU layout; 328 GB of
  bf16 does not fit one GPU, so the shards run one after another with
  id_base = r * 1.25M), then the HIP merge of [8, 256, 100]: top-10 = planted,
  merged scores = the oracle's on the stored values.
* C5 -- 10M MXFP8 chunks resident in ONE HBM (167 GB), B = 256: top-10 =
  planted, oracle spot scores on the dequantised values within 2e-3, and the
  unsharded ids/scores equal eight shard views + merge bit for bit.
* C3 -- 1M chunks, the whole pipelined hybrid path (host BM25 + stage 2 + RRF +
  rerank): top-10 = planted; equal to the unpipelined path; and for 32 queries
  the final top-10 is re-derived on the CPU from the same stage-1/2 lists
  (oracle RRF, oracle MaxSim rerank of the fused 50) -- ids exact, scores 1e-3.

The reference defines these workloads only through BASELINE.json configs 2-5;
its own selection is torch.topk (local_rag_complete.py:767).
"""
import numpy as np
import pytest
import torch

from _parity import assert_ids_match_separated, assert_ranking_consistent, assert_selection_exact
from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex, merge_topk, quantize_mxfp8
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
B, K = 256, 100


def _planted_ok(ids, planted, rows=None):
    ids = ids.cpu().numpy() if isinstance(ids, torch.Tensor) else ids
    rows = range(len(ids)) if rows is None else rows
    return all(set(ids[j, :10].tolist()) == set(planted[b].tolist()) for j, b in enumerate(rows))


# --------------------------------------------------------------------------- C2
@pytest.fixture(scope="module")
def c2(dev):
    N = 100_000
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, seed=0)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    full = ix.score(Q)                                   # the B=256 scan's score bits
    return N, planted, tokens, ix, Q, full


@pytest.mark.parametrize("Bq", [1, 16, 64, 256])
def test_c2_100k_maxsim_top100(dev, c2, Bq):
    N, planted, tokens, ix, Q, full = c2
    q = Q[:Bq]
    s, i = ix.search(q, K)
    assert _planted_ok(i, planted[:Bq])
    assert torch.equal(ix.score(q), full[:Bq])           # every batch shape: the same bits
    assert_selection_exact(i.cpu().numpy(), s.cpu().numpy(), full[:Bq].cpu().numpy(), K)
    rows = [0, Bq // 2, Bq - 1]
    for b in sorted(set(rows)):
        ids = i[b].long()
        ref = orc.maxsim(q[b:b + 1].float().cpu().numpy(), tokens[ids].float().cpu().numpy())[0]
        np.testing.assert_allclose(s[b].cpu().numpy(), ref, atol=1e-3, rtol=0)
    # ranking vs the oracle over a 3000-doc slice holding query 0's planted docs
    sl = np.unique(np.concatenate([planted[0], np.arange(0, N, 37)]))
    ref = orc.maxsim(q[:1].float().cpu().numpy(), tokens[torch.from_numpy(sl).to(dev)].float().cpu().numpy())
    sub = ColbertIndex(tokens[torch.from_numpy(sl).to(dev)].contiguous(),
                       torch.full((len(sl),), 128, dtype=torch.int32, device=dev))
    _, si = sub.search(q[:1], K)
    assert_ranking_consistent(si.cpu().numpy(), ref, 1e-3)


# --------------------------------------------------------------------------- C4
def test_c4_10m_bf16_eight_serial_shards(dev):
    N, G = 10_000_000, 8
    per = N // G
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    Q = Qf.to(dev, torch.bfloat16)
    spot = (0, 77, 255)
    S, I, saved = [], [], {}
    for r in range(G):
        torch.cuda.empty_cache()
        tokens, doclens = synth.make_shard(r * per, (r + 1) * per, Qf, planted, dev, seed=0)
        ix = ColbertIndex(tokens, doclens, id_base=r * per)
        s, i = ix.search(Q, K)
        S.append(s)
        I.append(i)
        for b in spot:                                   # keep the tokens a spot check may need
            for gid in i[b, :12].tolist():
                saved[gid] = tokens[gid - r * per].float().cpu().numpy()
        del ix, tokens, doclens
    ms, mi = merge_topk(torch.stack(S), torch.stack(I), K)
    assert _planted_ok(mi, planted)
    assert (torch.diff(ms, dim=1) <= 0).all()
    for b in spot:
        ids = mi[b, :12].tolist()
        ref = orc.maxsim(Q[b:b + 1].float().cpu().numpy(), np.stack([saved[x] for x in ids]))[0]
        np.testing.assert_allclose(ms[b, :12].cpu().numpy(), ref, atol=1e-3, rtol=0)
    eo = orc.merge_topk(torch.stack(S).cpu().numpy(), torch.stack(I).cpu().numpy(), K)
    assert np.array_equal(mi.cpu().numpy(), eo[1])


# --------------------------------------------------------------------------- C5
def test_c5_10m_mxfp8_one_hbm(dev):
    N, G = 10_000_000, 8
    torch.cuda.empty_cache()
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    q8, sc8, doclens = synth.make_shard_mxfp8(0, N, Qf, planted, dev, seed=0)
    ix = ColbertIndex(q8, doclens, scales=sc8)
    Q = Qf.to(dev, torch.bfloat16)
    s, i = ix.search(Q, K)
    assert _planted_ok(i, planted)
    assert (torch.diff(s, dim=1) <= 0).all()
    qq, qs = quantize_mxfp8(Q)
    Qd = orc.mxfp8_dequant(qq.cpu().numpy(), qs.cpu().numpy())
    for b in (0, 77, 255):
        ids = i[b, :12].long()
        ref = orc.maxsim(Qd[b:b + 1], orc.mxfp8_dequant(q8[ids].cpu().numpy(), sc8[ids].cpu().numpy()))[0]
        np.testing.assert_allclose(s[b, :12].cpu().numpy(), ref, atol=2e-3, rtol=0)
    per = N // G
    parts = [ColbertIndex(q8[r * per:(r + 1) * per], doclens[r * per:(r + 1) * per], id_base=r * per,
                          scales=sc8[r * per:(r + 1) * per]).search(Q, K) for r in range(G)]
    ms, mi = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), K)
    assert torch.equal(mi, i) and torch.equal(ms, s)


# --------------------------------------------------------------------------- C3
def test_c3_1m_pipelined_hybrid(dev):
    from hybrid_rag_colbertv2_amd import bm25 as bm25_mod
    from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher
    from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever, rrf_fuse
    N = 1_000_000
    torch.cuda.empty_cache()
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    terms, offs, vocab = synth.bm25_shard(0, N, planted)
    lex = bm25_mod.NativeBM25(terms, offs, vocab)
    del terms, offs
    qt, qo = synth.bm25_queries(B)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, seed=0)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    searcher = ShardedSearcher(ix, world=1)
    pipe = PipelinedRetriever(searcher, dev, colbert_k=100, fused=50, final_k=10)
    bm = lambda: lex.search(qt, qo, 100)                     # noqa: E731
    outs = pipe.run([(Q, bm)] * 3)
    fs, fi = outs[-1]
    for s_, i_ in outs[:-1]:                                 # every pipelined batch: the same result
        assert torch.equal(i_, fi) and torch.equal(s_, fs)
    assert _planted_ok(fi, planted)
    # unpipelined, stage by stage
    bm_ids, _ = lex.search(qt, qo, 100)
    s2, i2 = ix.search(Q, 100)
    cand = rrf_fuse(bm_ids, i2.cpu().numpy(), rrf_k=60, C=50)
    rs, ri, _ = ix.rerank(Q, torch.from_numpy(cand).to(dev), 10)
    assert torch.equal(ri, fi) and torch.equal(rs, fs)
    # CPU re-derivation for 32 queries: oracle RRF of the same lists, oracle MaxSim rerank of the fused 50
    i2h = i2.cpu().numpy()
    for b in range(0, B, 8):
        fused = [cid for cid, _ in orc.rrf(bm_ids[b].tolist(), i2h[b].tolist(), k=60)[:50]]
        assert fused == [int(x) for x in cand[b] if x >= 0], b
        docs = tokens[torch.tensor(fused, device=dev)].float().cpu().numpy()
        es, ei, ep = orc.rerank(Q[b:b + 1].float().cpu().numpy(), docs, np.full(len(fused), 128),
                                np.arange(len(fused))[None], 10)
        np.testing.assert_allclose(fs[b].cpu().numpy(), es[0], atol=1e-3, rtol=0)
        exp_ids = np.array([[fused[p] for p in ep[0]]])
        assert set(exp_ids[0].tolist()) == set(fi[b].tolist()), b          # the 10th/11th gap is >> 1e-3
        # the 10 planted docs' scores sit within ~1e-3 of each other (only ~6 % of
        # positions separate by more), so their ORDER is pinned bit for bit by the
        # exact-arithmetic 1M corpus of test_gpu_grid_exact.py, not here
        assert_ids_match_separated(fi[b:b + 1].cpu().numpy(), exp_ids, es, 1e-3, min_frac=0.0)
