"""GPU parity of the selections beyond one LDS sort: torch.topk takes any k
(local_rag_complete.py:767) and the rerank argsort any C (:789).  k > 1024
runs the multi-pass selection (passes bounded below the previous pass's last
key), C > 1024 the LDS-resident rerank, G*k > 8192 the in-place merge.  Each
is compared with the oracle's (score desc, index asc) selection bit for bit —
on the GPU's own score matrix, so the check is exact even with ties."""
import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd.index import ColbertIndex, merge_topk, select_topk, topk_rows
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def rand_unit(g, *shape):
    x = torch.randn(*shape, generator=g)
    return x / x.norm(dim=-1, keepdim=True)


def make_case(seed, N, B, lq=32):
    g = torch.Generator().manual_seed(seed)
    docs = rand_unit(g, N, 128, 128).bfloat16()
    doclens = torch.randint(1, 129, (N,), generator=g, dtype=torch.int32)
    Q = rand_unit(g, B, lq, 128).bfloat16()
    return docs, doclens, Q


@pytest.mark.parametrize("n,k", [(5000, 1025), (5000, 4096), (9000, 4097), (3000, 5000), (20000, 12345)])
def test_topk_rows_large_k(dev, n, k):
    g = np.random.default_rng(n + k)
    scores = g.integers(-50, 50, size=(3, n)).astype(np.float32)     # heavy ties across pass boundaries
    scores[1] = g.standard_normal(n).astype(np.float32)
    scores[2, ::5] = -np.inf
    s, i = topk_rows(torch.from_numpy(scores).to(dev), k, id_base=7)
    rs, ri = orc.topk(scores, k, id_base=7)
    assert np.array_equal(i.cpu().numpy(), ri)
    assert np.array_equal(s.cpu().numpy(), rs.astype(np.float32))


@pytest.mark.parametrize("N,B,k", [(6000, 3, 2000), (3000, 20, 3000), (2500, 2, 4000)])
def test_search_large_k(dev, N, B, k):
    docs, doclens, Q = make_case(N + k, N, B)
    ix = ColbertIndex(docs.to(dev), doclens.to(dev), id_base=11)
    s, i = ix.search(Q.to(dev), k=k)
    full = ix.score(Q.to(dev)).cpu().numpy()
    es, ei = orc.topk(full, k, id_base=11)                # the selection of the GPU's own scores
    assert np.array_equal(i.cpu().numpy(), ei)
    assert np.array_equal(s.cpu().numpy(), es.astype(np.float32))
    ref = orc.maxsim(Q.float().numpy(), docs.float().numpy(), doclens.numpy())
    kk = min(k, N)
    np.testing.assert_allclose(s.cpu().numpy()[:, :kk], orc.topk(ref, kk)[0], atol=1e-3, rtol=0)


@pytest.mark.parametrize("C,k", [(3000, 2000), (1025, 10), (5000, 6000), (32768, 100)])
def test_rerank_large_c(dev, C, k):
    N, B = 800, 3
    docs, doclens, Q = make_case(C + k, N, B)
    g = np.random.default_rng(C)
    cand = g.integers(0, N, size=(B, C)).astype(np.int32)       # many duplicates: exact ties
    cand[:, 1] = -1
    cand[:, 2] = N + 5
    ix = ColbertIndex(docs.to(dev), doclens.to(dev))
    ct = torch.from_numpy(cand).to(dev)
    raw = ix.rerank(Q.to(dev), ct, k=0)
    assert raw.shape == (B, C)
    full = ix.score(Q.to(dev))
    safe = torch.from_numpy(np.clip(cand, 0, N - 1)).to(dev).long()
    exp_raw = torch.gather(full, 1, safe)
    exp_raw[:, 1:3] = -float("inf")
    assert torch.equal(raw, exp_raw)
    s, i, p = ix.rerank(Q.to(dev), ct, k=k)
    raw_np = raw.cpu().numpy()
    for b in range(B):
        exp = orc.rerank_select(raw_np[b], k)
        got_p = p[b].cpu().numpy()
        assert [int(x) for x in got_p[:len(exp)]] == [e[0] for e in exp], b
        assert (got_p[len(exp):] == -1).all()
        assert np.array_equal(i[b].cpu().numpy()[:len(exp)], cand[b, got_p[:len(exp)]])
        assert np.array_equal(s[b].cpu().numpy()[:len(exp)], raw_np[b, got_p[:len(exp)]])


def test_select_topk_large_c(dev):
    g = np.random.default_rng(5)
    sc = g.integers(-30, 30, size=(4, 7000)).astype(np.float32)
    ids = g.integers(0, 10 ** 6, size=(4, 7000)).astype(np.int32)
    for k in (10, 1500, 7000, 8000):
        s, i, p = select_topk(torch.from_numpy(sc).to(dev), k, ids=torch.from_numpy(ids).to(dev))
        for b in range(4):
            exp = orc.rerank_select(sc[b], k)
            got = p[b].cpu().numpy()
            assert [int(x) for x in got[:len(exp)]] == [e[0] for e in exp]
            assert np.array_equal(i[b].cpu().numpy()[:len(exp)], ids[b, got[:len(exp)]])
            assert (got[len(exp):] == -1).all()


@pytest.mark.parametrize("G,k", [(4, 3000), (9, 1000), (2, 5000)])
def test_merge_topk_large(dev, G, k):
    g = np.random.default_rng(G * 10 + k)
    B = 3
    S, I = [], []
    for gg in range(G):
        sc = g.integers(-100, 100, size=(B, k + 17)).astype(np.float32)
        s, i = orc.topk(sc, k, id_base=gg * (k + 17))
        if gg == 1:
            s[:, k // 3:] = -np.inf
            i[:, k // 3:] = -1
        S.append(s.astype(np.float32))
        I.append(i.astype(np.int32))
    S, I = np.stack(S), np.stack(I)
    ms, mi = merge_topk(torch.from_numpy(S).to(dev), torch.from_numpy(I).to(dev), k)
    es, ei = orc.merge_topk(S, I, k)
    assert np.array_equal(mi.cpu().numpy(), ei)
    assert np.array_equal(ms.cpu().numpy(), es.astype(np.float32))


@pytest.mark.parametrize("k", [2000, 17000])
def test_faithful_search_large_k(dev, k):
    """fp32-faithful search with k past one LDS sort (band of k <= cap) and past
    any band (k > 16384: every row takes the full faithful scan, status -1)."""
    N, B = 18000, 2
    g = torch.Generator().manual_seed(k)
    x = rand_unit(g, N, 128, 128)
    doclens = torch.randint(1, 129, (N,), generator=g, dtype=torch.int32)
    Q = rand_unit(g, B, 32, 128)
    ix = ColbertIndex.faithful_f32(x.to(dev), doclens.to(dev))
    s, i = ix.search(Q.to(dev), k=k)
    st = ix.last_band.cpu().numpy()
    assert (st == -1).all() if k > 16384 else (st >= k).all()
    full = ix.score(Q.to(dev)).cpu().numpy()            # faithful scores of every doc
    es, ei = orc.topk(full, k)
    assert np.array_equal(i.cpu().numpy(), ei)
    assert np.array_equal(s.cpu().numpy(), es.astype(np.float32))
