"""GPU: the block-max top-k (CBV2_OPT_TOPK_BMAX, topk_bmax_kernel + the scans'
bmax_fold epilogue) returns exactly what the sampled filter + select and the
oracle's selection return (torch.topk semantics, LRC:767, ties -> lower id).

Every scan that feeds it is covered -- the direct scan (B <= 2), the 4-wave
shapes (B = 3..16), the 8-wave scan (B > 16), MXFP8 (direct, 4-wave and 8x8)
-- with ragged and empty docs, n not a multiple of 64 (the last block is
partial; dynamic-tail tasks start off the 64-doc grid), k = 1 .. 1024, heavy
ties (duplicated docs) and the fallback when ties at the threshold overflow
the candidate buffer (every doc identical)."""
import numpy as np
import pytest
import torch

from _parity import assert_selection_exact
from hybrid_rag_colbertv2_amd import _lib, synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex

pytestmark = pytest.mark.gpu


def _corpus(dev, n, B, seed):
    Qf = synth.make_queries(B, 32, seed=seed)
    planted = synth.planted_ids(B, n, 10, seed=seed + 1)
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=seed)
    g = torch.Generator(device=dev).manual_seed(seed)
    sel = torch.randperm(n, generator=g, device=dev)[: n // 50]
    doclens[sel] = torch.randint(0, 129, (len(sel),), generator=g, device=dev, dtype=torch.int32)
    doclens[sel[:20]] = 0                                     # empty docs score -inf
    dup = torch.randperm(n, generator=g, device=dev)[: n // 100]
    tokens[dup] = tokens[dup[0]].clone()                     # exact ties across many ids
    doclens[dup] = doclens[dup[0]].clone()
    return Qf.to(dev, torch.bfloat16), tokens, doclens


def _both(ix, Q, k):
    ix.set_option(_lib.OPT_TOPK_BMAX, 1)
    s1, i1 = ix.search(Q, k)
    ix.set_option(_lib.OPT_TOPK_BMAX, 0)
    s0, i0 = ix.search(Q, k)
    ix.set_option(_lib.OPT_TOPK_BMAX, 1)
    return (s1, i1), (s0, i0)


@pytest.mark.parametrize("n,B,k", [(65536, 1, 100), (100_003, 2, 100), (125_000, 5, 10), (100_000, 16, 100),
                                   (70_001, 40, 1), (131_072, 64, 1024), (100_000, 256, 100),
                                   # k large against the superblock count (k * 8 > n / 256): the
                                   # threshold from block keys (advisor, round 4), streaming scan and
                                   # the one-launch block-max select (B = 3-8)
                                   (70_001, 1, 1024), (70_001, 4, 1024), (262_143, 2, 1024)])
def test_bmax_equals_sampled_and_oracle_selection(dev, n, B, k):
    Q, tokens, doclens = _corpus(dev, n, B, seed=n % 97 + B)
    ix = ColbertIndex(tokens, doclens, id_base=17)
    (s1, i1), (s0, i0) = _both(ix, Q, k)
    assert torch.equal(i1, i0) and torch.equal(s1, s0), "block-max top-k differs from the sampled filter + select"
    full = ix.score(Q).cpu().numpy()
    assert_selection_exact(i1.cpu().numpy(), s1.cpu().numpy(), full, k, id_base=17)


@pytest.mark.parametrize("B", [1, 8, 16, 256])
def test_bmax_mxfp8(dev, B):
    n, k = 100_000, 100
    Q, tokens, doclens = _corpus(dev, n, B, seed=3 + B)
    ix = ColbertIndex.mxfp8(tokens, doclens)
    (s1, i1), (s0, i0) = _both(ix, Q, k)
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    assert_selection_exact(i1.cpu().numpy(), s1.cpu().numpy(), ix.score(Q).cpu().numpy(), k)


def test_bmax_all_ties_fall_back_exactly(dev):
    """Every doc identical: all blocks tie at t, the gathered candidates overflow
    kBmCand, and the row takes the exact full-row select -- still ids 0..k-1."""
    n, B, k = 70_000, 3, 100
    g = torch.Generator().manual_seed(0)
    one = torch.randn(1, 128, 128, generator=g).bfloat16().to(dev)
    tokens = one.expand(n, 128, 128).contiguous()
    doclens = torch.full((n,), 128, dtype=torch.int32, device=dev)
    Q = torch.randn(B, 32, 128, generator=g).bfloat16().to(dev)
    ix = ColbertIndex(tokens, doclens)
    (s1, i1), (s0, i0) = _both(ix, Q, k)
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    assert (i1.cpu() == torch.arange(k, dtype=torch.int32)).all()


def test_bmax_workspace_and_small_rows(dev):
    """Rows shorter than the sampled threshold keep the exact row select; the
    any-k workspace covers both layouts."""
    n = 5000
    Q, tokens, doclens = _corpus(dev, n, 4, seed=9)
    ix = ColbertIndex(tokens, doclens)
    (s1, i1), (s0, i0) = _both(ix, Q, 50)
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    L = _lib.lib()
    big = ColbertIndex(*_corpus(dev, 100_000, 2, seed=4)[1:])
    any_k = int(L.cbv2_search_workspace_bytes(big._h, 256))
    for k in (1, 100, 1024, 4096):
        assert int(L.cbv2_search_workspace_size(big._h, 256, k, 0)) <= any_k


@pytest.mark.parametrize("B", [1, 16])
def test_bmax_faithful_search(dev, B):
    """The fp32-faithful search's bf16 phase takes the same block-max top-k."""
    n, k = 80_000, 100
    Qf = synth.make_queries(B, 32, seed=40 + B)
    planted = synth.planted_ids(B, n, 10, seed=41)
    x, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=42, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(x, doclens)
    Q = Qf.to(dev)
    (s1, i1), (s0, i0) = _both(ix, Q, k)
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    assert all(set(i1[b, :10].tolist()) == set(planted[b].tolist()) for b in range(B))


@pytest.mark.parametrize("B", [1, 2, 3, 8])
def test_bmax_one_launch_dense_docs(dev, B):
    """Dense-doc index (every doc 128 tokens: the 4 x 1 scan, whose keys the
    one-launch bmax_topk_kernel writes and selects from, B <= 8) and a
    repeated call (its arrival counters are re-zeroed by the last workgroup):
    equal to the sampled path and to the oracle's selection."""
    n, k = 125_000, 100
    Qf = synth.make_queries(B, 32, seed=B)
    planted = synth.planted_ids(B, n, 10, seed=B + 1)
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=B)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    (s1, i1), (s0, i0) = _both(ix, Q, k)
    s2, i2 = ix.search(Q, k)
    assert torch.equal(i1, i0) and torch.equal(s1, s0) and torch.equal(i2, i1) and torch.equal(s2, s1)
    assert_selection_exact(i1.cpu().numpy(), s1.cpu().numpy(), ix.score(Q).cpu().numpy(), k)
