"""GPU parity of the fused scan + top-k (cbv2_search with k <= 104 on the
bf16 doc-interleaved scan, B > 16; the MXFP8 scan's fused build, slower and
off by default, is forced with CBV2_OPT_FUSED_TOPK = 2 for its own test).

The fused path never writes the [B, n] score matrix: each workgroup keeps its
best k keys per query in LDS and select_keys_kernel picks the global top-k.
Its results must be those of the unfused path (score matrix + radix top-k)
BIT FOR BIT -- ids and score bits, ties included -- and exactly the oracle's
selection (score desc, id asc) of the GPU's own score matrix.
"""
import numpy as np
import pytest
import torch

from _parity import assert_selection_exact
from hybrid_rag_colbertv2_amd import _lib
from hybrid_rag_colbertv2_amd.index import ColbertIndex
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _corpus(dev, N, seed, ragged=True, dup=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    docs = torch.randn(N, 128, 128, device=dev, generator=g)
    docs = (docs / docs.norm(dim=-1, keepdim=True)).bfloat16()
    if ragged:
        doclens = torch.randint(0, 129, (N,), device=dev, generator=g, dtype=torch.int32)
    else:
        doclens = torch.full((N,), 128, dtype=torch.int32, device=dev)
    if dup:   # exact ties: copies of doc 0 spread over the corpus
        pos = torch.randperm(N, device=dev, generator=g)[:dup]
        docs[pos] = docs[0].clone()
        doclens[pos] = doclens[0] = 128
    return docs, doclens


def _queries(dev, B, seed, near=None):
    g = torch.Generator(device=dev).manual_seed(seed)
    Q = torch.randn(B, 32, 128, device=dev, generator=g)
    if near is not None:
        Q[: B // 2] = near[:32].float() + 0.05 * Q[: B // 2]
    return (Q / Q.norm(dim=-1, keepdim=True)).bfloat16()


def _both(ix, Q, k, mode=1):
    ix.set_option(_lib.OPT_FUSED_TOPK, mode)
    fs, fi = ix.search(Q, k)
    ix.set_option(_lib.OPT_FUSED_TOPK, 0)
    us, ui = ix.search(Q, k)
    ix.set_option(_lib.OPT_FUSED_TOPK, 1)
    return fs, fi, us, ui


@pytest.mark.parametrize("N,B,k", [(70000, 64, 100), (24000, 200, 104), (9000, 17, 10), (3000, 40, 1),
                                   (50, 40, 100), (700, 256, 100)])
def test_fused_equals_unfused_bf16(dev, N, B, k):
    docs, doclens = _corpus(dev, N, N + B)
    Q = _queries(dev, B, k)
    ix = ColbertIndex(docs, doclens, id_base=7)
    fs, fi, us, ui = _both(ix, Q, k)
    assert torch.equal(fi, ui) and torch.equal(fs.view(torch.int32), us.view(torch.int32))
    assert_selection_exact(fi.cpu().numpy(), fs.cpu().numpy(), ix.score(Q).cpu().numpy(), k, id_base=7)
    kk = min(k, N)
    assert (fi[:, kk:] == -1).all() and torch.isneginf(fs[:, kk:]).all()


def test_fused_ties_and_empty_docs(dev):
    """Hundreds of exact copies of one doc (exact score ties, broken by the lower
    id) and empty docs (-inf) inside the top-k."""
    docs, doclens = _corpus(dev, 40000, 5, dup=600)
    doclens[1::9] = 0
    Q = _queries(dev, 64, 6, near=docs[0])
    ix = ColbertIndex(docs, doclens)
    fs, fi, us, ui = _both(ix, Q, 100)
    assert torch.equal(fi, ui) and torch.equal(fs.view(torch.int32), us.view(torch.int32))
    full = ix.score(Q).cpu().numpy()
    assert_selection_exact(fi.cpu().numpy(), fs.cpu().numpy(), full, 100)
    tied = (fs[:32] == fs[:32, :1]).sum(dim=1)
    assert (tied >= 100).all(), "the planted copies should fill the top-100 with exact ties"
    # rows of a query far from everything: a few empty docs at the end when k > live docs
    small, sl = docs[:150].contiguous(), doclens[:150].clone()
    sl[:100] = 0
    sl[100:] = 128                               # exactly 50 live docs
    ix2 = ColbertIndex(small, sl)
    fs2, fi2, us2, ui2 = _both(ix2, Q, 100)
    assert torch.equal(fi2, ui2) and torch.isneginf(fs2[:, 50:]).all()
    assert (fi2[:, 50:] == torch.arange(50, dtype=torch.int32, device=dev)).all()   # -inf ties: lower id first


@pytest.mark.parametrize("N,B,k", [(70000, 64, 100), (5000, 9, 50), (30000, 256, 104)])
def test_fused_equals_unfused_fp8(dev, N, B, k):
    docs, doclens = _corpus(dev, N, 3 * N + B)
    Q = _queries(dev, B, 2 * k)
    ix = ColbertIndex.mxfp8(docs, doclens)
    assert ix.fused_topk_slots(B, k) == 0            # off by default: the fused f8 build spills
    ix.set_option(_lib.OPT_FUSED_TOPK, 2)
    # the product library leaves the spilling fused MXFP8 scan out (lab builds
    # only): mode 2 searches an MXFP8 index unfused, with the same results
    assert ix.fused_topk_slots(B, k) == 0
    fs, fi, us, ui = _both(ix, Q, k, mode=2)
    assert torch.equal(fi, ui) and torch.equal(fs.view(torch.int32), us.view(torch.int32))


def test_fused_workspace_is_small_and_large_k_unfused(dev):
    docs, doclens = _corpus(dev, 100000, 1, ragged=False)
    ix = ColbertIndex(docs, doclens)
    L = _lib.lib()
    assert ix.fused_topk_slots(256, 100) == 0        # off by default (A/B: the unfused path is faster)
    ix.set_option(_lib.OPT_FUSED_TOPK, 1)
    fused = L.cbv2_search_workspace_size(ix._h, 256, 100, 0)
    unfused = L.cbv2_search_workspace_size(ix._h, 256, 200, 0)
    assert fused < 8 << 20 < 256 * 100000 * 4 <= unfused, (fused, unfused)   # unfused: the [B, n] score matrix
    Q = _queries(dev, 256, 3)
    s, i = ix.search(Q, 200)                 # k > 104: the unfused path
    s1, i1 = ix.search(Q, 100)               # fused
    assert torch.equal(i[:, :100], i1) and torch.equal(s[:, :100], s1)


def test_concurrent_streams_distinct_workspaces(dev):
    """Two searches in flight on two streams (each with its own workspace and
    dynamic-tail counters) return what they return alone."""
    docs, doclens = _corpus(dev, 60000, 8, ragged=False)
    ix = ColbertIndex(docs, doclens)
    Qa, Qb = _queries(dev, 64, 1), _queries(dev, 256, 2)
    ra, rb = ix.search(Qa, 50), ix.search(Qb, 100)
    ix2 = ColbertIndex(docs, doclens)        # second handle: its own cached workspace
    sa, sb = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(sa):
            oa = ix.search(Qa, 50)
        with torch.cuda.stream(sb):
            ob = ix2.search(Qb, 100)
        torch.cuda.synchronize()
        assert torch.equal(oa[1], ra[1]) and torch.equal(ob[1], rb[1])
        assert torch.equal(oa[0], ra[0]) and torch.equal(ob[0], rb[0])


def test_score_ring_slots_ordered_across_streams(dev):
    """cbv2_score's handle-owned counter ring: 300 launches (> 128 slots)
    alternating between two streams, every score row identical."""
    docs, doclens = _corpus(dev, 20000, 4, ragged=False)
    ix = ColbertIndex(docs, doclens)
    Q = _queries(dev, 64, 9)
    ref = ix.score(Q).clone()
    assert ix.last_scan_plan()["dynamic_tail"]
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    torch.cuda.synchronize()     # the side streams do not wait for the default stream's corpus/queries
    outs = []
    for j in range(300):
        with torch.cuda.stream(streams[j & 1]):
            outs.append(ix.score(Q)[:, ::997].clone())
    torch.cuda.synchronize()
    for o in outs:
        assert torch.equal(o, ref[:, ::997])
