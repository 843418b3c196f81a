"""GPU parity of the fp32-faithful index (cbv2_split_f32 / _score_f32 /
_search_f32 / _rerank_f32) against the exact fp64 MaxSim of the fp32 values
the reference stores (local_rag_complete.py:735-746, scored at :802-831).

Tolerances (north_star: MaxSim within 1e-3 of fp32, ranks identical): faithful
scores within 1e-4 of the fp64 oracle and within 1e-3 of the reference's own
fp32 arithmetic; top-k ids identical wherever neighbouring oracle scores are
more than 1e-4 apart.  The band certificate: every row status >= 0 (band size)
on these inputs, and rows forced past the band cap fall back to the full
faithful scan with identical results.
"""
import numpy as np
import pytest
import torch

from _parity import assert_ids_match_separated, assert_ranking_consistent
from hybrid_rag_colbertv2_amd import _lib
from hybrid_rag_colbertv2_amd.index import ColbertIndex
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ATOL = 1e-4


def rand_unit(g, *shape):
    x = torch.randn(*shape, generator=g)
    return x / x.norm(dim=-1, keepdim=True)


def make_case(seed, N, B, lq, ragged=True, planted=True):
    g = torch.Generator().manual_seed(seed)
    docs = rand_unit(g, N, 128, 128)
    doclens = torch.randint(1, 129, (N,), generator=g, dtype=torch.int32) if ragged \
        else torch.full((N,), 128, dtype=torch.int32)
    Q = rand_unit(g, B, lq, 128)
    if planted:
        for b in range(B):
            for j in range(3):
                d = (97 * b + 31 * j) % N
                docs[d, :lq] = Q[b] + 0.2 * rand_unit(g, lq, 128)
                doclens[d] = 128
    return docs, doclens, Q


def test_split_matches_oracle(dev):
    docs, doclens, _ = make_case(1, 300, 2, 32)
    docs[5, 100:] = 1e6            # garbage padding: split, but outside the bounds
    doclens[5] = 100
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    hi, lo, (E, M) = orc.split_f32(docs.numpy(), doclens.numpy())
    np.testing.assert_array_equal(ix.tokens.float().cpu().numpy(), hi)
    np.testing.assert_array_equal(ix.residual.float().cpu().numpy(), lo)
    assert E <= ix.bounds[0] <= E * (1 + 2 ** -9) and M <= ix.bounds[1] <= M * (1 + 2 ** -9)


@pytest.mark.parametrize("N,B,lq", [(1, 1, 32), (257, 3, 32), (2000, 9, 20)])
def test_score_f32(dev, N, B, lq):
    docs, doclens, Q = make_case(N + B, N, B, lq)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    got = ix.score(Q.to(dev)).cpu().numpy()
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    ref32 = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy(), dtype=np.float32)
    np.testing.assert_allclose(got, exact, atol=ATOL, rtol=0)
    np.testing.assert_allclose(got, ref32, atol=1e-3, rtol=0)


def test_faithful_beats_bf16_on_fp32_inputs(dev):
    docs, doclens, Q = make_case(7, 3000, 8, 32)
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    fx = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    bx = ColbertIndex(docs.bfloat16().to(dev), doclens.to(dev))
    e_f = np.abs(fx.score(Q.to(dev)).cpu().numpy() - exact).max()
    e_b = np.abs(bx.score(Q.bfloat16().to(dev)).cpu().numpy() - exact).max()
    assert e_f < ATOL < e_b, (e_f, e_b)


@pytest.mark.parametrize("N,B,k", [(5, 2, 10), (3000, 7, 100), (70000, 3, 100)])
def test_search_f32_certified(dev, N, B, k):
    docs, doclens, Q = make_case(N * 3 + k, N, B, 32)
    doclens[::11] = 0                                   # empty docs score -inf
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=1000)
    s, i = ix.search(Q.to(dev), k)
    status = ix.last_band.cpu().numpy()
    assert (status >= 0).all(), status
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    rs, ri = orc.topk(exact, k, id_base=1000)
    fin = np.isfinite(rs)
    np.testing.assert_allclose(s.cpu().numpy()[fin], rs[fin], atol=ATOL, rtol=0)
    assert_ranking_consistent(i.cpu().numpy(), exact, ATOL, id_base=1000)
    # planted docs (gap >> 1e-4) must be compared: at least the 3 planted ranks per query
    assert_ids_match_separated(i.cpu().numpy(), ri, rs, ATOL, min_frac=0.02 if N >= 1000 else 0.0)


def test_search_f32_overflow_falls_back(dev):
    docs, doclens, Q = make_case(9, 4000, 4, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    s_full, i_full = ix.search(Q.to(dev), 20)
    assert (ix.last_band >= 0).all()
    s_cap, i_cap = ix._search_f32(Q.to(dev).contiguous(), 4, 32, 20, cap=20)   # band > 20 -> status -1
    assert (ix.last_band < 0).any()
    torch.testing.assert_close(s_cap, s_full, atol=0, rtol=0)
    assert torch.equal(i_cap, i_full)


def test_rerank_f32(dev):
    docs, doclens, Q = make_case(13, 900, 5, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=50)
    g = torch.Generator().manual_seed(3)
    cand = torch.randint(40, 960, (5, 50), generator=g, dtype=torch.int32)   # some out of shard
    s, i, p = ix.rerank(Q.to(dev), cand.to(dev), 10)
    rs, ri, rp = orc.rerank(Q.numpy(), docs.numpy(), doclens.numpy(), cand.numpy(), 10, id_base=50)
    np.testing.assert_allclose(s.cpu().numpy(), rs, atol=ATOL, rtol=0)
    assert_ids_match_separated(i.cpu().numpy(), ri, rs, ATOL)
    raw = ix.rerank(Q.to(dev), cand.to(dev), 0).cpu().numpy()
    assert raw.shape == (5, 50)


def test_f32_abi_validation(dev):
    docs, doclens, Q = make_case(2, 10, 1, 32)
    bx = ColbertIndex(docs.bfloat16().to(dev), doclens.to(dev))
    L = _lib.lib()
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    out = torch.empty((1, 10), device=dev)
    q = Q.to(dev).contiguous()
    assert L.cbv2_score_f32(bx._h, q.data_ptr(), 1, 32, ws.data_ptr(), ws.numel(), out.data_ptr(), 10,
                            None) == _lib.ERR_ESTATE
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    assert L.cbv2_score_f32(ix._h, q.data_ptr(), 1, 33, ws.data_ptr(), ws.numel(), out.data_ptr(), 10,
                            None) == _lib.ERR_EINVAL
    assert L.cbv2_score_f32(ix._h, q.data_ptr(), 1, 32, ws.data_ptr(), 16, out.data_ptr(), 10,
                            None) == _lib.ERR_EINVAL
    fk = torch.empty((1, 10), device=dev)
    oi = torch.empty((1, 10), dtype=torch.int32, device=dev)
    stt = torch.empty((1,), dtype=torch.int32, device=dev)
    assert L.cbv2_search_f32_finish(bx._h, 1, 32, 10, 64, ws.data_ptr(), ws.numel(), fk.data_ptr(), out.data_ptr(),
                                    oi.data_ptr(), stt.data_ptr(), None) == _lib.ERR_ESTATE
    assert L.cbv2_search_f32_begin(ix._h, q.data_ptr(), 1, 32, 10, 5, ws.data_ptr(), ws.numel(), fk.data_ptr(),
                                   out.data_ptr(), oi.data_ptr(), stt.data_ptr(), None) == _lib.ERR_EINVAL  # cap < k
    assert L.cbv2_search_f32_begin(ix._h, q.data_ptr(), 1, 32, 10, 64, ws.data_ptr(), ws.numel(), None,
                                   out.data_ptr(), oi.data_ptr(), stt.data_ptr(), None) == _lib.ERR_EINVAL  # null fk


def test_faithful_shards_merge_equal_unsharded(dev):
    """Per-shard faithful top-k lists + the HIP merge == the unsharded faithful
    search (what each rank of the torch.distributed exchange returns)."""
    from hybrid_rag_colbertv2_amd.index import merge_topk
    docs, doclens, Q = make_case(21, 5000, 6, 32)
    full = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    fs, fi = full.search(Q.to(dev), 50)
    parts = [ColbertIndex.faithful_f32(docs[a:b].to(dev), doclens[a:b].to(dev), id_base=a).search(Q.to(dev), 50)
             for a, b in ((0, 1800), (1800, 5000))]
    ms, mi = merge_topk(torch.stack([p[0] for p in parts]), torch.stack([p[1] for p in parts]), 50)
    assert torch.equal(mi, fi) and torch.equal(ms, fs)


@pytest.mark.parametrize("N,dups,mode", [(6000, 1, 1), (3000, 9, 1), (6000, 1, 3), (3000, 9, 3), (6000, 1, 4), (3000, 9, 4)])
def test_band_doc_major_equals_pair_major(dev, N, dups, mode):
    """Doc-major band rescoring (pairs grouped by doc, each band doc's tiles
    read once per batch; batches of more than 8 queries) returns the
    pair-by-pair rescoring's results bit for bit.  dups > 1 repeats queries,
    so every band doc has > 4 pairs (several passes of one wave over the
    doc).  modes 3 / 4: the doc split over a workgroup of 4 / 2 waves
    (rescore_docs_split_kernel)."""
    docs, doclens, Q = make_case(N + dups, N, 12, 32)
    if dups > 1:
        Q = torch.cat([Q[:1].expand(dups, -1, -1), Q[1:]]).contiguous()
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=5)
    ix.set_option(_lib.OPT_BAND_DOC_MAJOR, mode)
    s1, i1 = ix.search(Q.to(dev), 100)
    b1 = ix.last_band.clone()
    ix.set_option(_lib.OPT_BAND_DOC_MAJOR, 0)
    s0, i0 = ix.search(Q.to(dev), 100)
    assert torch.equal(ix.last_band, b1) and (b1 >= 100).all()
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    rs, _ = orc.topk(exact, 100, id_base=5)
    fin = np.isfinite(rs)
    np.testing.assert_allclose(s1.cpu().numpy()[fin], rs[fin], atol=ATOL, rtol=0)


@pytest.mark.parametrize("N,k", [(20000, 100), (3000, 10), (50, 100)])
def test_band_lower_bound_equals_plain_band(dev, N, k):
    """The two-pass band (the bf16 top-k rescored first; its minimum faithful
    score lb bounds the k-th from below; band T >= lb - beta) returns the plain
    band's (T >= T_k - 2 beta) results bit for bit, with a band no wider."""
    docs, doclens, Q = make_case(N + k, N, 5, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=11)
    s1, i1 = ix.search(Q.to(dev), k)
    b1 = ix.last_band.clone()
    ix.set_option(_lib.OPT_BAND_LOWER_BOUND, 0)
    s0, i0 = ix.search(Q.to(dev), k)
    b0 = ix.last_band.clone()
    assert torch.equal(i1, i0) and torch.equal(s1, s0)
    assert (b1 >= 0).all() and (b1 <= b0).all(), (b1, b0)
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    rs, _ = orc.topk(exact, k, id_base=11)
    fin = np.isfinite(rs)
    np.testing.assert_allclose(s1.cpu().numpy()[fin], rs[fin], atol=ATOL, rtol=0)


@pytest.mark.parametrize("N,k,parts", [(12000, 100, (0, 3000, 7000, 12000)), (3000, 10, (0, 1500, 3000)),
                                       (600, 100, (0, 550, 600))])
def test_sharded_global_lower_bound_equals_unsharded(dev, N, k, parts):
    """cbv2_search_f32_begin / _finish as ShardedSearcher uses them: the
    shards' faithful scores of their bf16 top-k, gathered, give the k-th
    largest as a bound of the GLOBAL k-th score for every shard's band; the
    merge of the per-shard lists equals the unsharded faithful search bit for
    bit, and no shard's band is wider than with its own bound (the minimum of
    its own list; shard 550..600 has < k docs)."""
    from hybrid_rag_colbertv2_amd.index import merge_topk
    docs, doclens, Q = make_case(N + k, N, 6, 32)
    Qd = Q.to(dev)
    fs, fi = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev)).search(Qd, k)
    shards = [ColbertIndex.faithful_f32(docs[a:b].to(dev), doclens[a:b].to(dev), id_base=a)
              for a, b in zip(parts[:-1], parts[1:])]
    fks, own_band = [], []

    def own(fk):                                      # pass 1: every shard alone (its lists are the gather's inputs)
        fks.append(fk.clone())
        return fk.min(dim=1).values
    for sh in shards:
        sh.search(Qd, k, lb_reduce=own)
        own_band.append(sh.last_band.clone())
    glob = torch.cat(fks, dim=1).topk(k, dim=1).values[:, k - 1]
    lists, bands = [], []
    for sh in shards:                                 # pass 2: what each rank does after the all-gather
        lists.append(sh.search(Qd, k, lb_reduce=lambda fk: glob))
        bands.append(sh.last_band.clone())
    ms, mi = merge_topk(torch.stack([x[0] for x in lists]), torch.stack([x[1] for x in lists]), k)
    assert torch.equal(mi, fi) and torch.equal(ms, fs)
    for own, b in zip(own_band, bands):
        assert ((b >= 0) & (b <= own)).all(), (own, b)
    assert sum(int(b.sum()) for b in bands) < sum(int(b.sum()) for b in own_band)


def test_small_batch_band_pair_major_equals_batched(dev):
    """Batches of at most 8 queries rescore their band pair by pair, one band
    doc per wave (no doc-major passes): every row
    equals the same query's row of a 12-query batch (doc-major, bitonic or
    counting by band size) bit for bit, band sizes included."""
    docs, doclens, Q = make_case(77, 20000, 12, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=3)
    sb, ib = ix.search(Q.to(dev), 100)
    bb = ix.last_band.clone()
    for rows in ((0,), (1, 2, 3), tuple(range(4, 12))):
        s1, i1 = ix.search(Q[list(rows)].to(dev), 100)
        assert torch.equal(i1, ib[list(rows)]) and torch.equal(s1, sb[list(rows)])
        assert torch.equal(ix.last_band, bb[list(rows)])


@pytest.mark.parametrize("copies", [300, 1500, 5000])
def test_band_select_wide_bands_ties(dev, copies):
    """Bands of identical docs (every copy ties at the k-th score): 300 copies
    (+ the band's other docs) are ranked by counting after the radix select,
    1,500 / 5,000 tie past 512 keys and the whole band is sorted; every path
    returns the lowest ids among the tied copies first, with the oracle's
    scores."""
    g = torch.Generator().manual_seed(copies)
    base = rand_unit(g, 1, 128, 128)
    docs = torch.cat([rand_unit(g, 300, 128, 128), base.expand(copies, -1, -1)]).contiguous()
    doclens = torch.full((docs.shape[0],), 128, dtype=torch.int32)
    Q = (base[:, :32] + 0.3 * rand_unit(g, 1, 32, 128))
    Q = (Q / Q.norm(dim=-1, keepdim=True)).contiguous()
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev))
    for B in (1, 12):                                   # pair-major and doc-major band
        s, i = ix.search(Q.expand(B, -1, -1).contiguous().to(dev), 100)
        band = ix.last_band.cpu().numpy()
        assert (band >= copies).all(), band
        assert (i.cpu().numpy() == np.arange(300, 400)[None, :]).all()
        exact = orc.maxsim(Q.numpy(), docs[300:301].numpy(), doclens[300:301].numpy())[0, 0]
        np.testing.assert_allclose(s.cpu().numpy(), exact, atol=ATOL, rtol=0)


@pytest.mark.parametrize("B,copies", [(1, 0), (5, 0), (8, 0), (1, 3000), (3, 3000)])
def test_band_fused_equals_separate_launches(dev, B, copies):
    """Batches of at most 8 queries collect and rescore their band in ONE
    launch (band_collect_rescore_kernel, CBV2_OPT_BAND_FUSED): scores, ids and
    band sizes equal the collect-then-rescore launches bit for bit -- also
    when 3,000 tied copies put more hits in one workgroup than its LDS list
    holds (the overflow hits are rescored as they come) and when the band
    overflows cap (the full faithful scan takes the row)."""
    docs, doclens, Q = make_case(101 + B, 20000, B, 32)
    if copies:
        docs[5000:5000 + copies] = docs[97 % 20000]          # query 0's planted doc, copied: ties
        doclens[5000:5000 + copies] = 128
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=11)
    Qd = Q.to(dev)
    for cap in (16384, 64):
        ix.set_option(_lib.OPT_BAND_FUSED, 1)
        s1, i1 = ix._search_f32(Qd.contiguous(), B, 32, 100, cap=cap)
        b1 = ix.last_band.clone()
        ix.set_option(_lib.OPT_BAND_FUSED, 0)
        s0, i0 = ix._search_f32(Qd.contiguous(), B, 32, 100, cap=cap)
        b0 = ix.last_band.clone()
        assert torch.equal(i1, i0) and torch.equal(s1, s0), cap
        assert torch.equal(b1, b0), (cap, b1, b0)
    ix.set_option(_lib.OPT_BAND_FUSED, 1)
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    assert_ranking_consistent(i1.cpu().numpy(), exact, ATOL, id_base=11)


@pytest.mark.parametrize("B,ld", [(1, 128), (5, 128), (12, 128), (3, 256)])
def test_rescore_split_equals_one_wave_per_pair(dev, B, ld):
    """One pair per workgroup, the doc's rows split over its 4 waves
    (rescore_split_kernel, CBV2_OPT_RESCORE_SPLIT) vs one pair per wave
    (rescore_x3_kernel): search (bf16 top-k rescoring, band, fallback), rerank
    and the full faithful scores equal bit for bit; ragged and empty docs, and
    docs past 128 tokens (ld 256: the 128-token blocks carried)."""
    docs, doclens, Q = make_case(301 + B + ld, 6000, B, 32)
    if ld > 128:
        docs = torch.cat([docs, torch.flip(docs, dims=(1,))], dim=1).contiguous()
        doclens = torch.randint(0, ld + 1, doclens.shape, generator=torch.Generator().manual_seed(ld),
                                dtype=torch.int32)
    doclens[::17] = 0
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=5)
    Qd = Q.to(dev)
    cand = torch.randint(0, 6010, (B, 50), generator=torch.Generator().manual_seed(B), dtype=torch.int32).to(dev)
    got = {}
    for split in (1, 0):
        ix.set_option(_lib.OPT_RESCORE_SPLIT, split)
        s, i = ix.search(Qd, 100)
        sc, si = ix._search_f32(Qd.contiguous(), B, 32, 100, cap=100)        # forces the full-scan fallback
        rs, ri, rp = ix.rerank(Qd, cand, 10)
        got[split] = [x.clone() for x in (s, i, sc, si, rs, ri, rp, ix.score(Qd), ix.rerank(Qd, cand, 0))]
    ix.set_option(_lib.OPT_RESCORE_SPLIT, 1)
    for a, b, name in zip(got[1], got[0], ("s", "i", "sc", "si", "rs", "ri", "rp", "score", "raw")):
        assert torch.equal(a, b), name
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    np.testing.assert_allclose(got[1][7].cpu().numpy(), exact, atol=ATOL, rtol=0)


@pytest.mark.parametrize("B,mode", [(1, 1), (6, 1), (12, 1), (12, 3), (12, 4), (12, 0)])
def test_band_reuse_equals_full_band(dev, B, mode):
    """CBV2_OPT_BAND_REUSE: the two-pass band keeps phase 1's faithful scores of
    the bf16 top-k as its first k slots (band_collect leaves out every doc at
    or above the k-th key) and rescores only the rest -- pair by pair (B <= 8),
    doc-major (modes 1, 3) or pair by pair at any B (mode 0).  Top-k, scores
    and band sizes equal the full band's bit for bit, with exact copies of row
    0's k-th doc (k = 40, 100) at other ids: T ties straddling the k-th key."""
    docs, doclens, Q = make_case(911 + B + mode, 5000, B, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=3)
    _, i0 = ix.search(Q.to(dev), 100)
    for j, r in enumerate((39, 99)):              # copies right after the original's key: ties at the k-th
        src = int(i0[0, r]) - 3
        docs[4990 + j], doclens[4990 + j] = docs[src], doclens[src]
    del ix
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=3)
    ix.set_option(_lib.OPT_BAND_DOC_MAJOR, mode)
    Qd = Q.to(dev)
    got = {}
    for k in (40, 100):
        for reuse in (1, 0):
            ix.set_option(_lib.OPT_BAND_REUSE, reuse)
            s, i = ix.search(Qd, k)
            got[(k, reuse)] = (s.clone(), i.clone(), ix.last_band.clone())
        for a, b, name in zip(got[(k, 1)], got[(k, 0)], ("s", "i", "band")):
            assert torch.equal(a, b), (k, name)
    ix.set_option(_lib.OPT_BAND_REUSE, 1)
    ix.set_option(_lib.OPT_BAND_DOC_MAJOR, 1)
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    assert_ranking_consistent(got[(100, 1)][1].cpu().numpy(), exact, ATOL, id_base=3)


@pytest.fixture(scope="module")
def bmax_corpus(dev):
    """70,000 docs of the bench's synthetic corpus (fp32, 10 planted per query):
    past the block-max top-k's 65,536-doc threshold, so phase 1 leaves 64-doc
    block keys for the band collect."""
    from hybrid_rag_colbertv2_amd import synth
    n, B = 70_000, 12
    Qf = synth.make_queries(B, 32, seed=5)
    planted = synth.planted_ids(B, n, 10, seed=6)
    x, dl = synth.make_shard(0, n, Qf, planted, dev, seed=3, dtype=torch.float32)
    dl[::7] = torch.randint(0, 129, dl[::7].shape, device=dev, dtype=torch.int32)   # ragged and empty docs
    ix = ColbertIndex.faithful_f32(x, dl, id_base=9)
    del x
    torch.cuda.empty_cache()
    return ix, Qf.to(dev)


@pytest.mark.parametrize("B", [1, 3, 12])
def test_band_block_skip_equals_full_row(dev, bmax_corpus, B):
    """CBV2_OPT_BAND_BLOCK_SKIP: the band collect reads only the 64-doc blocks
    whose maximum reaches the threshold (the block-max top-k's keys).  Top-k,
    scores and band sizes equal the whole-row collect's bit for bit, with and
    without the phase-1 reuse, pair-by-pair (B <= 8) and doc-major (B = 12)."""
    ix, Q = bmax_corpus
    Qb = Q[:B].contiguous()
    got = {}
    for reuse in (1, 0):
        ix.set_option(_lib.OPT_BAND_REUSE, reuse)
        for skip in (1, 0):
            ix.set_option(_lib.OPT_BAND_BLOCK_SKIP, skip)
            s, i = ix.search(Qb, 100)
            got[(reuse, skip)] = (s.clone(), i.clone(), ix.last_band.clone())
    ix.set_option(_lib.OPT_BAND_REUSE, 1)
    ix.set_option(_lib.OPT_BAND_BLOCK_SKIP, 1)
    ref = got[(0, 0)]
    assert (ref[2] > 100).all()                    # a real band beyond the top-k
    for key, val in got.items():
        for a, b, name in zip(val, ref, ("s", "i", "band")):
            assert torch.equal(a, b), (key, name)


@pytest.mark.parametrize("B", [1, 3, 8])
def test_phase1_collect_fused_equals_two_launches(dev, bmax_corpus, B):
    """CBV2_OPT_P1_COLLECT_FUSED: phase 1 (the bf16 top-k's faithful scores)
    and the band collect in one launch, the collect's workgroups waiting in
    the launch for their row's phase 1 -- top-k, scores and band sizes equal
    the two launches' bit for bit, for k = 40 / 100 / 400 (threshold over
    superblock and block keys)."""
    ix, Q = bmax_corpus
    Qb = Q[:B].contiguous()
    got = {}
    for k in (40, 100, 400):
        for fused in (1, 0):
            ix.set_option(_lib.OPT_P1_COLLECT_FUSED, fused)
            s, i = ix.search(Qb, k)
            got[(k, fused)] = (s.clone(), i.clone(), ix.last_band.clone())
        assert (got[(k, 0)][2] > k).all()          # a real band beyond the top-k
        for a, b, name in zip(got[(k, 1)], got[(k, 0)], ("s", "i", "band")):
            assert torch.equal(a, b), (k, name)
    ix.set_option(_lib.OPT_P1_COLLECT_FUSED, 1)


@pytest.mark.parametrize("B", [1, 2, 4])
def test_fold_keys_equals_block_max_pass(dev, B):
    """CBV2_OPT_FOLD_KEYS: on a dense-doc index the 4 x 1 scan folds the
    block-max select's block / superblock keys in by atomic max (keys the
    query split zeroes; scan ranges of any alignment) -- top-k, scores and
    band sizes equal the separate block-max pass's bit for bit (k = 40 / 100
    / 400, twice in a row: the keys are zeroed per call)."""
    from hybrid_rag_colbertv2_amd import synth
    n = 70_003
    Qf = synth.make_queries(B, 32, seed=41)
    planted = synth.planted_ids(B, n, 10, seed=42)
    x, dl = synth.make_shard(0, n, Qf, planted, dev, seed=43, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(x, dl, id_base=5)
    del x
    assert ix.dense_docs
    Q = Qf.to(dev).contiguous()
    got = {}
    for k in (40, 100, 400):
        for fold in (1, 0, 1):
            ix.set_option(_lib.OPT_FOLD_KEYS, fold)
            s, i = ix.search(Q, k)
            got.setdefault((k, fold), []).append((s.clone(), i.clone(), ix.last_band.clone()))
        for run in got[(k, 1)]:
            for a, b, name in zip(run, got[(k, 0)][0], ("s", "i", "band")):
                assert torch.equal(a, b), (k, name)
    ix.set_option(_lib.OPT_FOLD_KEYS, 1)


@pytest.mark.parametrize("B", [1, 12])
def test_rescore_grid_equals_default(dev, B):
    """CBV2_OPT_RESCORE_GRID: fewer workgroups per row grid-stride over the
    row's pairs (band, top-k rescoring, forced overflow fallback, rerank): the
    same bits as the automatic grid."""
    docs, doclens, Q = make_case(77 + B, 5000, B, 32)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=2)
    Qd = Q.to(dev)
    cand = torch.randint(0, 5002, (B, 50), generator=torch.Generator().manual_seed(B), dtype=torch.int32).to(dev)
    got = {}
    for grid in (0, 7, 64):
        ix.set_option(_lib.OPT_RESCORE_GRID, grid)
        s, i = ix.search(Qd, 100)
        band = ix.last_band.clone()
        sc, si = ix._search_f32(Qd.contiguous(), B, 32, 100, cap=100)     # forces the fallback
        rs, ri, rp = ix.rerank(Qd, cand, 10)
        got[grid] = [x.clone() for x in (s, i, band, sc, si, rs, ri, rp)]
    ix.set_option(_lib.OPT_RESCORE_GRID, 0)
    for grid in (7, 64):
        for a, b, name in zip(got[grid], got[0], ("s", "i", "band", "sc", "si", "rs", "ri", "rp")):
            assert torch.equal(a, b), (grid, name)
