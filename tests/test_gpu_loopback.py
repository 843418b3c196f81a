"""GPU: the in-ABI sharded exchange (csrc/sharded.cpp: cbv2_search_sharded_local
/ _exchange, cbv2_rerank_sharded) at G = 2, 4, 8 on ONE GPU.

Each simulated rank holds a real shard (a ColbertIndex over docs [a, b) with
id_base = a) and its own doc-sharded BM25 (global statistics), and is driven
by its own host thread and HIP stream through the test-only loopback
communicator (cbv2_comm_loopback_init: all-gather = device copies of the G
send blocks, all-reduce(MAX) = a max kernel), so the packed
[scores | ids | bm25 scores | bm25 ids] blocks, the strided merges and the
rerank all-reduce run exactly as on G GPUs.  Done = every rank's results are
bit-equal to the unsharded search, rerank and BM25 top-k (SURVEY.md §8(e);
the seam is LRC:844).  Shards smaller than k pad with -inf / -1.
"""
import threading

import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
from hybrid_rag_colbertv2_amd.distributed import NativeExchange, loopback_comms
from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
from hybrid_rag_colbertv2_amd.index import ColbertIndex

pytestmark = pytest.mark.gpu


def _ranges(N, G, small):
    """Shard 0 gets ``small`` docs (fewer than k), the rest split evenly."""
    cuts = [0, small] + [small + (N - small) * (g + 1) // (G - 1) for g in range(G - 1)]
    return list(zip(cuts[:-1], cuts[1:]))


def _run_ranks(G, fn):
    out, errs = [None] * G, []

    def body(r):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                out[r] = fn(r)
            s.synchronize()
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            errs.append((r, e))

    ts = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a rank thread hung"
    if errs:
        raise errs[0][1]
    return out


@pytest.mark.parametrize("G,B,fp8", [(2, 12, False), (4, 5, False), (8, 12, False), (4, 12, True), (8, 3, True)])
def test_native_exchange_loopback_equals_unsharded(dev, G, B, fp8):
    N, k, kb, C, kf = 6000, 100, 100, 50, 10
    Qf = synth.make_queries(B, seed=21 + G)
    planted = synth.planted_ids(B, N, 10, seed=G)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev)
    doclens[::13] = torch.randint(0, 129, (len(doclens[::13]),), device=dev, dtype=torch.int32)
    doclens[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128     # planted docs keep their query copies
    mk = (lambda t, d, base: ColbertIndex.mxfp8(t, d, id_base=base)) if fp8 else \
        (lambda t, d, base: ColbertIndex(t, d, id_base=base))
    full = mk(tokens, doclens, 0)
    ranges = _ranges(N, G, small=40)
    shards = [mk(tokens[a:b].contiguous(), doclens[a:b].contiguous(), a) for a, b in ranges]
    Q = Qf.to(dev, torch.bfloat16)

    terms, off, V = synth.bm25_shard(0, N, planted)
    df = NativeBM25.doc_freq(terms, off, V)
    stats = (N, int(off[-1]), df)
    lex_full = NativeBM25(terms, off, V)
    lex = [NativeBM25(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a, stats=stats) for a, b in ranges]
    qt, qo = synth.bm25_queries(B)

    comms = loopback_comms(G)
    nxs = [NativeExchange(shards[r], comm=comms[r]) for r in range(G)]
    assert [nx.world for nx in nxs] == [G] * G and [nx.rank for nx in nxs] == list(range(G))

    es, ei = full.search(Q, k)
    cand = ei[:, :C].clone()
    cand[:, -1] = -1                                   # a padding candidate scores -inf on every shard
    cand[0, 3] = N + 5                                 # an id no shard owns
    cand = cand.contiguous()

    def rank(r):
        s, i, li, pool = nxs[r].search(Q, k, lexical=lambda: lex[r].search(qt, qo, kb), return_pool=True)
        s2, i2, _ = nxs[r].search(Q, 7)                # a second exchange without stage-1 lists
        rr = nxs[r].rerank(Q, cand, kf)                # candidates from elsewhere: the all-reduce form
        # stage 3 of the fused lists: scores from the first exchange's pool, no collective
        fused = torch.from_numpy(rrf_fuse(li.cpu().numpy(), i.cpu().numpy(), rrf_k=60, C=C)).to(dev)
        miss = torch.zeros(1, dtype=torch.int32, device=dev)
        c0 = nxs[r].comm_stats()
        pr = nxs[r].rerank(Q, fused, kf, pool=pool, misses=miss)
        c1 = nxs[r].comm_stats()
        return [x.cpu() for x in (s, i, li, s2, i2, *rr, *pr, miss)] + [(c1[0] - c0[0], c1[1] - c0[1])]

    outs = _run_ranks(G, rank)
    torch.cuda.synchronize()
    bi, _ = lex_full.search(qt, qo, kb)
    ers, eri, erp = full.rerank(Q, cand, kf)
    e7s, e7i = full.search(Q, 7)
    pws, pwi, pwp = (x.cpu() for x in full.rerank(Q, torch.from_numpy(rrf_fuse(bi, ei.cpu().numpy(), rrf_k=60,
                                                                                  C=C)).to(dev), kf))
    for r, (s, i, li, s2, i2, rs, ri, rp, ps, pi, pp, miss, dc) in enumerate(outs):
        assert torch.equal(i, ei.cpu()), f"rank {r}: ids differ from the unsharded search"
        assert torch.equal(s, es.cpu()), f"rank {r}: scores differ from the unsharded search"
        assert np.array_equal(li.numpy(), bi), f"rank {r}: merged BM25 lists differ from the unsharded BM25"
        assert torch.equal(i2, e7i.cpu()) and torch.equal(s2, e7s.cpu())
        assert torch.equal(ri, eri.cpu()) and torch.equal(rp, erp.cpu()) and torch.equal(rs, ers.cpu())
        assert torch.equal(pi, pwi) and torch.equal(pp, pwp) and torch.equal(ps, pws), \
            f"rank {r}: the prescored stage 3 differs from the unsharded rerank"
        assert int(miss) == 0 and dc == (0, 0), f"rank {r}: misses {int(miss)}, collectives {dc}"
    # the planted docs are the global top-10 whatever shard holds them
    for b in range(B):
        assert set(outs[0][1][b, :10].tolist()) == set(planted[b].tolist())
    del nxs


def test_loopback_shard_smaller_than_k_pads(dev):
    """G=2 with a 3-doc shard and k=8 > every shard's size on one side:
    the merged list is the unsharded top-8 and slots past n hold -inf / -1."""
    g = torch.Generator().manual_seed(3)
    N = 5
    docs = torch.randn(N, 128, 128, generator=g).bfloat16().to(dev)
    lens = torch.tensor([128, 0, 17, 128, 64], dtype=torch.int32, device=dev)
    Q = torch.randn(2, 32, 128, generator=g).bfloat16().to(dev)
    full = ColbertIndex(docs, lens)
    comms = loopback_comms(2)
    nxs = [NativeExchange(ColbertIndex(docs[a:b].contiguous(), lens[a:b].contiguous(), id_base=a), comm=comms[r])
           for r, (a, b) in enumerate([(0, 3), (3, 5)])]
    outs = _run_ranks(2, lambda r: [x.cpu() for x in nxs[r].search(Q, 8)[:2]])
    es, ei = full.search(Q, 8)
    for s, i in outs:
        assert torch.equal(s, es.cpu()) and torch.equal(i, ei.cpu())
        assert (i[:, N:] == -1).all() and torch.isinf(s[:, N:]).all()   # slots past n: -inf / -1
    del nxs


@pytest.mark.parametrize("G,B", [(2, 1), (4, 5), (8, 12)])
def test_native_exchange_loopback_faithful_equals_unsharded(dev, G, B):
    """fp32-faithful shards through the in-ABI exchange: the local call runs the
    faithful search against the GLOBAL k-th bound (one more all-gather of the
    bf16 top-k's faithful scores inside cbv2_search_sharded_local), the rerank
    scores the owned candidates faithfully.  Every rank equals the unsharded
    faithful search, rerank and BM25 lists bit for bit -- with a shard smaller
    than k, ragged docs, and exact ties: copies of planted docs placed N/2 ids
    away (another shard at G >= 4) score exactly like their originals, so the
    (score desc, id asc) rule decides between them.  B = 1 / 5 take the pair-by-pair band, B = 12 the
    doc-major one."""
    N, k, kb, C, kf = 6000, 100, 100, 50, 10
    Qf = synth.make_queries(B, seed=71 + G)
    planted = synth.planted_ids(B, N, 10, seed=70 + G)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, dtype=torch.float32)
    doclens[::13] = torch.randint(0, 129, (len(doclens[::13]),), device=dev, dtype=torch.int32)
    doclens[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128
    ranges = _ranges(N, G, small=40)
    # ties: the first planted doc of every query copied to an id in another shard
    src = torch.from_numpy(planted[:, 0].copy()).to(dev)
    dst = (src + N // 2) % N
    keep = ~torch.isin(dst, torch.from_numpy(planted.reshape(-1)).to(dev))
    tokens[dst[keep]] = tokens[src[keep]]
    doclens[dst[keep]] = doclens[src[keep]]
    full = ColbertIndex.faithful_f32(tokens, doclens)
    shards = [ColbertIndex.faithful_f32(tokens[a:b].contiguous(), doclens[a:b].contiguous(), id_base=a)
              for a, b in ranges]
    Q = Qf.to(dev)

    terms, off, V = synth.bm25_shard(0, N, planted)
    df = NativeBM25.doc_freq(terms, off, V)
    stats = (N, int(off[-1]), df)
    lex_full = NativeBM25(terms, off, V)
    lex = [NativeBM25(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a, stats=stats) for a, b in ranges]
    qt, qo = synth.bm25_queries(B)

    comms = loopback_comms(G)
    nxs = [NativeExchange(shards[r], comm=comms[r]) for r in range(G)]
    es, ei = full.search(Q, k)
    cand = ei[:, :C].clone()
    cand[:, -1] = -1
    cand = cand.contiguous()

    def rank(r):
        s, i, li, pool = nxs[r].search(Q, k, lexical=lambda: lex[r].search(qt, qo, kb), return_pool=True)
        rr = nxs[r].rerank(Q, cand, kf)
        fused = torch.from_numpy(rrf_fuse(li.cpu().numpy(), i.cpu().numpy(), rrf_k=60, C=C)).to(dev)
        miss = torch.zeros(1, dtype=torch.int32, device=dev)
        pr = nxs[r].rerank(Q, fused, kf, pool=pool, misses=miss)   # faithful prescores, no collective
        return [x.cpu() for x in (s, i, li, *rr, *pr, miss)]

    outs = _run_ranks(G, rank)
    torch.cuda.synchronize()
    bi, _ = lex_full.search(qt, qo, kb)
    ers, eri, erp = full.rerank(Q, cand, kf)
    pws, pwi, pwp = (x.cpu() for x in full.rerank(Q, torch.from_numpy(rrf_fuse(bi, ei.cpu().numpy(), rrf_k=60,
                                                                                  C=C)).to(dev), kf))
    for r, (s, i, li, rs, ri, rp, ps, pi, pp, miss) in enumerate(outs):
        assert torch.equal(i, ei.cpu()), f"rank {r}: ids differ from the unsharded faithful search"
        assert torch.equal(s, es.cpu()), f"rank {r}: scores differ from the unsharded faithful search"
        assert np.array_equal(li.numpy(), bi)
        assert torch.equal(ri, eri.cpu()) and torch.equal(rp, erp.cpu()) and torch.equal(rs, ers.cpu())
        assert torch.equal(pi, pwi) and torch.equal(pp, pwp) and torch.equal(ps, pws), \
            f"rank {r}: the faithful prescored stage 3 differs from the unsharded rerank"
        assert int(miss) == 0
    tied = 0
    for b in range(B):
        row = outs[0][0][b]
        tied += int((row[1:] == row[:-1]).sum())
        assert set(planted[b].tolist()) <= set(outs[0][1][b, :20].tolist())
    assert tied >= 1, "the copies must produce exact ties in the merged lists"
    del nxs
