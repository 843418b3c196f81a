"""GPU: the one-round-trip retrieve (csrc/retrieve.cpp: cbv2_retrieve_begin /
_finish, hybrid.OneTripRetriever) against the same stages called one by one
(search -> host RRF + [:C] -> rerank; LRC:894-935, 960-978, 916).

Done = scores, ids and positions equal bit for bit, for bf16, MXFP8 and
fp32-faithful shards, B = 1 / 5 / 40, with a BM25 callable, a host id array
and no stage 1; and at G = 2 / 4 / 8 through the test-only loopback
communicator, bf16, MXFP8 and fp32-faithful shards (every rank equals the
unsharded composed path).  The host results (``host=True``,
cbv2_retrieve_finish_host) equal the device ones, and one-shard bf16 /
faithful calls read them from the final select's host words (counted by
cbv2_retrieve_pool_stats [2])."""
import ctypes
import threading

import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import _lib, synth
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
from hybrid_rag_colbertv2_amd.distributed import NativeExchange, loopback_comms
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse
from hybrid_rag_colbertv2_amd.index import ColbertIndex

pytestmark = pytest.mark.gpu

K, KB, C, KF = 100, 100, 50, 10


def _corpus(dev, N, B, seed, dtype=torch.bfloat16):
    Qf = synth.make_queries(B, seed=seed)
    planted = synth.planted_ids(B, N, 10, seed=seed + 1)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, dtype=dtype)
    doclens[::11] = torch.randint(0, 129, (len(doclens[::11]),), device=dev, dtype=torch.int32)
    doclens[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128
    terms, off, V = synth.bm25_shard(0, N, planted)
    return Qf, planted, tokens, doclens, (terms, off, V)


def _composed(index, Q, lex_ids):
    """The stages one by one, as bench.step does."""
    _, ids = index.search(Q, K)
    bm = np.zeros((ids.shape[0], 0), np.int32) if lex_ids is None else lex_ids
    cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=60, C=C)
    return index.rerank(Q, torch.from_numpy(cand).to(index.device), KF)


def _final_words_calls():
    """finish_host calls served from host words: the final select's (GPU
    rerank) or the host rerank's."""
    st = (ctypes.c_int64 * 4)()
    _lib.lib().cbv2_retrieve_pool_stats(st, 4)
    return int(st[2]) + int(st[3])


def _host_rerank_calls():
    st = (ctypes.c_int64 * 4)()
    _lib.lib().cbv2_retrieve_pool_stats(st, 4)
    return int(st[3])


@pytest.mark.parametrize("kind", ["bf16", "fp8", "fp32"])
@pytest.mark.parametrize("B", [1, 5, 40])
def test_one_trip_equals_composed(dev, kind, B):
    N = 7000
    Qf, planted, tokens, doclens, (terms, off, V) = _corpus(
        dev, N, B, seed=31 + B, dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
    if kind == "fp32":
        ix, Q = ColbertIndex.faithful_f32(tokens, doclens), Qf.to(dev)
    elif kind == "fp8":
        ix, Q = ColbertIndex.mxfp8(tokens, doclens), Qf.to(dev, torch.bfloat16)
    else:
        ix, Q = ColbertIndex(tokens, doclens), Qf.to(dev, torch.bfloat16)
    lex = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(B)
    bm_i, bm_s = lex.search(qt, qo, KB)
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    for lexical, lex_ids in ((lambda: (bm_i, bm_s), bm_i), (bm_i, bm_i), (None, None)):
        h0 = _host_rerank_calls()
        got = [x.cpu() for x in one(Q, lexical)]
        if kind == "fp32" and B <= 8:      # the host rerank (stage 2's scores + stage 1's prescore)
            assert _host_rerank_calls() == h0 + 1, f"{kind} B={B}: not the host rerank"
        want = [x.cpu() for x in _composed(ix, Q, lex_ids)]
        for g, w, name in zip(got, want, ("scores", "ids", "positions")):
            assert torch.equal(g, w), f"{kind} B={B}: {name} differ from the composed stages"
        n0 = _final_words_calls()
        goth = one(Q, lexical, host=True)
        for g, w, name in zip(goth, want, ("scores", "ids", "positions")):
            assert isinstance(g, np.ndarray) and np.array_equal(g, w.numpy()), f"{kind} B={B}: host {name} differ"
        if kind == "fp32" or (kind == "bf16" and B <= 32):   # from the final select's host words
            assert _final_words_calls() == n0 + 1, f"{kind} B={B}: host results were copied, not mirrored"
    for b in range(B):                     # the planted docs win stage 3
        assert set(got[1][b].tolist()) == set(planted[b].tolist())


@pytest.mark.parametrize("kind", ["bf16", "fp32"])
def test_begin_probe_marks_and_results(dev, kind):
    """The latency lab's begin probe (tools/launch_latency.py): with it on,
    begin stamps entry <= search returned <= ready flags seen (the faithful
    search's split kernel always publishes them; a small bf16 shard's scan
    path may publish none: 0) and the results equal the probe-off call's;
    off again, begin stamps nothing."""
    L = _lib.lib()
    L.cbv2_set_begin_probe.argtypes = [ctypes.c_int32]
    L.cbv2_set_begin_probe.restype = None
    L.cbv2_retrieve_begin_marks.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    N, B = 5000, 1
    Qf, _, tokens, doclens, (terms, off, V) = _corpus(dev, N, B, seed=77,
                                                      dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
    ix = ColbertIndex.faithful_f32(tokens, doclens) if kind == "fp32" else ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.float32 if kind == "fp32" else torch.bfloat16)
    lex = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(B)
    bm = lambda: lex.search(qt, qo, KB)   # noqa: E731
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    want = one(Q, bm, host=True)
    marks = (ctypes.c_int64 * 3)()
    L.cbv2_set_begin_probe(1)
    try:
        got = one(Q, bm, host=True)
        assert L.cbv2_retrieve_begin_marks(marks, 3) == 0
    finally:
        L.cbv2_set_begin_probe(0)
    assert all(np.array_equal(g, w) for g, w in zip(got, want))
    assert 0 < marks[0] <= marks[1], list(marks)
    assert marks[1] <= marks[2] or (kind == "bf16" and marks[2] == 0), list(marks)
    one(Q, bm, host=True)
    again = (ctypes.c_int64 * 3)()
    L.cbv2_retrieve_begin_marks(again, 3)
    assert list(again) == list(marks)          # probe off: begin left the last probe's marks alone


def test_one_trip_long_queries_and_bad_input(dev):
    N = 300
    Qf, _, tokens, doclens, _ = _corpus(dev, N, 2, seed=5)
    ix = ColbertIndex(tokens, doclens)
    one = OneTripRetriever(ix)
    Ql = torch.randn(2, 40, 128, device=dev).to(torch.bfloat16)    # 40 query tokens: the stages by blocks
    got, want = one(Ql), _composed(ix, Ql, None)
    assert all(torch.equal(g, w) for g, w in zip(got, want))
    with pytest.raises(ValueError):                         # stage-1 rows != B
        one(Qf.to(dev, torch.bfloat16), lambda: (np.zeros((3, 5), np.int32), np.zeros((3, 5), np.float32)))


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


@pytest.mark.parametrize("G,B,kind,kb_ret", [(2, 1, "bf16", KB), (4, 9, "bf16", KB), (4, 6, "fp8", KB),
                                             (2, 3, "bf16", 60), (2, 1, "fp32", KB), (4, 5, "fp32", 60),
                                             (8, 12, "fp32", KB)])
def test_one_trip_sharded_loopback_equals_unsharded(dev, G, B, kind, kb_ret):
    """kb_ret < KB: the stage-1 callable returns fewer columns than begin's
    kb (an upper bound, include/colbert_mi355x.h), so finish lays out its
    workspace for a smaller kb than begin did.  fp32: faithful shards over the
    native exchange (the global k-th bound inside the local call)."""
    N = 6000
    Qf, planted, tokens, doclens, (terms, off, V) = _corpus(
        dev, N, B, seed=50 + G, dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
    mk = {"fp8": lambda t, d, base: ColbertIndex.mxfp8(t, d, id_base=base),
          "fp32": lambda t, d, base: ColbertIndex.faithful_f32(t, d, id_base=base),
          "bf16": lambda t, d, base: ColbertIndex(t, d, id_base=base)}[kind]
    full = mk(tokens, doclens, 0)
    cuts = [0, 40] + [40 + (N - 40) * (g + 1) // (G - 1) for g in range(G - 1)]   # shard 0 < k docs
    ranges = list(zip(cuts[:-1], cuts[1:]))
    shards = [mk(tokens[a:b].contiguous(), doclens[a:b].contiguous(), a) for a, b in ranges]
    Q = Qf.to(dev) if kind == "fp32" else Qf.to(dev, torch.bfloat16)
    df = NativeBM25.doc_freq(terms, off, V)
    stats = (N, int(off[-1]), df)
    lex_full = NativeBM25(terms, off, V)
    lex = [NativeBM25(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a, stats=stats) for a, b in ranges]
    qt, qo = synth.bm25_queries(B)
    comms = loopback_comms(G)
    ones = [OneTripRetriever(NativeExchange(shards[r], comm=comms[r]), colbert_k=K, fused=C, final_k=KF)
            for r in range(G)]
    c0 = [o._owner.comm_stats() for o in ones]
    outs = _run_ranks(G, lambda r: [x.cpu() for x in ones[r](Q, lambda: lex[r].search(qt, qo, kb_ret))])
    hosts = _run_ranks(G, lambda r: ones[r](Q, lambda: lex[r].search(qt, qo, kb_ret), host=True))
    torch.cuda.synchronize()
    # collectives per call: the stage-2 all-gather (+ the faithful band bound's),
    # and NO stage-3 all-reduce (the fused candidates' scores ride the all-gather)
    for r, o in enumerate(ones):
        g1, a1 = o._owner.comm_stats()
        assert (g1 - c0[r][0], a1 - c0[r][1]) == (2 * (2 if kind == "fp32" else 1), 0), \
            f"rank {r}: {(g1 - c0[r][0], a1 - c0[r][1])} collectives (all-gather, all-reduce) for two calls"
    bi, _ = lex_full.search(qt, qo, kb_ret)
    want = [x.cpu() for x in _composed(full, Q, bi)]
    for r, got in enumerate(outs):
        for g, w, name in zip(got, want, ("scores", "ids", "positions")):
            assert torch.equal(g, w), f"rank {r}: {name} differ from the unsharded composed stages"
        for g, w, name in zip(hosts[r], want, ("scores", "ids", "positions")):
            assert np.array_equal(g, w.numpy()), f"rank {r}: host {name} differ"
    for b in range(B):
        assert set(outs[0][1][b].tolist()) == set(planted[b].tolist())
    del ones
