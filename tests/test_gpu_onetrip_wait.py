"""GPU: the host side of the one-round-trip retrieve (csrc/retrieve.cpp) --
how cbv2_retrieve_finish waits for stage 2, which device it runs on, where
its host buffers come from, and when the fp32-faithful rerank may reuse
begin's query split (HybridRetriever.retrieve, LRC:894-935).

Done =
* the faithful host rerank is thread-safe (8 threads, host and device
  results, every call the host rerank);
* a B = 256 finish sleeps in its wait: the process CPU time of a whole
  one-trip call (begin + finish, no stage 1) stays <= 5 ms while the GPU
  scans for tens of ms (a polling wait would burn the whole scan);
* the one-shard call's device-mapped host buffers come from a pool: 1,000
  calls on 8 threads (B = 1 and B = 16) create at most 16, every one back in
  the pool at the end;
* the caller's current device is restored after begin / finish, from a
  thread that never selected one (one GPU on the box: the index-on-another-
  device case itself needs a second device);
* a faithful finish whose workspace got another query split between begin
  and finish (a search of other queries in the stage-1 callable) splits Q
  again: its results equal the composed stages on Q bit for bit."""
import ctypes
import threading
import time

import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import _lib, synth
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse
from hybrid_rag_colbertv2_amd.index import ColbertIndex, _stream_ptr

pytestmark = pytest.mark.gpu

K, C, KF = 100, 50, 10


def _index(dev, N, B, seed, dtype=torch.bfloat16):
    Qf = synth.make_queries(B, seed=seed)
    planted = synth.planted_ids(B, N, 10, seed=seed + 1)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, dtype=dtype)
    return Qf, planted, tokens, doclens


def _composed(index, Q):
    _, ids = index.search(Q, K)
    cand = rrf_fuse(np.zeros((ids.shape[0], 0), np.int32), ids.cpu().numpy(), rrf_k=60, C=C)
    return index.rerank(Q, torch.from_numpy(cand).to(index.device), KF)


def test_large_batch_wait_sleeps(dev):
    N, B = 200_000, 256
    Qf, _, tokens, doclens = _index(dev, N, B, seed=3)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    one(Q)
    torch.cuda.synchronize()
    cpu, wall = [], []
    for _ in range(3):
        t0, c0 = time.perf_counter(), time.process_time()
        out = one(Q)
        c1, t1 = time.process_time(), time.perf_counter()
        cpu.append(c1 - c0)
        wall.append(t1 - t0)
    torch.cuda.synchronize()
    assert min(wall) > 0.010, f"the call should wait for a scan of {N} docs x {B} queries (took {min(wall)} s)"
    assert sorted(cpu)[1] <= 0.005, f"a B=256 one-trip call used {cpu} s of CPU over {wall} s of wall time"
    assert out[1].shape == (B, KF)


def test_mapped_buffers_pooled_and_device_restored(dev):
    N = 3000
    L = _lib.lib()
    Qf, _, tokens, doclens = _index(dev, N, 16, seed=9)
    ix = ColbertIndex(tokens, doclens)
    Q1, Q16 = Qf[:1].to(dev, torch.bfloat16).contiguous(), Qf.to(dev, torch.bfloat16)
    want1, want16 = [x.cpu() for x in _composed(ix, Q1)], [x.cpu() for x in _composed(ix, Q16)]
    st0 = (ctypes.c_int64 * 2)()
    L.cbv2_retrieve_pool_stats(st0, 2)
    errs, devs = [], []

    def body(t):
        try:
            one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                for i in range(125):
                    Q, want = (Q1, want1) if (i + t) % 2 else (Q16, want16)
                    got = [x.cpu() for x in one(Q)]
                    if not all(torch.equal(g, w) for g, w in zip(got, want)):
                        raise AssertionError(f"thread {t} call {i}: results differ from the composed stages")
            devs.append(torch.cuda.current_device())
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            errs.append(e)

    ts = [threading.Thread(target=body, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a thread hung"
    if errs:
        raise errs[0]
    torch.cuda.synchronize()
    st1 = (ctypes.c_int64 * 2)()
    L.cbv2_retrieve_pool_stats(st1, 2)
    created = int(st1[0] - st0[0])
    assert created <= 16, f"1,000 calls on 8 threads created {created} mapped buffers"
    assert int(st1[1]) == int(st1[0]), "a mapped buffer was not returned to its pool"
    assert devs == [dev.index or 0] * 8


@pytest.mark.parametrize("kind", ["fp32", "bf16"])
def test_host_rerank_threads(dev, kind):
    """The host rerank (stage 2's scores + the stage-1 prescore, launched on
    each thread's second stream once the host has seen the search's ready
    flags in the call's mapped buffer: the faithful split's, one per row, or
    the bf16 counter zeroing's) under 8 threads x 40 calls, B = 1 and 4, host
    and device results: every call equals the composed stages, and every one
    took the host rerank.  (bf16: 70,000 dense docs -- the block-max select's
    one launch, whose counter zeroing publishes the flag.)  An in-kernel wait
    for the flag on the second stream starved the search here (bf16)."""
    N = 6000 if kind == "fp32" else 70_000
    L = _lib.lib()
    Qf, _, tokens, doclens = _index(dev, N, 4, seed=13, dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
    ix = ColbertIndex.faithful_f32(tokens, doclens) if kind == "fp32" else ColbertIndex(tokens, doclens)
    qdt = torch.float32 if kind == "fp32" else torch.bfloat16
    Q1, Q4 = Qf[:1].to(dev, qdt).contiguous(), Qf.to(dev, qdt).contiguous()
    bm = [np.stack([np.random.default_rng(b + 7 * B).permutation(N)[:K] for b in range(B)]).astype(np.int32)
          for B in (1, 4)]
    want = []
    for Q, bi in ((Q1, bm[0]), (Q4, bm[1])):
        _, ids = ix.search(Q, K)
        cand = rrf_fuse(bi, ids.cpu().numpy(), rrf_k=60, C=C)
        want.append([x.cpu() for x in ix.rerank(Q, torch.from_numpy(cand).to(dev), KF)])
    st0 = (ctypes.c_int64 * 4)()
    L.cbv2_retrieve_pool_stats(st0, 4)
    errs = []

    def body(t):
        try:
            one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
            s = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                for i in range(40):
                    j = (i + t) % 2
                    Q, bi = ((Q1, bm[0]), (Q4, bm[1]))[j]
                    if i % 3 == 0:
                        got = [torch.from_numpy(x) for x in one(Q, bi, host=True)]
                    else:
                        got = [x.cpu() for x in one(Q, bi)]
                    if not all(torch.equal(g, w) for g, w in zip(got, want[j])):
                        raise AssertionError(f"thread {t} call {i}: results differ from the composed stages")
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            errs.append(e)

    ts = [threading.Thread(target=body, args=(t,)) for t in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=240)
    assert not any(t.is_alive() for t in ts), "a thread hung"
    if errs:
        raise errs[0]
    torch.cuda.synchronize()
    st1 = (ctypes.c_int64 * 4)()
    L.cbv2_retrieve_pool_stats(st1, 4)
    assert int(st1[3] - st0[3]) == 8 * 40, "not every call took the host rerank"
    assert int(st1[1]) == int(st1[0]), "a mapped buffer was not returned to its pool"


def test_faithful_finish_resplits_after_foreign_split(dev):
    N, B = 6000, 4
    L = _lib.lib()
    Qf, planted, tokens, doclens = _index(dev, N, B, seed=21, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(tokens, doclens)
    Q = Qf.to(dev).contiguous()
    Q2 = torch.flip(Q, dims=[0]).contiguous() * 0.5          # other queries, same shape
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    want = [x.cpu() for x in _composed(ix, Q)]
    assert all(torch.equal(x.cpu(), w) for x, w in zip(one(Q), want))       # begin's split reused
    ws = one._sized[1][0]
    cap = 16384
    sw = int(L.cbv2_f32_workspace_bytes(ix._h, _lib.F32_SEARCH, B, Q.shape[1], cap))
    s2 = torch.empty((B, K), dtype=torch.float32, device=dev)
    i2 = torch.empty((B, K), dtype=torch.int32, device=dev)
    st2 = torch.empty((B,), dtype=torch.int32, device=dev)

    def foreign():     # stage 1 of this call: another search into the same workspace
        _lib.check(L.cbv2_search_f32(ix._h, Q2.data_ptr(), B, Q2.shape[1], K, cap, ws, sw, s2.data_ptr(),
                                     i2.data_ptr(), st2.data_ptr(), _stream_ptr(dev)))
        return np.full((B, 1), -1, np.int32), np.zeros((B, 1), np.float32)

    got = [x.cpu() for x in one(Q, foreign)]
    want_lex = [x.cpu() for x in _composed(ix, Q)]
    for g, w, name in zip(got, want_lex, ("scores", "ids", "positions")):
        assert torch.equal(g, w), f"{name}: the rerank did not re-split Q after a foreign split"
    for b in range(B):
        assert set(got[1][b].tolist()) == set(planted[b].tolist())


@pytest.mark.parametrize("kind", ["fp32", "bf16"])
def test_host_rerank_late_flag_path(dev, kind):
    """The host rerank's other prescore placement -- behind the search on the
    call's own stream, the path a ready flag not seen within its bound takes
    (lab knob cbv2_set_host_rerank(2) forces it): the same results as the
    composed stages, host and device, and the host rerank counted."""
    N = 6000 if kind == "fp32" else 70_000
    L = _lib.lib()
    Qf, _, tokens, doclens = _index(dev, N, 4, seed=17, dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
    ix = ColbertIndex.faithful_f32(tokens, doclens) if kind == "fp32" else ColbertIndex(tokens, doclens)
    qdt = torch.float32 if kind == "fp32" else torch.bfloat16
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    L.cbv2_set_host_rerank(2)
    try:
        for B in (1, 4):
            Q = Qf[:B].to(dev, qdt).contiguous()
            bi = np.stack([np.random.default_rng(b + 3 * B).permutation(N)[:K] for b in range(B)]).astype(np.int32)
            _, ids = ix.search(Q, K)
            cand = rrf_fuse(bi, ids.cpu().numpy(), rrf_k=60, C=C)
            want = [x.cpu() for x in ix.rerank(Q, torch.from_numpy(cand).to(dev), KF)]
            for host in (False, True):
                st0 = (ctypes.c_int64 * 4)()
                L.cbv2_retrieve_pool_stats(st0, 4)
                out = one(Q, bi, host=host)
                got = [torch.from_numpy(x) for x in out] if host else [x.cpu() for x in out]
                for g, w, name in zip(got, want, ("scores", "ids", "positions")):
                    assert torch.equal(g, w), f"{kind} B={B} host={host}: {name} differ"
                st1 = (ctypes.c_int64 * 4)()
                L.cbv2_retrieve_pool_stats(st1, 4)
                assert int(st1[3]) == int(st0[3]) + 1, f"{kind} B={B}: not the host rerank"
    finally:
        L.cbv2_set_host_rerank(1)
