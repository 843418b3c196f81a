"""GPU: every bounded in-kernel wait of the latency path fails loudly or
falls back exactly -- never a silent wrong result (errors are
negative codes + cbv2_last_error).

The waits, each forced once with the lab knob cbv2_set_wait_lab(ticks,
publish_delay_us) -- a 1 ms in-kernel bound and a host that publishes 50 ms
late:
* host_result_kernel (the host rerank's device copy of the final top-k,
  csrc/retrieve.cpp host_rerank): the call returns CBV2_EHIP;
* the pre-armed GPU rerank (rerank_split_kernel bf16, rescore_split_kernel
  fp32-faithful) waiting on the host's fused candidates: CBV2_EHIP;
* phase1_collect_kernel's wait for phase 1 (ticks 0: give up at once): the
  row takes the full faithful scan in the rescoring launch -- the results
  equal the normal run's bit for bit and the row's status reads -2.
After each forced failure the next normal call on the same retriever (the
same pooled mapped buffer) returns the composed stages' results."""
import ctypes

import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import _lib, synth
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse
from hybrid_rag_colbertv2_amd.index import ColbertIndex

pytestmark = pytest.mark.gpu

K, C, KF = 100, 50, 10
TICKS_1MS, DELAY_50MS = 100_000, 50_000


def _set_wait(ticks, delay_us):
    _lib.lib().cbv2_set_wait_lab(ctypes.c_int64(ticks), ctypes.c_int32(delay_us))


def _index(dev, N, B, seed, kind):
    Qf = synth.make_queries(B, seed=seed)
    planted = synth.planted_ids(B, N, 10, seed=seed + 1)
    dt = torch.float32 if kind == "fp32" else torch.bfloat16
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev, dtype=dt)
    ix = ColbertIndex.faithful_f32(tokens, doclens) if kind == "fp32" else ColbertIndex(tokens, doclens)
    return ix, Qf.to(dev, dt).contiguous()


def _want(ix, Q, bm):
    _, ids = ix.search(Q, K)
    cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=60, C=C)
    return [x.cpu() for x in ix.rerank(Q, torch.from_numpy(cand).to(ix.device), KF)]


@pytest.mark.parametrize("kind", ["fp32", "bf16"])
@pytest.mark.parametrize("host_rerank", [1, 0])
def test_forced_wait_timeout_fails_the_call(dev, kind, host_rerank):
    N = 6000 if kind == "fp32" else 70_000
    L = _lib.lib()
    ix, Q4 = _index(dev, N, 4, seed=31, kind=kind)
    Q = Q4[:1].contiguous()
    bm = np.random.default_rng(5).permutation(N)[:K][None].astype(np.int32)
    want = _want(ix, Q, bm)
    one = OneTripRetriever(ix, colbert_k=K, fused=C, final_k=KF)
    st0 = (ctypes.c_int64 * 4)()
    L.cbv2_retrieve_pool_stats(st0, 4)
    L.cbv2_set_host_rerank(host_rerank)
    try:
        for host in (False, True):
            _set_wait(TICKS_1MS, DELAY_50MS)
            try:
                with pytest.raises(_lib.Cbv2Error, match="gave up its wait") as ei:
                    one(Q, bm, host=host)
                    torch.cuda.synchronize()
                assert ei.value.code == _lib.ERR_EHIP
            finally:
                _set_wait(-1, 0)
            torch.cuda.synchronize()
            out = one(Q, bm, host=host)          # the same pooled buffer, normal bounds
            got = [torch.from_numpy(x) for x in out] if host else [x.cpu() for x in out]
            for g, w, name in zip(got, want, ("scores", "ids", "positions")):
                assert torch.equal(g, w), f"{kind} host_rerank={host_rerank} host={host}: {name} after a timeout"
    finally:
        L.cbv2_set_host_rerank(1)
    torch.cuda.synchronize()
    st1 = (ctypes.c_int64 * 4)()
    L.cbv2_retrieve_pool_stats(st1, 4)
    assert int(st1[1]) == int(st1[0]), "a mapped buffer was not returned to its pool"
    if host_rerank:
        assert int(st1[3] - st0[3]) == 2, "the normal calls should take the host rerank"


def test_phase1_wait_timeout_takes_exact_fallback(dev):
    """ticks 0: every band-collect workgroup gives up its wait for phase 1;
    the rows fall back to the full faithful scan (status -2) with the same
    top-k bits as the certified band."""
    N, B = 70_000, 4
    ix, Q = _index(dev, N, B, seed=41, kind="fp32")
    s0, i0 = ix.search(Q, K)
    band0 = ix.last_band.cpu()
    assert (band0 >= K).all(), f"the normal run should certify a band: {band0}"
    _set_wait(0, 0)
    try:
        s1, i1 = ix.search(Q, K)
        band1 = ix.last_band.cpu()
        torch.cuda.synchronize()
    finally:
        _set_wait(-1, 0)
    assert (band1 == -2).all(), f"status after a forced phase-1 timeout: {band1}"
    assert torch.equal(s0.cpu(), s1.cpu()) and torch.equal(i0.cpu(), i1.cpu()), \
        "the full-scan fallback differs from the certified band's top-k"
    s2, i2 = ix.search(Q, K)
    assert torch.equal(ix.last_band.cpu(), band0) and torch.equal(i2.cpu(), i0.cpu())
