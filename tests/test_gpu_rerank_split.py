"""GPU: the candidate-parallel rerank (cbv2_rerank_ws: one wave per (query,
candidate) + select_small_kernel, batches <= 32) returns the same scores, ids
and positions, bit for bit, as the one-workgroup-per-query rerank_kernel
(cbv2_rerank), and the raw k == 0 rows equal too -- bf16 and MXFP8, invalid
and out-of-shard ids, duplicates, C = 1 .. 1024 and the C > 1024 fallback
(LRC:779-800: argsort of the candidates' MaxSim scores)."""
import ctypes

import pytest
import torch

from hybrid_rag_colbertv2_amd import _lib, synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex, _stream_ptr

pytestmark = pytest.mark.gpu


def _index(dev, n, fp8, seed):
    Qf = synth.make_queries(40, 32, seed=seed)
    planted = synth.planted_ids(40, n, 10, seed=seed + 1)
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=seed)
    g = torch.Generator(device=dev).manual_seed(seed)
    doclens[torch.randperm(n, generator=g, device=dev)[: n // 7]] = torch.randint(
        0, 129, (n // 7,), generator=g, device=dev, dtype=torch.int32)
    ix = ColbertIndex.mxfp8(tokens, doclens, id_base=100) if fp8 else ColbertIndex(tokens, doclens, id_base=100)
    return ix, Qf.to(dev, torch.bfloat16)


def _one_wg(ix, Q, cand, k):
    """cbv2_rerank (no workspace): the one-workgroup-per-query kernel for k > 0."""
    _keep, qptr, _, B, lq = ix._prep_query(Q, "maxsim")
    C = cand.shape[1]
    out = [torch.empty((B, k), dtype=t, device=ix.device) for t in (torch.float32, torch.int32, torch.int32)]
    _lib.check(_lib.lib().cbv2_rerank(ix._h, qptr, B, lq, cand.data_ptr(), C, k, *(o.data_ptr() for o in out),
                                      _stream_ptr(ix.device)))
    return out


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("B,C,k", [(1, 50, 10), (1, 1, 1), (5, 100, 100), (32, 1024, 37), (33, 50, 10),
                                   (2, 1025, 10), (8, 300, 500)])
def test_split_rerank_equals_one_workgroup(dev, fp8, B, C, k):
    n = 20_000
    ix, Q = _index(dev, n, fp8, seed=3 + B + C)
    g = torch.Generator(device=dev).manual_seed(B * 1000 + C)
    cand = torch.randint(100, 100 + n, (B, C), generator=g, device=dev, dtype=torch.int32)
    cand[:, ::11] = -1                                    # invalid ids score -inf
    cand[:, 3::13] = 100 + n + 7                          # outside this shard
    if C > 4:
        cand[:, 1] = cand[:, 2]                           # a duplicated candidate: tie -> lower position
    Qb = Q[:B].contiguous()
    got = ix.rerank(Qb, cand, k)
    ref = _one_wg(ix, Qb, cand, k)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
    raw = ix.rerank(Qb, cand, 0)                          # k == 0: candidate-parallel when B <= 32
    _keep, qptr, _, _, lq = ix._prep_query(Qb, "maxsim")
    if B <= 32 and C <= 1024:
        full = ix.rerank(Qb, cand, C)[0]                  # every candidate, best first
        assert torch.equal(raw.sort(dim=1, descending=True).values, full)


def test_workspace_bytes_and_short_workspace(dev):
    L = _lib.lib()
    assert int(L.cbv2_rerank_workspace_bytes(1, 50)) >= 200
    assert int(L.cbv2_rerank_workspace_bytes(0, 50)) == 0
    ix, Q = _index(dev, 5000, False, seed=1)
    cand = torch.arange(100, 150, dtype=torch.int32, device=dev).unsqueeze(0)
    _keep, qptr, _, B, lq = ix._prep_query(Q[:1].contiguous(), "maxsim")
    outs = [torch.empty((1, 10), dtype=t, device=dev) for t in (torch.float32, torch.int32, torch.int32)]
    ws = torch.empty(16, dtype=torch.uint8, device=dev)   # too short: the one-workgroup path, same result
    _lib.check(L.cbv2_rerank_ws(ix._h, qptr, 1, lq, cand.data_ptr(), 50, 10, ws.data_ptr(), ws.numel(),
                                *(o.data_ptr() for o in outs), _stream_ptr(ix.device)))
    ref = _one_wg(ix, Q[:1].contiguous(), cand, 10)
    for a, b in zip(outs, ref):
        assert torch.equal(a, b)
