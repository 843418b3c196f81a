"""GPU: the MXFP8 path (config 5) — device quantizer, fp8 scan / search /
rerank — against the oracle computed on the SAME dequantized values.

Tolerance: the block-scaled fp8 MFMA does not accumulate its 128 products in
exact fp32 (tools/probes/mx_probe3.hip measured ~3e-5 relative to the largest
term), so fp8 scores are compared at 2e-3 absolute (scores are sums of 32
dot products of unit-norm tokens, |S| <= 32); bf16 keeps 1e-3.
"""
import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd.index import ColbertIndex, quantize_mxfp8
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ATOL8 = 2e-3


def _case(seed, N, B, lq=32, ragged=True):
    g = torch.Generator().manual_seed(seed)
    d = torch.randn(N, 128, 128, generator=g)
    d = d / d.norm(dim=-1, keepdim=True)
    q = torch.randn(B, lq, 128, generator=g)
    q = q / q.norm(dim=-1, keepdim=True)
    dl = torch.randint(1, 129, (N,), generator=g, dtype=torch.int32) if ragged else torch.full((N,), 128, dtype=torch.int32)
    return d.bfloat16(), dl, q.bfloat16()


def _deq(q, s):
    return orc.mxfp8_dequant(q.cpu().numpy(), s.cpu().numpy())


def test_quantizer_matches_oracle(dev):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(3000, 128, generator=g) * torch.exp(torch.randn(3000, 1, generator=g) * 3)
    x[0] = 0.0
    x[1, :64] = 0.0
    x[2] = 448.0
    for t in (x, x.bfloat16()):
        q, s = quantize_mxfp8(t.to(dev))
        eq, es = orc.mxfp8_quantize(t.float().numpy())
        assert np.array_equal(s.cpu().numpy(), es)
        qb = q.cpu().numpy()
        assert np.array_equal(qb, eq), np.argwhere(qb != eq)[:5]
        back = orc.mxfp8_dequant(qb, es)
        rel = np.abs(back - t.float().numpy()) / np.maximum(np.abs(t.float().numpy()), 1e-30)
        assert (rel[np.abs(t.float().numpy()) > 2.0 ** -6 * np.exp2(es.repeat(64, -1).astype(float) - 127)] <= 2 ** -4 + 1e-9).all()


def test_quantizer_rounding_boundaries_match_oracle(dev):
    """Byte-exact at the quantizer's boundaries: block maxima exactly at powers
    of two and at the e4m3 top (the E8M0 scale choice), elements at exact
    midpoints between neighbouring e4m3 codes under the block's scale (ties
    to even), in the e4m3 subnormal range, signed zeros, fp32 subnormals and
    values near the fp32 top -- f32 and bf16 inputs."""
    rng = np.random.default_rng(23)
    rows = []
    e4 = torch.arange(0, 127, dtype=torch.uint8).view(torch.float8_e4m3fn).float().numpy()   # e4m3 grid, >= 0
    mids = (e4[1:] + e4[:-1]) / 2                                        # exact midpoints
    for r in range(600):
        E = int(rng.integers(-20, 21))
        top = float(rng.choice([1.0, 1.5, 1.75, 1.875, 448.0 / 256.0])) * 2.0 ** E
        row = np.zeros(128, np.float32)
        for half in (0, 64):
            scale = 2.0 ** (E - 8)
            pick = rng.integers(0, len(mids), 64)
            v = np.where(rng.random(64) < 0.5, mids[pick], e4[pick]) * scale
            v *= np.where(rng.random(64) < 0.5, -1.0, 1.0)
            v[0] = top * (1 if r % 2 else -1)
            v[rng.random(64) < 0.05] = -0.0
            row[half:half + 64] = v
        rows.append(row)
    x = np.stack(rows).astype(np.float32)
    x[0, :5] = [1e-40, -1e-40, 3e38, -3e38, 1e-45]                       # fp32 subnormals, near the top
    x[1, 64:] = 2.0 ** -140
    for t in (torch.from_numpy(x), torch.from_numpy(x).bfloat16()):
        q, sc = quantize_mxfp8(t.to(dev))
        eq, es = orc.mxfp8_quantize(t.float().numpy())
        assert np.array_equal(sc.cpu().numpy(), es), np.argwhere(sc.cpu().numpy() != es)[:5]
        qb = q.cpu().numpy()
        assert np.array_equal(qb, eq), (t.dtype, np.argwhere(qb != eq)[:5])


@pytest.mark.parametrize("N,B,lq,ragged", [(300, 3, 32, True), (2000, 70, 32, True), (513, 1, 20, False),
                                           (1500, 9, 32, True)])
def test_fp8_score_matches_oracle(dev, N, B, lq, ragged):
    d, dl, q = _case(N + B, N, B, lq, ragged)
    ix = ColbertIndex.mxfp8(d.to(dev), dl.to(dev))
    got = ix.score(q.to(dev)).cpu().numpy()
    qq, qs = quantize_mxfp8(q.to(dev))
    ref = orc.maxsim(_deq(qq, qs), _deq(ix.tokens, ix.scales), dl.numpy())
    fin = np.isfinite(ref)
    assert (np.isneginf(got) == np.isneginf(ref)).all()
    np.testing.assert_allclose(got[fin], ref[fin], atol=ATOL8, rtol=0)


def test_fp8_paths_bit_identical(dev):
    """direct (B<=8), LDS (B>8) and rerank scores of the fp8 path: same bits."""
    d, dl, q = _case(5, 1200, 20)
    ix = ColbertIndex.mxfp8(d.to(dev), dl.to(dev))
    full = ix.score(q.to(dev))
    for lo, hi in [(0, 1), (2, 5), (8, 16)]:
        assert torch.equal(ix.score(q[lo:hi].to(dev)), full[lo:hi])
    cand = torch.randint(0, 1200, (20, 50), device=dev, dtype=torch.int32)
    raw = ix.rerank(q.to(dev), cand, 0)
    assert torch.equal(raw, torch.gather(full, 1, cand.long()))


def test_fp8_search_planted(dev):
    from hybrid_rag_colbertv2_amd import synth
    B, N = 70, 30000
    Qf = synth.make_queries(B)
    planted = synth.planted_ids(B, N, 10)
    tok, dl = synth.make_shard(0, N, Qf, planted, dev)
    ix = ColbertIndex.mxfp8(tok, dl)
    s, i = ix.search(Qf.to(dev), k=10)
    hits = np.mean([set(i[b].tolist()) == set(planted[b].tolist()) for b in range(B)])
    assert hits == 1.0
    assert ix.tokens.numel() == tok.numel() and ix.tokens.element_size() * 2 == tok.element_size()


def test_quantizer_beyond_32bit_work_items(dev):
    """70M rows: the launch would exceed 2^32 work-items without the grid-stride loop."""
    rows = 70_000_000
    x = torch.ones(rows, 128, dtype=torch.bfloat16, device=dev)
    x[-1] *= 3.0
    q, s = quantize_mxfp8(x)
    assert int(s[0, 0]) == 119 and int(q[0, 0]) == 0x78            # 1.0 -> 256 * 2^-8
    assert int(s[-1, 1]) == 120 and int(q[-1, 127]) == 0x7C         # 3.0 -> 384 * 2^-7
    back = orc.mxfp8_dequant(q[-2:].cpu().numpy(), s[-2:].cpu().numpy())
    assert np.array_equal(back, np.array([[1.0] * 128, [3.0] * 128]))
    del x, q, s
