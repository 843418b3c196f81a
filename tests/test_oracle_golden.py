"""CPU: the oracle against the reference's golden vectors (tests/golden/).

These pin the oracle BEFORE it is trusted as the checker of the HIP path.
"""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle as orc


def test_meanpool_cosine_matches_reference():
    """oracle.meanpool_cosine == the reference's _maxsim_score (LRC:802-831) outputs."""
    z = np.load(os.path.join(GOLDEN, "literal_maxsim.npz"))
    for case in "abc":
        got = orc.meanpool_cosine(z[f"{case}_q"], z[f"{case}_docs"])[0]
        np.testing.assert_allclose(got, z[f"{case}_scores"], atol=2e-6, rtol=0)


def test_maxsim_single_token_ranking_equals_reference():
    """At one unit-norm doc token the reference's literal ranking IS MaxSim's."""
    z = np.load(os.path.join(GOLDEN, "single_token.npz"))
    s = orc.maxsim(z["q"], z["docs"])
    _, ids = orc.topk(s, 25)
    assert np.array_equal(ids[0], z["ref_ids"])
    # and the scores are the reference's cosine times Lq * |mean q|
    scale = z["q"].shape[0] * np.linalg.norm(z["q"].astype(np.float64).mean(0))
    np.testing.assert_allclose(s[0, ids[0]] / scale, z["ref_scores"], atol=1e-6)


def test_exact_grid_known_answers():
    z = np.load(os.path.join(GOLDEN, "exact_grid.npz"))
    q = z["q_num"].astype(np.float64) / 16
    d = z["docs_num"].astype(np.float64) / 16
    s = orc.maxsim(q, d, z["doclens"])
    assert np.array_equal(s, z["scores"])
    _, ids = orc.topk(s, s.shape[1])
    assert np.array_equal(ids, z["order"])
    # the fixture really exercises the tie rule
    assert any(len(np.unique(z["scores"][b])) < z["scores"].shape[1] for b in range(len(q)))


def test_exact_grid_fp32_order_independent():
    """k/16 grid: fp32 sums are exact in any order (why GPU == oracle bit-exactly)."""
    z = np.load(os.path.join(GOLDEN, "exact_grid.npz"))
    q = z["q_num"].astype(np.float32) / 16
    d = z["docs_num"].astype(np.float32) / 16
    s32 = orc.maxsim(q, d, z["doclens"], dtype=np.float32)
    assert np.array_equal(s32.astype(np.float64), z["scores"])
    perm = np.random.default_rng(0).permutation(128)
    s32p = orc.maxsim(q[..., perm], d[..., perm], z["doclens"], dtype=np.float32)
    assert np.array_equal(s32p, s32)


def test_rrf_matches_reference_ties():
    for case in json.load(open(os.path.join(GOLDEN, "rrf_ties.json"))):
        got = orc.rrf(case["bm25"], case["colbert"])
        assert got == [(f["chunk_id"], f["rrf_score"]) for f in case["fused"]]


def test_c_oracle_matches_numpy_oracle():
    try:
        orc.c_lib()
    except RuntimeError:
        pytest.skip("C oracle not built (make -C oracle)")
    rng = np.random.default_rng(0)
    q = rng.standard_normal((3, 32, 128)).astype(np.float32)
    d = rng.standard_normal((40, 128, 128)).astype(np.float32)
    dl = rng.integers(0, 129, size=40).astype(np.int32)
    qb, db = orc.to_bf16_bits(q), orc.to_bf16_bits(d)
    c = orc.c_maxsim_bf16(qb, db, dl)
    n = orc.maxsim(orc.from_bf16_bits(qb), orc.from_bf16_bits(db), dl)
    assert np.isneginf(c[:, dl == 0]).all()
    fin = np.isfinite(n)
    np.testing.assert_allclose(c[fin], n[fin], atol=1e-9, rtol=0)
    ties = rng.integers(-3, 4, size=500).astype(np.float64)
    assert np.array_equal(orc.c_topk(ties, 37), orc.topk(ties[None], 37)[1][0])


def test_bf16_rounding_matches_torch():
    import torch
    x = np.random.default_rng(1).standard_normal(10000).astype(np.float32) * 10
    ref = torch.from_numpy(x).bfloat16().float().numpy()
    assert np.array_equal(orc.bf16_round(x), ref)


def test_merge_and_topk_oracle_consistent():
    rng = np.random.default_rng(2)
    s = rng.integers(-10, 10, size=(2, 1000)).astype(np.float64)
    full_s, full_i = orc.topk(s, 50)
    parts = [orc.topk(s[:, a:b], 50, id_base=a) for a, b in [(0, 300), (300, 301), (301, 1000)]]
    ms, mi = orc.merge_topk(np.stack([p[0] for p in parts]), np.stack([p[1] for p in parts]), 50)
    assert np.array_equal(mi, full_i) and np.array_equal(ms, full_s)
