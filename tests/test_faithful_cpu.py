"""CPU: the fp32-faithful index's arithmetic (oracle restatement, no GPU).

The reference keeps fp32 embeddings (local_rag_complete.py:735-746) and scores
them in fp32 (:802-831).  The faithful search scans hi = bf16(x) with bf16(q)
(score T), then rescores every doc with T >= lb - beta(q) (lb: the minimum exact
score of the bf16 top-k; or T >= T_k - 2 beta(q)).  These tests pin
the two facts that make that exact: |T - S| <= beta(q) for every doc, and the
band therefore holds the exact top-k.  (Parity unpinned by reference fixtures:
the reference has no fp32-vs-bf16 case; the exact fp64 MaxSim of the fp32
values is the ground truth.)
"""
import numpy as np

from oracle import oracle as orc


def rand_unit(rng, *shape):
    x = rng.standard_normal(shape).astype(np.float32)
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


def case(seed, N=600, B=6, lq=32):
    rng = np.random.default_rng(seed)
    docs = rand_unit(rng, N, 128, 128)
    doclens = rng.integers(1, 129, N)
    doclens[:5] = 128
    Q = rand_unit(rng, B, lq, 128)
    # a few near-duplicates of query tokens so the top of the ranking is structured
    for b in range(B):
        docs[10 * b, :lq] = Q[b] + 0.05 * rand_unit(rng, lq, 128)
        doclens[10 * b] = 128
    return docs, doclens, Q


def test_split_reconstructs_and_matches_bf16_cast():
    import torch
    docs, doclens, _ = case(0, N=60)
    hi, lo, (E, M) = orc.split_f32(docs, doclens)
    np.testing.assert_array_equal(hi, torch.from_numpy(docs).bfloat16().float().numpy())
    err = np.abs(docs.astype(np.float64) - hi - lo)
    assert err.max() <= 2.0 ** -16 * np.abs(docs).max()
    assert 0 < E <= 2.0 ** -8 * 1.001 and 0.99 < M < 1.01


def test_bf16_scan_within_beta_of_exact():
    docs, doclens, Q = case(1)
    hi, _, (E, M) = orc.split_f32(docs, doclens)
    S = orc.maxsim(Q, docs, doclens)                                   # exact fp64 on the fp32 values
    T = orc.maxsim(orc.bf16_round(Q), hi, doclens)                     # the bf16 scan (exact products)
    beta = orc.band_beta(Q, E, M)
    dev = np.abs(T - S).max(axis=1)
    assert (dev <= beta).all(), (dev, beta)
    # the bound is what the certificate pays for: bf16 alone misses the 1e-3 tolerance
    assert dev.max() > 1e-4


def test_band_contains_exact_topk():
    docs, doclens, Q = case(2, N=1500)
    hi, _, (E, M) = orc.split_f32(docs, doclens)
    S = orc.maxsim(Q, docs, doclens)
    T = orc.maxsim(orc.bf16_round(Q), hi, doclens)
    beta = orc.band_beta(Q, E, M)
    k = 50
    _, ids_exact = orc.topk(S, k)
    for b in range(Q.shape[0]):
        tk = np.sort(T[b])[::-1][k - 1]
        band = set(np.nonzero(T[b] >= tk - 2 * beta[b])[0].tolist())
        assert set(ids_exact[b].tolist()) <= band
        assert len(band) < len(T[b])          # the band is a real filter on this data


def test_maxsim_additive_over_query_token_blocks():
    """The identity the long-query path (ColbertIndex._query_blocks) rests on:
    MaxSim sums over query tokens (LRC:807-812), so a query's score is the sum
    of its 32-token blocks' scores -- checked on the oracle in float64, with
    ragged and empty docs."""
    import numpy as np
    from oracle import oracle as orc
    g = np.random.default_rng(4)
    Q = g.standard_normal((3, 70, 128))
    docs = g.standard_normal((50, 128, 128))
    doclens = g.integers(0, 129, 50)
    full = orc.maxsim(Q, docs, doclens)
    parts = sum(orc.maxsim(Q[:, a:a + 32], docs, doclens) for a in range(0, 70, 32))
    fin = np.isfinite(full)
    assert (np.isneginf(full) == np.isneginf(parts)).all()
    np.testing.assert_allclose(parts[fin], full[fin], rtol=0, atol=1e-9)


def test_lower_bound_band_contains_exact_topk_and_is_narrower():
    """The two-pass band of cbv2_search_f32 (CBV2_OPT_BAND_LOWER_BOUND): lb =
    the minimum exact score of the k docs the bf16 scan ranks first is a lower
    bound of the exact k-th score, so every exact top-k doc has T >= lb - beta;
    that band is no wider than T >= T_k - 2 beta (lb >= T_k - beta)."""
    for seed, k in ((3, 10), (4, 50), (5, 100)):
        docs, doclens, Q = case(seed, N=1500)
        hi, _, (E, M) = orc.split_f32(docs, doclens)
        S = orc.maxsim(Q, docs, doclens)
        T = orc.maxsim(orc.bf16_round(Q), hi, doclens)
        beta = orc.band_beta(Q, E, M)
        _, tk = orc.topk(T, k)                                  # the bf16 scan's top-k (ids)
        lb = np.array([S[b, tk[b]].min() for b in range(len(Q))])
        _, ek = orc.topk(S, k)                                  # the exact top-k
        Tk = orc.topk(T, k)[0][:, -1]
        for b in range(len(Q)):
            band_lb = T[b] >= lb[b] - beta[b]
            band_plain = T[b] >= Tk[b] - 2 * beta[b]
            assert band_lb[ek[b]].all(), (seed, b)
            assert lb[b] >= Tk[b] - beta[b] - 1e-12
            assert band_lb.sum() <= band_plain.sum()
