"""Shared id-parity checks for the GPU tests.

Three checks, from strongest to weakest, used together:

* ``assert_selection_exact`` -- the ids/scores a search returned are exactly
  the oracle's top-k SELECTION (oracle.topk: score desc, index asc) applied to
  the GPU's own score matrix.  This pins the selection bit for bit on any data,
  ties included; the scoring itself is pinned by an allclose against the
  float64 oracle.
* ``assert_ranking_consistent`` -- every returned id's ORACLE score equals the
  oracle's score at that rank within ``tol`` (the GPU ranking is the oracle's
  up to fp32 accumulation order), ids unique, padding only past min(k, n).
* ``assert_ids_match_separated`` -- ids equal the oracle's wherever the
  oracle's neighbouring scores differ by more than ``gap``; -inf entries (empty
  docs, padding, out-of-shard candidates) are compared exactly (the tie rule
  orders them identically on both sides).  Returns the fraction of positions
  compared, and asserts it is at least ``min_frac`` (default 0.5, so a check
  that compares almost nothing fails; call sites whose data is dense near the
  cut pass a lower, measured floor).

Bit-exact ids, ORDER and score bits on data where fp32 is exact (k/16 grid
tokens, ties included) are pinned separately, at every size up to the 1M-doc
headline corpus, by tests/test_gpu_grid_exact.py.
"""
import numpy as np

from oracle import oracle as orc


def assert_selection_exact(ids, scores, gpu_score_matrix, k, id_base=0):
    rs, ri = orc.topk(np.asarray(gpu_score_matrix, np.float32), k, id_base=id_base)
    assert np.array_equal(np.asarray(ids, np.int64), ri), "ids differ from the oracle's selection of the GPU scores"
    assert np.array_equal(np.asarray(scores, np.float32), rs.astype(np.float32))


def assert_ranking_consistent(ids, ref_matrix, tol, id_base=0):
    """ids [B, k] (global); ref_matrix [B, n] oracle scores over the same docs."""
    ids = np.asarray(ids, np.int64)
    ref = np.asarray(ref_matrix, np.float64)
    B, k = ids.shape
    n = ref.shape[1]
    kk = min(k, n)
    ref_sorted = -np.sort(-ref, axis=1)[:, :kk]
    for b in range(B):
        row = ids[b]
        assert (row[kk:] == -1).all(), (b, "padding expected past min(k, n)")
        got = row[:kk] - id_base
        assert ((got >= 0) & (got < n)).all(), (b, "id out of range")
        assert len(set(got.tolist())) == kk, (b, "duplicate ids")
        gs = ref[b, got]
        fin = np.isfinite(ref_sorted[b])
        assert np.array_equal(np.isfinite(gs), fin), (b, "-inf entries differ")
        np.testing.assert_allclose(gs[fin], ref_sorted[b][fin], atol=tol, rtol=0)


def assert_ids_match_separated(ids, ref_ids, ref_scores, gap, min_frac=0.5):
    ids = np.asarray(ids)
    ref_scores = np.asarray(ref_scores, np.float64)
    compared = total = 0
    for b in range(ids.shape[0]):
        s = ref_scores[b]
        for j in range(ids.shape[1]):
            total += 1
            if np.isneginf(s[j]):
                assert ids[b, j] == ref_ids[b, j], (b, j, ids[b, j], ref_ids[b, j], "-inf")
                compared += 1
                continue
            lo = s[j - 1] - s[j] if j > 0 else np.inf
            hi = s[j] - s[j + 1] if j + 1 < len(s) else np.inf     # s[j+1] = -inf -> gap inf
            if min(lo, hi) > gap:
                assert ids[b, j] == ref_ids[b, j], (b, j, ids[b, j], ref_ids[b, j])
                compared += 1
    frac = compared / max(total, 1)
    assert frac >= min_frac, f"only {frac:.1%} of positions were separated enough to compare (< {min_frac:.0%})"
    return frac
