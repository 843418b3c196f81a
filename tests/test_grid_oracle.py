"""CPU: the codebook oracle (oracle.codebook_*, oracle/cbv2_oracle.c
oracle_codebook_topk) and the exact-grid corpus it scores (tests/_grid.py).

The 1M-doc rank-order parity test (tests/test_gpu_grid_exact.py) trusts that
  (a) the codebook evaluation equals the plain maxsim oracle -- checked here on
      a small corpus of the same construction, planted docs and ties included;
  (b) the grid values are exact in bf16 and MXFP8 and every fp32 accumulation
      order gives the exact score -- checked here by rounding the inputs and by
      scoring in float32 vs float64.
"""
import numpy as np

from _grid import GridCorpus
from oracle import oracle as orc


def _small():
    return GridCorpus(1500, 4, seed=7)


def test_codebook_topk_equals_maxsim_oracle():
    g = _small()
    rows = g.rows_f32(0, g.N)
    ref = orc.maxsim(g.Q, rows, g.doclens)                       # float64, generic
    for k in (1, 10, 100, 1500, 1600):
        es, ei = orc.topk(ref, k)
        s, i = g.topk(k)
        assert np.array_equal(i, ei), k
        assert np.array_equal(s, es), k
    # planted docs lead, the last two of each query tie exactly (lower id first)
    s, i = g.topk(10)
    for b in range(g.B):
        assert set(i[b].tolist()) == set(g.planted[b].tolist())
        a, c = g.planted[b, -2], g.planted[b, -1]
        assert ref[b, a] == ref[b, c]
        pa, pc = list(i[b]).index(a), list(i[b]).index(c)
        assert abs(pa - pc) == 1 and (pa < pc) == (a < c)
    # exact_scores at arbitrary ids (codebook, planted, padding -1)
    ids = np.stack([np.r_[g.planted[b], np.arange(b, 300, 7)[:30], -1] for b in range(g.B)])
    got = g.exact_scores(range(g.B), ids)
    want = np.where(ids >= 0, np.take_along_axis(ref, np.maximum(ids, 0), axis=1), -np.inf)
    assert np.array_equal(got, want)
    assert np.isneginf(ref[:, g.doclens == 0]).all()


def test_grid_values_exact_in_bf16_mxfp8_fp32():
    g = _small()
    rows = g.rows_f32(0, 600)
    for x in (g.codebook, g.Q, rows, g.copy_vals):
        assert np.array_equal(orc.bf16_round(x), x)
        q, sc = orc.mxfp8_quantize(x)
        assert np.array_equal(orc.mxfp8_dequant(q, sc), x.astype(np.float64))
        hi, lo, _ = orc.split_f32(x.reshape(-1, 1, 128))
        assert np.array_equal(hi.reshape(x.shape), x) and not lo.any()
    # float32 accumulation (numpy's einsum order) == float64: every order is exact on the grid
    f32 = orc.maxsim(g.Q, rows, g.doclens[:600], dtype=np.float32)
    f64 = orc.maxsim(g.Q, rows, g.doclens[:600])
    assert np.array_equal(f32.astype(np.float64), f64)
    assert np.all(np.abs(f64[np.isfinite(f64)]) * 256 < 2 ** 24)
    assert np.array_equal(np.round(f64[np.isfinite(f64)] * 256), f64[np.isfinite(f64)] * 256)


def test_corpus_is_deterministic_and_ragged():
    a, b = GridCorpus(700, 2, seed=9), GridCorpus(700, 2, seed=9)
    assert np.array_equal(a.codes, b.codes) and np.array_equal(a.doclens, b.doclens)
    assert np.array_equal(a.planted_scores, b.planted_scores)
    assert a.doclens.min() >= 0 and a.doclens.max() == 128 and len(np.unique(a.doclens)) > 50
    # padding rows never hold a code of the doc's own set (reading them would change scores)
    for d in range(0, 700, 37):
        if d in set(a.planted_flat.tolist()):
            continue
        own = set(a.codes[d, : a.doclens[d]].tolist())
        assert not own & set(a.codes[d, a.doclens[d]:].tolist())
