"""CPU: the C-ABI library loads and exports every declared symbol; argument
validation fails before any launch; host-side logic (native RRF, BM25 stand-in,
sharding, synthetic corpus helpers) is exact."""
import ctypes
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN, ROOT
from hybrid_rag_colbertv2_amd import _lib
from oracle import oracle as orc


@pytest.fixture(scope="module")
def L():
    if not os.path.exists(_lib.LIB_PATH):
        pytest.skip("libcolbert_mi355x.so not built")
    return _lib.lib()


def test_library_exports_every_header_symbol(L):
    syms = _lib.header_symbols()
    assert len(syms) >= 13
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib._SIGS), "ctypes signatures out of sync with the header"
    assert L.cbv2_abi_version() == 2


def test_library_stamp_is_the_sources_content_hash(L, tmp_path):
    """Build provenance: the loaded library was compiled from exactly the tree's
    sources and flags; a library with another stamp is refused by the loader."""
    from hybrid_rag_colbertv2_amd import _build
    stamp = _build.source_stamp()
    assert L.cbv2_build_stamp().decode() == f"cbv2-build-stamp:{stamp}"
    assert _build.library_stamp(_lib.LIB_PATH) == stamp
    fake = tmp_path / "lib.so"
    fake.write_bytes(b"\0ELF... cbv2-build-stamp:0123456789abcdef ...")
    assert _build.library_stamp(str(fake)) == "0123456789abcdef" != stamp
    assert _build.library_stamp(str(tmp_path / "missing.so")) is None


def test_validation_errors_without_gpu(L):
    h = ctypes.c_void_p()
    assert L.cbv2_index_create(0, None, 7, 10, 128, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EUNSUPPORTED
    assert b"dtype" in L.cbv2_last_error()
    assert L.cbv2_index_create(0, None, 1, 10, 64, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EUNSUPPORTED
    assert L.cbv2_index_create(0, None, 1, 10, 200, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EUNSUPPORTED  # long docs: 256/512/1024
    assert L.cbv2_index_create(0, None, 1, 10, 2048, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EUNSUPPORTED
    assert L.cbv2_index_create_mxfp8(0, None, None, 10, 384, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EUNSUPPORTED
    assert L.cbv2_index_create_mxfp8(0, None, None, 10, 256, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EINVAL  # null
    assert L.cbv2_index_create(0, None, 1, -1, 128, 128, None, 0, ctypes.byref(h)) == _lib.ERR_EINVAL
    assert L.cbv2_index_create(0, None, 1, 10, 128, 128, None, 0, None) == _lib.ERR_EINVAL
    assert L.cbv2_topk_rows(None, 1, 10, 10, 5, 0, None, 0, None, None, None) == _lib.ERR_EINVAL
    assert L.cbv2_select_topk(ctypes.c_void_p(16), None, 1, 10, 0, ctypes.c_void_p(16), None, None, None) \
        == _lib.ERR_EINVAL
    assert L.cbv2_merge_topk(ctypes.c_void_p(16), ctypes.c_void_p(16), 65, 1, 10, ctypes.c_void_p(16),
                             ctypes.c_void_p(16), None) == _lib.ERR_EINVAL
    assert L.cbv2_score(None, 0, None, 1, 1, 32, None, 0, None) == _lib.ERR_EINVAL
    with pytest.raises(ValueError):
        _lib.check(_lib.ERR_EINVAL)


def test_native_rrf_matches_reference_golden(L):
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    for case in json.load(open(os.path.join(GOLDEN, "rrf_ties.json"))):
        bm = np.array(case["bm25"], np.int32).reshape(1, -1)
        cb = np.array(case["colbert"], np.int32).reshape(1, -1)
        ids, sc, cnt = rrf_fuse(bm, cb, C=200, return_scores=True)
        n = int(cnt[0])
        assert [(int(i), float(s)) for i, s in zip(ids[0, :n], sc[0, :n])] == \
            [(f["chunk_id"], f["rrf_score"]) for f in case["fused"]]
        assert (ids[0, n:] == -1).all()


def test_native_rrf_batch_equals_python(L):
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    rng = np.random.default_rng(0)
    B = 64
    bm = rng.integers(0, 300, size=(B, 100)).astype(np.int32)
    cb = rng.integers(0, 300, size=(B, 100)).astype(np.int32)
    cb[:, 90:] = -1
    ids = rrf_fuse(bm, cb, C=50)
    for b in range(B):
        exp = [i for i, _ in orc.rrf(list(bm[b]), [x for x in cb[b] if x >= 0])][:50]
        assert list(ids[b, : len(exp)]) == exp


@pytest.mark.parametrize("kb,kc,span", [(100, 100, 2**31 - 1), (3000, 2000, 4000), (0, 37, 50), (64, 0, 10)])
def test_native_rrf_hash_table_equals_python(L, kb, kc, span):
    """The id -> slot table (open addressing) against the reference dict semantics:
    ids over the whole int32 range, long lists (many probes), lists with many
    repeats, one empty list; ids AND float64 scores."""
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    rng = np.random.default_rng(kb + kc)
    B = 6
    bm = rng.integers(0, span, size=(B, kb)).astype(np.int32)
    cb = rng.integers(0, span, size=(B, kc)).astype(np.int32)
    if kc:
        cb[:, kc // 2:] = bm[:, : kc - kc // 2] if kb >= kc - kc // 2 else cb[:, kc // 2:]
    C = kb + kc + 3
    ids, sc, cnt = rrf_fuse(bm, cb, C=C, return_scores=True)
    for b in range(B):
        exp = orc.rrf(list(bm[b]), list(cb[b]))
        assert int(cnt[b]) == len(exp)
        assert [(int(i), float(s)) for i, s in zip(ids[b, : len(exp)], sc[b, : len(exp)])] == \
            [(int(i), float(s)) for i, s in exp]
        assert (ids[b, len(exp):] == -1).all()


def test_host_bm25_basic(tmp_path):
    from hybrid_rag_colbertv2_amd.bm25 import HostBM25
    corpus = ["the cat sat on the mat", "dogs chase cats", "a bird in the hand", "cats and dogs and cats"]
    bm = HostBM25()
    bm.index(bm.tokenize(corpus))
    ids, sc = bm.retrieve(bm.tokenize("cats"), k=3)
    assert ids[0][0] == 3 and sc[0][0] > sc[0][1] > 0
    bm.save(str(tmp_path))
    bm2 = HostBM25.load(str(tmp_path))
    ids2, sc2 = bm2.retrieve(bm2.tokenize("cats"), k=3)
    assert np.array_equal(ids, ids2) and np.allclose(sc, sc2)


def test_shard_range_partitions():
    from hybrid_rag_colbertv2_amd.distributed import shard_range
    for n in (0, 1, 7, 1000, 1_000_001):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(r, r[1:]))
            assert max(e - s for s, e in r) - min(e - s for s, e in r) <= 1


def test_synth_helpers():
    from hybrid_rag_colbertv2_amd import synth
    p = synth.planted_ids(16, 5000, 10)
    assert len(np.unique(p)) == p.size
    bm = synth.bm25_lists(16, 5000, p, k=100)
    assert bm.shape == (16, 100)
    for b in range(16):
        assert set(p[b, :5]) <= set(bm[b])
    q = synth.make_queries(4)
    assert np.allclose(q.norm(dim=-1).numpy(), 1.0, atol=1e-5)
