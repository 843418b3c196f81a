"""CPU: the native index file (csrc/index_file.cpp) through its
host-pointer entry points: layout, round trips of whole files and doc ranges,
and validation.  The device entry points (HBM in/out) are covered by
tests/test_gpu_api.py::test_native_index_file_roundtrip."""
import os
import struct

import numpy as np
import pytest


def _lib():
    from hybrid_rag_colbertv2_amd import _lib
    return _lib


def _write(path, dtype, tokens, scales, doclens, id_base=0):
    L = _lib()
    L.check(L.lib().cbv2_index_file_write_host(os.fsencode(path), dtype, len(doclens), tokens.ctypes.data,
                                               scales.ctypes.data if scales is not None else None,
                                               doclens.ctypes.data, id_base))


def _read(path, begin, end, elem, fp8):
    L = _lib()
    m = end - begin
    tok = np.zeros((m, 128, 128), elem)
    sc = np.zeros((m, 128, 2), np.uint8) if fp8 else None
    dl = np.zeros(m, np.int32)
    L.check(L.lib().cbv2_index_file_read_host(os.fsencode(path), begin, end, tok.ctypes.data if m else None,
                                              sc.ctypes.data if (fp8 and m) else None, dl.ctypes.data if m else None))
    return tok, sc, dl


@pytest.mark.parametrize("fp8", [False, True])
def test_roundtrip_and_ranges(tmp_path, fp8):
    L = _lib()
    rng = np.random.default_rng(3)
    n = 37
    elem = np.uint8 if fp8 else np.uint16
    tokens = rng.integers(0, 255 if fp8 else 65535, size=(n, 128, 128)).astype(elem)
    scales = rng.integers(0, 255, size=(n, 128, 2)).astype(np.uint8) if fp8 else None
    doclens = rng.integers(0, 129, size=n).astype(np.int32)
    path = str(tmp_path / "ix.cbv2")
    dt = L.DTYPE_MXFP8 if fp8 else L.DTYPE_BF16
    _write(path, dt, tokens, scales, doclens, id_base=1000)
    from hybrid_rag_colbertv2_amd.index import index_file_info
    assert index_file_info(path) == (dt, n, 1000)
    # header layout as documented in include/colbert_mi355x.h
    with open(path, "rb") as f:
        head = f.read(4096)
    assert head[:8] == b"CBV2IDX1"
    version, dtype, nn = struct.unpack_from("<IiQ", head, 8)
    doclens_off, tokens_off, scales_off, file_bytes = struct.unpack_from("<QQQQ", head, 40)
    assert (version, dtype, nn) == (1, dt, n) and doclens_off == 4096 and tokens_off % 4096 == 0
    assert os.path.getsize(path) == file_bytes
    assert (scales_off % 4096 == 0 and scales_off > 0) if fp8 else scales_off == 0
    for a, b in [(0, n), (0, 1), (5, 17), (36, 37), (12, 12)]:
        tok, sc, dl = _read(path, a, b, elem, fp8)
        assert np.array_equal(tok, tokens[a:b]) and np.array_equal(dl, doclens[a:b])
        if fp8:
            assert np.array_equal(sc, scales[a:b])


def test_validation(tmp_path):
    L = _lib()
    path = str(tmp_path / "ix.cbv2")
    tokens = np.zeros((4, 128, 128), np.uint16)
    doclens = np.full(4, 128, np.int32)
    _write(path, L.DTYPE_BF16, tokens, None, doclens)
    with pytest.raises(ValueError):
        _read(path, 2, 5, np.uint16, False)                 # past the end
    with pytest.raises(ValueError):
        _write(str(tmp_path / "bad.cbv2"), 2, tokens, None, doclens)   # f32 is not a storable dtype
    bad = tmp_path / "junk.cbv2"
    bad.write_bytes(b"x" * 8192)
    from hybrid_rag_colbertv2_amd.index import index_file_info
    with pytest.raises(ValueError):
        index_file_info(str(bad))
    with open(path, "r+b") as f:                            # truncate the token section
        f.truncate(4096 + 4096 + 100)
    with pytest.raises(ValueError):
        index_file_info(path)


@pytest.mark.parametrize("fp8", [False, True])
def test_streaming_writer_host_batches(tmp_path, fp8):
    """cbv2_index_writer_*: contiguous batches appended (host pointers) give the
    same file as one whole write; the header appears only at a complete close."""
    import ctypes
    L = _lib()
    rng = np.random.default_rng(5)
    n = 29
    elem = np.uint8 if fp8 else np.uint16
    tokens = rng.integers(0, 255 if fp8 else 65535, size=(n, 128, 128)).astype(elem)
    scales = rng.integers(0, 255, size=(n, 128, 2)).astype(np.uint8) if fp8 else None
    doclens = rng.integers(0, 129, size=n).astype(np.int32)
    dt = L.DTYPE_MXFP8 if fp8 else L.DTYPE_BF16
    whole, streamed = str(tmp_path / "whole.cbv2"), str(tmp_path / "streamed.cbv2")
    _write(whole, dt, tokens, scales, doclens, id_base=77)
    h = ctypes.c_void_p()
    L.check(L.lib().cbv2_index_writer_open(os.fsencode(streamed), dt, n, 77, ctypes.byref(h)))
    for a, b in [(0, 10), (10, 11), (11, 11), (11, 29)]:
        t, d = np.ascontiguousarray(tokens[a:b]), np.ascontiguousarray(doclens[a:b])
        sc = np.ascontiguousarray(scales[a:b]) if fp8 else None
        L.check(L.lib().cbv2_index_writer_append(h, b - a, t.ctypes.data, sc.ctypes.data if fp8 else None,
                                                 d.ctypes.data, 0, None))
    assert L.lib().cbv2_index_writer_count(h) == n
    with pytest.raises(ValueError):                         # past the declared count
        L.check(L.lib().cbv2_index_writer_append(h, 1, tokens.ctypes.data, None, doclens.ctypes.data, 0, None))
    L.check(L.lib().cbv2_index_writer_close(h))
    assert open(whole, "rb").read() == open(streamed, "rb").read()


def test_streaming_writer_incomplete_file_is_invalid(tmp_path):
    import ctypes
    L = _lib()
    path = str(tmp_path / "partial.cbv2")
    tokens = np.zeros((3, 128, 128), np.uint16)
    doclens = np.full(3, 128, np.int32)
    h = ctypes.c_void_p()
    L.check(L.lib().cbv2_index_writer_open(os.fsencode(path), L.DTYPE_BF16, 10, 0, ctypes.byref(h)))
    L.check(L.lib().cbv2_index_writer_append(h, 3, tokens.ctypes.data, None, doclens.ctypes.data, 0, None))
    with pytest.raises(ValueError, match="partial file removed"):
        L.check(L.lib().cbv2_index_writer_close(h))
    assert not os.path.exists(path)                  # no full-size headerless file left behind
    from hybrid_rag_colbertv2_amd.index import index_file_info
    with pytest.raises(ValueError):
        index_file_info(path)


@pytest.mark.parametrize("ld", [256, 1024])
def test_long_document_file(tmp_path, ld):
    """bf16 long-document files (ld = 256 / 512 / 1024 token slots, the layout
    of a long-document index): the header records ld, ranges read back exactly,
    the streaming writer gives the same bytes; other ld are refused (MXFP8
    long files: tests/test_gpu_long_docs.py)."""
    import ctypes
    L = _lib()
    from hybrid_rag_colbertv2_amd.index import index_file_info, index_file_layout
    rng = np.random.default_rng(ld)
    n = 9
    tokens = rng.integers(0, 65535, size=(n, ld, 128)).astype(np.uint16)
    doclens = rng.integers(0, ld + 1, size=n).astype(np.int32)
    path, streamed = str(tmp_path / "long.cbv2"), str(tmp_path / "long_s.cbv2")
    L.check(L.lib().cbv2_index_file_write_host_ld(os.fsencode(path), L.DTYPE_BF16, n, ld, tokens.ctypes.data, None,
                                                  doclens.ctypes.data, 40))
    assert index_file_layout(path) == (L.DTYPE_BF16, n, 40, ld)
    assert index_file_info(path) == (L.DTYPE_BF16, n, 40)
    assert os.path.getsize(path) == 8192 + n * ld * 256
    for a, b in [(0, n), (3, 7), (8, 9)]:
        tok = np.zeros((b - a, ld, 128), np.uint16)
        dl = np.zeros(b - a, np.int32)
        L.check(L.lib().cbv2_index_file_read_host(os.fsencode(path), a, b, tok.ctypes.data, None, dl.ctypes.data))
        assert np.array_equal(tok, tokens[a:b]) and np.array_equal(dl, doclens[a:b])
    h = ctypes.c_void_p()
    L.check(L.lib().cbv2_index_writer_open_ld(os.fsencode(streamed), L.DTYPE_BF16, n, ld, 40, ctypes.byref(h)))
    for a, b in [(0, 4), (4, 9)]:
        t, d = np.ascontiguousarray(tokens[a:b]), np.ascontiguousarray(doclens[a:b])
        L.check(L.lib().cbv2_index_writer_append(h, b - a, t.ctypes.data, None, d.ctypes.data, 0, None))
    L.check(L.lib().cbv2_index_writer_close(h))
    assert open(path, "rb").read() == open(streamed, "rb").read()
    for dt, bad_ld in [(L.DTYPE_MXFP8, 384), (L.DTYPE_BF16, 384), (L.DTYPE_BF16, 64)]:
        with pytest.raises(ValueError):
            L.check(L.lib().cbv2_index_file_write_host_ld(os.fsencode(str(tmp_path / "x.cbv2")), dt, n, bad_ld,
                                                          tokens.ctypes.data, tokens.ctypes.data,
                                                          doclens.ctypes.data, 0))
