"""ctypes binding of libcolbert_mi355x.so (the C ABI in include/colbert_mi355x.h).

There is no CPU fallback: if the library is missing or no HIP device is
present, every compute entry point raises.  ctypes releases the GIL for the
duration of each foreign call.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG, "libcolbert_mi355x.so")
HEADER = os.path.join(os.path.dirname(PKG), "include", "colbert_mi355x.h")

DTYPE_BF16 = 1
DTYPE_F32 = 2
DTYPE_MXFP8 = 3
SCORER_MAXSIM = 0
SCORER_REF_MEANPOOL_COSINE = 1
SCORERS = {"maxsim": SCORER_MAXSIM, "ref_meanpool_cosine": SCORER_REF_MEANPOOL_COSINE}
ERR_EINVAL, ERR_EUNSUPPORTED, ERR_EHIP, ERR_ESTATE = -1, -2, -3, -4
F32_SCORE, F32_SEARCH, F32_RERANK = 0, 1, 2
(OPT_FUSED_TOPK, OPT_DYNAMIC_TAIL, OPT_BAND_DOC_MAJOR, OPT_BAND_LOWER_BOUND, OPT_TOPK_BMAX, OPT_BAND_FUSED,
 OPT_RESCORE_SPLIT, OPT_BAND_REUSE, OPT_BAND_BLOCK_SKIP, OPT_RESCORE_GRID, OPT_DENSE_DOCS, OPT_P1_COLLECT_FUSED,
 OPT_FOLD_KEYS) = (1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13)

_p, _i32, _i64, _sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
_SIGS = {
    "cbv2_abi_version": (ctypes.c_int, []),
    "cbv2_last_error": (ctypes.c_char_p, []),
    "cbv2_build_stamp": (ctypes.c_char_p, []),
    "cbv2_index_create": (ctypes.c_int, [ctypes.c_int, _p, _i32, _i64, _i32, _i32, _p, _i64,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_index_destroy": (ctypes.c_int, [_p]),
    "cbv2_hbm_alloc": (ctypes.c_int, [ctypes.c_int, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                      ctypes.POINTER(ctypes.c_int32)]),
    "cbv2_hbm_free": (ctypes.c_int, [ctypes.c_int, _p]),
    "cbv2_index_time_scans": (ctypes.c_int, [_p, _i32]),
    "cbv2_index_scan_times": (ctypes.c_int, [_p, _p, _i32, ctypes.POINTER(ctypes.c_int32)]),
    "cbv2_index_band_times": (ctypes.c_int, [_p, _p, _i32, ctypes.POINTER(ctypes.c_int32)]),
    "cbv2_index_scan_clock": (ctypes.c_int, [_p, _p, _i32]),
    "cbv2_index_create_mxfp8": (ctypes.c_int, [ctypes.c_int, _p, _p, _i64, _i32, _i32, _p, _i64,
                                               ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_quantize_mxfp8": (ctypes.c_int, [_p, _i32, _i64, _p, _p, _p]),
    "cbv2_index_build_means": (ctypes.c_int, [_p, _p, _i32, _p, _p]),
    "cbv2_score": (ctypes.c_int, [_p, _i32, _p, _i32, _i32, _i32, _p, _i64, _p]),
    "cbv2_search_workspace_bytes": (_sz, [_p, _i32]),
    "cbv2_search_workspace_size": (_sz, [_p, _i32, _i32, _i32]),
    "cbv2_index_set_option": (ctypes.c_int, [_p, _i32, _i64]),
    "cbv2_search_fused_slots": (_i64, [_p, _i32, _i32, _i32]),
    "cbv2_index_last_scan_plan": (ctypes.c_int, [_p, _p]),
    "cbv2_search": (ctypes.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _p, _sz, _p, _p, _p]),
    "cbv2_rerank": (ctypes.c_int, [_p, _p, _i32, _i32, _p, _i32, _i32, _p, _p, _p, _p]),
    "cbv2_rerank_workspace_bytes": (_sz, [_i32, _i32]),
    "cbv2_rerank_ws": (ctypes.c_int, [_p, _p, _i32, _i32, _p, _i32, _i32, _p, _sz, _p, _p, _p, _p]),
    "cbv2_select_topk": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p]),
    "cbv2_topk_workspace_bytes": (_sz, [_i32, _i64]),
    "cbv2_topk_rows": (ctypes.c_int, [_p, _i32, _i64, _i64, _i32, _i64, _p, _sz, _p, _p, _p]),
    "cbv2_merge_topk": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _p, _p, _p]),
    "cbv2_rrf_fuse": (ctypes.c_int, [_p, _i32, _p, _i32, _i32, _i32, _i32, _p, _p, _p]),
    "cbv2_bm25_build": (ctypes.c_int, [_p, _p, _i64, _i32, ctypes.c_float, ctypes.c_float,
                                       ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_bm25_search": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _p, _p]),
    "cbv2_bm25_doc_freq": (ctypes.c_int, [_p, _p, _i64, _i32, _p]),
    "cbv2_bm25_build_shard": (ctypes.c_int, [_p, _p, _i64, _i32, ctypes.c_float, ctypes.c_float, _i64, _i64,
                                             _i64, _p, ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_bm25_num_docs": (_i64, [_p]),
    "cbv2_stem_en": (ctypes.c_int, [_p, _p, _i64, _p, _i64, _p]),
    "cbv2_index_file_info": (ctypes.c_int, [ctypes.c_char_p, _p, _p, _p]),
    "cbv2_index_file_write": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _p, _p, _p, _i64, _p]),
    "cbv2_index_file_read": (ctypes.c_int, [ctypes.c_char_p, _i64, _i64, _p, _p, _p, _p]),
    "cbv2_index_file_write_host": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _p, _p, _p, _i64]),
    "cbv2_index_file_read_host": (ctypes.c_int, [ctypes.c_char_p, _i64, _i64, _p, _p, _p]),
    "cbv2_index_writer_open": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _i64, ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_index_file_info_ld": (ctypes.c_int, [ctypes.c_char_p, _p, _p, _p, _p]),
    "cbv2_index_file_write_ld": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _i32, _p, _p, _p, _i64, _p]),
    "cbv2_index_file_write_host_ld": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _i32, _p, _p, _p, _i64]),
    "cbv2_index_writer_open_ld": (ctypes.c_int, [ctypes.c_char_p, _i32, _i64, _i32, _i64,
                                                 ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_index_writer_append": (ctypes.c_int, [_p, _i64, _p, _p, _p, _i32, _p]),
    "cbv2_index_writer_count": (_i64, [_p]),
    "cbv2_index_writer_close": (ctypes.c_int, [_p]),
    "cbv2_comm_init": (ctypes.c_int, [_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_comm_loopback_init": (ctypes.c_int, [_i32, ctypes.POINTER(ctypes.c_void_p)]),
    "cbv2_comm_size": (ctypes.c_int, [_p]),
    "cbv2_comm_rank": (ctypes.c_int, [_p]),
    "cbv2_comm_destroy": (ctypes.c_int, [_p]),
    "cbv2_sharded_workspace_bytes": (_sz, [_p, _p, _i32, _i32, _i32, _i32]),
    "cbv2_search_sharded": (ctypes.c_int, [_p, _p, _i32, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _sz, _p, _p,
                                           _p, _p]),
    "cbv2_search_sharded_local": (ctypes.c_int, [_p, _p, _i32, _p, _i32, _i32, _i32, _i32, _i32, _p, _sz, _p]),
    "cbv2_search_sharded_exchange": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _p, _sz, _p,
                                                    _p, _p, _p]),
    "cbv2_rerank_sharded": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _p, _i32, _i32, _p, _sz, _p, _p, _p, _p]),
    "cbv2_rerank_sharded_prescored": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _p, _i32, _i32, _p, _sz, _p, _p, _p,
                                                     _p, _p]),
    "cbv2_comm_stats": (ctypes.c_int, [_p, _p]),
    "cbv2_bm25_destroy": (ctypes.c_int, [_p]),
    "cbv2_split_f32": (ctypes.c_int, [_p, _i64, _i32, _p, _p, _p, _p, _p]),
    "cbv2_index_attach_residual": (ctypes.c_int, [_p, _p, ctypes.c_float, ctypes.c_float]),
    "cbv2_f32_workspace_bytes": (_sz, [_p, _i32, _i32, _i32, _i32]),
    "cbv2_score_f32": (ctypes.c_int, [_p, _p, _i32, _i32, _p, _sz, _p, _i64, _p]),
    "cbv2_search_f32": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _p, _sz, _p, _p, _p, _p]),
    "cbv2_search_f32_begin": (ctypes.c_int, [_p, _p, _i32, _i32, _i32, _i32, _p, _sz, _p, _p, _p, _p, _p]),
    "cbv2_search_f32_finish": (ctypes.c_int, [_p, _i32, _i32, _i32, _i32, _p, _sz, _p, _p, _p, _p, _p]),
    "cbv2_rerank_f32": (ctypes.c_int, [_p, _p, _i32, _i32, _p, _i32, _i32, _p, _sz, _p, _p, _p, _p]),
    "cbv2_index_kind": (ctypes.c_int, [_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
    "cbv2_retrieve_workspace_bytes": (_sz, [_p, _p, _i32, _i32, _i32, _i32, _i32]),
    "cbv2_retrieve_host_bytes": (_sz, [_i32, _i32, _i32, _i32]),
    "cbv2_retrieve_host_marks": (ctypes.c_int, [_p, _i32]),
    "cbv2_retrieve_cancel": (ctypes.c_int, [_p, _p, _p]),
    "cbv2_retrieve_pool_stats": (ctypes.c_int, [_p, _i32]),
    "cbv2_retrieve_begin": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _p, _sz, _p]),
    "cbv2_retrieve_finish": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _i32, _i32, _i32,
                                            _p, _sz, _p, _sz, _p, _p, _p, _p]),
    "cbv2_retrieve_finish_host": (ctypes.c_int, [_p, _p, _p, _i32, _i32, _i32, _i32, _p, _p, _i32, _i32, _i32,
                                                 _i32, _p, _sz, _p, _sz, _p, _p, _p, _p, _p, _p, _p]),
}

_lib = None


def header_symbols(path: str = HEADER):
    """Every function the public header declares (used by the export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:[\w\s\*]+?)\b(cbv2_\w+)\s*\(", text, re.M)))


def lib():
    global _lib
    if _lib is None:
        from . import _build
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
        want, have = _build.source_stamp(), _build.library_stamp(LIB_PATH)
        if have != want:     # never run a library built from other sources than the tree's
            raise RuntimeError(f"{LIB_PATH} was built from other sources (stamp {have}, sources {want}): "
                               "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


class Cbv2Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"cbv2 error {code}: {msg}")
        self.code = code


def check(rc: int):
    if rc != 0:
        msg = lib().cbv2_last_error().decode(errors="replace")
        if rc == ERR_EINVAL:
            raise ValueError(msg)
        raise Cbv2Error(rc, msg)
    return rc
