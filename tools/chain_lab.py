#!/usr/bin/env python3
"""Where the B=1 post-scan chain of the fp32-faithful one-trip retrieve spends
its time, per kernel and inside it: a lab build of the library
(-DCBV2_LAB_STAMPS, tools/_lab/libcolbert_lab.so, the same sources) stamps
s_memrealtime (100 MHz) at every workgroup's start and end and at the row
selects' phases of the block-max select, the phase-1 rescoring, the band
collect, the band rescoring + select and the rerank + select; this tool runs
OneTripRetriever (host results) at B=1 on the bench's corpus and prints the
median timeline relative to the block-max launch's first workgroup start.

usage: chain_lab.py [--docs 125000] [--iters 60] [--build]"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LAB = os.path.join(ROOT, "tools", "_lab", "libcolbert_lab.so")
KINDS = ("bmax_select", "phase1(+collect)", "band_collect", "band_rescore_select", "rerank_select")
STRIDE = 16 + 2 * 4096


def build():
    from hybrid_rag_colbertv2_amd import _build as B
    os.makedirs(os.path.dirname(LAB), exist_ok=True)
    cmd = [B.HIPCC, *B.FLAGS, f'-DCBV2_BUILD_STAMP="{B.source_stamp()}"', "-DCBV2_LAB_STAMPS=1", "-I",
           os.path.join(ROOT, "include"), B.SRC, *B.SRC_HOST, "-ldl", "-o", LAB]
    subprocess.run(cmd, check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=125000)
    ap.add_argument("--iters", type=int, default=60)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--grid", type=int, default=0, help="CBV2_OPT_RESCORE_GRID for the run (0: automatic)")
    a = ap.parse_args()
    if a.build:
        build()
        return
    from hybrid_rag_colbertv2_amd import _lib
    _lib.LIB_PATH = LAB                      # the stamped build of the same sources
    import torch
    from hybrid_rag_colbertv2_amd import bm25 as bm25_mod
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    L = _lib.lib()
    L.cbv2_lab_set_stamps.argtypes = [ctypes.c_void_p]
    L.cbv2_lab_set_stamps.restype = None
    dev = torch.device("cuda:0")
    n = a.docs
    Qf = synth.make_queries(256, 32, seed=1)
    planted = synth.planted_ids(256, n, 10, seed=2)
    terms, off, V = synth.bm25_shard(0, n, planted)
    lex = bm25_mod.sharded(terms, off, V, id_base=0, device=dev)
    qt, qo = synth.bm25_queries(256)
    bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], 100)   # noqa: E731
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(tokens, doclens)
    del tokens
    if a.grid:
        ix.set_option(_lib.OPT_RESCORE_GRID, a.grid)
    Q1 = Qf[:1].to(dev).contiguous()
    one = OneTripRetriever(ix)
    stamps = torch.zeros((len(KINDS), STRIDE), dtype=torch.int64, device=dev)
    L.cbv2_lab_set_stamps(stamps.data_ptr())
    rows = []
    lat = []
    for it in range(a.iters + 5):
        stamps.zero_()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        one(Q1, bm_one, host=True)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        if it < 5:
            continue
        lat.append((t1 - t0) * 1e6)
        S = stamps.cpu().numpy()
        r = {}
        base = None
        for k, name in enumerate(KINDS):
            st, en = S[k, 16::2], S[k, 17::2]
            used = st > 0
            if not used.any():
                continue
            first = int(st[used].min())
            if base is None:
                base = first
            ends = en[en > 0]
            r[name + ":first_wg_start"] = (first - base) * 0.01
            if len(ends):
                r[name + ":last_wg_end"] = (int(ends.max()) - base) * 0.01
            if S[k, 6] > 0:
                r[name + ":select_start"] = (int(S[k, 6]) - base) * 0.01
            if S[k, 4] > 0:
                r[name + ":select_end"] = (int(S[k, 4]) - base) * 0.01
            if k == 0 and S[k, 4] > 0:   # the block-max select's own phase stamps
                for j, ph in ((0, "keys"), (1, "threshold"), (2, "qualify"), (3, "gather")):
                    r["bmax:" + ph] = (int(S[k, j]) - base) * 0.01
            r[name + ":wgs"] = int(used.sum())
            if k in (1, 2, 3):
                r[name + ":count"] = int(S[k, 5])
        rows.append(r)
    keys = sorted({k for r in rows for k in r}, key=lambda k: statistics.median(r[k] for r in rows if k in r))
    out = {"docs": n, "iters": a.iters, "grid": a.grid, "p50_us": round(statistics.median(lat), 1),
           "timeline_us_from_bmax_start": {k: round(statistics.median(r[k] for r in rows if k in r), 2) for k in keys}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
