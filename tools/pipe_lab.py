#!/usr/bin/env python3
"""Can the fp32-faithful B=256 step hide its band work behind the scan?  The
batch is cut into row chunks; each chunk runs cbv2_search_f32_begin (split,
bf16 scan, top-k, the top-k's faithful scores fk) on the main stream and
cbv2_search_f32_finish (band with lb = min(fk), rescoring, select) on a side
stream, so chunk j's band overlaps chunk j+1's scan.  Compared with the
one-call search (cbv2_search_f32) and with the same chunks run serially;
every variant's top-k is checked bit-for-bit against the one-call search.
Also the plain bf16 search at B = 256 vs the same rows in chunks (does the
scan keep its rate at smaller batches?).  One JSON line per variant.
usage: pipe_lab.py [--docs N] [--reps R]"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import _lib, synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import BAND_CAP, ColbertIndex  # noqa: E402


def timed(fn, reps, side=None):
    ts = []
    for _ in range(reps):
        main = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(main)
        fn()
        if side is not None:
            main.wait_stream(side)
        e1.record(main)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return round(statistics.median(ts), 3), round(min(ts), 3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n, B, k, lq = a.docs, a.batch, 100, 32
    Qf = synth.make_queries(B, lq, seed=1)
    planted = synth.planted_ids(B, n, 10, seed=2)
    x, dl = synth.make_shard(0, n, Qf, planted, dev, seed=0, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(x, dl)
    del x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    Q = Qf.to(dev).contiguous()
    ref_s, ref_i = ix.search(Q, k)
    torch.cuda.synchronize()
    L = _lib.lib()
    cap = max(BAND_CAP, k)
    side = torch.cuda.Stream(dev)
    bufs = {}

    def chunk_bufs(c0, c1):
        key = (c0, c1)
        if key not in bufs:
            nb = c1 - c0
            need = int(L.cbv2_f32_workspace_bytes(ix._h, _lib.F32_SEARCH, nb, lq, cap))
            bufs[key] = dict(ws=torch.empty(((need + 3) // 4,), dtype=torch.float32, device=dev),
                             fk=torch.empty((nb, k), dtype=torch.float32, device=dev),
                             s=torch.empty((nb, k), dtype=torch.float32, device=dev),
                             i=torch.empty((nb, k), dtype=torch.int32, device=dev),
                             st=torch.empty((nb,), dtype=torch.int32, device=dev))
        return bufs[key]

    def run_chunks(sizes, overlap):
        main = torch.cuda.current_stream()
        bounds, c0 = [], 0
        for s in sizes:
            bounds.append((c0, c0 + s))
            c0 += s
        evs = []
        for (c0, c1) in bounds:   # phase 1 of every chunk, back to back on the main stream
            b = chunk_bufs(c0, c1)
            _lib.check(L.cbv2_search_f32_begin(ix._h, Q[c0:c1].data_ptr(), c1 - c0, lq, k, cap, b["ws"].data_ptr(),
                                               b["ws"].numel() * 4, b["fk"].data_ptr(), b["s"].data_ptr(),
                                               b["i"].data_ptr(), b["st"].data_ptr(), main.cuda_stream))
            ev = torch.cuda.Event()
            ev.record(main)
            evs.append(ev)
            if not overlap:
                finish(b, c1 - c0, main)
        if overlap:
            for (c0, c1), ev in zip(bounds, evs):
                side.wait_event(ev)
                finish(chunk_bufs(c0, c1), c1 - c0, side)

    def finish(b, nb, stream):
        with torch.cuda.stream(stream):
            b["lb"] = b["fk"].min(dim=1).values.contiguous()
        _lib.check(L.cbv2_search_f32_finish(ix._h, nb, lq, k, cap, b["ws"].data_ptr(), b["ws"].numel() * 4,
                                            b["lb"].data_ptr(), b["s"].data_ptr(), b["i"].data_ptr(),
                                            b["st"].data_ptr(), stream.cuda_stream))

    def same(sizes):
        c0, ok = 0, True
        for s in sizes:
            b = chunk_bufs(c0, c0 + s)
            ok = ok and torch.equal(b["s"], ref_s[c0:c0 + s]) and torch.equal(b["i"], ref_i[c0:c0 + s])
            c0 += s
        return bool(ok)

    print(json.dumps({"variant": "one_call", "B": B, "ms": timed(lambda: ix.search(Q, k), a.reps)}), flush=True)
    for sizes in ([128, 128], [96, 96, 64], [112, 112, 32], [64, 64, 64, 64], [80, 80, 64, 32]):
        for overlap in (False, True):
            run_chunks(sizes, overlap)
            torch.cuda.synchronize()
            ok = same(sizes)
            ms = timed(lambda: run_chunks(sizes, overlap), a.reps, side if overlap else None)
            print(json.dumps({"variant": "chunks_overlap" if overlap else "chunks_serial", "sizes": sizes,
                              "identical": ok, "ms": ms}), flush=True)
    bix = ColbertIndex(ix.tokens, ix.doclens)
    Qb = Qf.to(dev, torch.bfloat16).contiguous()
    for sizes in ([256], [128, 128], [64] * 4):
        def go():
            c0 = 0
            for s in sizes:
                bix.search(Qb[c0:c0 + s], k)
                c0 += s
        go()
        print(json.dumps({"variant": "bf16_search_chunks", "sizes": sizes, "ms": timed(go, a.reps)}), flush=True)


if __name__ == "__main__":
    main()
