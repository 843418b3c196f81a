#!/usr/bin/env python3
"""A/B of the dynamic-tail modes (CBV2_OPT_DYNAMIC_TAIL: 1 = 8 XCD-local
slices, 2 = one shared tail, 0 = static split) on cbv2_search top-100, one
GPU, interleaved rounds (modes alternate in launch order, so a rocprofv3 PMC
pass can attribute dispatches: dispatch i ran mode modes[i % len(modes)]).

    python tools/tail_ab.py [--docs 1000000] [--batch 256] [--reps 5] [--modes 1,2]"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import _lib, synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="1,2")
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(a.batch, 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 8), a.docs, 10, seed=2)[: a.batch]
    if a.dtype == "fp8":
        q8, sc8, dl = synth.make_shard_mxfp8(0, a.docs, Qf, planted, dev, seed=0)
        ix = ColbertIndex(q8, dl, scales=sc8)
    else:
        tok, dl = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0)
        ix = ColbertIndex(tok, dl)
    Q = Qf.to(dev, torch.bfloat16)
    modes = [int(m) for m in a.modes.split(",")]
    ts = {m: [] for m in modes}
    outs = {}
    for r in range(a.reps + 1):
        for m in modes:
            ix.set_option(_lib.OPT_DYNAMIC_TAIL, m)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            outs[m] = ix.search(Q, 100)
            e1.record()
            e1.synchronize()
            if r:
                ts[m].append(e0.elapsed_time(e1))
    same = all(torch.equal(outs[m][0], outs[modes[0]][0]) and torch.equal(outs[m][1], outs[modes[0]][1])
               for m in modes)
    print(json.dumps({"docs": a.docs, "batch": a.batch, "dtype": a.dtype,
                      "ms": {str(m): round(statistics.median(ts[m]), 3) for m in modes},
                      "min_ms": {str(m): round(min(ts[m]), 3) for m in modes}, "identical": same}))


if __name__ == "__main__":
    main()
