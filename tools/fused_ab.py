#!/usr/bin/env python3
"""A/B of the fused scan + top-k against the unfused path (score matrix + radix
top-k) on one GPU, interleaved, HIP events around each cbv2_search call.

    python tools/fused_ab.py [--docs 1000000] [--batch 256] [--reps 5] [--dtype bf16|fp8]

Prints one JSON line per (dtype, batch): median ms of fused / unfused search,
the unfused scan alone (cbv2_score), and whether the results are identical.
"""
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


def timed(fn, reps):
    out, ts = None, []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return out, statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batches", default="256")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Bmax = max(int(b) for b in a.batches.split(","))
    Qf = synth.make_queries(Bmax, 32, seed=1)
    planted = synth.planted_ids(Bmax, a.docs, 10, seed=2)
    if a.dtype == "fp8":
        q8, sc8, dl = synth.make_shard_mxfp8(0, a.docs, Qf, planted, dev, seed=0)
        ix = ColbertIndex(q8, dl, scales=sc8)
    else:
        tokens, dl = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0)
        ix = ColbertIndex(tokens, dl)
    for B in (int(b) for b in a.batches.split(",")):
        Q = Qf[:B].to(dev, torch.bfloat16)
        ix.search(Q, a.k)                                  # warm up both paths
        ix.set_option(_lib.OPT_FUSED_TOPK, 0)
        ix.search(Q, a.k)
        ix.score(Q)
        rows = {"fused": [], "unfused": [], "score": []}
        same = True
        for _ in range(a.reps):
            ix.set_option(_lib.OPT_FUSED_TOPK, 1)
            f, t = timed(lambda: ix.search(Q, a.k), 1)
            rows["fused"].append(t)
            ix.set_option(_lib.OPT_FUSED_TOPK, 0)
            u, t = timed(lambda: ix.search(Q, a.k), 1)
            rows["unfused"].append(t)
            _, t = timed(lambda: ix.score(Q), 1)
            rows["score"].append(t)
            same = same and torch.equal(f[1], u[1]) and torch.equal(f[0], u[0])
        ix.set_option(_lib.OPT_FUSED_TOPK, 1)
        med = {k: round(statistics.median(v), 3) for k, v in rows.items()}
        flop = B * a.docs * 2 * 32 * 128 * 128
        peak = 5000.0 if a.dtype == "fp8" else 2500.0
        print(json.dumps({"dtype": a.dtype, "docs": a.docs, "batch": B, "k": a.k, "fused_slots": ix.fused_topk_slots(B, a.k),
                          "ms": med, "identical": same,
                          "frac_fused": round(flop / (med["fused"] * 1e-3) / 1e12 / peak, 4),
                          "frac_score": round(flop / (med["score"] * 1e-3) / 1e12 / peak, 4)}), flush=True)


if __name__ == "__main__":
    main()
