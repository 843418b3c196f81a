#!/usr/bin/env python3
"""Small-shard stage-2 workload for a rocprofv3 kernel trace:
cbv2_search top-100 over n docs (default 100k = BASELINE C2 and 125k = one
rank's shard of 1M at 8 GPUs) at B = 1 / 16 / 64 / 256, each search followed
by a device sync and a 2 ms host sleep, so the trace splits into one window
per search (tools/split_search_trace.py).  Also prints HIP-event medians.

usage: small_shard_trace.py [--docs 100000,125000] [--batches 1,16,64,256]
                            [--reps 10] [--dtype bf16|fp8]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", default="100000,125000")
    ap.add_argument("--batches", default="1,16,64,256")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--bmax", type=int, default=1, help="CBV2_OPT_TOPK_BMAX (1: block-max top-k, 0: sampled)")
    ap.add_argument("--sleep-ms", type=float, default=2.0,
                    help="host sleep after each search (0: back to back, as tools/config_sweep.py times them)")
    a = ap.parse_args()
    from hybrid_rag_colbertv2_amd import _lib
    dev = torch.device("cuda:0")
    batches = [int(x) for x in a.batches.split(",")]
    plan = []
    for n in (int(x) for x in a.docs.split(",")):
        Qf = synth.make_queries(max(batches), 32, seed=1)
        planted = synth.planted_ids(max(batches), n, 10, seed=2)
        tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0)
        ix = ColbertIndex.mxfp8(tokens, doclens) if a.dtype == "fp8" else ColbertIndex(tokens, doclens)
        del tokens
        ix.set_option(_lib.OPT_TOPK_BMAX, a.bmax)
        for B in batches:
            Q = Qf[:B].to(dev, torch.bfloat16)
            torch.cuda.synchronize()
            ts = []
            for r in range(a.warmup + a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ix.search(Q, a.k)
                e1.record()
                torch.cuda.synchronize()
                if r >= a.warmup:
                    ts.append(e0.elapsed_time(e1))
                if a.sleep_ms > 0:
                    time.sleep(a.sleep_ms / 1e3)
            med = sorted(ts)[len(ts) // 2]
            plan.append({"docs": n, "batch": B, "dtype": a.dtype, "bmax": a.bmax, "searches": a.warmup + a.reps,
                         "warmup": a.warmup, "event_ms_median": round(med, 4), "plan": ix.last_scan_plan()})
            print(json.dumps(plan[-1]), flush=True)
        del ix
        torch.cuda.empty_cache()
    print("PLAN " + json.dumps(plan), flush=True)


if __name__ == "__main__":
    main()
