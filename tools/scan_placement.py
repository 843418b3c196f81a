#!/usr/bin/env python3
"""Is the B=1 streaming scan's rate a property of the index's memory?  The
same 1M-doc bf16 tokens scanned through four handles, interleaved in one
process: the fp32-faithful index (its hi, cbv2_search_f32), a plain bf16
handle over that same hi tensor (cbv2_search), a plain handle over a copy of
hi in torch's caching allocator, and a plain handle over tokens generated
directly as bf16 (index.hbm_empty, like hi).  One
JSON line per round: median scan event times (ms) per handle."""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex, hbm_placement  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--batch", type=int, default=1)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    n = a.docs
    Qf = synth.make_queries(max(a.batch, 1), 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 1), n, 10, seed=2)
    x, dl = synth.make_shard(0, n, Qf, planted, dev, seed=0, dtype=torch.float32)
    fix = ColbertIndex.faithful_f32(x, dl)
    del x
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    same = ColbertIndex(fix.tokens, fix.doclens)
    copy = ColbertIndex(fix.tokens.clone(), fix.doclens)          # torch's caching allocator
    bt, bdl = synth.make_shard(0, n, Qf, planted, dev, seed=0, dtype=torch.bfloat16)
    fresh = ColbertIndex(bt, bdl)
    print(json.dumps({"bitwise_same_tokens": bool(torch.equal(bt.view(torch.int16), fix.tokens.view(torch.int16))),
                      "placement": {k: [hex(v.tokens.data_ptr()), hbm_placement(v.tokens)] for k, v in
                                    (("faithful_hi", fix), ("copy", copy), ("fresh", fresh))}}), flush=True)
    Q32 = Qf[: a.batch].to(dev).contiguous()
    Qb = Qf[: a.batch].to(dev, torch.bfloat16).contiguous()
    legs = {"faithful_search_f32": (fix, Q32), "plain_over_hi": (same, Qb), "plain_over_copy": (copy, Qb),
            "plain_fresh_bf16": (fresh, Qb)}
    for r in range(a.rounds):
        rec = {"round": r, "docs": n, "B": a.batch}
        for name, (ix, Q) in legs.items():
            ix.search(Q, 100)                     # warm
            torch.cuda.synchronize()
            ix.time_scans(True)
            for _ in range(a.reps):
                ix.search(Q, 100)
            torch.cuda.synchronize()
            rec[name] = round(statistics.median(ix.scan_times()), 4)
            if ix.faithful:
                ix.band_times()
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
