#!/usr/bin/env python3
"""A/B of the faithful search's rescoring grid (CBV2_OPT_RESCORE_GRID:
workgroups per row of a split rescoring launch) on the bench corpus:
interleaved rounds, the library's band events (end of the bf16 top-k -> end
of the band select) per search; checks every grid's top-k equals the first's.
usage: grid_ab.py [--docs N] [--batches 256,64,16,1] [--grids 1024,512,256]"""
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
    ap.add_argument("--batches", default="256,64,16,1")
    ap.add_argument("--grids", default="1024,512,256")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    batches = [int(x) for x in a.batches.split(",")]
    grids = [int(x) for x in a.grids.split(",")]
    Bmax = max(batches)
    Qf = synth.make_queries(Bmax, 32, seed=1)
    planted = synth.planted_ids(Bmax, a.docs, 10, seed=2)
    x, dl = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(x, dl)
    del x
    torch.cuda.empty_cache()
    Q = Qf.to(dev)
    for B in batches:
        Qb = Q[:B].contiguous()
        bs = {g: [] for g in grids}
        outs = {}
        for r in range(a.reps + 1):
            for g in grids:
                ix.set_option(_lib.OPT_RESCORE_GRID, g)
                ix.time_scans(True)
                outs[g] = ix.search(Qb, 100)
                torch.cuda.synchronize()
                band = ix.band_times()
                if r:
                    bs[g].append(band[-1])
        ix.set_option(_lib.OPT_RESCORE_GRID, 0)
        same = all(torch.equal(outs[g][0], outs[grids[0]][0]) and torch.equal(outs[g][1], outs[grids[0]][1])
                   for g in grids)
        print(json.dumps({"docs": a.docs, "batch": B, "band_ms": {str(g): round(statistics.median(bs[g]), 4)
                                                                 for g in grids}, "identical": same}), flush=True)


if __name__ == "__main__":
    main()
