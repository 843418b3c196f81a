#!/usr/bin/env python3
"""A/B of the fp32-faithful search's band rescoring (CBV2_OPT_BAND_DOC_MAJOR:
0 pair by pair, 1 doc-major with the doc's tiles held per half, 2 doc-major
pair-outer, 3 / 4 doc-major with the doc split over a workgroup of 4 / 2
waves) on one GPU, interleaved rounds, HIP events around each search and the
library's band events (end of the bf16 top-k -> end of the band select).

    python tools/band_ab.py [--docs 1000000] [--batch 256] [--reps 5]

Prints one JSON line: median search ms and band ms per mode and whether every
mode's ids and scores equal the first mode's."""
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
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--modes", default="0,1,3,4")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(a.batch, 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 8), a.docs, 10, seed=2)[: a.batch]
    f32, dl = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0, dtype=torch.float32)
    ix = ColbertIndex.faithful_f32(f32, dl)
    del f32
    Q = Qf.to(dev)
    modes = [int(m) for m in a.modes.split(",")]
    ts = {m: [] for m in modes}
    bs = {m: [] for m in modes}
    outs = {}
    for r in range(a.reps + 1):
        for m in modes:
            ix.set_option(_lib.OPT_BAND_DOC_MAJOR, m)
            ix.time_scans(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            outs[m] = ix.search(Q, a.k)
            e1.record()
            e1.synchronize()
            band = ix.band_times()
            if r:
                ts[m].append(e0.elapsed_time(e1))
                bs[m].append(band[-1])
    same = all(torch.equal(outs[m][0], outs[modes[0]][0]) and torch.equal(outs[m][1], outs[modes[0]][1])
               for m in modes)
    print(json.dumps({"docs": a.docs, "batch": a.batch, "k": a.k, "band_mean": round(float(ix.last_band.float().mean()), 1),
                      "ms": {str(m): round(statistics.median(ts[m]), 3) for m in modes},
                      "band_ms": {str(m): round(statistics.median(bs[m]), 3) for m in modes}, "identical": same}),
          flush=True)


if __name__ == "__main__":
    main()
