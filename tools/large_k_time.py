#!/usr/bin/env python3
"""Time the k > 1024 selection (topk_multi_kernel: passes of 4,096 keys; the
path of torch.topk at any k, LRC:767) on [B, n] random score rows, HIP events
around each call, median of --iters.  `--root` runs another tree's package
(a before/after A/B of two builds of the library on one box).

  python3 tools/large_k_time.py --n 1000000 --k 2048 --B 1 16"""
import argparse
import json
import os
import statistics
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1_000_000)
ap.add_argument("--k", type=int, nargs="+", default=[2048])
ap.add_argument("--B", type=int, nargs="+", default=[1, 16])
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--root", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ap.add_argument("--tag", default="")
a = ap.parse_args()
sys.path.insert(0, a.root)
import torch  # noqa: E402

from hybrid_rag_colbertv2_amd import _lib  # noqa: E402
from hybrid_rag_colbertv2_amd.index import topk_rows  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
for B in a.B:
    sc = torch.randn(B, a.n, device=dev, generator=g)
    for k in a.k:
        ref = None
        ts = []
        for it in range(a.iters + 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s, i = topk_rows(sc, k, sampled=False)
            e1.record()
            torch.cuda.synchronize()
            if it >= 2:
                ts.append(e0.elapsed_time(e1))
            ref = (s, i)
        want = torch.topk(sc, k, dim=1)
        ok = bool(torch.equal(ref[0], want.values))
        print(json.dumps({"tag": a.tag, "lib": _lib.lib().cbv2_build_stamp().decode(), "n": a.n, "B": B, "k": k,
                          "ms_median": round(statistics.median(ts), 4), "ms_min": round(min(ts), 4),
                          "scores_equal_torch_topk": ok}), flush=True)
