#!/usr/bin/env python3
"""Where the B=1 block-max top-k spends its time (tools/topk_lab.hip): the
production one-launch kernel (bmax_topk_kernel) with its lab stamps -- the
block-max phase (first workgroup start -> the row's last arrival), then the
last workgroup's select phases -- on the bench's scores of one query, checked
against the production search's top-100.
usage: topk_lab.py [--docs 125000,1000000] [--reps R] [--build]"""
import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex, _stream_ptr  # noqa: E402

LAB = os.path.join(ROOT, "tools", "_lab", "libtopklab.so")
PHASES = ("block_max+arrival", "keys", "threshold", "qualify", "gather", "rank+write")
SUB = ()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", default="125000,1000000")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--warm", type=int, default=1, help="1: a scan right before each timed select")
    a = ap.parse_args()
    if a.build or not os.path.exists(LAB):
        os.makedirs(os.path.dirname(LAB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-fno-honor-nans", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tools", "topk_lab.hip"), "-o", LAB], check=True)
        if a.build:
            return
    lab = ctypes.CDLL(LAB)
    dev = torch.device("cuda:0")
    for n in (int(x) for x in a.docs.split(",")):
        B, k = 1, 100
        Qf = synth.make_queries(B, 32, seed=1)
        planted = synth.planted_ids(B, n, 10, seed=2)
        tok, dl = synth.make_shard(0, n, Qf, planted, dev, seed=0)
        ix = ColbertIndex(tok, dl)
        Q = Qf.to(dev, torch.bfloat16)
        scores = ix.score(Q).contiguous()
        ref_s, ref_i = ix.search(Q, k)
        nb = (n + 63) // 64
        bm = torch.empty((B, nb + (n + 255) // 256), dtype=torch.int32, device=dev)
        out_s = torch.empty((B, k), dtype=torch.float32, device=dev)
        out_i = torch.empty((B, k), dtype=torch.int32, device=dev)
        done = torch.zeros((B,), dtype=torch.int32, device=dev)
        G = lab.lab_bmax_grid(ctypes.c_int64(n))
        stamps = torch.zeros((16 + 2 * G,), dtype=torch.int64, device=dev)
        st = _stream_ptr(dev)
        ph = {p: [] for p in PHASES + SUB}
        tot, spread = [], []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            if a.warm:        # a scan just before, as in the search (the clock of a loaded chip)
                ix.score(Q)
            e0.record()
            rc = lab.lab_bmax_topk(ctypes.c_void_p(scores.data_ptr()), B, ctypes.c_int64(n), k,
                                   ctypes.c_void_p(bm.data_ptr()), ctypes.c_void_p(out_s.data_ptr()),
                                   ctypes.c_void_p(out_i.data_ptr()), ctypes.c_void_p(done.data_ptr()),
                                   ctypes.c_void_p(stamps.data_ptr()), ctypes.c_void_p(st))
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            tot.append(e0.elapsed_time(e1) * 1e3)
            s = stamps.tolist()
            starts = s[16::2][:G]
            t = [min(starts), s[6], s[0], s[1], s[2], s[3], s[4]]
            for j, p in enumerate(PHASES):
                ph[p].append((t[j + 1] - t[j]) * 0.01)      # 100 MHz ticks -> us

            spread.append((max(starts) - min(starts)) * 0.01)
        same = bool(torch.equal(out_s, ref_s) and torch.equal(out_i, ref_i))
        nq, nc = stamps[5].item() >> 32, stamps[5].item() & 0xffffffff
        print(json.dumps({"docs": n, "grid": G, "identical_to_search": same,
                          "event_us": round(statistics.median(tot), 1),
                          "wg_start_spread_us": round(statistics.median(spread), 2),
                          "phases_us": {p: round(statistics.median(v), 2) for p, v in ph.items()},
                          "qualifying_blocks": nq, "candidates": nc}), flush=True)
        del ix, tok, scores


if __name__ == "__main__":
    main()
