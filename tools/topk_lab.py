#!/usr/bin/env python3
"""Where the B=1 block-max top-k spends its time (tools/topk_lab.hip): phase
durations of the production select (variant 0, s_memrealtime stamps at its
phase boundaries) and of the superblock-key variant (1), on the bench's 1M-doc
scores of one query; both checked against the production search's top-100.
usage: topk_lab.py [--docs N] [--batch B] [--reps R]"""
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

LAB = os.path.join(ROOT, "tools", "_build", "libtopklab.so")
PHASES = ("keys", "pass0", "pass1", "qualify", "gather", "rank+write")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--build", action="store_true")
    a = ap.parse_args()
    if a.build or not os.path.exists(LAB):
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-fno-honor-nans", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "tools", "topk_lab.hip"), "-o", LAB], check=True)
        if a.build:
            return
    lab = ctypes.CDLL(LAB)
    dev = torch.device("cuda:0")
    n, B, k = a.docs, a.batch, 100
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, n, 10, seed=2)
    tok, dl = synth.make_shard(0, n, Qf, planted, dev, seed=0)
    ix = ColbertIndex(tok, dl)
    Q = Qf.to(dev, torch.bfloat16)
    scores = ix.score(Q).contiguous()
    ref_s, ref_i = ix.search(Q, k)
    nb = (n + 63) // 64
    bm = torch.empty((B, nb + (n + 255) // 256), dtype=torch.int32, device=dev)   # block + superblock keys
    out_s = torch.empty((B, k), dtype=torch.float32, device=dev)
    out_i = torch.empty((B, k), dtype=torch.int32, device=dev)
    stamps = torch.zeros((B, 8), dtype=torch.int64, device=dev)
    st = _stream_ptr(dev)
    for variant in (0, 1, 2, 0, 1, 2):
        ph = {p: [] for p in PHASES}
        tot = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = lab.lab_topk_bmax(ctypes.c_void_p(scores.data_ptr()), B, ctypes.c_int64(n), k,
                                   ctypes.c_void_p(bm.data_ptr()), ctypes.c_void_p(out_s.data_ptr()),
                                   ctypes.c_void_p(out_i.data_ptr()), ctypes.c_void_p(stamps.data_ptr()), variant,
                                   ctypes.c_void_p(st))
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, rc
            tot.append(e0.elapsed_time(e1) * 1e3)
            s = stamps[0].tolist()
            for j, p in enumerate(PHASES):
                if variant != 2:                                  # the production kernel records no stamps
                    ph[p].append((s[j + 1] - s[j]) * 0.01)      # 100 MHz ticks -> us
        same = bool(torch.equal(out_s, ref_s) and torch.equal(out_i, ref_i))
        nq, nc = stamps[0, 7].item() >> 32, stamps[0, 7].item() & 0xffffffff
        print(json.dumps({"variant": variant, "docs": n, "B": B, "identical_to_search": same,
                          "block_max+select_event_us": round(statistics.median(tot), 1),
                          "phases_us": {p: round(statistics.median(v), 2) for p, v in ph.items() if v},
                          "qualifying_blocks": nq, "candidates": nc}), flush=True)


if __name__ == "__main__":
    main()
