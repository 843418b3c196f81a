#!/usr/bin/env python3
"""A/B the scan-kernel variants in ONE process, interleaved rounds (guide §5.4
rule 24), on the bench's synthetic corpus; check every variant's scores
against variant 0 and the oracle.  usage: scan_lab.py [--docs N] [--batch B] [--rounds R] [--variants 0,1,2]"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402
from oracle import oracle as orc  # noqa: E402

LAB = os.path.join(ROOT, "tools", "_build", "libscanlab.so")


def build():
    src = os.path.join(ROOT, "tools", "scan_lab.hip")
    if not os.path.exists(LAB) or os.path.getmtime(LAB) < max(os.path.getmtime(src), os.path.getmtime(
            os.path.join(ROOT, "hybrid-rag-colbertv2_amd", "csrc", "colbert_mi355x.hip"))):
        os.makedirs(os.path.dirname(LAB), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                        "-fno-honor-nans", "-I", os.path.join(ROOT, "include"), src, "-o", LAB], check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=200_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--build-only", action="store_true")
    a = ap.parse_args()
    build()
    if a.build_only:
        return
    L = ctypes.CDLL(LAB)
    L.lab_scan.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(a.batch, 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 8), a.docs, 10, seed=2)[: a.batch]
    tokens, doclens = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0)
    # ragged tail so every variant's masking path runs
    doclens[-1000:] = torch.randint(0, 129, (1000,), device=dev, dtype=torch.int32)
    ix = ColbertIndex(tokens, doclens)
    Q = Qf.to(dev, torch.bfloat16)
    st = torch.cuda.current_stream()
    variants = [int(v) for v in a.variants.split(",")]
    outs = {v: torch.empty((a.batch, a.docs), device=dev) for v in variants}

    def run(v):
        rc = L.lab_scan(ix._h, v, Q.data_ptr(), a.batch, 32, outs[v].data_ptr(), a.docs, st.cuda_stream)
        assert rc == 0, rc

    for v in variants:
        run(v)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            run(v)
            e1.record(st)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1))
    # oracle on a slice (first 64 and last 200 docs, 8 queries)
    sl = torch.cat([torch.arange(64), torch.arange(a.docs - 200, a.docs)]).to(dev)
    nq = min(8, a.batch)
    ref = orc.maxsim(Q[:nq].float().cpu().numpy(), tokens[sl].float().cpu().numpy(), doclens[sl].cpu().numpy())
    flop = a.batch * a.docs * 2 * 32 * 128 * 128
    base = outs[variants[0]]
    for v in variants:
        med = statistics.median(times[v])
        got = outs[v][:nq, sl].cpu().numpy()
        fin = np.isfinite(ref)
        err = float(np.abs(got[fin] - ref[fin]).max())
        inf_ok = bool((np.isneginf(got) == np.isneginf(ref)).all())
        dv = float((outs[v] - base).abs().nan_to_num(0).max())
        gbs = a.docs * 32768 / med / 1e6
        print(f"B={a.batch} variant {v}: median {med:.3f} ms  min {min(times[v]):.3f}  {gbs:.0f} GB/s doc bytes  "
              f"{flop / med / 1e9:.1f} TFLOP/s "
              f"({flop / med / 1e9 / 2500 * 100:.1f}% of bf16 peak)  oracle_err {err:.2e} inf_ok {inf_ok} "
              f"max|d vs v{variants[0]}| {dv:.2e}", flush=True)


if __name__ == "__main__":
    main()
