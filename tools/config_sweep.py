#!/usr/bin/env python3
"""Stage-2 (MaxSim scan + top-k) timings for BASELINE.json's configs on ONE
MI355X, HIP events on the launching stream, synthetic corpus of bench.py:

  C2      100k docs, MaxSim-only top-100, B in {1, 16, 64, 256}
  C4/C5   one GPU's shard of 10M docs over 8 GPUs (1.25M docs), B=256, bf16 / MXFP8
  C3      1M docs at B in {1, 16, 64, 256} (the scan dispatch by batch size)

Each line: {"config", "docs", "batch", "dtype", "ms", "qps", "roofline"}; the
roofline is MFMA (B >= 16: B*n*1,048,576 FLOP / time vs 2.5 / 5.0 PF) or HBM
(B < 16: index bytes / time vs 8 TB/s).  usage: config_sweep.py [--out FILE]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

FLOP = 2 * 32 * 128 * 128


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def run(config, n, batches, dtype, out):
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(max(batches), 32, seed=1)
    planted = synth.planted_ids(max(batches), n, 10, seed=2)
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0)
    ix = ColbertIndex.mxfp8(tokens, doclens) if dtype == "fp8" else ColbertIndex(tokens, doclens)
    del tokens
    docbytes = 16384 + 256 if dtype == "fp8" else 32768
    for B in batches:
        Q = Qf[:B].to(dev, torch.bfloat16)
        ms = timed(lambda: ix.search(Q, 100))
        ids = ix.search(Q, 100)[1].cpu()
        ok = float(sum(set(ids[b, :10].tolist()) == set(planted[b].tolist()) for b in range(B)) / B)
        if B >= 16:
            ach = B * n * FLOP / (ms * 1e-3) / 1e12
            peak = 5000.0 if dtype == "fp8" else 2500.0
            roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4)}
        else:
            ach = n * docbytes / (ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                    "frac": round(ach / 8000.0, 4)}
        line = {"config": config, "docs": n, "batch": B, "dtype": dtype, "k": 100, "ms": round(ms, 3),
                "qps": round(B / (ms * 1e-3), 1), "roofline": roof, "top10_equals_planted": ok}
        print(json.dumps(line), flush=True)
        out.write(json.dumps(line) + "\n")
    del ix
    torch.cuda.empty_cache()


def run_long(n, ld, batches, out, dtype="bf16"):
    """Long documents (not a BASELINE config): n docs of ld token slots, all
    full, random unit tokens (the index bytes of n * ld / 128 standard docs).
    dtype bf16, fp8 (MXFP8) or fp32 (fp32-faithful: the whole certified search,
    priced against the bf16 scan's FLOP)."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
    tokens = torch.empty((n, ld, 128), dtype=tdt, device=dev)
    for a in range(0, n, 8192):
        x = torch.randn((min(8192, n - a), ld, 128), device=dev, generator=g)
        tokens[a:a + x.shape[0]] = (x / x.norm(dim=-1, keepdim=True)).to(tdt)
    doclens = torch.full((n,), ld, dtype=torch.int32, device=dev)
    if dtype == "fp8":
        ix = ColbertIndex.mxfp8(tokens, doclens)
    elif dtype == "fp32":
        ix = ColbertIndex.faithful_f32(tokens, doclens)
    else:
        ix = ColbertIndex(tokens, doclens)
    del tokens
    torch.cuda.empty_cache()
    Qf = synth.make_queries(max(batches), 32, seed=1)
    flop = 2 * 32 * ld * 128
    peak = 5000.0 if dtype == "fp8" else 2500.0
    docbytes = ld * 130 if dtype == "fp8" else ld * 256
    for B in batches:
        Q = Qf[:B].to(dev, torch.float32 if dtype == "fp32" else torch.bfloat16)
        ms = timed(lambda: ix.search(Q, 100))
        if B >= 16:
            ach = B * n * flop / (ms * 1e-3) / 1e12
            roof = {"bound": "mfma", "achieved": round(ach, 1), "peak": peak, "unit": "TFLOP/s",
                    "frac": round(ach / peak, 4)}
        else:
            ach = n * docbytes / (ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": 8000.0, "unit": "GB/s",
                    "frac": round(ach / 8000.0, 4)}
        line = {"config": f"long documents (ld={ld})", "docs": n, "ld": ld, "batch": B, "dtype": dtype, "k": 100,
                "ms": round(ms, 3), "qps": round(B / (ms * 1e-3), 1), "roofline": roof}
        if dtype == "fp32":
            line["band_mean"] = round(float(ix.last_band.float().mean()), 1)
        print(json.dumps(line), flush=True)
        out.write(json.dumps(line) + "\n")
    del ix
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "config_sweep.jsonl"))
    ap.add_argument("--long-only", action="store_true", help="only the long-document rows")
    ap.add_argument("--long-dtypes", default="bf16", help="comma list of bf16 / fp8 / fp32 for --long-only")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as out:
        if a.long_only:
            for dt in a.long_dtypes.split(","):
                run_long(250_000, 512, [1, 256], out, dt)
                run_long(125_000, 1024, [1, 256], out, dt)
            return
        run("C2 (100k docs, MaxSim-only top-100)", 100_000, [1, 16, 64, 256], "bf16", out)
        run("C3 stage 2 (1M docs)", 1_000_000, [1, 16, 64, 256], "bf16", out)
        run("C4 per-GPU shard (10M / 8)", 1_250_000, [256], "bf16", out)
        run("C5 per-GPU shard (10M / 8, MXFP8)", 1_250_000, [1, 256], "fp8", out)
        run_long(250_000, 512, [1, 256], out)


if __name__ == "__main__":
    main()
