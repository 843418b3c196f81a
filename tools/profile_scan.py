#!/usr/bin/env python3
"""Scan-only workload for rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE,
GRBM_GUI_ACTIVE, SQ_VALU_MFMA_BUSY_CYCLES: one counter per pass); --op search
runs cbv2_search (the fused scan + top-k the bench runs), --op score the
unfused scan that writes the [B, n] score matrix.

Builds the bench's synthetic 1M-doc index (bf16, or MXFP8 via the HIP
quantizer) and runs the MaxSim scan kernel (B=256) a few times;
tools/pmc_summary.py turns the counter CSVs into profiles/pmc_scan.json, which
bench.py reports as roofline.traffic.
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=1_000_000)
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16")
ap.add_argument("--op", choices=["search", "score"], default="search",
                help="search: cbv2_search top-100 (the fused scan, as the bench runs it); score: the unfused scan")
a = ap.parse_args()
dev = torch.device("cuda:0")
Qf = synth.make_queries(a.batch, 32, seed=1)
planted = synth.planted_ids(a.batch, a.docs, 10, seed=2)
if a.dtype == "fp8":
    q8, sc8, doclens = synth.make_shard_mxfp8(0, a.docs, Qf, planted, dev, seed=0)
    ix = ColbertIndex(q8, doclens, scales=sc8)
else:
    tokens, doclens = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0)
    ix = ColbertIndex(tokens, doclens)
Q = Qf.to(dev, torch.bfloat16)
for _ in range(a.reps):
    if a.op == "search":
        ix.search(Q, 100)
    else:
        ix.score(Q)
torch.cuda.synchronize()
print("done", a.dtype, a.docs, a.batch, a.reps)
