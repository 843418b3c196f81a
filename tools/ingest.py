#!/usr/bin/env python3
"""Bounded-memory ingest: encode a corpus in batches and
stream it into the native index file (or into HBM), never holding the corpus's
embeddings on the host.

    python tools/ingest.py --docs 1000000 --out /path/index.cbv2 [--dtype bf16|fp8] [--batch 4096]
    python tools/ingest.py --docs 1000000 --hbm [--dtype fp32]   # build the HBM index only

The encoder is the synthetic corpus's (synth.SyntheticDocEncoder: the bench's
1M-chunk corpus); with a real model, pass any object with encode(texts).
Prints one JSON line: docs, seconds, docs/s, peak host RSS growth, and a
top-10 = planted check of a B=64 search over the result.
"""
import argparse
import json
import os
import sys
import time

import psutil
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex, IndexBuilder, IndexWriter  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--dtype", choices=["bf16", "fp8", "fp32"], default="bf16",
                    help="fp32: the fp32-faithful index (hi + residual), --hbm only")
    ap.add_argument("--out", default=None, help="native index file to write")
    ap.add_argument("--hbm", action="store_true", help="build the HBM index instead of a file")
    a = ap.parse_args()
    if a.dtype == "fp32" and not a.hbm:
        ap.error("the fp32-faithful index is built in HBM (--hbm); its file form is ColbertIndex.save")
    dev = torch.device("cuda:0")
    B = 64
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, a.docs, 10, seed=2)
    enc = synth.SyntheticDocEncoder(Qf, planted, dev)
    proc = psutil.Process()
    rss0 = peak = proc.memory_info().rss
    t0 = time.time()
    sink = IndexBuilder(a.docs, dev, a.dtype) if a.hbm else IndexWriter(a.out, a.docs, a.dtype, device=dev)
    for s in range(0, a.docs, a.batch):
        sink.append(enc.encode(enc.texts(s, min(a.docs, s + a.batch))))
        peak = max(peak, proc.memory_info().rss)
    ix = sink.finish() if a.hbm else None
    if not a.hbm:
        sink.close()
    torch.cuda.synchronize()
    dt = time.time() - t0
    if ix is None:
        ix = ColbertIndex.load(a.out, device=dev)
    _, ids = ix.search(Qf.to(dev, torch.float32 if ix.faithful else torch.bfloat16), 100)
    ids = ids.cpu().numpy()
    ok = float(sum(set(ids[b, :10]) == set(planted[b]) for b in range(B)) / B)
    print(json.dumps({"docs": a.docs, "dtype": a.dtype, "sink": "hbm" if a.hbm else "file", "seconds": round(dt, 2),
                      "docs_per_s": round(a.docs / dt, 1), "host_rss_growth_gb": round((peak - rss0) / 2**30, 3),
                      "host_rss_gb": round(peak / 2**30, 3), "top10_equals_planted": ok}), flush=True)


if __name__ == "__main__":
    main()
