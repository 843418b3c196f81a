#!/usr/bin/env python3
"""fp32-faithful search of a corpus split into G shards in ONE process (what
each rank of a G-GPU run does): per shard, the search bounded by its own k-th
score vs by the GLOBAL bound (the k-th largest of all shards' faithful top-k
scores, as ShardedSearcher gathers them), band sizes and HIP-event times; and
whether the merge of the globally bounded shard lists equals the unsharded
search.

    python tools/shard_band.py [--docs 1000000] [--shards 8] [--batch 256] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.distributed import shard_range  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex, merge_topk  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--no-unsharded", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(a.batch, 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 8), a.docs, 10, seed=2)[: a.batch]
    Q = Qf.to(dev)
    full = None
    if not a.no_unsharded:
        f32, dl = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0, dtype=torch.float32)
        full = ColbertIndex.faithful_f32(f32, dl)
        del f32, dl
        torch.cuda.empty_cache()
    shards = []
    for r in range(a.shards):
        b0, b1 = shard_range(a.docs, r, a.shards)
        f32, dl = synth.make_shard(b0, b1, Qf, planted, dev, seed=0, dtype=torch.float32)
        shards.append(ColbertIndex.faithful_f32(f32, dl, id_base=b0))
        del f32, dl
        torch.cuda.empty_cache()
    fks = []
    for sh in shards:          # the all-gather's inputs: each shard's faithful scores of its bf16 top-k
        sh.search(Q, a.k, lb_reduce=lambda fk: fks.append(fk.clone()) or fk.min(dim=1).values)
    glob = torch.cat(fks, dim=1).topk(a.k, dim=1).values[:, a.k - 1]
    rows = []
    lists = []
    for r, sh in enumerate(shards):
        t_own, _ = timed(lambda: sh.search(Q, a.k), a.reps)
        band_own = float(sh.last_band.float().mean())
        t_glob, out = timed(lambda: sh.search(Q, a.k, lb_reduce=lambda fk: glob), a.reps)
        band_glob = float(sh.last_band.float().mean())
        lists.append(out)
        rows.append({"shard": r, "docs": sh.n, "ms_own_bound": round(t_own, 3), "ms_global_bound": round(t_glob, 3),
                     "band_own": round(band_own, 1), "band_global": round(band_glob, 1)})
        print(json.dumps(rows[-1]), flush=True)
    ms, mi = merge_topk(torch.stack([x[0] for x in lists]), torch.stack([x[1] for x in lists]), a.k)
    res = {"docs": a.docs, "shards": a.shards, "batch": a.batch, "k": a.k,
           "ms_own_bound_max": max(r["ms_own_bound"] for r in rows),
           "ms_global_bound_max": max(r["ms_global_bound"] for r in rows)}
    if full is not None:
        fs, fi = full.search(Q, a.k)
        res["merged_equals_unsharded"] = bool(torch.equal(mi, fi) and torch.equal(ms, fs))
        res["unsharded_band"] = round(float(full.last_band.float().mean()), 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
