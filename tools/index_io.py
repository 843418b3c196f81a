#!/usr/bin/env python3
"""Native index file throughput on the GPU box (SURVEY §8 f2 measurement):
build the synthetic corpus in HBM, save it (HBM -> file), then load it back
whole and as 8 rank shards (file -> HBM, O_DIRECT where aligned) and check
the bytes.  usage: index_io.py [--docs N] [--dir /tmp]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.distributed import shard_range  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=250_000)
ap.add_argument("--dir", default="/tmp")
a = ap.parse_args()
dev = torch.device("cuda:0")
Qf = synth.make_queries(8)
planted = synth.planted_ids(8, a.docs, 10)
tokens, doclens = synth.make_shard(0, a.docs, Qf, planted, dev)
ix = ColbertIndex(tokens, doclens)
path = os.path.join(a.dir, "cbv2_io_test.cbv2")
nbytes = a.docs * 32768
torch.cuda.synchronize()
t = time.perf_counter()
ix.save(path)
w = time.perf_counter() - t
os.sync()
t = time.perf_counter()
back = ColbertIndex.load(path, device=dev)
torch.cuda.synchronize()
r_full = time.perf_counter() - t
ok = torch.equal(back.tokens, ix.tokens) and torch.equal(back.doclens, ix.doclens)
del back
t = time.perf_counter()
parts = [ColbertIndex.load(path, device=dev, begin=b, end=e) for b, e in (shard_range(a.docs, r, 8) for r in range(8))]
torch.cuda.synchronize()
r_sh = time.perf_counter() - t
ok = ok and all(torch.equal(p.tokens, ix.tokens[p.id_base:p.id_base + p.n]) for p in parts)
os.remove(path)
print(json.dumps({"docs": a.docs, "bytes": nbytes, "write_GBps": round(nbytes / w / 1e9, 2),
                  "read_full_GBps": round(nbytes / r_full / 1e9, 2), "read_8_shards_GBps": round(nbytes / r_sh / 1e9, 2),
                  "bit_exact": bool(ok)}))
