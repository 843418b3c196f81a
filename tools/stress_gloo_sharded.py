#!/usr/bin/env python3
"""Soak of the N > 1 main line (distributed.ShardedSearcher with the
torch.distributed exchange: stage 1 + 2 in one all-gather, stage 3 from the
gathered pool with no collective) for a bounded time.  Launch with
torch.distributed.run, every rank on cuda:0 over gloo (the one-GPU box's
rehearsal setup; the driver's node runs the same code over RCCL):

  BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nproc-per-node 2 \\
      --master-addr 127.0.0.1 --master-port 29541 tools/stress_gloo_sharded.py --seconds 150

Every rank draws the same random (dtype, B, k, kb, C, final_k) per step;
rank 0 also holds the whole corpus and checks every rank's result against
the unsharded stages called one by one (bit for bit).  A lab tool, not a
test."""
import argparse
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import bm25 as bm25_mod, synth  # noqa: E402
from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, shard_range  # noqa: E402
from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

BATCHES = (1, 2, 5, 8, 17, 64)
SHAPES = ((100, 100, 50, 10), (40, 30, 20, 7), (10, 1, 1, 1), (100, 0, 50, 10), (150, 50, 100, 50))  # k, kb, C, fk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--docs", type=int, default=60_000)
    a = ap.parse_args()
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    N, bmax = a.docs, max(BATCHES)
    Qf = synth.make_queries(bmax, seed=61)
    planted = synth.planted_ids(bmax, N, 10, seed=62)
    lo, hi = shard_range(N, rank, world)
    terms, off, V = synth.bm25_shard(lo, hi, planted)
    lex = bm25_mod.sharded(terms, off, V, id_base=lo)              # global statistics: one all-reduce
    qt, qo = synth.bm25_queries(bmax)
    searchers, full = {}, {}
    for kind in ("bf16", "fp32"):
        dt = torch.float32 if kind == "fp32" else torch.bfloat16
        tok, dl = synth.make_shard(lo, hi, Qf, planted, dev, dtype=dt)
        ix = ColbertIndex.faithful_f32(tok, dl, id_base=lo) if kind == "fp32" else ColbertIndex(tok, dl, id_base=lo)
        searchers[kind] = ShardedSearcher(ix, lexical_k=100)
        if rank == 0:
            ftok, fdl = synth.make_shard(0, N, Qf, planted, dev, dtype=dt)
            full[kind] = ColbertIndex.faithful_f32(ftok, fdl) if kind == "fp32" else ColbertIndex(ftok, fdl)
    if rank == 0:
        fterms, foff, _ = synth.bm25_shard(0, N, planted)
        lex_full = bm25_mod.NativeBM25(fterms, foff, V)
    rng = np.random.default_rng(8)          # the same draws on every rank
    t0 = time.time()
    t_print = t0
    steps = mism = misses = 0
    while True:
        go = torch.tensor([1 if time.time() - t0 < a.seconds else 0])
        dist.broadcast(go, 0)                                       # rank 0's clock ends the run everywhere
        if not int(go):
            break
        kind = ("bf16", "fp32")[rng.integers(2)]
        B = int(BATCHES[rng.integers(len(BATCHES))])
        b0 = int(rng.integers(0, bmax - B + 1))
        k, kb, C, fk = SHAPES[rng.integers(len(SHAPES))]
        ss = searchers[kind]
        Q = Qf[b0:b0 + B].to(dev, torch.float32 if kind == "fp32" else torch.bfloat16).contiguous()
        q_t, q_o = qt[qo[b0]:qo[b0 + B]], qo[b0:b0 + B + 1] - qo[b0]
        lexical = (lambda: lex.search(q_t, q_o, kb)) if kb else None
        _, ids, bm, pool = ss.search_hybrid(Q, k, lexical, return_pool=True)
        bm = bm.cpu().numpy() if isinstance(bm, torch.Tensor) else (bm if bm is not None
                                                                      else np.zeros((B, 0), np.int32))
        cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=60, C=C)
        s, i, p = ss.rerank(Q, torch.from_numpy(cand).to(dev), fk, pool=pool)
        got = torch.stack([s.view(torch.int32), i, p]).cpu()
        miss = int(ss.last_pool_misses) if ss.last_pool_misses is not None else 0
        outs = [torch.zeros_like(got) for _ in range(world)]
        dist.all_gather(outs, got)
        mv = torch.tensor([miss])
        dist.all_reduce(mv)
        steps += 1
        misses += int(mv)
        if rank == 0:
            fx = full[kind]
            _, fi = fx.search(Q, k)
            fbm = lex_full.search(q_t, q_o, kb)[0] if kb else np.zeros((B, 0), np.int32)
            fc = rrf_fuse(fbm, fi.cpu().numpy(), rrf_k=60, C=C)
            ws, wi, wp = fx.rerank(Q, torch.from_numpy(fc).to(dev), fk)
            want = torch.stack([ws.view(torch.int32), wi, wp]).cpu()
            bad = [r for r, o in enumerate(outs) if not torch.equal(o, want)]
            if bad or not np.array_equal(cand, fc):
                mism += 1
                if mism <= 5:
                    print(f"MISMATCH #{mism}: {kind} B={B} (k, kb, C, fk)={(k, kb, C, fk)} ranks {bad} "
                          f"cand_equal {np.array_equal(cand, fc)}", flush=True)
            if time.time() - t_print > 20:
                t_print = time.time()
                print(f"{t_print - t0:.0f}s: {steps} steps, {mism} mismatches, {misses} pool misses", flush=True)
    if rank == 0:
        print({"steps": steps, "mismatches": mism, "pool_misses": misses, "world": world,
               "seconds": round(time.time() - t0, 1), "docs": N}, flush=True)
    bad = torch.tensor([1 if (mism or misses) else 0])
    dist.broadcast(bad, 0)
    dist.destroy_process_group()
    sys.exit(int(bad))


if __name__ == "__main__":
    main()
