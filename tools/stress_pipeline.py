#!/usr/bin/env python3
"""Soak of the bench's throughput path (hybrid.PipelinedRetriever: batch j+1's
scan enqueued before the host fuses batch j, pinned staging buffers reused
every other batch) against each batch run alone through the stages called
one by one, for a bounded time: random sequences of 1-6 batches of random
sizes (1-64) with stage-1 callables / host id arrays, over bf16 and
fp32-faithful shards of one index.  A lab tool (GPU box), not a test.
usage: stress_pipeline.py [--seconds S] [--docs N]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25  # noqa: E402
from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever, rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

K, KB, C, KF = 100, 100, 50, 10


def step(index, Q, lex_ids):
    _, ids = index.search(Q, K)
    cand = rrf_fuse(lex_ids, ids.cpu().numpy(), rrf_k=60, C=C)
    s, i, _ = index.rerank(Q, torch.from_numpy(cand).to(index.device), KF)
    return s, i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--docs", type=int, default=125_000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, qmax = a.docs, 64
    Qf = synth.make_queries(qmax, seed=51)
    planted = synth.planted_ids(qmax, N, 10, seed=52)
    tok32, dl = synth.make_shard(0, N, Qf, planted, dev, dtype=torch.float32)
    dl[::9] = torch.randint(0, 129, (len(dl[::9]),), device=dev, dtype=torch.int32)
    dl[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128
    terms, off, V = synth.bm25_shard(0, N, planted)
    lex = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(qmax)
    shards = {"bf16": (ColbertIndex(tok32.to(torch.bfloat16), dl), torch.bfloat16),
              "fp32": (ColbertIndex.faithful_f32(tok32, dl), torch.float32)}
    del tok32
    pipes = {name: PipelinedRetriever(ix, dev, colbert_k=K, fused=C, final_k=KF) for name, (ix, _) in shards.items()}
    rng = np.random.default_rng(6)
    t0 = time.time()
    t_print = t0
    seqs = batches = mism = 0
    while time.time() - t0 < a.seconds:
        name = ("bf16", "fp32")[rng.integers(2)]
        ix, qdt = shards[name]
        jobs, refs = [], []
        for _ in range(int(rng.integers(1, 7))):
            B = int(rng.integers(1, 65))
            b0 = int(rng.integers(0, qmax - B + 1))
            Q = Qf[b0:b0 + B].to(dev, qdt).contiguous()
            bm_i, bm_s = lex.search(qt[qo[b0]:qo[b0 + B]], qo[b0:b0 + B + 1] - qo[b0], KB)
            lexical = (lambda bm_i=bm_i, bm_s=bm_s: (bm_i, bm_s)) if rng.integers(2) else bm_i
            jobs.append((Q, lexical))
            refs.append((Q, bm_i))
        out = pipes[name].run(jobs)
        torch.cuda.synchronize()
        got = [(s.cpu(), i.cpu()) for s, i in out]
        for (Q, bm_i), (gs, gi) in zip(refs, got):
            ws, wi = step(ix, Q, bm_i)
            batches += 1
            if not (torch.equal(gs, ws.cpu()) and torch.equal(gi, wi.cpu())):
                mism += 1
                if mism <= 5:
                    print(f"MISMATCH #{mism}: {name} B={Q.shape[0]} (sequence of {len(jobs)})", flush=True)
        seqs += 1
        if time.time() - t_print > 20:
            t_print = time.time()
            print(f"{t_print - t0:.0f}s: {seqs} sequences, {batches} batches, {mism} mismatches", flush=True)
    print({"sequences": seqs, "batches": batches, "mismatches": mism, "seconds": round(time.time() - t0, 1),
           "docs": N}, flush=True)
    sys.exit(1 if mism else 0)


if __name__ == "__main__":
    main()
