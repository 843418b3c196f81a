#!/usr/bin/env python3
"""Soak of the one-round-trip retrieve (cbv2_retrieve_begin / _finish[_host],
hybrid.OneTripRetriever) against the same stages called one by one, for a
bounded time: random batch sizes (the host-rerank B <= 8 path, the GPU-rerank
path beyond), bf16 / fp32-faithful / MXFP8 shards, dense-doc (one-workgroup
B <= 2 scan with its task hand-off) and ragged indexes, a BM25 callable / a
host id array / no stage 1, device or host results.  Every call must equal
the composed stages bit for bit; the first mismatch is printed and counted.
A lab tool (GPU box), not a test: the tests pin each path once, this looks
for rare host/device protocol races over thousands of calls.  --threads T:
T host threads, each on its own stream with its own retrievers (the mapped
buffer pool is process-wide); --cancel P: a stage-1 callable raises with
probability P (the call is cancelled: cbv2_retrieve_cancel) and later calls
must still be right.
usage: stress_onetrip.py [--seconds S] [--docs N] [--threads T] [--cancel P]"""
import threading
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
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

K, KB, C, KF = 100, 100, 50, 10
SHAPES = ((100, 50, 10), (10, 1, 1), (200, 100, 50), (100, 100, 100), (40, 20, 7))   # --shapes: (k, C, final_k)
BATCHES = (1, 1, 1, 2, 2, 3, 5, 8, 17)


def composed(index, Q, lex_ids, k=K, c=C, kf=KF):
    _, ids = index.search(Q, k)
    bm = np.zeros((ids.shape[0], 0), np.int32) if lex_ids is None else lex_ids
    cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=60, C=c)
    return index.rerank(Q, torch.from_numpy(cand).to(index.device), kf)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--docs", type=int, default=125_000)
    ap.add_argument("--threads", type=int, default=1)
    ap.add_argument("--cancel", type=float, default=0.0)
    ap.add_argument("--shapes", action="store_true", help="random (k, C, final_k) per call (several layouts)")
    ap.add_argument("--ties", action="store_true", help="a corpus of copies of 300 docs (exact score ties)")
    ap.add_argument("--busy-stage1", action="store_true",
                    help="also a stage-1 callable that first runs a search on another shard (same stream)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bmax = max(BATCHES)
    Qf = synth.make_queries(bmax, seed=11)
    planted = synth.planted_ids(bmax, a.docs, 10, seed=12)
    tok32, dl = synth.make_shard(0, a.docs, Qf, planted, dev, dtype=torch.float32)
    if a.ties:   # every doc a copy of one of 300: exact ties in stage 2, the fusion and stage 3
        pick = torch.randint(0, 300, (a.docs,), device=dev, generator=torch.Generator(device=dev).manual_seed(3))
        tok32 = tok32[:300][pick].contiguous()
        dl = dl[:300][pick].contiguous()
    tok16 = tok32.to(torch.bfloat16)
    dl_ragged = dl.clone()
    dl_ragged[::3] = torch.randint(0, 129, (len(dl_ragged[::3]),), device=dev, dtype=torch.int32)
    dl_ragged[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128
    terms, off, V = synth.bm25_shard(0, a.docs, planted)
    lex = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(bmax)
    shards = {
        "bf16 dense": (ColbertIndex(tok16, dl), torch.bfloat16),
        "bf16 ragged": (ColbertIndex(tok16, dl_ragged), torch.bfloat16),
        "fp32 dense": (ColbertIndex.faithful_f32(tok32, dl), torch.float32),
        "fp8 dense": (ColbertIndex.mxfp8(tok16, dl), torch.bfloat16),
    }
    del tok32
    combos = {(b0, B): lex.search(qt[qo[b0]:qo[b0 + B]], qo[b0:b0 + B + 1] - qo[b0], KB)
              for B in set(BATCHES) for b0 in range(bmax - B + 1)}   # stage 1 once, off the threads
    t0 = time.time()
    stats = {"calls": 0, "mismatches": 0, "cancelled": 0, "per": {}}
    lock = threading.Lock()
    # the composed reference reuses the index object's own workspace: one
    # thread at a time per shard (the one-trip calls run unserialized)
    ref_lock = {name: threading.Lock() for name in shards}

    class Cancelled(RuntimeError):
        pass

    def worker(wid):
        rets = {}

        def ret(name, shape):   # one retriever per (shard, k / C / final_k): their buffers' layouts differ
            if (name, shape) not in rets:
                rets[name, shape] = OneTripRetriever(shards[name][0], colbert_k=shape[0], fused=shape[1],
                                                     final_k=shape[2])
            return rets[name, shape]
        rng = np.random.default_rng(5 + wid)
        stream = torch.cuda.Stream() if a.threads > 1 else torch.cuda.current_stream()
        prev = None
        t_print = t0
        with torch.cuda.stream(stream):
            while time.time() - t0 < a.seconds:
                name = list(shards)[rng.integers(len(shards))]
                ix, qdt = shards[name]
                B = int(BATCHES[rng.integers(len(BATCHES))])
                b0 = int(rng.integers(0, bmax - B + 1))
                Q = Qf[b0:b0 + B].to(dev, qdt).contiguous()
                bm_i, bm_s = combos[b0, B]
                mode = int(rng.integers(4 if a.busy_stage1 else 3))
                if a.cancel > 0 and rng.random() < a.cancel:   # a stage 1 that fails mid-call
                    def boom():
                        raise Cancelled()
                    try:
                        ret(name, (K, C, KF))(Q, boom, host=bool(rng.integers(2)))
                    except Cancelled:
                        pass
                    with lock:
                        stats["cancelled"] += 1
                    prev = (name, B, "cancelled")
                    continue
                if mode == 3:   # a stage 1 that runs GPU work of its own on the call's stream first
                    other_ix, other_qdt = shards[list(shards)[rng.integers(len(shards))]]

                    def busy(other_ix=other_ix, other_qdt=other_qdt, bm_i=bm_i, bm_s=bm_s):
                        other_ix.search(Qf[:2].to(dev, other_qdt).contiguous(), 50)
                        return bm_i, bm_s
                    lexical, lex_ids = busy, bm_i
                else:
                    lexical, lex_ids = (((lambda: (bm_i, bm_s)), bm_i) if mode == 0
                                        else ((bm_i, bm_i) if mode == 1 else (None, None)))
                host = bool(rng.integers(2))
                shape = SHAPES[rng.integers(len(SHAPES))] if a.shapes else (K, C, KF)
                got = ret(name, shape)(Q, lexical, host=host)
                with ref_lock[name]:
                    want = composed(ix, Q, lex_ids, *shape)
                    stream.synchronize()
                ok = all(np.array_equal(np.asarray(g if host else g.cpu()), w.cpu().numpy()) for g, w in zip(got, want))
                with lock:
                    stats["calls"] += 1
                    stats["per"][name] = stats["per"].get(name, 0) + 1
                    if not ok:
                        stats["mismatches"] += 1
                    mism = stats["mismatches"]
                if not ok and mism <= 6:
                    print(f"MISMATCH #{mism} (thread {wid}): {name} B={B} rows {b0}.. mode {mode} host {host}; "
                          f"previous call {prev}", flush=True)
                    for nm, g, w in zip(("scores", "ids", "pos"), got, want):
                        g = np.asarray(g if host else g.cpu())
                        w = w.cpu().numpy()
                        bad = np.argwhere(g != w)
                        if len(bad):
                            r = int(bad[0][0])
                            print(f"  {nm}: {len(bad)} entries differ, rows {sorted(set(int(x) for x in bad[:, 0]))}; "
                                  f"row {r} got {g[r].tolist()} want {w[r].tolist()}", flush=True)
                prev = (name, B, mode, host)
                if wid == 0 and time.time() - t_print > 20:
                    t_print = time.time()
                    print(f"{t_print - t0:.0f}s: {stats['calls']} calls, {stats['mismatches']} mismatches, "
                          f"{stats['cancelled']} cancelled", flush=True)

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(a.threads)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    calls, mism, per = stats["calls"], stats["mismatches"], stats["per"]
    print({"calls": calls, "mismatches": mism, "cancelled": stats["cancelled"], "per_shard": per,
           "seconds": round(time.time() - t0, 1), "docs": a.docs, "threads": a.threads}, flush=True)
    sys.exit(1 if mism else 0)


if __name__ == "__main__":
    main()
