#!/usr/bin/env python3
"""Soak of the sharded one-trip retrieve inside the C ABI (NativeExchange over
the test-only in-process loopback communicator, G ranks on one GPU, one host
thread and stream per rank) against the UNSHARDED stages called one by one,
for a bounded time: random G in {2, 4, 8}, bf16 / fp32-faithful / MXFP8
shards, batch sizes, stage-1 widths below begin's kb (kb_ret) and device or
host results.  Every rank's result must equal the unsharded one bit for bit,
and every call must issue exactly its collectives (the stage-2 all-gather,
+1 for a faithful shard's band bound; no stage-3 all-reduce).  A lab tool
(GPU box), not a test.  usage: stress_sharded.py [--seconds S] [--docs N]"""
import argparse
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.bm25 import NativeBM25  # noqa: E402
from hybrid_rag_colbertv2_amd.distributed import NativeExchange, loopback_comms  # noqa: E402
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

K, KB, C, KF = 100, 100, 50, 10
BATCHES = (1, 1, 2, 3, 8, 17)


def composed(index, Q, lex_ids):
    _, ids = index.search(Q, K)
    cand = rrf_fuse(lex_ids, ids.cpu().numpy(), rrf_k=60, C=C)
    return index.rerank(Q, torch.from_numpy(cand).to(index.device), KF)


def run_ranks(G, fn):
    out, errs = [None] * G, []

    def body(r):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                out[r] = fn(r)
            s.synchronize()
        except BaseException as e:  # noqa: BLE001 - reported by the caller
            errs.append((r, repr(e)))

    ts = [threading.Thread(target=body, args=(r,)) for r in range(G)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return out, errs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--docs", type=int, default=60_000)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N, bmax = a.docs, max(BATCHES)
    Qf = synth.make_queries(bmax, seed=21)
    planted = synth.planted_ids(bmax, N, 10, seed=22)
    tok32, dl = synth.make_shard(0, N, Qf, planted, dev, dtype=torch.float32)
    dl[::7] = torch.randint(0, 129, (len(dl[::7]),), device=dev, dtype=torch.int32)
    dl[torch.from_numpy(planted.reshape(-1)).to(dev)] = 128
    tok16 = tok32.to(torch.bfloat16)
    terms, off, V = synth.bm25_shard(0, N, planted)
    df = NativeBM25.doc_freq(terms, off, V)
    stats = (N, int(off[-1]), df)
    lex_full = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(bmax)
    mk = {"bf16": lambda a_, b_: ColbertIndex(tok16[a_:b_].contiguous(), dl[a_:b_].contiguous(), id_base=a_),
          "fp8": lambda a_, b_: ColbertIndex.mxfp8(tok16[a_:b_].contiguous(), dl[a_:b_].contiguous(), id_base=a_),
          "fp32": lambda a_, b_: ColbertIndex.faithful_f32(tok32[a_:b_].contiguous(), dl[a_:b_].contiguous(),
                                                           id_base=a_)}
    full = {kind: mk[kind](0, N) for kind in mk}
    groups = {}
    for kind in mk:
        for G in (2, 4, 8):
            cuts = [N * g // G for g in range(G + 1)]
            ranges = list(zip(cuts[:-1], cuts[1:]))
            comms = loopback_comms(G)
            ones = [OneTripRetriever(NativeExchange(mk[kind](lo, hi), comm=comms[r]), colbert_k=K, fused=C,
                                     final_k=KF) for r, (lo, hi) in enumerate(ranges)]
            lex = [NativeBM25(terms[off[lo]:off[hi]], off[lo:hi + 1] - off[lo], V, id_base=lo, stats=stats)
                   for lo, hi in ranges]
            groups[kind, G] = (ones, lex)
    del tok32
    rng = np.random.default_rng(9)
    t0 = time.time()
    t_print = t0
    calls = mism = coll_bad = errors = 0
    while time.time() - t0 < a.seconds:
        kind = ("bf16", "fp32", "fp8")[rng.integers(3)]
        G = (2, 4, 8)[rng.integers(3)]
        B = int(BATCHES[rng.integers(len(BATCHES))])
        b0 = int(rng.integers(0, bmax - B + 1))
        kb_ret = int((100, 100, 60, 1)[rng.integers(4)])
        host = bool(rng.integers(2))
        ones, lex = groups[kind, G]
        Q = Qf[b0:b0 + B].to(dev, torch.float32 if kind == "fp32" else torch.bfloat16).contiguous()
        q_t, q_o = qt[qo[b0]:qo[b0 + B]], qo[b0:b0 + B + 1] - qo[b0]
        c0 = [o._owner.comm_stats() for o in ones]
        outs, errs = run_ranks(G, lambda r: (lambda x: x if host else [y.cpu() for y in x])(
            ones[r](Q, lambda: lex[r].search(q_t, q_o, kb_ret), host=host)))
        calls += 1
        if errs:
            errors += 1
            if errors <= 3:
                print(f"ERROR {kind} G={G} B={B}: {errs[:2]}", flush=True)
            continue
        bad_c = [r for r, o in enumerate(ones)
                 if tuple(np.subtract(o._owner.comm_stats(), c0[r])) != ((2 if kind == "fp32" else 1), 0)]
        if bad_c:
            coll_bad += 1
        bi, _ = lex_full.search(q_t, q_o, kb_ret)
        want = [x.cpu().numpy() for x in composed(full[kind], Q, bi)]
        torch.cuda.synchronize()
        ok = all(np.array_equal(np.asarray(g), w) for got in outs for g, w in zip(got, want))
        if not ok:
            mism += 1
            if mism <= 5:
                print(f"MISMATCH #{mism}: {kind} G={G} B={B} rows {b0}.. kb_ret {kb_ret} host {host}", flush=True)
                for r, got in enumerate(outs):
                    for nm, g, w in zip(("scores", "ids", "pos"), got, want):
                        g = np.asarray(g)
                        bad = np.argwhere(g != w)
                        if len(bad):
                            row = int(bad[0][0])
                            print(f"  rank {r} {nm}: {len(bad)} differ; row {row} got {g[row].tolist()} "
                                  f"want {w[row].tolist()}", flush=True)
        if time.time() - t_print > 20:
            t_print = time.time()
            print(f"{t_print - t0:.0f}s: {calls} calls, {mism} mismatches, {coll_bad} collective-count misses, "
                  f"{errors} errors", flush=True)
    print({"calls": calls, "mismatches": mism, "collective_count_misses": coll_bad, "errors": errors,
           "seconds": round(time.time() - t0, 1), "docs": N}, flush=True)
    sys.exit(1 if (mism or coll_bad or errors) else 0)


if __name__ == "__main__":
    main()
