#!/usr/bin/env python3
"""Host time before the first kernel of a B=1 one-trip call, with no profiler
attached (a latency lab).  A kernel trace times the first
kernel's start but its interception of every dispatch adds host time of its
own; this measures without it.  cbv2_set_begin_probe(1) makes begin poll for
the search's ready flags -- the first kernel's LAST store, system-scope, to
the call's mapped host buffer -- and stamp when the host saw them, so

  Python entry -> flags seen  >=  Python entry -> first kernel start

(the bound also holds the first kernel's run and the flag's trip to the host).
Per call (steady_clock ns, medians over --iters calls, the GPU idle 2 ms
before each as in the bench's latency loop): Python prep (entry -> the ctypes
call), ctypes -> begin entered, begin entered -> the search returned (every
launch enqueued), entry -> flags seen.  Run it bare and under rocprofv3
--kernel-trace to see what the trace adds.

  python3 tools/launch_latency.py --docs 125000 --dtype both"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=125_000)
    ap.add_argument("--dtype", default="both", choices=["bf16", "fp32", "both"])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--label", default="bare", help="names the run in the output (bare / traced)")
    ap.add_argument("--idle", default="sleep", choices=["sleep", "spin"],
                    help="how the host waits out the 2 ms between calls: sleep (the bench's latency loop) or "
                         "spin (the CPU stays awake)")
    a = ap.parse_args()
    import torch
    sys.path.insert(0, ROOT)
    from hybrid_rag_colbertv2_amd import _lib, bm25 as bm25_mod, synth
    from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    L = _lib.lib()
    L.cbv2_set_begin_probe.argtypes = [ctypes.c_int32]
    L.cbv2_set_begin_probe.restype = None
    L.cbv2_retrieve_begin_marks.argtypes = [ctypes.c_void_p, ctypes.c_int32]
    L.cbv2_retrieve_begin_marks.restype = ctypes.c_int
    dev = torch.device("cuda:0")
    n = a.docs
    Qf = synth.make_queries(8, 32, seed=1)
    planted = synth.planted_ids(8, n, 10, seed=2)
    terms, off, V = synth.bm25_shard(0, n, planted)
    lex = bm25_mod.sharded(terms, off, V, id_base=0, device=dev)
    qt, qo = synth.bm25_queries(8)
    bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], 100)   # noqa: E731
    f32 = a.dtype in ("fp32", "both")
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0,
                                       dtype=torch.float32 if f32 else torch.bfloat16)
    ix = ColbertIndex.faithful_f32(tokens, doclens) if f32 else ColbertIndex(tokens, doclens)
    del tokens
    torch.cuda.synchronize()
    legs = {"fp32" if f32 else "bf16": (OneTripRetriever(ix), Qf[:1].to(dev, torch.float32 if f32 else torch.bfloat16))}
    if a.dtype == "both":   # a bf16 handle over the faithful index's hi
        legs["bf16"] = (OneTripRetriever(ColbertIndex(ix.tokens, ix.doclens)), Qf[:1].to(dev, torch.bfloat16))
    for one, _ in legs.values():
        one.record_marks = True
    rows = {k: [] for k in legs}
    bm = (ctypes.c_int64 * 3)()
    L.cbv2_set_begin_probe(1)
    try:
        for it in range(a.iters + 10):
            for name, (one, Q1) in legs.items():
                Q1 = Q1.contiguous()
                torch.cuda.synchronize()
                if a.idle == "sleep":
                    time.sleep(0.002)
                else:
                    t_end = time.perf_counter() + 0.002
                    while time.perf_counter() < t_end:
                        pass
                one(Q1, bm_one, host=True)
                L.cbv2_retrieve_begin_marks(bm, 3)
                m = one.marks
                if it >= 10 and bm[2] > 0:
                    rows[name].append({"prep": m["prep"] - m["enter"], "ctypes_to_begin": bm[0] - m["prep"],
                                       "begin_to_search_returned": bm[1] - bm[0],
                                       "entry_to_flags_seen": bm[2] - m["enter"],
                                       "search_returned_to_flags_seen": bm[2] - bm[1]})
    finally:
        L.cbv2_set_begin_probe(0)
    for name, rs in rows.items():
        out = {"leg": name, "docs": n, "calls": len(rs), "run": a.label, "idle": a.idle}
        for key in (rs[0] if rs else {}):
            v = sorted(r[key] for r in rs)
            out[key + "_us"] = {"p50": round(statistics.median(v) / 1e3, 2), "p10": round(v[len(v) // 10] / 1e3, 2),
                                "p90": round(v[(9 * len(v)) // 10] / 1e3, 2)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
