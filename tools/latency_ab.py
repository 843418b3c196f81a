#!/usr/bin/env python3
"""B=1 latency of the whole hot path (host BM25 + scan + top-100 + RRF + rerank
top-10), the stages called one by one from Python (bench.py's ``step``) vs
the one-round-trip C++ path (hybrid.OneTripRetriever: cbv2_retrieve_begin /
_finish), interleaved in one process on the same index.  Prints one JSON line
per (docs, dtype) with p50 / p99 of each and the scan's own event time.

usage: latency_ab.py [--docs 125000,1000000] [--dtype bf16] [--iters 200] [--root TREE --tag T]
(--root: another tree's package, for a before/after of two builds on one box;
`one_trip_minus_scan_us` = one-trip p50 - the scan's own event p50.)"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "--root" in sys.argv:
    ROOT = os.path.abspath(sys.argv[sys.argv.index("--root") + 1])
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import bm25 as bm25_mod  # noqa: E402
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", default="125000,1000000")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8", "fp32"])
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--root", default=ROOT)
    ap.add_argument("--tag", default="")
    ap.add_argument("--ab-opt", default="",
                    help="OPT:v0,v1 -- the host-results one-trip leg once per value of that handle option "
                         "(cbv2_index_set_option, e.g. BAND_LOWER_BOUND:1,0), interleaved")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for n in (int(x) for x in a.docs.split(",")):
        B = 1
        Qf = synth.make_queries(256, 32, seed=1)
        planted = synth.planted_ids(256, n, 10, seed=2)
        terms, off, V = synth.bm25_shard(0, n, planted)
        lex = bm25_mod.sharded(terms, off, V, id_base=0, device=dev)
        del terms, off
        qt, qo = synth.bm25_queries(256)
        bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], 100)   # noqa: E731
        f32 = a.dtype == "fp32"
        tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0,
                                           dtype=torch.float32 if f32 else torch.bfloat16)
        ix = (ColbertIndex.faithful_f32(tokens, doclens) if f32 else
              ColbertIndex.mxfp8(tokens, doclens) if a.dtype == "fp8" else ColbertIndex(tokens, doclens))
        del tokens
        Q1 = Qf[:B].to(dev, torch.float32 if f32 else torch.bfloat16).contiguous()
        one = OneTripRetriever(ix)

        def composed():
            _, ids = ix.search(Q1, 100)
            bi, _ = bm_one()
            cand = rrf_fuse(bi, ids.cpu().numpy(), rrf_k=60, C=50)
            return ix.rerank(Q1, torch.from_numpy(cand).to(dev), 10)

        def onetrip():
            return one(Q1, bm_one)

        def onetrip_host():   # returns with the top-10 on the host: no synchronize in the timed region
            return one(Q1, bm_one, host=True)

        legs = {"composed": composed, "one_trip": onetrip}
        try:
            onetrip_host()
            legs["one_trip_host"] = onetrip_host
        except TypeError:     # a tree without host results
            pass
        ab_out = {}
        if a.ab_opt:
            from hybrid_rag_colbertv2_amd import _lib
            oname, vals = a.ab_opt.split(":")
            oid = getattr(_lib, "OPT_" + oname)
            for v in (int(x) for x in vals.split(",")):
                def leg(v=v):
                    ix.set_option(oid, v)
                    r = one(Q1, bm_one, host=True)
                    ix.set_option(oid, int(vals.split(",")[0]))
                    return r
                legs[f"one_trip_host[{oname}={v}]"] = leg
                ab_out[v] = leg()
        lat = {k: [] for k in legs}
        for it in range(a.iters + 5):
            for name, fn in legs.items():
                torch.cuda.synchronize()
                t = time.perf_counter()
                out = fn()
                if not name.startswith("one_trip_host"):
                    torch.cuda.synchronize()
                if it >= 5:
                    lat[name].append((time.perf_counter() - t) * 1e3)
        a_out, b_out = composed(), onetrip()
        same = all(torch.equal(x, y) for x, y in zip(a_out, b_out))
        if "one_trip_host" in legs:
            same = same and all(np.array_equal(x.cpu().numpy(), y) for x, y in zip(a_out, onetrip_host()))
        for r in ab_out.values():   # every option value: the same results
            same = same and all(np.array_equal(x.cpu().numpy(), y) for x, y in zip(a_out, r))
        band = None
        if f32:   # the faithful band of the query (docs rescored exactly), as the call sizes it
            ix.search(Q1, 100)
            band = int(getattr(ix, "last_band").cpu()[0])
        ix.time_scans(True)
        for _ in range(20):
            ix.search(Q1, 100)
        torch.cuda.synchronize()
        scan = statistics.median(ix.scan_times()[-20:])
        ix.time_scans(False)
        from hybrid_rag_colbertv2_amd import _lib
        rec = {"tag": a.tag, "lib": _lib.lib().cbv2_build_stamp().decode(), "docs": n, "dtype": a.dtype, "B": B,
               "iters": a.iters, "scan_event_ms_p50": round(scan, 4),
               "identical": same, "top10": [int(x) for x in b_out[1][0][:3]], "faithful_band_docs": band}
        for name, v in lat.items():
            rec[name] = {"p50_ms": round(statistics.median(v), 4), "p99_ms": round(float(np.percentile(v, 99)), 4),
                         "min_ms": round(min(v), 4)}
        rec["p50_gain_us"] = round((rec["composed"]["p50_ms"] - rec["one_trip"]["p50_ms"]) * 1e3, 1)
        rec["one_trip_minus_scan_us"] = round((rec["one_trip"]["p50_ms"] - scan) * 1e3, 1)
        for name in list(rec):
            if name.startswith("one_trip_host"):
                rec[name + "_minus_scan_us"] = round((rec[name]["p50_ms"] - scan) * 1e3, 1)
        print(json.dumps(rec), flush=True)
        del ix, one, lex


if __name__ == "__main__":
    main()
