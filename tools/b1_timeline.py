#!/usr/bin/env python3
"""Where the B=1 latency goes: the one-round-trip path (hybrid.OneTripRetriever)
on one index, run --iters times back to back, for a rocprofv3 kernel +
memory-copy trace; then `--parse <dir>` folds the trace into a per-iteration
timeline (median over iterations): every kernel and copy after the scan, its
duration and the idle gap before it, and the scan-end -> last-event total.

  run:    rocprofv3 --kernel-trace --memory-copy-trace -f csv -d D -o t -- \
              python3 tools/b1_timeline.py --dtype fp32 --docs 1000000
  parse:  python3 tools/b1_timeline.py --parse D

--marks F (run) records the host timestamps of every timed call (monotonic
ns: Python entry, begin returned, cbv2_retrieve_host_marks of finish, exit,
synchronize returned) into F; `--parse D --marks F` prints them on the
kernel timeline (rocprofv3's timestamps are on the same clock when the first
kernel of an iteration starts a few us after the Python entry)."""
import argparse
import csv
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(a):
    import torch
    sys.path.insert(0, ROOT)
    from hybrid_rag_colbertv2_amd import bm25 as bm25_mod
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    dev = torch.device("cuda:0")
    n = a.docs
    Qf = synth.make_queries(256, 32, seed=1)
    planted = synth.planted_ids(256, n, 10, seed=2)
    terms, off, V = synth.bm25_shard(0, n, planted)
    lex = bm25_mod.sharded(terms, off, V, id_base=0, device=dev)
    del terms, off
    qt, qo = synth.bm25_queries(256)
    bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], 100)   # noqa: E731
    f32 = a.dtype in ("fp32", "both")
    tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0,
                                       dtype=torch.float32 if f32 else torch.bfloat16)
    ix = (ColbertIndex.faithful_f32(tokens, doclens) if f32 else
          ColbertIndex.mxfp8(tokens, doclens) if a.dtype == "fp8" else ColbertIndex(tokens, doclens))
    del tokens
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    legs = {a.dtype if a.dtype != "both" else "fp32":
            (OneTripRetriever(ix), Qf[:1].to(dev, torch.float32 if f32 else torch.bfloat16).contiguous())}
    if a.dtype == "both":   # a bf16 handle over the faithful index's hi: the same memory, interleaved
        legs["bf16"] = (OneTripRetriever(ColbertIndex(ix.tokens, ix.doclens)),
                        Qf[:1].to(dev, torch.bfloat16).contiguous())
    lat = {k: [] for k in legs}
    marks = []
    for name, (one, _) in legs.items():
        one.record_marks = bool(a.marks)
    for it in range(a.iters + 5):
        for name, (one, Q1) in legs.items():
            torch.cuda.synchronize()
            time.sleep(0.002)          # the GPU idles between queries, as in the bench's latency loop
            t = time.perf_counter()
            one(Q1, bm_one, host=bool(a.host))
            if not a.host:
                torch.cuda.synchronize()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            if it >= 5:
                lat[name].append((t1 - t) * 1e3)
                if a.marks:
                    marks.append(dict(one.marks, leg=name, it=it, synced=time.monotonic_ns()))
    if a.marks:
        with open(a.marks, "w") as f:
            for m in marks:
                f.write(json.dumps(m) + "\n")
        for name in legs:   # host-only view (valid without a profiler attached)
            ms = [m for m in marks if m["leg"] == name]
            med = lambda f: round(statistics.median(f(m) for m in ms) / 1e3, 1)   # noqa: E731
            print(json.dumps({"leg": name, "host_us": {
                "prep": med(lambda m: m["prep"] - m["enter"]),
                "begin_call": med(lambda m: m["begun"] - m["prep"]),
                "begin_return_to_finish": med(lambda m: m["finish"][0] - m["begun"]),
                "finish_to_D2H_issued": med(lambda m: m["finish"][1] - m["finish"][0]),
                "D2H_issued_to_wait_done": med(lambda m: m["finish"][2] - m["finish"][1]),
                "fusion": med(lambda m: m["finish"][3] - m["finish"][2]),
                "rerank_enqueue_or_host_select": med(lambda m: m["finish"][4] - m["finish"][3]),
                "finish_tail": med(lambda m: m["finish"][5] - m["finish"][4]),
                "finish_exit_to_python_exit": med(lambda m: m["exit"] - m["finish"][5]),
                "python_exit_to_synced": med(lambda m: m["synced"] - m["exit"]),
                "total": med(lambda m: m["synced"] - m["enter"])}}), flush=True)
    from hybrid_rag_colbertv2_amd.index import hbm_placement
    for name, v in lat.items():
        print(json.dumps({"docs": n, "dtype": name, "iters": a.iters, "p50_ms": round(statistics.median(v), 4),
                          "min_ms": round(min(v), 4), "placement": hbm_placement(ix.tokens)}), flush=True)


def short(name):
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return name.split("(")[0][:60]


def parse(d, scan_key, marks_path=None):
    kf = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    mf = glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True)
    ev = []
    for f in kf:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    for f in mf:
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "?")))
    ev.sort()
    groups, cur = [], []   # iterations: runs of events separated by > 1 ms idle (the sleep between queries)
    for e in ev:
        if cur and e[0] - max(x[1] for x in cur) > 1_000_000:
            groups.append(cur)
            cur = []
        cur.append(e)
    if cur:
        groups.append(cur)
    per_kind = {}
    marks = [json.loads(x) for x in open(marks_path)] if marks_path else []
    host = {}
    for g in groups:
        if not any(scan_key in e[2] for e in g):
            continue
        if marks:   # the call whose entry precedes this iteration's first kernel by < 1 ms
            t0 = g[0][0]
            near = [m for m in marks if 0 <= t0 - m["enter"] < 1_000_000]
            if near:
                m = max(near, key=lambda m: m["enter"])
                f = m["finish"]
                last_end = max(e[1] for e in g)
                copies = [e[1] for e in g if e[2].startswith("copy") and e[1] <= f[2]]
                row = {"python entry -> first kernel start": t0 - m["enter"],
                       "python prep (entry -> begin call)": m["prep"] - m["enter"],
                       "begin returned (from first kernel start)": m["begun"] - t0,
                       "finish entered": f[0] - t0, "D2H issued": f[1] - t0,
                       "wait done - D2H copy end": f[2] - max(copies) if copies else None,
                       "fusion": f[3] - f[2], "rerank enqueued / host select done - wait done": f[4] - f[2],
                       "finish exit - wait done": f[5] - f[2], "python exit - last kernel end": m["exit"] - last_end,
                       "synchronize returned - last kernel end": m["synced"] - last_end}
                host.setdefault(m["leg"], []).append(row)
        rows, prev = [], g[0][0]
        for (a, b, nm) in g:
            rows.append((nm, (b - a) / 1e3, max(0, a - prev) / 1e3))
            prev = max(prev, b)
        kind = "fp32-faithful" if any("split_query" in e[2] for e in g) else "bf16 / other"
        per_kind.setdefault(kind, []).append((rows, (prev - g[0][0]) / 1e3))
    if not per_kind:
        print("no iterations found")
        return
    for kind, per in per_kind.items():
        print(f"[{kind}]")
        _fold(per, scan_key)
    af = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)
    if af and marks:
        _api(af, marks, groups, scan_key)
    for leg, rows in host.items():
        print(f"[host marks, {leg}: {len(rows)} calls; medians in us]")
        for key in rows[0]:
            vals = [r[key] for r in rows if r[key] is not None]
            if vals:
                print(f"  {key:45s} {statistics.median(vals) / 1e3:9.1f}")


def _api(files, marks, groups, scan_key):
    """HIP runtime calls of each timed call (a --hip-runtime-trace run), from
    the Python entry to the call's exit: start offset from the entry and
    duration, medians over the calls of the modal call sequence, with the
    iteration's first kernel start and the scan's end on the same axis."""
    api = []
    for f in files:
        for r in csv.DictReader(open(f)):
            api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Function") or r.get("Operation", "?")))
    api.sort()
    per_leg = {}
    for g in groups:
        if not any(scan_key in e[2] for e in g):
            continue
        t0 = g[0][0]
        near = [m for m in marks if 0 <= t0 - m["enter"] < 1_000_000]
        if not near:
            continue
        m = max(near, key=lambda m: m["enter"])
        calls = [(a - m["enter"], b - a, nm) for (a, b, nm) in api if m["enter"] <= a <= m["exit"]]
        scan_end = max(e[1] for e in g if scan_key in e[2])
        per_leg.setdefault(m["leg"], []).append((calls, t0 - m["enter"], scan_end - m["enter"], m["exit"] - m["enter"]))
    for leg, per in per_leg.items():
        L = statistics.mode(len(c) for c, *_ in per)
        same = [p for p in per if len(p[0]) == L]
        print(f"[HIP calls, {leg}: {len(same)} of {len(per)} calls with the modal {L}; us from the Python entry]")
        for k in range(L):
            nm = same[0][0][k][2]
            st = statistics.median(p[0][k][0] for p in same) / 1e3
            du = statistics.median(p[0][k][1] for p in same) / 1e3
            print(f"  {st:9.1f} +{du:7.1f}  {nm}")
        for lab, j in (("first kernel start", 1), ("scan end", 2), ("python exit", 3)):
            print(f"  {statistics.median(p[j] for p in same) / 1e3:9.1f}           <{lab}>")


def _fold(per, scan_key):
    L = statistics.mode(len(r) for r, _ in per)
    same = [p for p in per if len(p[0]) == L]
    print(f"{len(per)} iterations ({len(same)} with the modal {L} events); medians:")
    tot_d = tot_g = scan = 0.0
    for k in range(L):
        nm = same[0][0][k][0]
        dur = statistics.median(p[0][k][1] for p in same)
        gap = statistics.median(p[0][k][2] for p in same)
        if scan_key in nm:
            scan = dur
        else:
            tot_d += dur
        tot_g += gap
        print(f"  {nm:60s} {dur:9.1f} us  gap {gap:7.1f} us")
    span = statistics.median(t for _, t in same)
    print(f"outside the scan: busy {tot_d:.1f} us + gaps {tot_g:.1f} us; first -> last event {span:.1f} us "
          f"(scan {scan:.1f} us)")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp8", "fp32", "both"],
                    help="both: the faithful index and a bf16 handle over its hi, interleaved in one process")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--parse", default=None, help="a rocprofv3 output directory to fold")
    ap.add_argument("--scan", default="maxsim_scan", help="substring naming the scan kernel")
    ap.add_argument("--marks", default=None, help="host timestamps file (run: written; parse: read)")
    ap.add_argument("--host", type=int, default=1, help="1: the call returns host results (cbv2_retrieve_finish_host)")
    a = ap.parse_args()
    if a.parse:
        parse(a.parse, a.scan, a.marks)
    else:
        run(a)
