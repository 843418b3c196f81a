#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of tools/small_shard_trace.py into searches
(windows separated by > 1 ms idle gaps that contain a MaxSim scan) and report,
per (docs, batch), the median of: each kernel's duration, the search's GPU
span (first start -> last end) and the idle gaps between its kernels.

usage: split_search_trace.py <kernel_trace.csv> <small_shard_trace stdout log>"""
import csv
import json
import statistics
import sys


def short_name(full: str) -> str:
    """'void (anonymous namespace)::maxsim_scan16x4_kernel<8, 4, ...>(...)' -> 'maxsim_scan16x4_kernel'."""
    name = full.replace("(anonymous namespace)::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].split("<")[0]


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    plan = None
    for line in open(sys.argv[2]):
        if line.startswith("PLAN "):
            plan = json.loads(line[5:])
    groups, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and s - last_end > 1_000_000 and cur:
            groups.append(cur)
            cur = []
        cur.append((short_name(r["Kernel_Name"]), s, e))
        last_end = max(last_end or e, e)
    if cur:
        groups.append(cur)
    searches = [g for g in groups if any("maxsim_scan" in k for k, _, _ in g)]
    i = 0
    for p in plan:
        mine = searches[i + p["warmup"]: i + p["searches"]]
        i += p["searches"]
        per = {}
        spans, gaps = [], []
        for g in mine:
            g = [x for x in g if "maxsim_scan" in x[0] or "topk" in x[0] or "select" in x[0] or "rocclr_fill" in x[0] or "block_max" in x[0]]
            spans.append((g[-1][2] - g[0][1]) / 1e3)
            gaps.append(sum(max(0, b[1] - a[2]) for a, b in zip(g, g[1:])) / 1e3)
            for k, s, e in g:
                per.setdefault(k, []).append((e - s) / 1e3)
        out = {"docs": p["docs"], "batch": p["batch"], "dtype": p["dtype"], "bmax": p.get("bmax"),
               "event_ms": p["event_ms_median"],
               "gpu_span_us": round(statistics.median(spans), 1), "idle_gaps_us": round(statistics.median(gaps), 1),
               "kernels_us": {k: round(statistics.median(v), 1) for k, v in per.items()},
               "launches_per_search": {k: len(v) // max(len(mine), 1) for k, v in per.items()}}
        print(json.dumps(out))


if __name__ == "__main__":
    main()
