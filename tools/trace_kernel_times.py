#!/usr/bin/env python3
"""Median duration of the top-k kernels in a rocprofv3 --kernel-trace CSV
(the filter split by batch: grid.y 256 = the B=256 steps, 1 = the B=1 latency
samples).  usage: trace_kernel_times.py <..._kernel_trace.csv>"""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for kn in ("topk_filter", "topk_select", "topk_rows", "select_small"):
    for y in ("256", "1"):
        d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
                   if kn in r["Kernel_Name"] and (r["Grid_Size_Y"] == y if kn == "topk_filter" else y == "256"))
        if d:
            print(kn, y, d[len(d) // 2], len(d))
