#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs for one kernel: per-launch HBM bytes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half of the
bytes of a wide coalesced read -> x2; WRITE_SIZE is exact for 16-B stores.
Both counters are in KB (x1024).
usage: pmc_summary.py <fetch_counter_collection.csv> <write_counter_collection.csv> <kernel-substr> <out.json> [batch docs]
"""
import csv
import json
import sys


def per_dispatch(path, kernel, counter):
    vals = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


fetch = per_dispatch(sys.argv[1], sys.argv[3], "FETCH_SIZE")
write = per_dispatch(sys.argv[2], sys.argv[3], "WRITE_SIZE")
f_avg = sum(fetch) / len(fetch)
w_avg = sum(write) / len(write)
out = {"kernel": sys.argv[3], "dispatches": [len(fetch), len(write)],
       "fetch_size_kb_raw": f_avg, "write_size_kb": w_avg,
       "hbm_bytes_per_launch": (2.0 * f_avg + w_avg) * 1024.0,
       "correction": "FETCH_SIZE x2 (gfx950 wide-read under-count), both KB x1024"}
if len(sys.argv) > 6:
    out["batch"], out["docs_per_gpu"] = int(sys.argv[5]), int(sys.argv[6])
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
