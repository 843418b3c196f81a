#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one counter per pass) for one kernel.

usage: pmc_summary.py <out.json> <kernel-substr> <batch> <docs> <dtype> <variant> <csv>...
(variant: "fused" = the scan with the top-k fused in, "unfused" = the scan
that writes the score matrix)
Each CSV is a counter_collection.csv of one pass.  Per-launch values are the
median over the kernel's dispatches (min and max kept beside it).  Derived (MI355X_MICROARCH.md):
  hbm_bytes_per_launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024
      (gfx950: FETCH_SIZE reports half of a wide coalesced read; both in KB)
  clock_ghz = GRBM_GUI_ACTIVE / 8 / launch duration (summed over 8 XCDs)
The output file holds one entry per (kernel, dtype, batch, docs); an existing
entry for the same key is replaced.
"""
import csv
import json
import os
import sys

out_path, kernel, batch, docs, dtype = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
variant = sys.argv[6]
vals, durs = {}, []
for path in sys.argv[7:]:
    per = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel not in row.get("Kernel_Name", ""):
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            c = row["Counter_Name"]
            per.setdefault(c, {}).setdefault(d, 0.0)
            per[c][d] += float(row["Counter_Value"])
            if c.startswith("GRBM_GUI_ACTIVE"):
                durs.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    for c, byd in per.items():   # median over the dispatches: robust to one outlier launch
        v = sorted(byd.values())
        vals[c] = {"per_launch": v[len(v) // 2], "dispatches": len(v), "min": v[0], "max": v[-1]}
e = {"kernel": kernel, "dtype": dtype, "batch": batch, "docs_per_gpu": docs, "variant": variant, "counters": vals}
if "FETCH_SIZE" in vals and "WRITE_SIZE" in vals:
    e["hbm_bytes_per_launch"] = (2.0 * vals["FETCH_SIZE"]["per_launch"] + vals["WRITE_SIZE"]["per_launch"]) * 1024.0
    e["correction"] = "FETCH_SIZE x2 (gfx950 wide-read under-count), both KB x1024"
if "GRBM_GUI_ACTIVE" in vals and durs:
    d = sorted(durs)[len(durs) // 2]
    e["profiled_launch_s"] = d
    e["clock_ghz"] = vals["GRBM_GUI_ACTIVE"]["per_launch"] / 8.0 / d / 1e9
doc = {"entries": []}
if os.path.exists(out_path):
    with open(out_path) as f:
        old = json.load(f)
    key = (kernel, dtype, batch, docs, variant)
    doc.update({k: v for k, v in old.items() if k != "entries"})   # other sections kept as they are
    doc["entries"] = [x for x in old.get("entries", [])
                      if (x["kernel"], x.get("dtype"), x.get("batch"), x.get("docs_per_gpu"),
                          x.get("variant", "unfused")) != key]
doc["entries"].append(e)
with open(out_path, "w") as f:
    json.dump(doc, f, indent=1)
print(json.dumps(e))
