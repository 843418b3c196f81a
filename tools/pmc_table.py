#!/usr/bin/env python3
"""One rocprofv3 --pmc pass (counter_collection.csv) folded per kernel
(template arguments kept): per-dispatch medians of the SQ wave-state
fractions, MFMA-busy and the effective clock.  usage: pmc_table.py <csv> [substr]"""
import collections
import csv
import statistics
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:90]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    wall = {}
    for r in rows:
        if sub not in r["Kernel_Name"]:
            continue
        key = (short(r["Kernel_Name"]), r["Dispatch_Id"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        if "End_Timestamp" in r:
            wall[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    agg = collections.defaultdict(list)
    for (k, d), c in per.items():
        c = dict(c)
        if (k, d) in wall:
            c["wall_s"] = wall[(k, d)]
        agg[k].append(c)
    for k, lst in agg.items():
        c = {n: statistics.median(x.get(n, 0.0) for x in lst) for n in lst[0]}
        gui = c.get("GRBM_GUI_ACTIVE", 0.0) / 8            # summed over the 8 XCDs
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        out = {"dispatches": len(lst)}
        if "wall_s" in c and c["wall_s"] > 0:
            out["wall_ms"] = round(c["wall_s"] * 1e3, 3)
            if gui:
                out["clock_ghz"] = round(gui / c["wall_s"] / 1e9, 3)
        if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            out["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * gui), 3)
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                  "SQ_WAIT_INST_LDS"):
            if n in c:
                out[n.replace("SQ_", "").lower() + "_frac"] = round(c[n] / wc, 3)
        print(k, out)


if __name__ == "__main__":
    main()
