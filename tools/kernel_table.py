#!/usr/bin/env python3
"""Per-kernel durations from a rocprofv3 --kernel-trace CSV, grouped by kernel
and grid y (the batch for the row-parallel kernels: 256 = B=256 steps, 1 =
B=1 latency samples).  usage: kernel_table.py <..._kernel_trace.csv> [min_calls]"""
import collections
import csv
import re
import statistics
import sys


def short(name):
    name = name.replace("(anonymous namespace)::", "")
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)                       # drop the argument list
    return name[:60]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    min_calls = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    g = collections.defaultdict(list)
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        g[(short(r["Kernel_Name"]), r.get("Grid_Size_Y", "?"))].append(d)
    print(f"{'kernel':60s} {'grid_y':>7s} {'calls':>6s} {'median_us':>10s} {'mean_us':>10s} {'total_ms':>9s}")
    for (k, y), d in sorted(g.items(), key=lambda kv: -sum(kv[1])):
        if len(d) >= min_calls:
            print(f"{k:60s} {y:>7s} {len(d):6d} {statistics.median(d):10.1f} {statistics.mean(d):10.1f} "
                  f"{sum(d) / 1e3:9.2f}")


if __name__ == "__main__":
    main()
