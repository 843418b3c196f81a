#!/usr/bin/env python3
"""Median of one rocprofv3 --pmc counter per dispatch, grouped by kernel name
(template arguments kept, so the lab's variants stay apart).

usage: pmc_by_kernel.py <counter_collection.csv> [name-substring]"""
import collections
import csv
import statistics
import sys

per = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for row in csv.DictReader(open(sys.argv[1])):
    name = row["Kernel_Name"]
    if len(sys.argv) > 2 and sys.argv[2] not in name:
        continue
    d = row.get("Dispatch_Id") or row.get("Correlation_Id")
    per[name][d] += float(row["Counter_Value"])
    names[name] = row["Counter_Name"]
for name, byd in per.items():
    v = sorted(byd.values())
    short = name.split("(")[0].replace("(anonymous namespace)::", "")
    print(f"{names[name]} median {statistics.median(v):.4g} min {v[0]:.4g} max {v[-1]:.4g} n={len(v)}  {short[-140:]}")
