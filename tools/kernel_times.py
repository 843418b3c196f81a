#!/usr/bin/env python3
"""Per-kernel launch count and median / mean duration from a rocprofv3
results database (rocpd SQLite, the default output of ROCm 7.2's rocprofv3).
usage: kernel_times.py <run_results.db> [...]"""
import re
import sqlite3
import statistics
import sys


def short(name):
    """Kernel name without argument list and namespace: 'topk_filter_kernel', 'maxsim_scan16x4_kernel<8, 4, ...>'."""
    n = re.sub(r"^void\s+", "", name)
    n = n.replace("(anonymous namespace)::", "")
    depth, out = 0, []
    for ch in n:                      # cut the parameter list (the first '(' at template depth 0)
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            break
        out.append(ch)
    return "".join(out).strip()


def main():
    for path in sys.argv[1:]:
        con = sqlite3.connect(path)
        by = {}
        for name, dur in con.execute("select name, duration from kernels"):
            by.setdefault(short(name), []).append(dur / 1e3)
        print(f"== {path}")
        for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
            print(f"  {len(v):4d} x  median {statistics.median(v):10.1f} us  mean {statistics.mean(v):10.1f} us  {k[:110]}")


if __name__ == "__main__":
    main()
