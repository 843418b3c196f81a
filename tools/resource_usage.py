#!/usr/bin/env python3
"""Per-kernel register / spill / LDS usage of the gfx950 build (CPU only).

Compiles the device side of a .hip file with -Rpass-analysis=kernel-resource-usage
and prints one line per kernel matching the optional filter:
    python tools/resource_usage.py [filter] [--src path.hip]
"""
import argparse
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("filter", nargs="?", default="")
    ap.add_argument("--src", default=os.path.join(ROOT, "hybrid-rag-colbertv2_amd", "csrc", "colbert_mi355x.hip"))
    ap.add_argument("-D", action="append", default=[])
    a = ap.parse_args()
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-fno-honor-nans", "-c",
           "--offload-device-only", "-I", os.path.join(ROOT, "include"), a.src, "-o", "/tmp/_ru.o",
           "-Rpass-analysis=kernel-resource-usage"] + [f"-D{d}" for d in a.D]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    cur = None
    rows = []
    for line in out.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|VGPRs Spill|SGPRs Spill|LDS Size \[bytes/block\]|"
                      r"Occupancy \[waves/SIMD\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for r in rows:
        if a.filter and a.filter not in r["name"]:
            continue
        name = subprocess.run(["c++filt", r["name"]], capture_output=True,
                              text=True).stdout.strip()
        name = name.replace("(anonymous namespace)::", "")
        print(f"vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>3} vspill {r.get('VGPRs Spill', '?'):>3} "
              f"sspill {r.get('SGPRs Spill', '?'):>3} lds {r.get('LDS Size [bytes/block]', '?'):>6} "
              f"occ {r.get('Occupancy [waves/SIMD]', '?')}  {name[:150]}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
