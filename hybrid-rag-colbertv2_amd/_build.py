"""Build libcolbert_mi355x.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build()."""
from __future__ import annotations

import os
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "colbert_mi355x.hip")
SRC_HOST = [os.path.join(PKG, "csrc", f) for f in ("host_bm25.cpp", "host_rrf.cpp", "sharded.cpp", "index_file.cpp", "text_en.cpp")]
HDR = os.path.join(ROOT, "include", "colbert_mi355x.h")
LIB = os.path.join(PKG, "libcolbert_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-honor-nans: lets fmaxf on MFMA results lower to bare v_max3_f32 (no
# canonicalising v_max per operand); the path never feeds NaNs on purpose.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-honor-nans", "-pthread",
         "-Wall", "-Wno-unused-function"]


def stale(out: str, deps) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build_lib(force: bool = False, verbose: bool = True) -> str:
    if force or stale(LIB, [SRC, *SRC_HOST, HDR, __file__]):
        cmd = [HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), SRC, *SRC_HOST, "-ldl", "-o", LIB + ".tmp"]
        if verbose:
            print("[build]", " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    return LIB
