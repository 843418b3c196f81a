"""Build libcolbert_mi355x.so in-tree (hipcc, gfx950).  Used by __graft_entry__.build().

Provenance: the library embeds a content stamp -- a SHA-256 prefix over the
compiler flags and the bytes of every source and header it is built from
(``source_stamp()``) -- returned by ``cbv2_build_stamp()``.  ``build_lib``
rebuilds whenever the library's embedded stamp differs from the tree's
(never on file times), and ``_lib.lib()`` refuses to load a library whose
stamp differs, so a shipped ``.so`` is used only if it was compiled from
exactly the sources beside it.
"""
from __future__ import annotations

import hashlib
import os
import re
import subprocess

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(PKG, "csrc", "colbert_mi355x.hip")
SRC_HOST = [os.path.join(PKG, "csrc", f) for f in ("host_bm25.cpp", "host_rrf.cpp", "sharded.cpp", "index_file.cpp", "text_en.cpp", "retrieve.cpp")]
HDR = os.path.join(ROOT, "include", "colbert_mi355x.h")
LIB = os.path.join(PKG, "libcolbert_mi355x.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -fno-honor-nans: lets fmaxf on MFMA results lower to bare v_max3_f32 (no
# canonicalising v_max per operand); the path never feeds NaNs on purpose.
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-honor-nans", "-pthread",
         "-Wall", "-Wno-unused-function"]
_STAMP_RE = re.compile(rb"cbv2-build-stamp:([0-9a-f]{16}|unstamped)")


def source_stamp() -> str:
    """SHA-256 prefix of the flags and the bytes of every input of the library."""
    h = hashlib.sha256()
    h.update(" ".join(FLAGS).encode())
    for path in (SRC, *SRC_HOST, HDR):
        with open(path, "rb") as f:
            data = f.read()
        h.update(os.path.basename(path).encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    return h.hexdigest()[:16]


def library_stamp(path: str = LIB):
    """The stamp embedded in a built library (read from its bytes, not loaded); None if absent."""
    if not os.path.exists(path):
        return None
    with open(path, "rb") as f:
        m = _STAMP_RE.search(f.read())
    return m.group(1).decode() if m else None


def build_lib(force: bool = False, verbose: bool = True) -> str:
    stamp = source_stamp()
    have = library_stamp()
    if force or have != stamp:
        cmd = [HIPCC, *FLAGS, f'-DCBV2_BUILD_STAMP="{stamp}"', "-I", os.path.join(ROOT, "include"), SRC, *SRC_HOST,
               "-ldl", "-o", LIB + ".tmp"]
        if verbose:
            print(f"[build] stamp {stamp} (library had {have}): " + " ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        os.replace(LIB + ".tmp", LIB)
    elif verbose:
        print(f"[build] {os.path.basename(LIB)} is current: stamp {stamp}", flush=True)
    return LIB
