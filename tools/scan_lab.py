#!/usr/bin/env python3
"""A/B the scan-kernel variants in ONE process, interleaved rounds (guide §5.4
rule 24), on the bench's synthetic corpus; check every variant's scores
against variant 0 and a float64 torch MaxSim of a slice.  usage: scan_lab.py [--docs N] [--batch B] [--rounds R] [--variants 0,1,2]
Variants: an int = a production/lab scan variant (lab_scan); "f<frac>t<docs>" =
the production B > 16 scan with that dynamic-tail split (lab_scan16x4), e.g.
f0t128 (static), f0.1t128; a suffix k<kind> selects a lab kernel build of lab_scan16x4; a prefix "n:" runs the variant
from the alternate build (-D flags in env SCANLAB_ALT_DEFS)."""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402


def _dequant_mxfp8(q: torch.Tensor, sc: torch.Tensor) -> torch.Tensor:
    """e4m3 bytes [..., 128] + E8M0 scales [..., 2] -> f32 (one scale per 64 dims)."""
    v = q.contiguous().view(torch.float8_e4m3fn).float()
    return v * torch.exp2(sc.float() - 127.0).repeat_interleave(64, dim=-1)


def _maxsim_ref(Q: torch.Tensor, D: torch.Tensor, dl: torch.Tensor) -> torch.Tensor:
    """Plain torch float64 MaxSim of queries [q, 32, 128] over docs [n, L, 128]
    (rows >= doclens never score; empty docs -inf) -- the lab's check (the
    oracle is test infrastructure: tests, smoke and the bench's CPU baseline)."""
    sims = torch.einsum("qid,ntd->qnit", Q.double(), D.double())
    mask = torch.arange(D.shape[1], device=D.device)[None, :] >= dl[:, None].long()
    sims = sims.masked_fill(mask[None, :, None, :], float("-inf"))
    return sims.max(dim=-1).values.sum(dim=-1).float()

LAB = os.path.join(ROOT, "tools", "_build", "libscanlab.so")
# "n:" variants run in a second build with the -D flags of ALT_DEFS (env
# SCANLAB_ALT_DEFS; default: the round-1 CAS task grab of the dynamic tail)
LAB_NT = os.environ.get("SCANLAB_ALT_LIB") or os.path.join(ROOT, "tools", "_build", "libscanlab_alt.so")
ALT_DEFS = os.environ.get("SCANLAB_ALT_DEFS", "-DCBV2_TAIL_CAS=1").split()


def build():
    if os.environ.get("SCANLAB_NO_BUILD") == "1" and os.path.exists(LAB) and os.path.exists(LAB_NT):
        return   # (the GPU box: the libraries built in the container travel with the tree)
    src = os.path.join(ROOT, "tools", "scan_lab.hip")
    stamp = LAB_NT + ".defs"
    if not os.path.exists(stamp) or open(stamp).read() != " ".join(ALT_DEFS):
        if os.path.exists(LAB_NT):
            os.remove(LAB_NT)
    for lib, defs in ((LAB, []), (LAB_NT, ALT_DEFS)):
        if not os.path.exists(lib) or os.path.getmtime(lib) < max(os.path.getmtime(src), os.path.getmtime(
                os.path.join(ROOT, "hybrid-rag-colbertv2_amd", "csrc", "colbert_mi355x.hip"))):
            os.makedirs(os.path.dirname(lib), exist_ok=True)
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                            "-fno-honor-nans", *defs, "-I", os.path.join(ROOT, "include"), src, "-o", lib],
                           check=True)
    with open(stamp, "w") as f:
        f.write(" ".join(ALT_DEFS))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=200_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2,3,4")
    ap.add_argument("--build-only", action="store_true")
    ap.add_argument("--chain", type=int, default=1,
                    help="launches back to back between the timing events (reported per launch)")
    ap.add_argument("--dtype", choices=["bf16", "fp8"], default="bf16", help="fp8: lab_scan_f8 variants 0/1")
    ap.add_argument("--stamps", default="",
                    help="comma list of f<frac>t<docs> splits: after the A/B, run each with per-workgroup "
                         "s_memtime/s_memrealtime stamps and report the duration spread, tail and in-kernel clock")
    a = ap.parse_args()
    build()
    if a.build_only:
        return
    libs = {}
    for key, path in (("", LAB), ("n:", LAB_NT)):
        L = ctypes.CDLL(path)
        L.lab_scan.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.lab_scan_f8.argtypes = L.lab_scan.argtypes
        L.lab_scan16x4.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_int64, ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_int]
        libs[key] = L
    dev = torch.device("cuda:0")
    Qf = synth.make_queries(a.batch, 32, seed=1)
    planted = synth.planted_ids(max(a.batch, 8), a.docs, 10, seed=2)[: a.batch]
    tokens, doclens = synth.make_shard(0, a.docs, Qf, planted, dev, seed=0)
    # ragged tail so every variant's masking path runs
    doclens[-1000:] = torch.randint(0, 129, (1000,), device=dev, dtype=torch.int32)
    fp8 = a.dtype == "fp8"
    if fp8:
        from hybrid_rag_colbertv2_amd.index import quantize_mxfp8
        ix = ColbertIndex.mxfp8(tokens, doclens)
        Q = Qf.to(dev, torch.bfloat16)
        qq, qs = quantize_mxfp8(Q)
        qbuf = torch.cat([qq.reshape(-1), qs.reshape(-1)])
        qptr = qbuf.data_ptr()
        Qd = _dequant_mxfp8(qq, qs)
    else:
        ix = ColbertIndex(tokens, doclens)
        Q = Qf.to(dev, torch.bfloat16)
        qptr = Q.data_ptr()
    st = torch.cuda.current_stream()
    variants = a.variants.split(",")
    outs = {v: torch.empty((a.batch, a.docs), device=dev) for v in variants}

    def split(v):
        kind = 0
        if "k" in v:
            v, kind = v.split("k")
        fr, td = v[1:].split("t")
        return float(fr), int(td), int(kind)

    def run(v, stamps=None):
        L = libs["n:" if v.startswith("n:") else ""]
        v0 = v[2:] if v.startswith("n:") else v
        if v0.startswith("f"):
            fr, td, kind = split(v0)
            rc = L.lab_scan16x4(ix._h, qptr, a.batch, 32, outs[v].data_ptr(), a.docs, st.cuda_stream, fr, td,
                                stamps, kind)
        else:
            fn = L.lab_scan_f8 if fp8 else L.lab_scan
            rc = fn(ix._h, int(v0), qptr, a.batch, 32, outs[v].data_ptr(), a.docs, st.cuda_stream)
        assert rc == 0, rc

    for v in variants:
        run(v)
    torch.cuda.synchronize()
    times = {v: [] for v in variants}
    for _ in range(a.rounds):
        for v in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.chain):
                run(v)
            e1.record(st)
            e1.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.chain)
    # a float64 torch reference on a slice (first 64 and last 200 docs, 8 queries)
    sl = torch.cat([torch.arange(64), torch.arange(a.docs - 200, a.docs)]).to(dev)
    nq = min(8, a.batch)
    qref = Qd[:nq] if fp8 else Q[:nq].float()
    if fp8:   # the dequantized values of the slice
        dsl = _dequant_mxfp8(ix.tokens[sl], ix.scales[sl])
    else:
        dsl = tokens[sl].float()
    ref = _maxsim_ref(qref, dsl, doclens[sl]).cpu().numpy()
    flop = a.batch * a.docs * 2 * 32 * 128 * 128
    base = outs[variants[0]]
    for v in variants:
        med = statistics.median(times[v])
        got = outs[v][:nq, sl].cpu().numpy()
        fin = np.isfinite(ref)
        err = float(np.abs(got[fin] - ref[fin]).max())
        inf_ok = bool((np.isneginf(got) == np.isneginf(ref)).all())
        dv = float((outs[v] - base).abs().nan_to_num(0).max())
        gbs = a.docs * 32768 / med / 1e6
        print(f"B={a.batch} variant {v}: median {med:.3f} ms  min {min(times[v]):.3f}  {gbs:.0f} GB/s doc bytes  "
              f"{flop / med / 1e9:.1f} TFLOP/s "
              f"({flop / med / 1e9 / (5000 if fp8 else 2500) * 100:.1f}% of {a.dtype} peak)  ref_err {err:.2e} inf_ok {inf_ok} "
              f"max|d vs v{variants[0]}| {dv:.2e}", flush=True)
    for v in [x for x in a.stamps.split(",") if x] if not fp8 else []:
        outs.setdefault(v, torch.empty((a.batch, a.docs), device=dev))
        print(f"split {v}:", flush=True)
        stamps_report(lambda sp: run(v, sp))


def stamps_report(run_stamped, n_wg_max=1 << 16):
    """Per-workgroup [realtime start, end, memtime start, end] of the last of 3 stamped launches."""
    buf = torch.zeros((n_wg_max, 4), dtype=torch.int64, device="cuda")
    for _ in range(3):
        run_stamped(buf.data_ptr())
    torch.cuda.synchronize()
    st = buf.cpu().numpy()[:16384]                  # rows >= 16384 hold the per-wave phase sums
    st = st[st[:, 1] > 0]
    r0, r1, t0, t1 = (st[:, i].astype(np.float64) for i in range(4))
    dur = (r1 - r0) / 100.0                         # s_memrealtime: 100 MHz -> us
    clk = (t1 - t0) / (r1 - r0) * 0.1               # GHz
    span = (r1.max() - r0.min()) / 100.0
    print(f"stamps: {len(st)} workgroups; duration us min {dur.min():.1f} median {np.median(dur):.1f} "
          f"max {dur.max():.1f}; launch span {span:.1f} us; start skew {(r0.max() - r0.min()) / 100:.1f} us; "
          f"tail loss (span/median - 1) {span / np.median(dur) - 1:.2%}; clock GHz min {clk.min():.3f} "
          f"median {np.median(clk):.3f} max {clk.max():.3f}", flush=True)
    ph = buf.cpu().numpy()[16384:].astype(np.float64)          # per-wave phase cycles (s_memtime)
    wv = np.arange(len(ph)) % 8                                 # row 16384 + 8 * bid + wave
    keep = ph[:, 3] > 0
    ph, wv = ph[keep], wv[keep]
    for lo, hi in ((0, 4), (4, 8)):                            # SPLITLOAD: loader waves 0-3 vs 4-7
        sel = (wv >= lo) & (wv < hi)
        if sel.any():
            p2 = ph[sel]
            print(f"  waves {lo}-{hi - 1}: per iteration cycles wait {np.median(p2[:, 0] / p2[:, 3]):.0f} "
                  f"issue {np.median(p2[:, 1] / p2[:, 3]):.0f} compute {np.median(p2[:, 2] / p2[:, 3]):.0f}",
                  flush=True)
    if len(ph):
        tot = ph[:, :3].sum(axis=1)
        fr = ph[:, :3] / tot[:, None]
        print(f"phases over {len(ph)} waves (median fraction of loop cycles): wait {np.median(fr[:, 0]):.2%}  "
              f"issue {np.median(fr[:, 1]):.2%}  compute {np.median(fr[:, 2]):.2%}; per iteration cycles: "
              f"wait {np.median(ph[:, 0] / ph[:, 3]):.0f} issue {np.median(ph[:, 1] / ph[:, 3]):.0f} "
              f"compute {np.median(ph[:, 2] / ph[:, 3]):.0f}", flush=True)
    bid = np.nonzero(buf.cpu().numpy()[:16384, 1] > 0)[0]
    for x in range(8):
        sel = (bid & 7) == x
        if sel.any():
            print(f"  blockIdx%8={x}: duration median {np.median(dur[sel]):.1f} max {dur[sel].max():.1f} us, "
                  f"clock median {np.median(clk[sel]):.3f} GHz", flush=True)


if __name__ == "__main__":
    main()
