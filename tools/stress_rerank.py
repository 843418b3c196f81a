#!/usr/bin/env python3
"""Soak of stage 3 (cbv2_rerank / cbv2_rerank_f32 through ColbertIndex.rerank:
gather-by-id MaxSim + the (score desc, position asc) select) against the
index's own score matrix for a bounded time: random batch sizes, candidate
counts C (1 .. 1,500: the LDS select and the multi-pass one), k (0 = the raw
scores), candidates drawn from the shard with duplicates, -1 paddings and
out-of-shard ids (which score -inf), over bf16 (dense, ragged), MXFP8 and
fp32-faithful indexes.  A lab tool (GPU box), not a test.
usage: stress_rerank.py [--seconds S]"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex  # noqa: E402

BATCHES = (1, 1, 2, 3, 5, 8, 9, 17, 33, 64)
CS = (1, 7, 50, 50, 100, 257, 1000, 1024, 1500)
BASE = 11


def expected(sc: torch.Tensor, cand: torch.Tensor, k: int):
    B, n = sc.shape
    loc = cand.long() - BASE
    ok = (loc >= 0) & (loc < n)
    raw = torch.where(ok, torch.gather(sc, 1, loc.clamp(0, n - 1)), torch.full_like(sc[:, :1], float("-inf")))
    if k == 0:
        return (raw,)
    s, p = torch.sort(raw, dim=1, descending=True, stable=True)   # ties: lower position first
    kk = min(k, cand.shape[1])
    out_s = torch.full((B, k), float("-inf"), device=sc.device)
    out_p = torch.full((B, k), -1, dtype=torch.int32, device=sc.device)
    out_i = torch.full((B, k), -1, dtype=torch.int32, device=sc.device)
    out_s[:, :kk] = s[:, :kk]
    out_p[:, :kk] = p[:, :kk].to(torch.int32)
    out_i[:, :kk] = torch.gather(cand, 1, p[:, :kk]).to(torch.int32)
    return out_s, out_i, out_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    qmax = max(BATCHES)
    idx = {}
    for name, n, ragged, kind in (("bf16 dense 50k", 50_000, False, "bf16"), ("bf16 ragged 60k", 60_001, True, "bf16"),
                                  ("fp8 dense 50k", 50_000, False, "fp8"), ("fp32 ragged 40k", 40_003, True, "fp32"),
                                  ("bf16 ties 50k", 50_000, "ties", "bf16"), ("fp32 ties 40k", 40_003, "ties", "fp32"),
                                  ("bf16 long512 20k", 20_003, "long512", "bf16"),
                                  ("fp32 long256 15k", 15_001, "long256", "fp32"),
                                  ("fp32 wild 30k", 30_011, "wild", "fp32"), ("bf16 wild 30k", 30_011, "wild", "bf16")):
        Qf = synth.make_queries(qmax, seed=41)
        planted = synth.planted_ids(qmax, n, 10, seed=42)
        if str(ragged).startswith("long"):   # long documents: ld token slots, random lengths up to ld
            ld = int(str(ragged)[4:])
            g = torch.Generator(device=dev).manual_seed(n)
            tok = torch.randn(n, ld, 128, device=dev, generator=g)
            tok = tok / tok.norm(dim=-1, keepdim=True)
            tok = tok if kind == "fp32" else tok.to(torch.bfloat16)
            dl = torch.randint(0, ld + 1, (n,), device=dev, generator=g, dtype=torch.int32)
        else:
            tok, dl = synth.make_shard(0, n, Qf, planted, dev,
                                       dtype=torch.float32 if kind == "fp32" else torch.bfloat16)
        if ragged == "wild":   # token norms over ~6 orders of magnitude
            g = torch.Generator(device=dev).manual_seed(n + 1)
            scale = torch.exp(torch.randn(n, 128, 1, device=dev, generator=g) * 2.5)
            tok = (tok.float() * scale).to(tok.dtype)
            dl = torch.randint(0, 129, (n,), device=dev, generator=g, dtype=torch.int32)
        if ragged == "ties":   # every doc a copy of one of 200: exact ties between candidates
            pick = torch.randint(0, 200, (n,), device=dev)
            tok = tok[:200][pick].contiguous()
            dl = dl[:200][pick].contiguous()
        elif ragged is True:
            dl[::5] = torch.randint(0, 129, (len(dl[::5]),), device=dev, dtype=torch.int32)
            dl[::89] = 0
        ix = (ColbertIndex.faithful_f32(tok, dl, id_base=BASE) if kind == "fp32" else
              ColbertIndex.mxfp8(tok, dl, id_base=BASE) if kind == "fp8" else ColbertIndex(tok, dl, id_base=BASE))
        Qs = Qf.float()
        if ragged == "wild":
            Qs = Qs * torch.exp(torch.randn(Qs.shape[0], Qs.shape[1], 1, generator=torch.Generator().manual_seed(5)) * 2)
        Q = Qs.to(dev, torch.float32 if kind == "fp32" else torch.bfloat16)
        idx[name] = (ix, Q, ix.score(Q).clone())     # every query's scores, once
        del tok
    rng = np.random.default_rng(4)
    t0 = time.time()
    t_print = t0
    calls = mism = 0
    while time.time() - t0 < a.seconds:
        name = list(idx)[rng.integers(len(idx))]
        ix, Qall, scall = idx[name]
        n = scall.shape[1]
        B = int(BATCHES[rng.integers(len(BATCHES))])
        C = int(CS[rng.integers(len(CS))])
        k = int((0, 1, 10, 50, C)[rng.integers(5)])
        b0 = int(rng.integers(0, qmax - B + 1))
        cand = rng.integers(BASE, BASE + n, size=(B, C))
        flip = rng.random((B, C))
        cand[flip < 0.05] = -1                                        # paddings
        cand[(flip >= 0.05) & (flip < 0.08)] = BASE + n + 3           # out of the shard
        cand[(flip >= 0.08) & (flip < 0.1)] = BASE - 2
        if C > 1:
            cand[:, -1] = cand[:, 0]                                  # a duplicate per row
        cand_d = torch.from_numpy(cand.astype(np.int32)).to(dev)
        Q = Qall[b0:b0 + B].contiguous()
        got = ix.rerank(Q, cand_d, k)
        got = got if isinstance(got, tuple) else (got,)
        want = expected(scall[b0:b0 + B], cand_d, k)
        ok = len(got) == len(want) and all(torch.equal(g, w) for g, w in zip(got, want))
        calls += 1
        if not ok:
            mism += 1
            if mism <= 5:
                print(f"MISMATCH #{mism}: {name} B={B} C={C} k={k} rows {b0}..", flush=True)
                for nm, g, w in zip(("scores", "ids", "pos"), got, want):
                    bad = (g != w)
                    if bool(bad.any()):
                        r = int(bad.any(dim=1).nonzero()[0])
                        c = int(bad[r].nonzero()[0])
                        print(f"  {nm}: {int(bad.sum())} differ; row {r} col {c} got {g[r, c].item()} "
                              f"want {w[r, c].item()}", flush=True)
        if time.time() - t_print > 20:
            t_print = time.time()
            print(f"{t_print - t0:.0f}s: {calls} calls, {mism} mismatches", flush=True)
    print({"calls": calls, "mismatches": mism, "seconds": round(time.time() - t0, 1)}, flush=True)
    sys.exit(1 if mism else 0)


if __name__ == "__main__":
    main()
