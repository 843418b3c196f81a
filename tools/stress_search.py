#!/usr/bin/env python3
"""Soak of the stage-2 selection (cbv2_search / cbv2_search_f32: block-max
top-k, radix selects, multi-pass k > 1,024, the faithful band) against the
index's own score matrix for a bounded time: random batch sizes and k over
bf16 (dense, ragged, tiny), MXFP8 and fp32-faithful indexes.  The expected
top-k is the score matrix (cbv2_score / cbv2_score_f32: the same bits the
scan gives the search) sorted by (score desc, id asc) with torch -- every
call must return exactly those scores and ids.  A lab tool (GPU box), not a
test.  usage: stress_search.py [--seconds S]"""
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

BATCHES = (1, 1, 2, 3, 4, 5, 8, 9, 16, 17, 33, 64, 100)
KS = (1, 10, 50, 100, 100, 128, 500, 1024, 1500)


def expected(sc: torch.Tensor, k: int, id_base: int):
    B, n = sc.shape
    kk = min(k, n)
    s, i = torch.sort(sc, dim=1, descending=True, stable=True)   # ties: lower id first
    out_s = torch.full((B, k), float("-inf"), device=sc.device)
    out_i = torch.full((B, k), -1, dtype=torch.int32, device=sc.device)
    out_s[:, :kk] = s[:, :kk]
    out_i[:, :kk] = (i[:, :kk] + id_base).to(torch.int32)
    return out_s, out_i


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    qmax = max(BATCHES)
    idx = {}
    for name, n, ragged, kind in (("bf16 dense 70k", 70_000, False, "bf16"),
                                  ("bf16 ragged 200k", 200_003, True, "bf16"),
                                  ("bf16 tiny 3k", 3_001, True, "bf16"),
                                  ("fp8 dense 70k", 70_000, False, "fp8"),
                                  ("fp32 dense 70k", 70_000, False, "fp32"),
                                  ("fp32 ragged 90k", 90_001, True, "fp32"),
                                  ("bf16 ties 70k", 70_000, "ties", "bf16"),
                                  ("fp32 ties 50k", 50_003, "ties", "fp32"),
                                  ("fp8 ties 70k", 70_000, "ties", "fp8"),
                                  ("bf16 long512 20k", 20_003, "long512", "bf16"),
                                  ("fp8 long256 20k", 20_000, "long256", "fp8"),
                                  ("fp32 long256 15k", 15_001, "long256", "fp32"),
                                  ("fp32 wild 30k", 30_011, "wild", "fp32"),
                                  ("bf16 wild 30k", 30_011, "wild", "bf16")):
        Qf = synth.make_queries(qmax, seed=31)
        planted = synth.planted_ids(qmax, n, 10, seed=32)
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
        if ragged == "wild":   # token norms over ~6 orders of magnitude: the faithful band's bound at every scale
            g = torch.Generator(device=dev).manual_seed(n + 1)
            scale = torch.exp(torch.randn(n, 128, 1, device=dev, generator=g) * 2.5)
            tok = (tok.float() * scale).to(tok.dtype)
            dl = torch.randint(0, 129, (n,), device=dev, generator=g, dtype=torch.int32)
        if ragged == "ties":   # every doc a copy of one of 300: exact score ties across the whole index
            pick = torch.randint(0, 300, (n,), device=dev)
            tok = tok[:300][pick].contiguous()
            dl = dl[:300][pick].contiguous()
        elif ragged is True:
            dl[::5] = torch.randint(0, 129, (len(dl[::5]),), device=dev, dtype=torch.int32)
            dl[::97] = 0                                     # empty docs (-inf)
        ix = (ColbertIndex.faithful_f32(tok, dl, id_base=7) if kind == "fp32" else
              ColbertIndex.mxfp8(tok, dl, id_base=7) if kind == "fp8" else ColbertIndex(tok, dl, id_base=7))
        Qs = Qf.float()
        if ragged == "wild":
            Qs = Qs * torch.exp(torch.randn(Qs.shape[0], Qs.shape[1], 1, generator=torch.Generator().manual_seed(5)) * 2)
        Q = Qs.to(dev, torch.float32 if kind == "fp32" else torch.bfloat16)
        idx[name] = (ix, Q)
        del tok
    rng = np.random.default_rng(3)
    t0 = time.time()
    t_print = t0
    calls = mism = 0
    per = {}
    while time.time() - t0 < a.seconds:
        name = list(idx)[rng.integers(len(idx))]
        ix, Qall = idx[name]
        B = int(BATCHES[rng.integers(len(BATCHES))])
        k = int(KS[rng.integers(len(KS))])
        b0 = int(rng.integers(0, qmax - B + 1))
        Q = Qall[b0:b0 + B].contiguous()
        s, i = ix.search(Q, k)
        es, ei = expected(ix.score(Q), k, 7)
        ok = torch.equal(s, es) and torch.equal(i, ei)
        calls += 1
        per[name] = per.get(name, 0) + 1
        if not ok:
            mism += 1
            if mism <= 5:
                bad = (s != es) | (i != ei)
                r = int(bad.any(dim=1).nonzero()[0])
                c = int(bad[r].nonzero()[0])
                print(f"MISMATCH #{mism}: {name} B={B} k={k} rows {b0}..: {int(bad.sum())} entries; row {r} col {c}: "
                      f"got ({float(s[r, c])}, {int(i[r, c])}) want ({float(es[r, c])}, {int(ei[r, c])})", flush=True)
        if time.time() - t_print > 20:
            t_print = time.time()
            print(f"{t_print - t0:.0f}s: {calls} calls, {mism} mismatches", flush=True)
    print({"calls": calls, "mismatches": mism, "per_index": per, "seconds": round(time.time() - t0, 1)}, flush=True)
    sys.exit(1 if mism else 0)


if __name__ == "__main__":
    main()
