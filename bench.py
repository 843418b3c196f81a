#!/usr/bin/env python3
"""Benchmark: queries/s (+ p50 latency) of the hybrid ColBERT retrieval path on a
1M-chunk x 128-token synthetic corpus, top-10 rerank (BASELINE.json metric,
config 3).

The headline line runs on the fp32-FAITHFUL index (the default, and the
package's: RAGConfig.index_dtype = "fp32"): the reference keeps fp32
embeddings and scores them in fp32 (LRC:735-746, 802-831), and this index
returns those scores within 1e-4 (bf16 hi scanned on the MFMA, every doc that
can reach the top-k rescored with the bf16 residual).

One STEP = one batch of B=256 queries through the whole path:
  stage 1  host BM25 top-100 (native C++, csrc/host_bm25.cpp) over the
           synthetic 1M-doc term corpus -- run while the GPU scans,
  stage 2  HIP MaxSim scan + top-100 (+ the faithful band: rescoring of the
           docs the bf16 scan cannot rule out); sharded over ranks: per-rank
           top-100 -> RCCL all-gather -> HIP merge (the ranks' BM25 lists over
           their doc shards ride the same all-gather),
  fusion   host RRF (native C++, reference semantics) -> top-50 candidates,
  stage 3  HIP gather-by-id MaxSim rerank -> top-10 (sharded: no collective -- the
           fused candidates' rerank scores ride the stage-2 all-gather: each
           rank's top-k scores and its prescored BM25 list).
Inputs (the query batch and term ids, both indexes) are resident before the
timed region; every stage runs in full inside every timed step.

The JSON line also carries, measured in the same run:
  bf16             (fp32 main) the same K steps + p50 on a bf16 index of the
                   same corpus (the faithful index's hi tokens, no copy);
                   `--dtype bf16` swaps the two (main bf16, side leg "faithful");
  roofline.band_ms the faithful band work per step (HIP events, timed region);
  native_exchange  (N > 1, RCCL) the same K steps with the exchange inside the
                   C ABI (cbv2_search_sharded_* / cbv2_rerank_sharded);
  cpu_baseline     (N = 1 only; null at N > 1) the CPU restatements timed on
                   this host (numpy fp32 BLAS = `value`; the scalar C
                   restatement; the literal mean-pool scorer), with the CPU
                   model and thread count;
  p50 / p99        single-query latency of the whole hot path.
Every optional leg agrees across ranks before its collectives (run_leg): a
rank that fails one records the error in the line with every other rank.

N>1: the SAME 1M-doc corpus is split into N contiguous shards, one per rank
(strong scaling); value = B*K / max-over-ranks wall time.

Run:  python bench.py [--gpus N --steps K --warmup W] [--dtype fp32|bf16|fp8]
      torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from hybrid_rag_colbertv2_amd import bm25 as bm25_mod  # noqa: E402
from hybrid_rag_colbertv2_amd import synth  # noqa: E402
from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, shard_range  # noqa: E402
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever, PipelinedRetriever, rrf_fuse  # noqa: E402
from hybrid_rag_colbertv2_amd.index import ColbertIndex, quantize_mxfp8  # noqa: E402

LQ, LD, DIM = 32, 128, 128
PEAK_FP8_TFLOPS = 5000.0                   # MI355X dense fp8 (block-scaled MFMA)
FLOP_PER_PAIR = 2 * LQ * LD * DIM          # 1,048,576 algorithmic FLOP per (query, doc)
PEAK_BF16_TFLOPS = 2500.0                  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
NOMINAL_GHZ = 2.4                          # the clock the dense peaks are quoted at (MI355X_MICROARCH.md: max clock)
JSON_FD = 1                                # set in main(): the real stdout, for the JSON line only
SCAN_KERNEL = "maxsim_scan16x4_kernel"    # the B=256 scan (auto dispatch: doc-interleaved tiles, 32 queries / workgroup)


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def host_info():
    model = platform.processor() or platform.machine()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def cpu_baseline(Q: torch.Tensor, tokens: torch.Tensor, n_total: int, budget_s: float):
    """The CPU restatements of the reference path, timed on this host on bounded
    samples of the same corpus and queries, extrapolated to n_total docs:
      numpy   oracle.maxsim fp32 (einsum -> max -> sum, BLAS threads) + top-100:
              the reference's own CPU arithmetic (torch fp32 on "cpu", LRC:802-831
              in its MaxSim form) -- this row is `value`;
      c       oracle/cbv2_oracle.c, scalar C (double accumulation, one core);
      literal the reference's code as written (LRC:821-829: mean-pool both sides,
              doc means recomputed per call, cosine), numpy float64.
    Threads: OMP_NUM_THREADS (the box's CPU share for this GPU) or the affinity
    mask -- this host's cores available to the process."""
    from threadpoolctl import threadpool_limits
    from oracle import oracle as orc
    info = host_info()
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or info["affinity_cpus"]
    n_s = min(20000, tokens.shape[0])
    docs = tokens[:n_s].float().cpu().numpy()
    q = Q.float().cpu().numpy()
    rows = []
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        s = orc.maxsim(q[:2], docs, dtype=np.float32)
        orc.topk(s, 100)
        per_q = (time.perf_counter() - t0) / 2
        b_s = int(max(2, min(q.shape[0], budget_s / max(per_q, 1e-6))))
        t0 = time.perf_counter()
        s = orc.maxsim(q[:b_s], docs, dtype=np.float32)
        orc.topk(s, 100)
        dt = time.perf_counter() - t0
        qps = b_s / (dt * n_total / n_s)
        rows.append({"impl": "numpy fp32 einsum->max->sum + top-100 (oracle.maxsim)", "value": round(qps, 6),
                     "cores": threads, "sample": f"{b_s} queries x {n_s} docs, {dt:.1f}s"})
        # literal scorer (per-call doc means, as LRC:822 recomputes them)
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < budget_s / 6 or reps == 0:
            orc.meanpool_cosine(q[reps % q.shape[0]: reps % q.shape[0] + 1], docs)
            reps += 1
        dt_l = time.perf_counter() - t0
        rows.append({"impl": "literal mean-pool cosine (LRC:821-829, doc means per call; oracle.meanpool_cosine)",
                     "value": round(reps / (dt_l * n_total / n_s), 6), "cores": threads,
                     "sample": f"{reps} queries x {n_s} docs, {dt_l:.1f}s"})
    try:   # scalar C restatement on the same bf16 values (oracle/cbv2_oracle.c)
        qb = Q[:1].to(torch.bfloat16).contiguous().cpu().view(torch.int16).numpy().view(np.uint16)
        n_c = 64
        t0 = time.perf_counter()
        while True:
            db = tokens[:n_c].to(torch.bfloat16).contiguous().cpu().view(torch.int16).numpy().view(np.uint16)
            t1 = time.perf_counter()
            orc.c_maxsim_bf16(qb, db, np.full(n_c, LD, np.int32))
            dt_c = time.perf_counter() - t1
            if dt_c > budget_s / 6 or n_c >= n_s or time.perf_counter() - t0 > budget_s / 3:
                break
            n_c *= 4
        rows.append({"impl": "scalar C, double accumulation (oracle/cbv2_oracle.c)",
                     "value": round(1.0 / (dt_c * n_total / n_c), 8), "cores": 1,
                     "sample": f"1 query x {n_c} docs, {dt_c:.2f}s"})
    except Exception as e:  # the C library is built by __graft_entry__.build(); report, do not fail
        rows.append({"impl": "scalar C (oracle/cbv2_oracle.c)", "error": str(e)[:200]})
    return {"value": round(qps, 6), "unit": "queries/s", "cores": threads, "kind": "port",
            "sample": f"{b_s} queries x {n_s} docs (fp32 numpy einsum->max->sum + top-100, "
                      f"{threads} BLAS threads, {dt:.1f}s), extrapolated to {n_total} docs",
            "cpu": info["cpu_model"], "nproc": info["nproc"], "affinity_cpus": info["affinity_cpus"],
            "omp_num_threads": info["omp_num_threads"], "rows": rows}


def timed_steps(run_steps, K, W, world, on_start=None):
    """W untimed warmup steps, then EXACTLY K steps bracketed by barrier + sync on
    both sides; returns (outputs, max-over-ranks elapsed seconds).  on_start()
    runs after the warmup, before the timed region (arms measurement records)."""
    if W:
        run_steps(W)
    if on_start is not None:
        on_start()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = run_steps(K)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        e = torch.tensor([elapsed], device=torch.device("cuda", torch.cuda.current_device()), dtype=torch.float64)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return outs, elapsed


def clock_view(flop_per_launch, avg_ms, peak_tflops, clock_ghz, nominal_ghz=NOMINAL_GHZ):
    """The roofline fraction split into this run's held clock and the MFMA
    busy fraction at that clock: frac = (clock / nominal) x busy, so
    flop_per_launch / (busy x peak x clock / nominal) reproduces avg_ms.
    clock_ghz: the scans' in-kernel clock probe of the timed region
    (cbv2_index_scan_clock); None -> no split."""
    achieved = flop_per_launch / (avg_ms * 1e-3) / 1e12
    if not clock_ghz:
        return {"clock_ghz_this_run": None, "mfma_busy_this_run": None}
    peak_at_clock = peak_tflops * clock_ghz / nominal_ghz
    busy = achieved / peak_at_clock
    return {"clock_ghz_this_run": round(clock_ghz, 4), "peak_tflops_at_this_clock": round(peak_at_clock, 1),
            "mfma_busy_this_run": round(busy, 4),
            "avg_ms_from_clock_and_busy": round(flop_per_launch / (busy * peak_at_clock * 1e12) * 1e3, 3)}


def main_line(qps, ms_per_step, p50, p99, native, native_is_main):
    """The numbers the line reports as its own.  At N > 1 the product's
    exchange is the one inside the C ABI (cbv2_search_sharded_* /
    cbv2_rerank_sharded); the torch.distributed exchange is the
    risk-free leg that runs first.  Once the native leg has validated on every
    rank (its results equal the torch exchange's, its one-trip results equal
    the stages', every top-10 planted), `value`, `ms_per_step`, p50 and p99
    come from it, with the torch.distributed numbers kept beside; otherwise
    (no native leg, a failed or unvalidated one) the torch.distributed numbers
    stay the line's.  With --native-exchange the main legs already ran native.
    Returns (dict of the line's numbers, dict of the torch exchange's or None)."""
    own = {"value": qps, "ms_per_step": ms_per_step, "p50_ms_b1": p50, "p99_ms_b1": p99}
    if native_is_main:
        return dict(own, exchange="native (--native-exchange)"), None
    if (native is not None and native.get("validated_on_every_rank") and native.get("value") is not None
            and native.get("ms_per_step") is not None and native.get("p50_ms_b1") is not None):
        return ({"value": native["value"], "ms_per_step": native["ms_per_step"], "p50_ms_b1": native["p50_ms_b1"],
                 "p99_ms_b1": native.get("p99_ms_b1"), "exchange": "native (validated on every rank)"},
                dict(own, exchange="torch.distributed"))
    return dict(own, exchange="torch.distributed" if native is not None else None), None


def gather_floats(vals, world, dev, backend):
    """Every rank's list of floats (same length on every rank) -> [rank][i] on all ranks."""
    if world == 1:
        return [list(vals)]
    t = torch.tensor(vals, dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
    out = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def spot_check(fs, fi_h, Qd, docs_fn, begin, end, queries, tol, world, dev):
    """Oracle MaxSim of the final top-10 of a few queries, each id checked on the
    rank that owns it; the mismatch count is summed over ranks."""
    from oracle import oracle as orc
    bad = 0
    for b in queries:
        pos = [j for j, x in enumerate(fi_h[b]) if begin <= x < end]
        if not pos:
            continue
        sel = torch.tensor([int(fi_h[b][j]) for j in pos], device=dev) - begin
        ref = orc.maxsim(Qd[b:b + 1], docs_fn(sel))[0]
        got = fs[b, pos].cpu().numpy()
        bad += int(np.abs(got - ref).max() > tol)
    if world > 1:
        t = torch.tensor([bad], device=dev, dtype=torch.int64)
        dist.all_reduce(t)
        bad = int(t.item())
    return bad


def c45_legs(args, B, world, rank, dev, backend):
    """BASELINE configs 4 and 5: ``args.c45_docs`` (10M) docs split into one
    contiguous shard per rank (1.25M at 8 ranks), B=256, stage 2 = scan +
    top-100 + ONE RCCL all-gather + HIP merge, K timed steps after W warmups:
    config 4 on bf16 tokens, config 5 on MXFP8 e4m3 tokens (block-scaled fp8
    MFMA).  Checks: the merged top-10 of every query = its planted docs.  Each
    config is a ``run_leg``: a rank whose shard build fails (e.g. out of
    memory) records the error with every other rank instead of stranding them
    in the all-gather."""
    n_c = args.c45_docs
    b, e = shard_range(n_c, rank, world)
    Qf = synth.make_queries(B, LQ, seed=1)
    planted = synth.planted_ids(B, n_c, 10, seed=2)
    Q = Qf.to(dev, torch.bfloat16)
    out = {"corpus_docs": n_c, "docs_per_gpu": e - b, "global_batch": B, "stage": "MaxSim top-100 + all-gather merge"}
    for name, fp8 in (("config4_bf16", False), ("config5_mxfp8", True)):
        def prepare(fp8=fp8, name=name):
            t0 = time.time()
            if fp8:
                q8, sc8, dl = synth.make_shard_mxfp8(b, e, Qf, planted, dev, seed=0)
                ix = ColbertIndex(q8, dl, id_base=b, scales=sc8)
            else:
                tok, dl = synth.make_shard(b, e, Qf, planted, dev, seed=0)
                ix = ColbertIndex(tok, dl, id_base=b)
            ix.search(Q, args.k)           # local only: allocates the search workspace before any collective
            torch.cuda.synchronize()
            log(f"{name}: shard [{b},{e}) built in {time.time() - t0:.1f}s")
            return ix

        def run(ix, fp8=fp8):
            srch = ShardedSearcher(ix, lexical_k=args.k)
            ix.time_scans(True)
            outs, el = timed_steps(lambda K: [srch.search(Q, args.k) for _ in range(K)], args.steps, args.warmup,
                                   world)
            scans = ix.scan_times()[-args.steps:]
            avg = sum(scans) / len(scans) if scans else float("nan")
            per_rank = [r[0] for r in gather_floats([avg], world, dev, backend)]
            ih = outs[-1][1].cpu().numpy()
            peak = PEAK_FP8_TFLOPS if fp8 else PEAK_BF16_TFLOPS
            achieved = B * (n_c // world) * FLOP_PER_PAIR / (max(per_rank) * 1e-3) / 1e12
            return {"value": round(B * args.steps / el, 2), "unit": "queries/s",
                    "ms_per_step": round(el / args.steps * 1e3, 3),
                    "scan_avg_ms_by_rank": [round(x, 3) for x in per_rank],
                    "roofline_frac_slowest_rank": round(achieved / peak, 4), "peak_tflops": peak,
                    "top10_equals_planted": float(np.mean([set(ih[q, :10]) == set(planted[q]) for q in range(B)])),
                    "sorted": bool((torch.diff(outs[-1][0], dim=1) <= 0).all().item())}

        out[name] = run_leg(name, prepare, run, world, rank, dev, backend)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    return out


def agree(ok: bool, world: int, dev, backend: str) -> bool:
    """True on every rank iff ``ok`` on every rank (one all-reduce MIN; no-op at N = 1)."""
    if world == 1:
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev if backend == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t.item()))


def _maybe_fail(name: str, rank: int):
    """Failure injection for the N > 1 rehearsals (never set by the driver):
    BENCH_FAIL_LEG=<leg> BENCH_FAIL_RANK=<r> raises inside that leg's local
    preparation on rank r only."""
    if os.environ.get("BENCH_FAIL_LEG") == name and int(os.environ.get("BENCH_FAIL_RANK", "-1")) == rank:
        raise RuntimeError(f"injected failure (BENCH_FAIL_LEG={name}, rank {rank})")


def run_leg(name: str, prepare, run, world: int, rank: int, dev, backend: str):
    """An optional leg of the line, with symmetric failure handling across ranks.

    ``prepare()`` does the leg's LOCAL work (index build, workspace warm-up with
    a local search; no collectives) and may fail on one rank only (e.g. an OOM
    from uneven free memory); ``run(state)`` runs the leg's collectives.  The
    ranks agree (one all-reduce MIN) after ``prepare``: every rank then either
    enters ``run`` or records the same error, so a failing rank never strands
    its peers inside a collective.  ``run`` executes the same code on the same
    shapes on every rank; its result is agreed on again afterwards.  Returns
    the leg's dict, or {"error": ...} (the line still prints)."""
    state, err = None, None
    try:
        _maybe_fail(name, rank)
        state = prepare()
    except Exception as e:   # noqa: BLE001  reported in the line
        err = f"{type(e).__name__}: {str(e)[:300]}"
    if not agree(err is None, world, dev, backend):
        state = None
        if dev.type == "cuda":
            torch.cuda.synchronize()
            torch.cuda.empty_cache()
        return {"error": err or f"{name}: failed on another rank (local preparation)"}
    out, err = None, None
    try:
        out = run(state)
    except Exception as e:   # noqa: BLE001
        err = f"{type(e).__name__}: {str(e)[:300]}"
    if not agree(err is None, world, dev, backend):
        out = {"error": err or f"{name}: failed on another rank"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--docs", type=int, default=1_000_000)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--fused", type=int, default=50)
    ap.add_argument("--final-k", type=int, default=10)
    ap.add_argument("--p50-iters", type=int, default=100)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side-leg", "--no-faithful", dest="no_side_leg", action="store_true",
                    help="skip the side leg (fp32 main: the bf16 leg; bf16 main: the fp32-faithful leg)")
    ap.add_argument("--check-queries", type=int, default=8)
    ap.add_argument("--no-pipeline", action="store_true", help="time unpipelined steps")
    ap.add_argument("--native-exchange", action="store_true",
                    help="N>1: the MAIN timing uses the exchange inside the C ABI (the native leg always runs too)")
    ap.add_argument("--fused-topk", action="store_true", help="stage 2 with the top-k fused into the scan (A/B)")
    ap.add_argument("--c45", choices=["auto", "on", "off"], default="auto",
                    help="BASELINE configs 4 / 5 (10M docs sharded over the ranks, stage 2, bf16 and MXFP8) as "
                         "extra legs of the line; auto = at 8 ranks (the configs' node)")
    ap.add_argument("--c45-docs", type=int, default=10_000_000, help="corpus of the config-4/5 legs")
    ap.add_argument("--replicas", action="store_true",
                    help="N>1: query-level data-parallel replicas (SURVEY §8(e), the alternative for config 3): "
                         "every rank holds the WHOLE corpus and runs its own query batches, no collective; "
                         "value = N x the per-rank rate (weak scaling).  Default: the corpus sharded (strong).")
    ap.add_argument("--dtype", choices=["fp32", "bf16", "fp8"], default="fp32",
                    help="index: fp32-faithful (default: the reference's fp32 arithmetic, LRC:735-746 / 802-831, "
                         "within 1e-4 -- bf16 hi scanned + residual-certified band, DESIGN §3.7), bf16 tokens, "
                         "or MXFP8 e4m3 + E8M0 (config 5)")
    args = ap.parse_args()
    # stdout carries exactly the ONE JSON line: everything else any layer prints
    # to fd 1 (Python, RCCL / gloo C++ logging) is sent to stderr from here on
    global JSON_FD
    JSON_FD = os.dup(1)
    os.dup2(2, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal knobs for a one-GPU box (never used by the driver): several ranks
    # on cuda:0 over gloo.  The real multi-GPU run is one rank per GPU over RCCL.
    backend = os.environ.get("BENCH_BACKEND", "nccl")
    if os.environ.get("BENCH_SAME_DEVICE") == "1":
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    B, n_total = args.batch, args.docs
    replicas = args.replicas and world > 1
    begin, end = (0, n_total) if replicas else shard_range(n_total, rank, world)
    n_local = end - begin
    t_setup = time.time()
    Qf = synth.make_queries(B, LQ, seed=1)
    planted = synth.planted_ids(B, n_total, 10, seed=2)
    t_bm = time.time()
    bm_terms, bm_off, vocab = synth.bm25_shard(begin, end, planted)
    if replicas:   # the whole BM25 index on every rank (its own statistics: no all-reduce)
        lex = bm25_mod.NativeBM25(bm_terms, bm_off, vocab)
    else:
        lex = bm25_mod.sharded(bm_terms, bm_off, vocab, id_base=begin, device=dev)   # global stats: 1 all-reduce
    del bm_terms, bm_off
    qt, qo = synth.bm25_queries(B)
    log(f"host BM25 shard built in {time.time() - t_bm:.1f}s ({lex.n_docs} docs, {len(lex.doc_terms)} terms)")
    bm_all = lambda: lex.search(qt, qo, args.k)                 # noqa: E731  stage 1, whole batch
    bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], args.k)     # noqa: E731  stage 1, query 0
    faithful = args.dtype == "fp32"
    fp8 = args.dtype == "fp8"
    tokens, doclens = synth.make_shard(begin, end, Qf, planted, dev, seed=0,
                                       dtype=torch.float32 if faithful else torch.bfloat16)
    if faithful:
        # fp32-faithful index: bf16 hi scanned, bf16 residual gathered for the band (HIP split)
        ix = ColbertIndex.faithful_f32(tokens, doclens, id_base=begin)
    elif fp8:
        ix = ColbertIndex.mxfp8(tokens, doclens, id_base=begin)   # quantized on the GPU (HIP kernel)
    else:
        ix = ColbertIndex(tokens, doclens, id_base=begin)
    if args.fused_topk:
        from hybrid_rag_colbertv2_amd import _lib
        ix.set_option(_lib.OPT_FUSED_TOPK, 1)
    nccl = world > 1 and backend == "nccl" and not replicas
    searcher = (ShardedSearcher(ix, world=1, lexical_k=args.k) if replicas else   # a replica: the one-shard path
                ShardedSearcher(ix, native=args.native_exchange and nccl, lexical_k=args.k))
    Q = Qf.to(dev, torch.float32 if faithful else torch.bfloat16)
    Q1 = Q[:1].contiguous()
    torch.cuda.synchronize()
    log(f"setup {time.time() - t_setup:.1f}s: rank {rank}/{world} docs [{begin},{end}) B={B} index {args.dtype}")

    def step(srch, Qb, lexical):
        """One batch, unpipelined (used for the B=1 latency)."""
        _, ids, bm, pool = srch.search_hybrid(Qb, args.k, lexical, return_pool=True)
        bm = bm.cpu().numpy() if isinstance(bm, torch.Tensor) else bm
        cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=60, C=args.fused)
        cand_d = torch.from_numpy(cand).to(dev, non_blocking=False)
        return srch.rerank(Qb, cand_d, args.final_k, pool=pool)   # sharded: scores from the pool, no collective

    def stepper(srch, Qb):
        # K batches through the software-pipelined path (batch j+1's scan runs on
        # the GPU while the host runs its BM25 and fuses batch j; PipelinedRetriever)
        pipe = PipelinedRetriever(srch, dev, colbert_k=args.k, fused=args.fused, final_k=args.final_k)
        if args.no_pipeline:
            return lambda K: [step(srch, Qb, bm_all)[:2] for _ in range(K)]
        return lambda K: pipe.run([(Qb, bm_all)] * K)

    def one_trip(srch):
        if srch.world > 1 and srch._nx is None:
            return None
        return OneTripRetriever(srch, colbert_k=args.k, fused=args.fused, final_k=args.final_k, lexical_k=args.k)

    def latency(srch, Qb, one=None):
        lat = []
        for it in range(args.p50_iters + 3):
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t = time.perf_counter()
            if one is not None:
                one(Qb, bm_one, host=True)   # returns with the top-10 on the host (LRC:935 returns host results)
            else:
                step(srch, Qb, bm_one)
                torch.cuda.synchronize()
            if it >= 3:
                lat.append((time.perf_counter() - t) * 1e3)
        return lat, (statistics.median(lat) if lat else None), (float(np.percentile(lat, 99)) if lat else None)

    def same_as_step(srch, one, Qb):
        """The one-trip result equals the stages called one by one (bit for bit)."""
        a, b, h = step(srch, Qb, bm_one), one(Qb, bm_one), one(Qb, bm_one, host=True)
        return (all(torch.equal(x, y) for x, y in zip(a, b))
                and all(np.array_equal(x.cpu().numpy(), y) for x, y in zip(a, h)))

    def planted_frac(ids_h):
        return float(np.mean([set(ids_h[b]) == set(planted[b]) for b in range(B)]))

    # ---- the main leg: K timed steps.  The scan launches (and, fp32-faithful,
    # each search's band work) are bracketed by HIP events recorded on their own
    # stream by the C ABI (cbv2_index_time_scans); the collective times are
    # read from a separate untimed pass below, not from the timed region
    # (+ the doc-interleaved scans' in-kernel clock probe, reset after the
    # warmup: the clock the K timed scans held)
    ix.time_scans(True, clock=True)
    outs, elapsed = timed_steps(stepper(searcher, Q), args.steps, args.warmup, world,
                                on_start=lambda: ix.scan_clock(reset=True))
    scan_ms = ix.scan_times()                           # the warmup + K scans; keep the K of the timed region
    scan_clk = ix.scan_clock()
    scan_ms = scan_ms[-args.steps:] if len(scan_ms) >= args.steps else scan_ms
    band_ms = ix.band_times()[-args.steps:] if faithful else []
    qps = B * args.steps / elapsed * (world if replicas else 1)   # replicas: every rank ran its own K batches
    band = None
    if faithful:                         # the band each query of the last timed batch rescored
        bs = ix.last_band.float()
        band = {"batch": B, "mean": round(float(bs.mean()), 1), "max": int(bs.max()),
                "overflow_rows": int((bs < 0).sum())}
    coll = {}
    if world > 1:                        # per-step collective times: 2 untimed steps, instrumented
        searcher.time_collectives(True)
        stepper(searcher, Q)(2)
        torch.cuda.synchronize()
        coll = {k: {f: v / 2 for f, v in d.items()} for k, d in searcher.collective_times().items()}

    # ---- correctness of the timed output (size-independent properties)
    fs, fi = outs[-1]
    fi_h = fi.cpu().numpy()
    top10_planted = planted_frac(fi_h)
    sorted_ok = bool((torch.diff(fs, dim=1) <= 0).all().item())

    # ---- p50 / p99 latency at batch 1 (whole hot path, one query).  One shard
    # (or the native exchange): the one-round-trip path (cbv2_retrieve_begin /
    # _finish: stages 2 -> host RRF -> 3 in C++, one host round trip); the
    # torch.distributed exchange at N > 1: the stages one by one (`step`)
    one = one_trip(searcher)
    one_same = same_as_step(searcher, one, Q1) if one is not None else None
    _, p50_step, _ = latency(searcher, Q1) if one is not None else (None, None, None)
    lat, p50, p99 = latency(searcher, Q1, one)
    latency_path = ("one host round trip (cbv2_retrieve_begin/_finish_host; the call returns with the top-10 "
                    "on the host)" if one is not None
                    else "stages one by one (torch.distributed exchange)")
    bm_ms = []
    for _ in range(3):                                  # stage 1 alone (host), for the record
        t = time.perf_counter()
        bm_all()
        bm_ms.append((time.perf_counter() - t) * 1e3)

    # ---- dominant kernel: the MaxSim scan launches of the timed region above
    # (fp32-faithful: the bf16 scan of hi, the same kernel and template)
    if len(scan_ms) != args.steps:
        log(f"warning: {len(scan_ms)} timed scans recorded for {args.steps} steps")
    scan_avg = sum(scan_ms) / len(scan_ms) if scan_ms else float("nan")
    band_avg = sum(band_ms) / len(band_ms) if band_ms else None
    achieved = B * n_local * FLOP_PER_PAIR / (scan_avg * 1e-3) / 1e12
    fused_topk = ix.fused_topk_slots(B, args.k) > 0
    # HBM bytes per launch from the committed PMC passes of the same kernel and
    # shape (tools/profile_round.sh -> tools/pmc_summary.py); null otherwise
    traffic = clock = traffic_src = mfma_busy = pmc_ref = None
    pmc = os.path.join(ROOT, "profiles", "pmc_scan.json")
    want = "maxsim_scan_f8x4_kernel" if fp8 else SCAN_KERNEL
    variant = "fused" if fused_topk else "unfused"
    if os.path.exists(pmc):
        with open(pmc) as f:
            entries = json.load(f).get("entries", [])
        for d in entries:
            if (d.get("batch") == B and d.get("docs_per_gpu") == n_local and d.get("kernel") == want
                    and d.get("variant", "unfused") == variant):
                traffic, clock = d.get("hbm_bytes_per_launch"), d.get("clock_ghz")
                ctr = d.get("counters", {})
                busy, gui = (ctr.get(c, {}).get("per_launch") for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"))
                if busy and gui:   # busy SIMD-cycles / (1024 SIMDs x GPU-busy cycles; GRBM summed over 8 XCDs)
                    mfma_busy = busy / (1024 * gui / 8)
                traffic_src = (f"committed PMC pass profiles/pmc_scan.json ({want}, {variant}, batch {B}, "
                               f"{n_local} docs/GPU, one MI355X), not this run")
                pmc_ref = {"clock_ghz": round(clock, 3) if clock else None,
                           "mfma_busy": round(mfma_busy, 4) if mfma_busy else None, "source": traffic_src}
    clk_view = clock_view(B * n_local * FLOP_PER_PAIR, scan_avg, PEAK_FP8_TFLOPS if fp8 else PEAK_BF16_TFLOPS,
                          scan_clk["clock_ghz"])
    # every rank's scan time and collective time per step (max-over-ranks view of N > 1)
    names = ("all_gather", "all_reduce_max")
    mine = [scan_avg] + [coll.get(k, {}).get(f, 0.0) for k in names for f in ("device_ms", "host_ms")] \
        + [coll.get(k, {}).get("calls", 0) for k in names]
    per_rank = gather_floats(mine, world, dev, backend)
    collectives = None
    if world > 1:
        collectives = {k: {"calls_per_step": per_rank[0][5 + j],
                           "device_ms_per_step_max": round(max(r[1 + 2 * j] for r in per_rank), 4),
                           "host_ms_per_step_max": round(max(r[2 + 2 * j] for r in per_rank), 4),
                           "device_ms_per_step_by_rank": [round(r[1 + 2 * j], 4) for r in per_rank]}
                       for j, k in enumerate(names)}
        collectives["timing"] = ("2 untimed steps after the timed region, instrumented: HIP events on the issuing "
                                 "stream (device_ms; RCCL) and host wall time of the call (host_ms; gloo blocks "
                                 "the host), per step")

    # ---- spot parity: oracle MaxSim of the final candidates, on the owning rank
    check_rows = list(range(min(args.check_queries, B)))
    if fp8:                              # the oracle scores the same dequantized fp8 values
        from oracle import oracle as orc
        qq, qs = quantize_mxfp8(Q)
        Qd = orc.mxfp8_dequant(qq.cpu().numpy(), qs.cpu().numpy())
        docs_fn = lambda sel: orc.mxfp8_dequant(ix.tokens[sel].cpu().numpy(), ix.scales[sel].cpu().numpy())  # noqa: E731
        tol = 2e-3
    else:                                # fp32: the fp32 values themselves; bf16: the stored bf16 values
        Qd = Q.float().cpu().numpy()
        docs_fn = lambda sel: tokens[sel].float().cpu().numpy()   # noqa: E731
        tol = 1e-4 if faithful else 1e-3
    bad = spot_check(fs, fi_h, Qd, docs_fn, begin, end, check_rows, tol, world, dev)

    # ---- N > 1 over RCCL: the same K steps with the native (in-ABI) exchange
    native = None
    if nccl:
        def native_prepare():
            return searcher if args.native_exchange else ShardedSearcher(ix, native=True, lexical_k=args.k)

        def native_run(nsearch):
            nouts, nel = timed_steps(stepper(nsearch, Q), args.steps, args.warmup, world)
            nfi = nouts[-1][1].cpu().numpy()
            none = one_trip(nsearch)
            _, np50, np99 = latency(nsearch, Q1, none)
            res = {"value": round(B * args.steps / nel, 2), "ms_per_step": round(nel / args.steps * 1e3, 3),
                   "p50_ms_b1": round(np50, 3) if np50 is not None else None,
                   "p99_ms_b1": round(np99, 3) if np99 is not None else None,
                   "top10_equals_planted": planted_frac(nfi),
                   "equals_torch_exchange": bool(np.array_equal(nfi, fi_h)),
                   "one_trip_equals_stages": same_as_step(nsearch, none, Q1),
                   "main_line": "native" if args.native_exchange else "torch.distributed"}
            # every rank's native results equal the torch exchange's and the
            # one-trip's equal the stages': the line's p50 may then come from it
            res["validated_on_every_rank"] = agree(res["equals_torch_exchange"] and res["one_trip_equals_stages"]
                                                   and res["top10_equals_planted"] == 1.0, world, dev, backend)
            return res

        native = run_leg("native_exchange", native_prepare, native_run, world, rank, dev, backend)
        if "error" in native and args.native_exchange:
            raise RuntimeError(f"native exchange (the main line's): {native['error']}")

    # ---- CPU baseline: N = 1 only (the contract times it once, on the host of
    # the one-GPU run; an N > 1 line carries null and the ranks do not idle)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(Q, tokens, n_total, args.cpu_budget)
    if world > 1:
        dist.barrier()

    # ---- the side leg, same K steps + p50 on the same corpus:
    #   fp32 main -> "bf16": a plain bf16 index over the faithful index's hi
    #                tokens (bf16(x), exactly what a bf16 index of the corpus
    #                holds; no copy), scores within 1e-3 of the bf16 values;
    #   bf16 main -> "faithful": the fp32-faithful index of the same corpus.
    side = None
    if not args.no_side_leg and args.dtype in ("fp32", "bf16"):
        side_name = "bf16" if faithful else "faithful"

        def side_prepare():
            if faithful:
                six = ColbertIndex(ix.tokens, ix.doclens, id_base=begin)
                ssrch = ShardedSearcher(six, world=1, lexical_k=args.k) if replicas else ShardedSearcher(
                    six, native=nccl and native is not None and "error" not in native,
                                        lexical_k=args.k)
                return six, ssrch, Q.to(torch.bfloat16), None
            f32, dl32 = synth.make_shard(begin, end, Qf, planted, dev, seed=0, dtype=torch.float32)
            six = ColbertIndex.faithful_f32(f32, dl32, id_base=begin)
            return six, ShardedSearcher(six, world=1 if replicas else None, lexical_k=args.k), Qf.to(dev), f32

        def side_run(st):
            six, ssrch, Qs, f32 = st
            six.time_scans(True)
            souts, sel = timed_steps(stepper(ssrch, Qs), args.steps, args.warmup, world)
            sscan = six.scan_times()[-args.steps:]
            sband = six.band_times()[-args.steps:] if six.faithful else []
            sfs, sfi = souts[-1]
            sfi_h = sfi.cpu().numpy()
            sone = one_trip(ssrch)
            _, sp50, sp99 = latency(ssrch, Qs[:1].contiguous(), sone)
            if six.faithful:
                sbad = spot_check(sfs, sfi_h, Qs.cpu().numpy(), lambda sel: f32[sel].cpu().numpy(), begin, end,
                                  check_rows, 1e-4, world, dev)
            else:
                sbad = spot_check(sfs, sfi_h, Qs.float().cpu().numpy(), lambda sel: six.tokens[sel].float().cpu().numpy(),
                                  begin, end, check_rows, 1e-3, world, dev)
            res = {"value": round(B * args.steps / sel * (world if replicas else 1), 2),
                   "ms_per_step": round(sel / args.steps * 1e3, 3),
                   "scan_avg_ms": round(sum(sscan) / len(sscan), 3) if sscan else None,
                   "p50_ms_b1": round(sp50, 3) if sp50 is not None else None,
                   "p99_ms_b1": round(sp99, 3) if sp99 is not None else None,
                   "latency_path": "one host round trip" if sone is not None else "stages one by one",
                   "tolerance": 1e-4 if six.faithful else 1e-3, "oracle_mismatch_queries": sbad,
                   "top10_equals_planted": planted_frac(sfi_h)}
            if six.faithful:
                bs = six.last_band.float()
                res["band_ms"] = round(sum(sband) / len(sband), 3) if sband else None
                res["band"] = {"mean": round(float(bs.mean()), 1), "max": int(bs.max()),
                               "overflow_rows": int((bs < 0).sum())}
                res["note"] = ("fp32 index (the reference stores fp32, LRC:735-746); scores vs float64 oracle "
                               "of the fp32 values")
            else:
                res["note"] = ("bf16 index over the same corpus (hi = bf16(x)); scores vs float64 oracle of "
                               "the bf16 values; ~5e-3 from the fp32 scores (DESIGN §3.7)")
            return res

        side = run_leg(side_name, side_prepare, side_run, world, rank, dev, backend)
        torch.cuda.synchronize()
        torch.cuda.empty_cache()

    # ---- BASELINE configs 4 and 5 on the node (8 ranks): the 10M-doc corpus
    # sharded over the ranks, stage 2 (scan + top-100 + ONE all-gather + merge)
    c45 = None
    if args.c45 == "on" or (args.c45 == "auto" and world == 8 and args.dtype in ("fp32", "bf16") and not replicas):
        one = searcher = ix = tokens = None   # noqa: F841  free HBM for the 10M-doc shards
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        c45 = c45_legs(args, B, world, rank, dev, backend)

    # N > 1: the product's exchange is the native one (the C ABI's RCCL calls,
    # no Python between the stages or around the collectives); once it has
    # validated on every rank, the line's throughput and latency come from it
    # and the torch.distributed leg's numbers stay beside (main_line)
    mine, torch_leg = main_line(round(qps, 2), round(elapsed / args.steps * 1e3, 3), p50, p99, native,
                                bool(args.native_exchange))
    if torch_leg is not None:
        latency_path = ("one host round trip over the native exchange (cbv2_retrieve_begin/_finish, "
                        "RCCL collectives inside the C ABI)")
    p50, p99 = mine["p50_ms_b1"], mine["p99_ms_b1"]
    if world > 1 and mine["exchange"] is None:   # no native leg (gloo): the torch.distributed exchange
        mine["exchange"] = "torch.distributed"

    peak = PEAK_FP8_TFLOPS if fp8 else PEAK_BF16_TFLOPS
    if rank == 0:
        workload = ("config 5 (MXFP8 e4m3 tokens, block-scaled fp8 MFMA)" if fp8 else
                    "config 3, fp32-faithful index (the reference's fp32 arithmetic within 1e-4: bf16 scan + "
                    "certified hi/lo band rescoring)" if faithful else "config 3, bf16 index")
        line = {
            "metric": "queries/sec + p50 retrieval latency, 1M-chunk corpus, top-10 rerank",
            "value": mine["value"], "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": mine["ms_per_step"],
            "higher_is_better": True, "scaling": "weak" if replicas else "strong", "vs_baseline": None,
            "dtype": "fp32 (faithful: bf16 hi/lo split, fp32 accumulate)" if faithful else args.dtype,
            "data": "synthetic (unit-norm N(0,I) tokens, Zipf term-id corpus for BM25, 10 planted positives/query)",
            "config": {"workload": workload + f": {n_total} chunks x 128 tokens x 128-d, host BM25 top-100 + "
                                              "ColBERT MaxSim top-100 + RRF + rerank top-10",
                       "corpus_docs": n_total, "docs_per_gpu": n_local, "global_batch": B, "lq": LQ, "ld": LD,
                       "dim": DIM, "colbert_k": args.k, "fused": args.fused, "final_k": args.final_k,
                       "index_dtype": args.dtype,
                       "parallelism": f"query replicas x{world} (the whole corpus on every GPU, no collective)"
                       if replicas else f"corpus sharded x{world}" + (
                           ((" (RCCL all-gather, stage 3 without a collective, " + (
                               "native in-ABI" if args.native_exchange else "torch.distributed") + " exchange)")
                            if nccl else f" ({backend} rehearsal: ranks share one GPU)")
                           if world > 1 else "")},
            "p50_ms_b1": round(p50, 3) if p50 is not None else None,
            "p99_ms_b1": round(p99, 3) if p99 is not None else None,
            "latency_samples": len(lat),
            "latency_path": latency_path,
            "p50_ms_b1_stages_one_by_one": round(p50_step, 3) if p50_step is not None else None,
            "exchange": mine["exchange"],
            "torch_exchange": ({k: (round(v, 3) if isinstance(v, float) and k.startswith("p") else v)
                                for k, v in torch_leg.items()} if torch_leg is not None else None),
            "one_trip_equals_stages": one_same,
            "host_bm25_ms_per_batch": round(min(bm_ms), 3),
            "roofline": {"bound": "mfma", "kernel": want, "variant": variant, "achieved": round(achieved, 2),
                         "peak": peak, "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                         "traffic": traffic, "traffic_source": traffic_src, "avg_ms": round(scan_avg, 3),
                         "launches_timed": len(scan_ms),
                         "avg_ms_by_rank": [round(r[0], 3) for r in per_rank],
                         "avg_ms_min_max": [round(min(r[0] for r in per_rank), 3),
                                            round(max(r[0] for r in per_rank), 3)],
                         "band_ms": round(band_avg, 3) if band_avg is not None else None,
                         "band_ms_note": ("fp32-faithful band work per step (HIP events in the timed region: end "
                                          "of the bf16 top-k -> end of the band select), rank 0; not part of avg_ms"
                                          if faithful else None),
                         **clk_view,
                         "clock_source": (f"in-kernel probe of the {len(scan_ms)} timed scans: sum of workgroup "
                                          f"s_memtime cycles / s_memrealtime ticks over {scan_clk['workgroups']} "
                                          "workgroups (cbv2_index_scan_clock)"
                                          if scan_clk["clock_ghz"] else None),
                         "pmc_reference": pmc_ref},
            "cpu_baseline": cpu,
            "checks": {"top10_equals_planted": top10_planted, "sorted": sorted_ok, "oracle_mismatch_queries": bad,
                       "oracle_checked_queries": len(check_rows), "oracle_tolerance": tol},
        }
        if band is not None:
            line["faithful_band"] = band
        if side is not None:
            line["bf16" if faithful else "faithful"] = side
        if native is not None:
            line["native_exchange"] = native
        if collectives is not None:
            line["collectives"] = collectives
        if c45 is not None:
            line["configs_4_5"] = c45
        os.write(JSON_FD, (json.dumps(line) + "\n").encode())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
