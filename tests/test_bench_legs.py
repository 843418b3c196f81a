"""CPU, gloo world 2 / 4: bench.py's optional legs fail symmetrically
(bench.run_leg).  A leg whose local preparation fails on ONE rank (an OOM
from uneven free memory, or the injected BENCH_FAIL_LEG failure the N > 1
rehearsals use) must end with the same {"error": ...} on every rank, with no
rank entering the leg's collectives -- otherwise the peers would block in the
next all-gather and the 8-GPU line would never print.  The leg that follows
still runs on every rank.  No reference counterpart (the reference is
single-process)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, port, q, fail_rank):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["BENCH_FAIL_LEG"] = "configs_x"
    os.environ["BENCH_FAIL_RANK"] = str(fail_rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        dev = torch.device("cpu")
        ran = []

        def prep():
            return torch.full((4,), float(rank))

        def run(t):
            ran.append(True)
            out = torch.empty((world, 4))
            dist.all_gather(list(out.unbind(0)), t)      # the leg's collective
            return {"sum": float(out.sum())}

        a = bench.run_leg("configs_x", prep, run, world, rank, dev, "gloo")   # fails on fail_rank
        first_ran = bool(ran)
        b = bench.run_leg("configs_y", prep, run, world, rank, dev, "gloo")   # still runs everywhere

        def bad_run(t):   # a run-phase error on every rank (same code, same shapes)
            raise ValueError("symmetric")

        c = bench.run_leg("configs_z", prep, bad_run, world, rank, dev, "gloo")
        q.put((rank, a, first_ran, b, c))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (4, 2), (2, -1)])
def test_run_leg_symmetric_failure(world, fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, fail_rank)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    expect_sum = 4.0 * sum(range(world))
    for rank, a, first_ran, b, c in res:
        if fail_rank >= 0:
            assert set(a) == {"error"}, a
            assert not first_ran                       # no rank entered the failed leg's collective
            if rank == fail_rank:
                assert "injected failure" in a["error"]
            else:
                assert "another rank" in a["error"]
        else:
            assert a == {"sum": expect_sum} and first_ran
        assert b == {"sum": expect_sum}
        assert "ValueError: symmetric" in c["error"]


def test_main_line_takes_native_numbers_once_validated():
    """bench.main_line: the N > 1 line's value / ms_per_step / p50 come from
    the in-ABI exchange when it validated
    on every rank, with the torch.distributed numbers beside; otherwise the
    torch.distributed numbers stay the line's.  No collective involved."""
    import bench
    own = (1000.0, 256.0, 0.9, 1.1)
    good = {"value": 1200.0, "ms_per_step": 213.3, "p50_ms_b1": 0.7, "p99_ms_b1": 0.8,
            "validated_on_every_rank": True}
    line, torch_leg = bench.main_line(*own, good, False)
    assert (line["value"], line["ms_per_step"], line["p50_ms_b1"]) == (1200.0, 213.3, 0.7)
    assert line["exchange"].startswith("native")
    assert torch_leg == {"value": 1000.0, "ms_per_step": 256.0, "p50_ms_b1": 0.9, "p99_ms_b1": 1.1,
                         "exchange": "torch.distributed"}
    for native in (dict(good, validated_on_every_rank=False), {"error": "failed on another rank"}, None,
                   dict(good, p50_ms_b1=None)):
        line, torch_leg = bench.main_line(*own, native, False)
        assert (line["value"], line["ms_per_step"], line["p50_ms_b1"]) == (1000.0, 256.0, 0.9)
        assert torch_leg is None
    line, torch_leg = bench.main_line(*own, good, True)     # --native-exchange: the main legs ran native
    assert line["value"] == 1000.0 and torch_leg is None and line["exchange"].startswith("native")


def test_clock_view_reproduces_avg_ms():
    """bench.clock_view: the line's roofline frac split into THIS run's held
    clock (the scans' in-kernel probe) and the MFMA-busy fraction at that
    clock -- frac = clock / 2.4 GHz x busy, and FLOP / (busy x peak x clock /
    2.4) gives back the measured avg_ms.  No probe -> no split."""
    import bench
    flop = 256 * 1_000_000 * bench.FLOP_PER_PAIR
    for avg_ms, ghz in ((144.677, 2.022), (138.12, 1.95), (4.6, 1.59)):
        v = bench.clock_view(flop, avg_ms, bench.PEAK_BF16_TFLOPS, ghz)
        frac = flop / (avg_ms * 1e-3) / 1e12 / bench.PEAK_BF16_TFLOPS
        assert v["clock_ghz_this_run"] == round(ghz, 4)
        assert abs(v["avg_ms_from_clock_and_busy"] - avg_ms) <= 1e-3
        assert abs(v["mfma_busy_this_run"] * ghz / bench.NOMINAL_GHZ - frac) < 1e-4
    assert bench.clock_view(flop, 140.0, bench.PEAK_BF16_TFLOPS, None)["mfma_busy_this_run"] is None
