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
