"""GPU: the scans' in-kernel clock probe (cbv2_index_time_scans(ix, 2) /
cbv2_index_scan_clock) that gives bench.py's roofline this run's clock
(SURVEY §8(d)): every probed workgroup is counted in and out, the clock
lands in the chip's range, the sums reset, and the probe changes no result
bit (it only adds run times to two sums).  bf16 doc-interleaved scans (B = 1
dense one-per-CU shape, B = 64) and the MXFP8 one (B = 64)."""
import pytest
import torch

from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fp8,B", [(False, 1), (False, 64), (True, 64)])
def test_clock_probe_counts_and_keeps_bits(dev, fp8, B):
    N = 60_000
    Qf = synth.make_queries(B, seed=5)
    planted = synth.planted_ids(B, N, 10, seed=6)
    tok, dl = synth.make_shard(0, N, Qf, planted, dev)
    ix = ColbertIndex.mxfp8(tok, dl) if fp8 else ColbertIndex(tok, dl)
    Q = Qf.to(dev, torch.bfloat16)
    want = [x.clone() for x in ix.search(Q, 100)]
    ix.time_scans(True, clock=True)
    got = [ix.search(Q, 100) for _ in range(3)]
    torch.cuda.synchronize()
    c = ix.scan_clock(reset=True)
    times = ix.scan_times()
    assert len(times) == 3
    assert c["complete"] and c["workgroups"] > 0 and c["workgroups"] % 3 == 0, c
    assert 0.5 < c["clock_ghz"] < 3.0, c
    assert ix.scan_clock()["workgroups"] == 0          # reset
    for s, i in got:
        assert torch.equal(i, want[1]) and torch.equal(s, want[0])
    ix.time_scans(True)                                  # events only: the probe stays off
    ix.search(Q, 100)
    torch.cuda.synchronize()
    assert ix.scan_clock()["workgroups"] == 0
    ix.time_scans(False)
