"""GPU: index memory placement (cbv2_hbm_alloc / cbv2_hbm_free, index.hbm_empty).

Large index arrays come from physically contiguous HBM when the driver can
provide it; the tensor torch sees must alias that block exactly, free it when
the last view dies, and index/search over it must return what the same tokens
in torch's allocator return."""
import gc

import pytest
import torch

from hybrid_rag_colbertv2_amd import synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex, hbm_empty, hbm_placement

pytestmark = pytest.mark.gpu


def _cycle(n, dev):
    t = hbm_empty((n // 2,), torch.bfloat16, dev)
    t.fill_(1.5)
    s = float(t[:: 1 << 20].float().sum())
    del t
    gc.collect()
    return s


def test_hbm_block_aliases_and_frees(dev):
    n = 1 << 28                                            # 256 MiB: above the torch-allocator threshold
    _cycle(n, dev)                                         # torch's kernels loaded, its small-block pool made
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info(dev)[0]
    t = hbm_empty((n // 2,), torch.bfloat16, dev)
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info(dev)[0] <= free0 - n + (16 << 20)     # the block is device memory
    assert hbm_placement(t) in ("contiguous", "hipMalloc")
    assert t.data_ptr() % 256 == 0 and t.numel() == n // 2 and t.device == dev
    t.fill_(1.5)
    assert float(t[:: 1 << 20].float().sum()) == 1.5 * ((n // 2) >> 20)
    v = t.view(torch.int16)[: 1 << 20]                     # a view keeps the block alive
    del t
    gc.collect()
    assert int(v[0]) == int(torch.tensor(1.5, dtype=torch.bfloat16).view(torch.int16))
    del v
    gc.collect()
    torch.cuda.synchronize()
    assert torch.cuda.mem_get_info(dev)[0] >= free0 - (16 << 20)   # returned to the device
    small = hbm_empty((1000,), torch.float32, dev)
    assert hbm_placement(small) == "torch"


def test_index_over_hbm_equals_torch_allocation(dev):
    N, B = 20000, 3
    Qf = synth.make_queries(B, seed=9)
    planted = synth.planted_ids(B, N, 10, seed=10)
    tok, dl = synth.make_shard(0, N, Qf, planted, dev)       # 655 MB of bf16: hbm_empty
    big = hbm_empty(tok.shape, tok.dtype, dev)
    big.copy_(tok)
    plain = tok.clone()
    assert hbm_placement(big) in ("contiguous", "hipMalloc")
    a = ColbertIndex(big, dl).search(Qf.to(dev, torch.bfloat16), 50)
    b = ColbertIndex(plain, dl).search(Qf.to(dev, torch.bfloat16), 50)
    assert all(torch.equal(x, y) for x, y in zip(a, b))
