"""CPU: distributed.pool_scores -- the lookup the collective-free sharded stage
3 runs (ShardedSearcher.rerank(..., pool=...); the HIP twin is
prescored_select_kernel): every candidate takes the score its id carries in
the row's pool of (id, rerank score) pairs; a negative id scores -inf (as the
rerank scores one, LRC:788-792 never sees one: the RRF pads with -1); an id
in no list scores -inf and is counted as a miss.  Duplicated pool entries
(a doc in its owner's stage-2 and stage-1 lists) carry the same bits."""
import numpy as np
import torch

from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, pool_scores


def test_pool_scores_lookup_padding_and_misses():
    ids = torch.tensor([[5, 9, -1, 7, 9], [3, -1, -1, 4, 8]], dtype=torch.int32)
    sc = torch.tensor([[0.5, 0.25, -np.inf, 0.75, 0.25], [1.0, -np.inf, -np.inf, 2.0, 3.0]], dtype=torch.float32)
    cand = torch.tensor([[9, 7, -1, 5], [8, 42, 3, -1]], dtype=torch.int32)
    raw, misses = pool_scores(cand, ids, sc)
    want = torch.tensor([[0.25, 0.75, -np.inf, 0.5], [3.0, -np.inf, 1.0, -np.inf]], dtype=torch.float32)
    assert torch.equal(raw, want)
    assert int(misses) == 1                      # id 42 is in no list; the -1 paddings are not misses


def test_pool_layout_from_gathered_blocks():
    """ShardedSearcher._pool: [G, B, k + 2 kb, 2] gathered (score bits, id)
    blocks -> per row every rank's k stage-2 pairs and kb prescored stage-1
    pairs (the BM25 scores in between are not rerank scores and stay out)."""
    G, B, k, kb = 3, 2, 4, 2
    rng = np.random.default_rng(1)
    allp = torch.from_numpy(rng.integers(0, 1000, size=(G, B, k + 2 * kb, 2)).astype(np.int32))
    pool = ShardedSearcher._pool(allp, k, kb)
    assert tuple(pool.ids.shape) == (B, G * (k + kb))
    for b in range(B):
        want = [allp[g, b, j, 1].item() for g in range(G) for j in list(range(k)) + list(range(k + kb, k + 2 * kb))]
        assert pool.ids[b].tolist() == want
        bits = pool.scores[b].view(torch.int32).tolist()
        assert bits == [allp[g, b, j, 0].item() for g in range(G)
                        for j in list(range(k)) + list(range(k + kb, k + 2 * kb))]
    p0 = ShardedSearcher._pool(allp[:, :, :k], k, 0)   # no stage-1 lists: the stage-2 pairs only
    assert tuple(p0.ids.shape) == (B, G * k)
