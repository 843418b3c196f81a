"""CPU, world_size 2 and 4 (gloo): the sharded search / rerank protocol of
hybrid-rag-colbertv2_amd/distributed.py (all-gather of packed (score, id)
pairs + merge; all-reduce MAX of candidate scores + select) equals the
unsharded oracle.  The per-shard compute is injected as oracle-backed CPU
objects (test-only); on the GPU box the same class drives the HIP kernels
over RCCL (tests/test_gpu_api.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import oracle as orc


class OracleShard:
    def __init__(self, Q, docs, doclens, begin):
        self.docs, self.doclens, self.begin = docs, doclens, begin

    def search(self, Q, k):
        s = orc.maxsim(Q.numpy(), self.docs, self.doclens)
        vs, ids = orc.topk(s, k, id_base=self.begin)
        return torch.from_numpy(vs.astype(np.float32)), torch.from_numpy(ids.astype(np.int32))

    def rerank(self, Q, cand, k):
        assert k == 0
        c = cand.numpy()
        out = np.full(c.shape, -np.inf, np.float32)
        for b in range(c.shape[0]):
            for j in range(c.shape[1]):
                loc = c[b, j] - self.begin
                if c[b, j] >= 0 and 0 <= loc < len(self.docs):
                    out[b, j] = orc.maxsim(Q[b:b + 1].numpy(), self.docs[loc:loc + 1], self.doclens[loc:loc + 1])[0, 0]
        return torch.from_numpy(out)


class OracleOps:
    @staticmethod
    def merge(S, I, k):
        s, i = orc.merge_topk(S.numpy(), I.numpy(), k)
        return torch.from_numpy(s.astype(np.float32)), torch.from_numpy(i.astype(np.int32))

    @staticmethod
    def select(scores, k, ids):
        sc = scores.numpy()
        out_s = np.full((sc.shape[0], k), -np.inf, np.float32)
        out_i = np.full((sc.shape[0], k), -1, np.int32)
        out_p = np.full((sc.shape[0], k), -1, np.int32)
        for b in range(sc.shape[0]):
            for r, (p, s, _) in enumerate(orc.rerank_select(sc[b], k)):
                out_s[b, r], out_i[b, r], out_p[b, r] = s, ids[b, p], p
        return torch.from_numpy(out_s), torch.from_numpy(out_i), torch.from_numpy(out_p)


def _data():
    rng = np.random.default_rng(7)
    N, B = 301, 3
    docs = orc.bf16_round(rng.standard_normal((N, 16, 128)).astype(np.float32))
    doclens = rng.integers(0, 17, size=N)
    Q = torch.from_numpy(orc.bf16_round(rng.standard_normal((B, 32, 128)).astype(np.float32)))
    cand = rng.integers(-1, N, size=(B, 20)).astype(np.int32)
    return Q, docs, doclens, cand


def _worker(rank, world, port, q, k=40):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, shard_range
        Q, docs, doclens, cand = _data()
        a, b = shard_range(len(docs), rank, world)
        ss = ShardedSearcher(OracleShard(Q, docs[a:b], doclens[a:b], a), ops=OracleOps())
        s, i = ss.search(Q, k)
        rs, ri, rp = ss.rerank(Q, torch.from_numpy(cand), 7)
        q.put((rank, s.numpy(), i.numpy(), rs.numpy(), ri.numpy(), rp.numpy()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,k", [(2, 40), (4, 100)])
def test_sharded_protocol_equals_unsharded(world, k):
    """world 4, k = 100: every shard (75-76 docs) is shorter than k, so every
    rank's list ends in -inf / -1 padding that the merge must skip."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Q, docs, doclens, cand = _data()
    full = orc.maxsim(Q.numpy(), docs, doclens)
    es, ei = orc.topk(full, k)
    rs, ri, rp = orc.rerank(Q.numpy(), docs, doclens, cand, 7)
    for _, s, i, gs, gi, gp in res:        # every rank holds the identical global answer
        assert np.array_equal(i, ei)
        np.testing.assert_allclose(s, es, atol=1e-5)
        assert np.array_equal(gp, rp) and np.array_equal(gi, ri)
        np.testing.assert_allclose(gs, rs, atol=1e-5)


def _bm25_data():
    rng = np.random.default_rng(9)
    N, V = 301, 30
    lens = rng.integers(0, 25, size=N)
    off = np.zeros(N + 1, np.int64)
    off[1:] = np.cumsum(lens)
    terms = rng.integers(0, V, size=int(off[-1])).astype(np.int32)
    qo = np.arange(4, dtype=np.int64) * 3
    qt = rng.integers(0, V, size=9).astype(np.int32)
    return terms, off, qt, qo, V


def _hybrid_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hybrid_rag_colbertv2_amd import bm25
        from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, shard_range
        from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
        Q, docs, doclens, _ = _data()
        terms, off, qt, qo, V = _bm25_data()
        a, b = shard_range(len(docs), rank, world)
        lex = bm25.sharded(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a)   # all-reduced stats
        ss = ShardedSearcher(OracleShard(Q, docs[a:b], doclens[a:b], a), ops=OracleOps())
        s, i, li = ss.search_hybrid(Q, 40, lambda: lex.search(qt, qo, 50))
        # stage 3 without a collective: the fused candidates' scores from the
        # pool (stage-2 lists + the ranks' prescored BM25 lists), for a full
        # and a narrower stage-1 width (kb 50 / 30)
        pooled = []
        for kb in (50, 30):
            ss.time_collectives(True)
            s3, i3, li3, pool = ss.search_hybrid(Q, 40, lambda: lex.search(qt, qo, kb), return_pool=True)
            cand = rrf_fuse(li3.numpy(), i3.numpy(), rrf_k=60, C=20)
            rs, ri, rp = ss.rerank(Q, torch.from_numpy(cand), 7, pool=pool)
            coll = ss.collective_times()
            pooled.append((cand, rs.numpy(), ri.numpy(), rp.numpy(), int(ss.last_pool_misses),
                           {n: d["calls"] for n, d in coll.items()}))
        q.put((rank, s.numpy(), i.numpy(), li.numpy(), pooled))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_hybrid_exchange_equals_unsharded(world):
    """Doc-sharded BM25 (global stats by all-reduce) + stage 2 in one all-gather;
    stage 3 of the fused lists with NO collective (every candidate's rerank
    score rides that all-gather) equals the unsharded rerank, at kb 50 and 30."""
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_hybrid_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Q, docs, doclens, _ = _data()
    es, ei = orc.topk(orc.maxsim(Q.numpy(), docs, doclens), 40)
    terms, off, qt, qo, V = _bm25_data()
    bi, _ = orc.bm25_topk(terms, off, qt, qo, V, 50)
    for _, s, i, li, pooled in res:
        assert np.array_equal(i, ei) and np.array_equal(li, bi)
        np.testing.assert_allclose(s, es, atol=1e-5)
        for kb, (cand, rs, ri, rp, misses, calls) in zip((50, 30), pooled):
            bk, _ = orc.bm25_topk(terms, off, qt, qo, V, kb)
            assert np.array_equal(cand, rrf_fuse(bk, ei, rrf_k=60, C=20))
            ws, wi, wp = orc.rerank(Q.numpy(), docs, doclens, cand, 7)
            assert np.array_equal(ri, wi) and np.array_equal(rp, wp), f"kb {kb}: pooled stage 3 differs"
            np.testing.assert_allclose(rs, ws, atol=1e-5)
            assert misses == 0 and calls == {"all_gather": 1}, (kb, misses, calls)


# randomized stage-1 width / k / C / final_k cases of the pooled stage 3 at
# world 3 (ragged shards): (k, kb, C, final_k); kb 0 = no stage 1
_POOL_CASES = [(40, 50, 20, 7), (5, 13, 7, 7), (100, 1, 20, 1), (17, 50, 64, 20), (40, 0, 20, 7),
               (100, 50, 1, 1), (5, 50, 64, 20), (17, 13, 20, 20), (120, 7, 50, 10)]


def _pool_cases_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hybrid_rag_colbertv2_amd import bm25
        from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher, shard_range
        from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
        Q, docs, doclens, _ = _data()
        terms, off, qt, qo, V = _bm25_data()
        a, b = shard_range(len(docs), rank, world)
        lex = bm25.sharded(terms[off[a]:off[b]], off[a:b + 1] - off[a], V, id_base=a)
        ss = ShardedSearcher(OracleShard(Q, docs[a:b], doclens[a:b], a), ops=OracleOps())
        out = []
        for k, kb, C, fk in _POOL_CASES:
            lexical = (lambda kb=kb: lex.search(qt, qo, kb)) if kb else None
            s3, i3, li3, pool = ss.search_hybrid(Q, k, lexical, return_pool=True)
            bm = li3.numpy() if li3 is not None else np.zeros((Q.shape[0], 0), np.int32)
            cand = rrf_fuse(bm, i3.numpy(), rrf_k=60, C=C)
            rs, ri, rp = ss.rerank(Q, torch.from_numpy(cand), fk, pool=pool)
            out.append((cand, rs.numpy(), ri.numpy(), rp.numpy(), int(ss.last_pool_misses)))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_pooled_stage3_cases_world3():
    """The collective-free stage 3 over many (k, kb, C, final_k) shapes at
    world 3: k above a shard's size (padding in the pool), kb = 1 and no
    stage 1, C = 1 and C above the fused list, final_k = C -- every rank
    equals the unsharded rerank of the same fused candidates, no misses."""
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pool_cases_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    Q, docs, doclens, _ = _data()
    full = orc.maxsim(Q.numpy(), docs, doclens)
    terms, off, qt, qo, V = _bm25_data()
    for _, out in res:
        for (k, kb, C, fk), (cand, rs, ri, rp, misses) in zip(_POOL_CASES, out):
            _, ei = orc.topk(full, k)
            bk = orc.bm25_topk(terms, off, qt, qo, V, kb)[0] if kb else np.zeros((Q.shape[0], 0), np.int32)
            assert np.array_equal(cand, rrf_fuse(bk, ei, rrf_k=60, C=C)), (k, kb, C)
            ws, wi, wp = orc.rerank(Q.numpy(), docs, doclens, cand, fk)
            assert np.array_equal(ri, wi) and np.array_equal(rp, wp), (k, kb, C, fk)
            np.testing.assert_allclose(rs, ws, atol=1e-5)
            assert misses == 0, (k, kb, C, fk, misses)


_QUERIES = ["what is late interaction", "colbert maxsim on mi355x", "bm25 and rrf fusion",
            "hbm3e bandwidth", "rerank the top fifty chunks"]


def _encode_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hybrid_rag_colbertv2_amd.distributed import encode_queries_sharded
        from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
        enc = FakeEncoder()
        # B = 5 (ragged over the ranks), 1 (empty slices on some ranks), 0
        outs = [encode_queries_sharded(enc, _QUERIES[:n]).float().numpy() for n in (5, 1, 0)]
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def test_sharded_query_encoding_equals_single_process():
    """Each rank encodes its slice of the batch; one all-gather rebuilds it in order."""
    from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
    for world in (2, 3):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_encode_worker, args=(r, world, port, q)) for r in range(world)]
        for p in procs:
            p.start()
        res = [q.get(timeout=300) for _ in range(world)]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
        enc = FakeEncoder()
        want = [enc.encode(_QUERIES[:n]).to(torch.bfloat16).float().numpy() for n in (5, 1)]
        for _, outs in res:
            assert np.array_equal(outs[0], want[0]) and np.array_equal(outs[1], want[1])
            assert outs[2].shape[0] == 0


class _UnpaddedEncoder:
    """Query encoder that does NOT pad to a fixed Lq: a batch comes out
    [b, max words in the batch, 128], shorter queries zero-padded."""

    def encode(self, texts, convert_to_tensor=True, **_):
        from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
        fe = FakeEncoder(maxlen=64)
        rows = [[w for w in fe.tokenize(t) if not w.startswith("[PAD]")] for t in texts]
        L = max([len(r) for r in rows] + [1])
        out = torch.zeros((len(texts), L, 128))
        for i, r in enumerate(rows):
            for j, w in enumerate(r):
                out[i, j] = torch.from_numpy(fe._vec(w))
        return out


def _ragged_encode_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hybrid_rag_colbertv2_amd.distributed import encode_queries_sharded
        q.put((rank, encode_queries_sharded(_UnpaddedEncoder(), _QUERIES).float().numpy()))
    finally:
        dist.destroy_process_group()


def test_sharded_query_encoding_unpadded_encoder():
    """Ranks whose slices encode to different Lq: the gathered batch is
    the single-process encode, zero rows added where a rank's Lq was shorter."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ragged_encode_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _UnpaddedEncoder().encode(_QUERIES).to(torch.bfloat16).float().numpy()
    for _, got in res:
        assert np.array_equal(got, want)
