"""GPU: the drop-in Python API (JinaColBERTRetriever / DualIndexer /
HybridRetriever) on the HIP kernels reproduces the reference's recorded
outputs (config 1, literal scorer) and the oracle's (maxsim scorer)."""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from hybrid_rag_colbertv2_amd import FakeEncoder, RAGConfig
from hybrid_rag_colbertv2_amd.hybrid import ChunkStore, DualIndexer, HybridRetriever
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
TOY = json.load(open(os.path.join(GOLDEN, "toy_c1.json")))


class RecordedBM25:
    """Stage-1 stand-in replaying the BM25 lists recorded with the golden run."""

    def __init__(self):
        self.lists = {q: bm for q, bm in zip(TOY["queries"], TOY["bm25"])}

    def tokenize(self, q):
        return q

    def retrieve(self, q, k):
        bm = self.lists[q]
        return np.array([bm["ids"][:k]]), np.array([bm["scores"][:k]])


def _system(tmp_path, scorer, index_dtype="bf16", encoder_cls=None):
    cfg = RAGConfig(scorer=scorer, colbert_index_path=str(tmp_path / "colbert"),
                    bm25_index_path=str(tmp_path / "bm25"), index_dtype=index_dtype)
    ind = DualIndexer(cfg, encoder=(encoder_cls or FakeEncoder)(**TOY["encoder"]))
    ind.colbert_retriever.index(TOY["corpus"])
    ind.bm25_retriever = RecordedBM25()
    store = ChunkStore([{"chunk_id": c["id"], "text": t, "document_id": c["document_id"],
                         "heading_path": c["heading_path"], "has_images": c["has_images"],
                         "metadata": json.loads(c["metadata"]) if c["metadata"] else {}}
                        for c, t in zip(TOY["chunks"], TOY["corpus"])])
    return cfg, ind, HybridRetriever(cfg, ind, store, verbose=False)


@pytest.mark.parametrize("strict", [False, True])
def test_c1_literal_search_rerank_retrieve_match_reference(dev, tmp_path, strict):
    """strict: the encoder has sentence-transformers 2.x's ``encode`` signature
    (no ``is_query``, no ``**kwargs``; LRC:758-761 / 782-783 pass only
    ``convert_to_tensor=True``) and the golden reference outputs are still
    reproduced through index, search, rerank and HybridRetriever.retrieve."""
    cfg, ind, hyb = _system(tmp_path, "ref_meanpool_cosine", encoder_cls=StrictEncoder if strict else None)
    r = ind.colbert_retriever
    for i, q in enumerate(TOY["queries"]):
        got = r.search(q, k=10)
        assert [g["document_id"] for g in got] == [x["document_id"] for x in TOY["search"][i]]
        np.testing.assert_allclose([g["score"] for g in got], [x["score"] for x in TOY["search"][i]], atol=1e-5)
        assert got[0]["text"] == TOY["corpus"][got[0]["document_id"]]
        rr = r.rerank(q, TOY["corpus"][0:50:3], k=5)
        ref = TOY["rerank"][i]["results"]
        assert [(x["result_index"], x["rank"]) for x in rr] == [(x["result_index"], x["rank"]) for x in ref]
        np.testing.assert_allclose([x["score"] for x in rr], [x["score"] for x in ref], atol=1e-5)
        fin = hyb.retrieve(q)
        ref = TOY["retrieve"][i]
        assert [f["chunk_id"] for f in fin] == [x["chunk_id"] for x in ref]
        for f, x in zip(fin, ref):
            assert f["text"] == TOY["corpus"][f["chunk_id"]]
            assert {k: v for k, v in f.items() if k not in ("score", "text")} == \
                {k: v for k, v in x.items() if k != "score"}
            assert abs(f["score"] - x["score"]) < 1e-5


class StrictEncoder:
    """sentence-transformers 2.x ``encode`` signature: no ``is_query``, no ``**kwargs``."""

    def __init__(self, **kw):
        self.fe = FakeEncoder(**kw)

    def encode(self, sentences, batch_size=32, show_progress_bar=None, output_value="sentence_embedding",
               convert_to_numpy=True, convert_to_tensor=False, device=None, normalize_embeddings=False):
        return self.fe.encode(sentences, convert_to_tensor=convert_to_tensor)


@pytest.mark.parametrize("scorer", ["maxsim", "ref_meanpool_cosine"])
def test_strict_signature_encoder_through_search_rerank_retrieve(dev, tmp_path, scorer):
    """LRC:758-761 / 782-783 call ``encode(x, convert_to_tensor=True)`` only: an
    encoder without ``is_query`` / ``**kwargs`` must work in index, search,
    rerank and retrieve, with results equal to the keyword-tolerant encoder's."""
    cfg, ind, hyb = _system(tmp_path / "a", scorer)
    cfg2 = RAGConfig(scorer=scorer, colbert_index_path=str(tmp_path / "b"), index_dtype="bf16")
    ind2 = DualIndexer(cfg2, encoder=StrictEncoder(**TOY["encoder"]))
    ind2.colbert_retriever.index(TOY["corpus"])
    ind2.bm25_retriever = RecordedBM25()
    hyb2 = HybridRetriever(cfg2, ind2, hyb.db_session, verbose=False)
    for q in TOY["queries"]:
        assert ind2.colbert_retriever.search(q, k=10) == ind.colbert_retriever.search(q, k=10)
        docs = TOY["corpus"][1:40:4]
        assert ind2.colbert_retriever.rerank(q, docs, k=5) == ind.colbert_retriever.rerank(q, docs, k=5)
        assert hyb2.retrieve(q) == hyb.retrieve(q)


def test_literal_maxsim_score_shapes_match_reference(dev, tmp_path):
    cfg = RAGConfig(scorer="ref_meanpool_cosine")
    from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever
    r = JinaColBERTRetriever(cfg, encoder=FakeEncoder())
    z = np.load(os.path.join(GOLDEN, "literal_maxsim.npz"))
    for case in "abc":
        got = r._maxsim_score(torch.from_numpy(z[f"{case}_q"]), torch.from_numpy(z[f"{case}_docs"]))
        assert tuple(got.shape) == z[f"{case}_scores"].shape
        np.testing.assert_allclose(got.cpu().numpy(), z[f"{case}_scores"], atol=1e-5)


def test_maxsim_pipeline_matches_oracle(dev, tmp_path):
    cfg, ind, hyb = _system(tmp_path, "maxsim")
    enc = FakeEncoder(**TOY["encoder"])
    docs = orc.bf16_round(enc.encode(TOY["corpus"], convert_to_tensor=False))
    for i, q in enumerate(TOY["queries"]):
        qe = orc.bf16_round(enc.encode(q, convert_to_tensor=False))
        s = orc.maxsim(qe, docs)
        es, ei = orc.topk(s, 10)
        got = ind.colbert_retriever.search(q, k=10)
        assert [g["document_id"] for g in got] == list(ei[0])
        np.testing.assert_allclose([g["score"] for g in got], es[0], atol=1e-3)
        fused = orc.rrf(TOY["bm25"][i]["ids"], list(orc.topk(s, 100)[1][0]))[:50]
        cand = [c for c, _ in fused]
        order = orc.rerank_select(s[0, cand], 10)
        fin = hyb.retrieve(q)
        assert [f["chunk_id"] for f in fin] == [cand[p] for p, _, _ in order]
        assert [f["rank"] for f in fin] == list(range(1, len(fin) + 1))


def test_fp32_index_pipeline_matches_exact_fp32(dev, tmp_path):
    """index_dtype="fp32": search / rerank / retrieve on the encoder's fp32
    values themselves (no bf16 rounding), scores within 1e-4 of fp64."""
    cfg, ind, hyb = _system(tmp_path, "maxsim", index_dtype="fp32")
    assert ind.colbert_retriever.corpus_embeddings.faithful
    enc = FakeEncoder(**TOY["encoder"])
    docs = np.asarray(enc.encode(TOY["corpus"], convert_to_tensor=False), np.float32)
    for i, q in enumerate(TOY["queries"]):
        qe = np.asarray(enc.encode(q, convert_to_tensor=False), np.float32)
        s = orc.maxsim(qe, docs)
        es, ei = orc.topk(s, 10)
        got = ind.colbert_retriever.search(q, k=10)
        assert [g["document_id"] for g in got] == list(ei[0])
        np.testing.assert_allclose([g["score"] for g in got], es[0], atol=1e-4)
        fused = orc.rrf(TOY["bm25"][i]["ids"], list(orc.topk(s, 100)[1][0]))[:50]
        cand = [c for c, _ in fused]
        order = orc.rerank_select(s[0, cand], 10)
        fin = hyb.retrieve(q)
        assert [f["chunk_id"] for f in fin] == [cand[p] for p, _, _ in order]
        np.testing.assert_allclose([f["score"] for f in fin], [sc for _, sc, _ in order], atol=1e-4)


def test_index_save_load_roundtrip_and_reference_format(dev, tmp_path):
    cfg, ind, _ = _system(tmp_path, "maxsim")
    r = ind.colbert_retriever
    before = r.search(TOY["queries"][0], k=7)
    r.corpus_embeddings = None
    r.load()
    assert r.search(TOY["queries"][0], k=7) == before
    # a file in the reference's own layout: {'embeddings': fp32 [N, L, D], 'corpus': [...]}
    enc = FakeEncoder(maxlen=20)
    emb = enc.encode(TOY["corpus"][:9], convert_to_tensor=True)
    os.makedirs(tmp_path / "ref", exist_ok=True)
    torch.save({"embeddings": emb, "corpus": TOY["corpus"][:9]}, tmp_path / "ref" / "index.pt")
    cfg2 = RAGConfig(colbert_index_path=str(tmp_path / "ref"))
    from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever
    r2 = JinaColBERTRetriever(cfg2, encoder=enc)
    r2.load()
    res = r2.search(TOY["queries"][1], k=20)
    assert len(res) == 9 and res[0]["text"] in TOY["corpus"][:9]


def test_pooled_query_and_docs_work(dev):
    """Pooled [D] encodings (SentenceTransformer's default) are 1-token inputs here."""
    from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever

    class Pooled:
        def encode(self, x, convert_to_tensor=True, **_):
            e = FakeEncoder(maxlen=1).encode(x, convert_to_tensor=True)
            return e[..., 0, :] if isinstance(x, list) else e[0]

    r = JinaColBERTRetriever(RAGConfig(), encoder=Pooled())
    r.index_embeddings(Pooled().encode(TOY["corpus"]), TOY["corpus"])
    res = r.search(TOY["corpus"][4], k=3)
    assert res[0]["document_id"] == 4


def test_retrieve_batch_equals_single(dev, tmp_path):
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    B, N = 8, 3000
    Qf = synth.make_queries(B)
    planted = synth.planted_ids(B, N, 10)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev)
    bm = synth.bm25_lists(B, N, planted)
    cfg = RAGConfig()
    ind = DualIndexer(cfg, encoder=FakeEncoder())
    ind.colbert_retriever.corpus_embeddings = ColbertIndex(tokens, doclens)
    hyb = HybridRetriever(cfg, ind, None, verbose=False)
    Q = Qf.to(dev, torch.bfloat16)
    s, i = hyb.retrieve_batch(Q, bm)
    for b in range(B):
        assert set(i[b].tolist()) == set(planted[b].tolist())
        s1, i1 = hyb.retrieve_batch(Q[b:b + 1], bm[b:b + 1])
        assert torch.equal(i1[0], i[b]) and torch.equal(s1[0], s[b])
    # the one-round-trip path equals the stages called one by one
    from hybrid_rag_colbertv2_amd.hybrid import rrf_fuse
    retr = ind.colbert_retriever
    _, ids = retr.search_embeddings(Q, cfg.colbert_top_k)
    cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=cfg.rrf_k, C=cfg.fused_candidates)
    es, ei, _ = retr.rerank_ids(Q, torch.from_numpy(cand).to(dev), cfg.final_top_k)
    assert torch.equal(ei, i) and torch.equal(es, s)


def test_sharded_searcher_single_process(dev):
    from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    g = torch.Generator().manual_seed(0)
    docs = torch.randn(500, 128, 128, generator=g).bfloat16()
    ix = ColbertIndex(docs.to(dev), torch.full((500,), 128, dtype=torch.int32, device=dev))
    Q = torch.randn(3, 32, 128, generator=g).bfloat16().to(dev)
    ss = ShardedSearcher(ix)
    a = ss.search(Q, 10)
    b = ix.search(Q, 10)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    cand = a[1][:, :5].contiguous()
    r1 = ss.rerank(Q, cand, 3)
    r2 = ix.rerank(Q, cand, 3)
    assert all(torch.equal(x, y) for x, y in zip(r1, r2))


def test_pipelined_batches_equal_unpipelined(dev):
    """PipelinedRetriever overlaps batch j+1's scan with batch j's host fusion;
    every batch's result must equal the plain sequential path."""
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever, rrf_fuse
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    N = 20000
    Qall = synth.make_queries(48, seed=5)
    planted = synth.planted_ids(48, N, 10)
    tokens, doclens = synth.make_shard(0, N, Qall, planted, dev)
    ix = ColbertIndex(tokens, doclens)
    bm = synth.bm25_lists(48, N, planted)
    batches = [(Qall[a:b].to(dev, torch.bfloat16), bm[a:b]) for a, b in [(0, 16), (16, 17), (17, 40), (40, 48)]]
    got = PipelinedRetriever(ix, dev).run(batches)
    for (Q, b), (s, i) in zip(batches, got):
        _, ids = ix.search(Q, 100)
        cand = torch.from_numpy(rrf_fuse(b, ids.cpu().numpy())).to(dev)
        es, ei, _ = ix.rerank(Q, cand, 10)
        assert torch.equal(i, ei) and torch.equal(s, es)


def test_pipelined_with_host_bm25_equals_sequential(dev):
    """Stage 1 as a host callable (native BM25 run while the GPU scans): every
    batch equals BM25 (oracle-checked lists) -> search -> RRF -> rerank done
    one step at a time, and the planted docs are the final top-10."""
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever, rrf_fuse
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    N, B = 20000, 40
    Qall = synth.make_queries(B, seed=6)
    planted = synth.planted_ids(B, N, 10)
    tokens, doclens = synth.make_shard(0, N, Qall, planted, dev)
    ix = ColbertIndex(tokens, doclens)
    terms, off, V = synth.bm25_shard(0, N, planted)
    lex = NativeBM25(terms, off, V)
    qt, qo = synth.bm25_queries(B)
    spans = [(0, 16), (16, 17), (17, 40)]

    def fn(a, b):
        return lambda: lex.search(qt[qo[a]:qo[b]], qo[a:b + 1] - qo[a], 100)
    batches = [(Qall[a:b].to(dev, torch.bfloat16), fn(a, b)) for a, b in spans]
    got = PipelinedRetriever(ix, dev).run(batches)
    oi, _ = orc.bm25_topk(terms[:off[2000]], off[:2001], qt, qo, V, 5)   # oracle spot check on a prefix
    pi, _ = NativeBM25(terms[:off[2000]], off[:2001], V).search(qt, qo, 5)
    assert np.array_equal(pi, oi)
    for (a, b), (Q, f), (s, i) in zip(spans, batches, got):
        bm, _ = f()
        _, ids = ix.search(Q, 100)
        cand = torch.from_numpy(rrf_fuse(bm, ids.cpu().numpy())).to(dev)
        es, ei, _ = ix.rerank(Q, cand, 10)
        assert torch.equal(i, ei) and torch.equal(s, es)
        for r in range(b - a):
            assert set(i[r].tolist()) == set(planted[a + r].tolist())


def test_native_exchange_rccl_world1(dev, tmp_path):
    """cbv2_search_sharded_local/_exchange and cbv2_rerank_sharded over torch's
    RCCL communicator (one rank on this box: the all-gather/all-reduce run for
    real with G=1; G>1 is the same code path with a longer receive buffer, and
    the protocol itself is covered at world 2 over gloo)."""
    import torch.distributed as dist
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.bm25 import NativeBM25
    from hybrid_rag_colbertv2_amd.distributed import ShardedSearcher
    from hybrid_rag_colbertv2_amd.hybrid import PipelinedRetriever
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        N, B = 5000, 12
        Qf = synth.make_queries(B, seed=8)
        planted = synth.planted_ids(B, N, 10)
        tokens, doclens = synth.make_shard(0, N, Qf, planted, dev)
        ix = ColbertIndex(tokens, doclens)
        terms, off, V = synth.bm25_shard(0, N, planted)
        lex = NativeBM25(terms, off, V)
        qt, qo = synth.bm25_queries(B)
        Q = Qf.to(dev, torch.bfloat16)
        ss = ShardedSearcher(ix, native=True)
        assert ss._nx.world == 1 and ss._nx.rank == 0
        s, i, li = ss.search_hybrid(Q, 100, lambda: lex.search(qt, qo, 100))
        es, ei = ix.search(Q, 100)
        bi, _ = lex.search(qt, qo, 100)
        assert torch.equal(s, es) and torch.equal(i, ei)
        assert np.array_equal(li.cpu().numpy(), bi)
        s2, i2 = ss.search(Q, 37)
        assert torch.equal(i2, ix.search(Q, 37)[1])
        cand = i[:, :50].contiguous()
        r = ss.rerank(Q, cand, 10)
        er = ix.rerank(Q, cand, 10)
        assert all(torch.equal(a, b) for a, b in zip(r, er))
        # the pipelined path over the native exchange equals the plain one
        batches = [(Q[a:b], (lambda a=a, b=b: lex.search(qt[qo[a]:qo[b]], qo[a:b + 1] - qo[a], 100)))
                   for a, b in [(0, 5), (5, 12)]]
        got = PipelinedRetriever(ss, dev).run(batches)
        ref = PipelinedRetriever(ix, dev).run(batches)
        for (gs, gi), (rs, ri) in zip(got, ref):
            assert torch.equal(gi, ri) and torch.equal(gs, rs)
        # sharded query encoding over RCCL (device tensors through the all-gather)
        from hybrid_rag_colbertv2_amd.distributed import encode_queries_sharded
        from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
        texts = ["late interaction on mi355x", "bm25 plus colbert", "top fifty to top ten"]
        qe = encode_queries_sharded(FakeEncoder(), texts)
        assert qe.device.type == "cuda" and qe.dtype == torch.bfloat16
        assert torch.equal(qe.cpu(), FakeEncoder().encode(texts).to(torch.bfloat16))
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


def test_native_index_file_roundtrip(dev, tmp_path):
    """HBM -> native file -> HBM, whole and by rank shards (multi-chunk staging:
    3000 docs = 98 MB > one 64 MiB pinned buffer), bf16 and MXFP8, and the
    retriever's save_native / load_native."""
    from hybrid_rag_colbertv2_amd import synth
    from hybrid_rag_colbertv2_amd.distributed import shard_range
    from hybrid_rag_colbertv2_amd.index import ColbertIndex, index_file_info
    from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever
    N = 3000
    Qf = synth.make_queries(4, seed=9)
    planted = synth.planted_ids(4, N, 10)
    tokens, doclens = synth.make_shard(0, N, Qf, planted, dev)
    doclens[::7] = torch.randint(0, 129, (len(doclens[::7]),), device=dev, dtype=torch.int32)
    Q = Qf.to(dev, torch.bfloat16)
    for fp8 in (False, True):
        ix = ColbertIndex.mxfp8(tokens, doclens, id_base=50) if fp8 else ColbertIndex(tokens, doclens, id_base=50)
        path = str(tmp_path / f"ix{int(fp8)}.cbv2")
        ix.save(path)
        assert index_file_info(path)[1:] == (N, 50)
        full = ColbertIndex.load(path, device=dev)
        assert full.fp8 == fp8 and full.id_base == 50
        assert torch.equal(full.tokens, ix.tokens) and torch.equal(full.doclens, ix.doclens)
        if fp8:
            assert torch.equal(full.scales, ix.scales)
        s0, i0 = ix.search(Q, 20)
        s1, i1 = full.search(Q, 20)
        assert torch.equal(s0, s1) and torch.equal(i0, i1)
        for r in range(3):
            a, b = shard_range(N, r, 3)
            sh = ColbertIndex.load(path, device=dev, begin=a, end=b)
            assert sh.id_base == 50 + a and torch.equal(sh.tokens, ix.tokens[a:b])
            assert torch.equal(sh.doclens, ix.doclens[a:b])
    cfg = RAGConfig()
    cfg.colbert_index_path = str(tmp_path / "colbert")
    r = JinaColBERTRetriever(cfg, encoder=FakeEncoder())
    r.index_embeddings([torch.randn(int(k), 128) for k in torch.randint(1, 129, (40,))], corpus=[f"d{i}" for i in range(40)])
    r.save_native()
    r2 = JinaColBERTRetriever(cfg, encoder=FakeEncoder())
    r2.load()                                   # no index.pt: the native file is loaded
    assert r2.corpus == r.corpus and torch.equal(r2.corpus_embeddings.tokens, r.corpus_embeddings.tokens)


def test_jina_encoder_gpu_matches_fp32_cpu(dev):
    """The encoder on PyTorch-ROCm (bf16, SDPA) vs an fp32 CPU forward of the
    same weights (tiny config of the same architecture), the HIP-graph replay
    vs eager, and the encoder driving the retriever end to end."""
    import copy
    from hybrid_rag_colbertv2_amd.jina_encoder import (HashTokenizer, JinaColBERTConfig, JinaColBERTEncoder,
                                                       JinaColBERTModel)
    from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever
    c = JinaColBERTConfig.tiny()
    torch.manual_seed(1)
    m = JinaColBERTModel(c)
    cpu = JinaColBERTEncoder(copy.deepcopy(m), HashTokenizer(c.vocab_size), device="cpu", dtype=torch.float32)
    gpu = JinaColBERTEncoder(m, HashTokenizer(c.vocab_size), device=dev, dtype=torch.bfloat16)
    qs = ["late interaction over token embeddings", "mi355x hbm bandwidth", "colbert"]
    a = cpu.encode(qs, is_query=True)
    b = gpu.encode(qs, is_query=True).cpu()
    cos = (a * b).sum(-1)
    assert float(cos.min()) > 0.99, float(cos.min())
    docs = ["a short doc", " ".join(f"token{i}" for i in range(60))]
    for x, y in zip(cpu.encode(docs, is_query=False), gpu.encode(docs, is_query=False)):
        assert x.shape == y.shape and float((x * y.cpu()).sum(-1).min()) > 0.99
    ids, mask = gpu.query_batch([gpu._ids(q) for q in qs])
    eager = gpu.encode_ids(ids, mask)
    gpu.capture_queries(len(qs))
    assert torch.equal(gpu.encode_ids(ids, mask), eager)
    cfg = RAGConfig(index_dtype="bf16")     # the check below scores the bf16 index's own values
    r = JinaColBERTRetriever(cfg, encoder=gpu)
    corpus = [f"doc {i} about topic {i % 7} and thing {i % 3}" for i in range(50)]
    r.index_embeddings(gpu.encode(corpus, is_query=False), corpus=corpus)
    res = r.search("doc 17 about topic 3", k=5)
    q = gpu.encode("doc 17 about topic 3", is_query=True)          # random weights: check arithmetic, not semantics
    ix = r.corpus_embeddings
    ref = orc.maxsim(orc.bf16_round(q[None].cpu().numpy()), ix.tokens.float().cpu().numpy(),
                     ix.doclens.cpu().numpy())[0]
    assert [x["document_id"] for x in res] == [int(i) for i in np.argsort(-ref, kind="stable")[:5]]
    np.testing.assert_allclose([x["score"] for x in res], np.sort(ref)[::-1][:5], atol=1e-3)


def test_faithful_index_native_file_roundtrip(dev, tmp_path):
    """An fp32-faithful index persists as hi + residual native files + bounds,
    and loads back (whole and by rank shard) with identical search results."""
    from hybrid_rag_colbertv2_amd.distributed import shard_range
    from hybrid_rag_colbertv2_amd.index import ColbertIndex
    g = torch.Generator().manual_seed(4)
    N = 2500
    x = torch.randn(N, 128, 128, generator=g)
    x = x / x.norm(dim=-1, keepdim=True)
    doclens = torch.randint(0, 129, (N,), generator=g, dtype=torch.int32)
    Q = torch.randn(5, 32, 128, generator=g)
    Q = (Q / Q.norm(dim=-1, keepdim=True)).to(dev)
    ix = ColbertIndex.faithful_f32(x.to(dev), doclens.to(dev), id_base=7)
    path = str(tmp_path / "f.cbv2")
    ix.save(path)
    back = ColbertIndex.load(path, device=dev)
    assert back.faithful and back.bounds == ix.bounds and back.id_base == 7
    assert torch.equal(back.residual, ix.residual) and torch.equal(back.tokens, ix.tokens)
    s0, i0 = ix.search(Q, 30)
    s1, i1 = back.search(Q, 30)
    assert torch.equal(s0, s1) and torch.equal(i0, i1)
    a, b = shard_range(N, 1, 3)
    sh = ColbertIndex.load(path, device=dev, begin=a, end=b)
    assert sh.faithful and sh.id_base == 7 + a and torch.equal(sh.residual, ix.residual[a:b])


def test_default_config_is_fp32_faithful():
    from hybrid_rag_colbertv2_amd.config import RAGConfig
    assert RAGConfig().index_dtype == "fp32"
