"""Long documents (index ld = 256 / 512 / 1024 token slots, bf16): the
reference's chunks run to 1024 BERT tokens (local_rag_complete.py:63-64);
MaxSim over a long doc is the same sum over query tokens of the max over ALL
its tokens (LRC:807-812 docstring / north_star).  The doc-interleaved scan
spans ld/64 iterations per doc group and the direct scan and the rerank work
128 tokens at a time, carrying the row maxima.  Checked against the float64
oracle (1e-3), the oracle's selection of the GPU's own scores (bit for bit),
and bit-identity with the 128-slot index on docs of <= 128 tokens."""
import numpy as np
import pytest
import torch

from _parity import assert_ranking_consistent, assert_selection_exact
from hybrid_rag_colbertv2_amd.index import ColbertIndex
from oracle import oracle as orc

pytestmark = pytest.mark.gpu
ATOL = 1e-3


def rand_unit(g, *shape):
    x = torch.randn(*shape, generator=g)
    return x / x.norm(dim=-1, keepdim=True)


def make_case(seed, N, ld, B):
    g = torch.Generator().manual_seed(seed)
    docs = rand_unit(g, N, ld, 128).bfloat16()
    doclens = torch.randint(0, ld + 1, (N,), generator=g, dtype=torch.int32)
    doclens[:6] = torch.tensor([0, 1, 127, 128, 129, ld], dtype=torch.int32)
    Q = rand_unit(g, B, 32, 128).bfloat16()
    return docs, doclens, Q


@pytest.mark.parametrize("ld,N", [(256, 3000), (512, 1200), (1024, 500)])
@pytest.mark.parametrize("B", [1, 5, 40])
def test_long_docs_score_search_rerank(dev, ld, N, B):
    docs, doclens, Q = make_case(ld + B, N, ld, B)
    ix = ColbertIndex(docs.to(dev), doclens.to(dev), id_base=3)
    assert ix.ld == ld
    got = ix.score(Q.to(dev)).cpu().numpy()
    ref = orc.maxsim(Q.float().numpy(), docs.float().numpy(), doclens.numpy())
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(got[fin], ref[fin], atol=ATOL, rtol=0)
    s, i = ix.search(Q.to(dev), 50)
    assert_selection_exact(i.cpu().numpy(), s.cpu().numpy(), got, 50, id_base=3)
    assert_ranking_consistent(i.cpu().numpy(), ref, ATOL, id_base=3)
    g = np.random.default_rng(ld)
    cand = g.integers(0, N, size=(B, 60)).astype(np.int32) + 3
    rs, ri, rp = ix.rerank(Q.to(dev), torch.from_numpy(cand).to(dev), 10)
    raw = ix.rerank(Q.to(dev), torch.from_numpy(cand).to(dev), 0).cpu().numpy()
    np.testing.assert_array_equal(raw, got[np.arange(B)[:, None], cand - 3])     # same bits as the scan
    for b in range(B):
        exp = orc.rerank_select(raw[b], 10)
        assert [int(x) for x in rp[b].cpu()] == [e[0] for e in exp], b


@pytest.mark.parametrize("ld", [256, 1024])
def test_long_index_of_short_docs_bit_identical(dev, ld):
    """Docs of <= 128 tokens in a long-doc index score exactly as in the
    128-slot index (every scan path: B = 1, 5, 40)."""
    g = torch.Generator().manual_seed(ld)
    N = 2000
    short = rand_unit(g, N, 128, 128).bfloat16()
    doclens = torch.randint(0, 129, (N,), generator=g, dtype=torch.int32)
    long = torch.zeros((N, ld, 128), dtype=torch.bfloat16)
    long[:, :128] = short
    long[:, 128:] = 7.0                                    # padding rows never score
    a = ColbertIndex(short.to(dev), doclens.to(dev))
    b = ColbertIndex(long.to(dev), doclens.to(dev))
    for B in (1, 5, 40):
        Q = rand_unit(g, B, 32, 128).bfloat16().to(dev)
        assert torch.equal(a.score(Q), b.score(Q)), B


def test_long_docs_dynamic_tail(dev):
    """ld = 256 over a corpus large enough for the dynamic tail (B = 40: two
    query groups): every score equals a small static-split index's."""
    N, ld, B = 12000, 256, 40
    g = torch.Generator(device=dev).manual_seed(3)
    docs = torch.randn(N, ld, 128, device=dev, generator=g)
    docs = (docs / docs.norm(dim=-1, keepdim=True)).bfloat16()
    doclens = torch.randint(0, ld + 1, (N,), device=dev, generator=g, dtype=torch.int32)
    Q = torch.randn(B, 32, 128, device=dev, generator=g)
    Q = (Q / Q.norm(dim=-1, keepdim=True)).bfloat16()
    ix = ColbertIndex(docs, doclens)
    full = ix.score(Q)
    assert ix.last_scan_plan()["dynamic_tail"]
    for a, e in [(0, 500), (N - 1500, N)]:
        part = ColbertIndex(docs[a:e].contiguous(), doclens[a:e].contiguous()).score(Q)
        assert torch.equal(part, full[:, a:e]), (a, e)


def test_from_embeddings_picks_long_ld(dev):
    g = torch.Generator().manual_seed(1)
    embs = [rand_unit(g, L, 128) for L in (5, 130, 300, 64)]
    ix = ColbertIndex.from_embeddings(embs, device=dev)
    assert ix.ld == 512 and ix.doclens.cpu().tolist() == [5, 130, 300, 64]
    Q = rand_unit(g, 2, 32, 128)
    docs = torch.zeros((4, 512, 128))
    for i, e in enumerate(embs):
        docs[i, : e.shape[0]] = e.bfloat16().float()
    ref = orc.maxsim(Q.bfloat16().float().numpy(), docs.numpy(), np.array([5, 130, 300, 64]))
    np.testing.assert_allclose(ix.score(Q.to(dev)).cpu().numpy(), ref, atol=ATOL, rtol=0)
    fx = ColbertIndex.from_embeddings(embs, device=dev, dtype="fp8")
    assert fx.fp8 and fx.ld == 512 and tuple(fx.scales.shape) == (4, 512, 2)


@pytest.mark.parametrize("ld,N", [(256, 2500), (1024, 400)])
@pytest.mark.parametrize("B", [1, 5, 40])
def test_mxfp8_long_docs(dev, ld, N, B):
    """MXFP8 index of long documents: every scan shape (B=1 direct, B=5 the
    4-wave x 2-query shape, B=40 8 waves x 8 queries) within 2e-3 of the
    float64 oracle on the dequantised values; search = the oracle's selection
    of the GPU's own scores; rerank raw scores = the scan's bits; docs of <=
    128 tokens score as in a 128-slot MXFP8 index."""
    from hybrid_rag_colbertv2_amd.index import quantize_mxfp8
    docs, doclens, Q = make_case(ld * 7 + B, N, ld, B)
    ix = ColbertIndex.mxfp8(docs.to(dev), doclens.to(dev), id_base=3)
    assert ix.fp8 and ix.ld == ld
    qq, qs = quantize_mxfp8(Q.to(dev))
    Qd = orc.mxfp8_dequant(qq.cpu().numpy(), qs.cpu().numpy())
    Dd = orc.mxfp8_dequant(ix.tokens.cpu().numpy(), ix.scales.cpu().numpy())
    ref = orc.maxsim(Qd, Dd, doclens.numpy())
    got = ix.score(Q.to(dev)).cpu().numpy()
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(ref))
    fin = np.isfinite(ref)
    np.testing.assert_allclose(got[fin], ref[fin], atol=2e-3, rtol=0)
    s, i = ix.search(Q.to(dev), 50)
    assert_selection_exact(i.cpu().numpy(), s.cpu().numpy(), got, 50, id_base=3)
    cand = np.random.default_rng(ld + B).integers(0, N, size=(B, 60)).astype(np.int32) + 3
    raw = ix.rerank(Q.to(dev), torch.from_numpy(cand).to(dev), 0).cpu().numpy()
    np.testing.assert_array_equal(raw, got[np.arange(B)[:, None], cand - 3])
    short = (doclens <= 128).nonzero().flatten()[:300]
    sx = ColbertIndex.mxfp8(docs[short, :128].contiguous().to(dev), doclens[short].contiguous().to(dev))
    assert np.array_equal(sx.score(Q.to(dev)).cpu().numpy(), got[:, short.numpy()])


def make_f32_case(seed, N, ld, B):
    """fp32 docs of up to ld tokens (the reference keeps fp32 encoder output,
    LRC:735-746) with 3 planted docs per query whose best-matching tokens sit
    past token 128."""
    g = torch.Generator().manual_seed(seed)
    docs = rand_unit(g, N, ld, 128)
    doclens = torch.randint(0, ld + 1, (N,), generator=g, dtype=torch.int32)
    doclens[:5] = torch.tensor([0, 1, 128, 129, ld], dtype=torch.int32)
    Q = rand_unit(g, B, 32, 128)
    for b in range(B):
        for j in range(3):
            d = 5 + (97 * b + 31 * j) % (N - 5)
            docs[d, ld - 40: ld - 8] = Q[b] + 0.2 * rand_unit(g, 32, 128)
            doclens[d] = ld
    return docs, doclens, Q


@pytest.mark.parametrize("ld,N", [(256, 2500), (512, 1200)])
def test_faithful_long_docs(dev, ld, N):
    """fp32-faithful index of long documents: scores within 1e-4 of the fp64
    oracle of the fp32 values, the certified band search, doc-major ==
    pair-major rescoring bit for bit, rerank."""
    from _parity import assert_ids_match_separated
    from hybrid_rag_colbertv2_amd import _lib
    B, k = 5, 50
    docs, doclens, Q = make_f32_case(ld + N, N, ld, B)
    ix = ColbertIndex.faithful_f32(docs.to(dev), doclens.to(dev), id_base=7)
    assert ix.ld == ld and ix.faithful
    exact = orc.maxsim(Q.numpy(), docs.numpy(), doclens.numpy())
    got = ix.score(Q.to(dev)).cpu().numpy()
    np.testing.assert_array_equal(np.isneginf(got), np.isneginf(exact))
    fin = np.isfinite(exact)
    np.testing.assert_allclose(got[fin], exact[fin], atol=1e-4, rtol=0)
    s, i = ix.search(Q.to(dev), k)
    assert (ix.last_band.cpu().numpy() >= k).all()
    rs, ri = orc.topk(exact, k, id_base=7)
    np.testing.assert_allclose(s.cpu().numpy(), rs, atol=1e-4, rtol=0)
    assert_ranking_consistent(i.cpu().numpy(), exact, 1e-4, id_base=7)
    assert_ids_match_separated(i.cpu().numpy(), ri, rs, 1e-4, min_frac=0.02)
    planted = {(b, 5 + (97 * b + 31 * j) % (N - 5) + 7) for b in range(B) for j in range(3)}
    assert planted <= {(b, int(x)) for b in range(B) for x in i[b, :3].cpu()}
    ix.set_option(_lib.OPT_BAND_DOC_MAJOR, 0)
    s0, i0 = ix.search(Q.to(dev), k)
    assert torch.equal(s0, s) and torch.equal(i0, i)
    cand = torch.from_numpy(np.random.default_rng(ld).integers(0, N, size=(B, 40)).astype(np.int32) + 7)
    cs, ci, cp = ix.rerank(Q.to(dev), cand.to(dev), 10)
    es, ei, ep = orc.rerank(Q.numpy(), docs.numpy(), doclens.numpy(), cand.numpy(), 10, id_base=7)
    np.testing.assert_allclose(cs.cpu().numpy(), es, atol=1e-4, rtol=0)
    assert_ids_match_separated(ci.cpu().numpy(), ei, es, 1e-4)


@pytest.mark.parametrize("dtype", ["bf16", "fp32", "fp8"])
def test_long_docs_native_file_and_builder(dev, tmp_path, dtype):
    """A long-document index (bf16, or fp32-faithful: hi + residual files)
    through the native file (whole and by doc range) scores bit-identically;
    IndexBuilder grows its token slots 128 -> 512 when a later batch holds a
    longer doc and equals from_embeddings of the whole list."""
    from hybrid_rag_colbertv2_amd.index import IndexBuilder, index_file_layout
    g = torch.Generator().manual_seed(11)
    lens = [int(x) for x in torch.randint(1, 129, (300,), generator=g)] + [300, 17, 512, 90] + [5] * 40
    embs = [rand_unit(g, L, 128) for L in lens]
    Q = rand_unit(g, 3, 32, 128).to(dev)
    Qs = Q if dtype == "fp32" else Q.bfloat16()
    ix = ColbertIndex.from_embeddings(embs, device=dev, dtype=dtype, id_base=100)
    assert ix.ld == 512
    ref = ix.score(Qs)
    b = IndexBuilder(len(embs), device=dev, dtype=dtype, id_base=100)
    for a in range(0, len(embs), 150):
        b.append(embs[a:a + 150])
    bx = b.finish()
    assert bx.ld == 512 and torch.equal(bx.score(Qs), ref)
    path = str(tmp_path / "long.cbv2")
    ix.save(path)
    assert index_file_layout(path)[1:] == (len(embs), 100, 512)
    assert torch.equal(ColbertIndex.load(path, device=dev).score(Qs), ref)
    part = ColbertIndex.load(path, device=dev, begin=290, end=310)
    assert part.id_base == 390 and part.faithful == (dtype == "fp32")
    assert torch.equal(part.score(Qs), ref[:, 290:310])


class _LongChunkEncoder:
    """Docs: one unit vector per word, no padding (chunks of 20-600 words, as
    the reference's 256-1024-token chunks, LRC:63-64); queries: 32 rows
    (words, then [PAD]<i> vectors) like Jina-ColBERT's query augmentation."""

    def __init__(self):
        from hybrid_rag_colbertv2_amd.encoder import FakeEncoder
        self.fe = FakeEncoder(maxlen=32)

    def encode(self, texts, convert_to_tensor=True, is_query=True, **_):
        if is_query:
            return self.fe.encode(texts, convert_to_tensor=True)
        one = isinstance(texts, str)
        out = [torch.from_numpy(np.stack([self.fe._vec(w) for w in t.lower().split()]))
               for t in ([texts] if one else texts)]
        return out[0] if one else out


def test_long_chunks_end_to_end_default_config(dev, tmp_path):
    """JinaColBERTRetriever with the DEFAULT config (fp32-faithful index) on
    chunks of up to 600 tokens, ingested in batches (the builder grows to 1024
    slots): search ids/scores vs the float64 oracle of the fp32 values (1e-4),
    the text rerank API, and index.pt persistence reloading bit-identically."""
    from hybrid_rag_colbertv2_amd import RAGConfig, JinaColBERTRetriever
    rng = np.random.default_rng(5)
    vocab = [f"w{i}" for i in range(400)]
    lens = rng.integers(20, 200, size=60)
    lens[[7, 33, 50]] = [600, 450, 300]
    corpus = [" ".join(rng.choice(vocab, size=int(L))) for L in lens]
    cfg = RAGConfig(colbert_index_path=str(tmp_path / "colbert"))
    assert cfg.index_dtype == "fp32"
    enc = _LongChunkEncoder()
    r = JinaColBERTRetriever(cfg, encoder=enc)
    r.index(corpus, batch_size=16)
    ix = r.corpus_embeddings
    assert ix.faithful and ix.ld == 1024 and ix.doclens.cpu().tolist() == [int(x) for x in lens]
    docs = np.zeros((60, 1024, 128), np.float32)
    for i, e in enumerate(enc.encode(corpus, is_query=False)):
        docs[i, : e.shape[0]] = e.numpy()
    queries = [" ".join(rng.choice(vocab, size=6)) for _ in range(4)] + [corpus[7][:60]]
    for q in queries:
        qe = enc.encode(q).numpy()[None]
        s = orc.maxsim(qe, docs, lens)
        es, ei = orc.topk(s, 10)
        got = r.search(q, k=10)
        np.testing.assert_allclose([g["score"] for g in got], es[0], atol=1e-4, rtol=0)
        sep = np.abs(np.diff(es[0])) > 1e-4
        for j, g in enumerate(got):
            if (j == 0 or sep[j - 1]) and (j == 9 or sep[j]):
                assert g["document_id"] == int(ei[0, j]), (q, j)
        assert got[0]["text"] == corpus[got[0]["document_id"]]
    cand = [3, 7, 50, 12]
    rr = r.rerank(queries[-1], [corpus[i] for i in cand], k=4)
    s_c = orc.maxsim(enc.encode(queries[-1]).numpy()[None], docs[cand], lens[cand])[0]
    np.testing.assert_allclose([x["score"] for x in rr], np.sort(s_c)[::-1], atol=1e-4, rtol=0)
    assert [x["rank"] for x in rr] == [1, 2, 3, 4]
    assert rr[0]["result_index"] == int(np.argmax(s_c))
    # stage 3 of HybridRetriever (_colbert_rerank -> rerank_ids): candidate tiles gathered by id
    qe = torch.from_numpy(enc.encode(queries[1]).numpy()).to(dev)[None]
    cand_ids = torch.tensor([[50, 7, 33, 0, 12, 59]], dtype=torch.int32, device=dev)
    rs, ri, rp = r.rerank_ids(qe, cand_ids, 4)
    s_ref = orc.maxsim(qe.cpu().numpy(), docs[[50, 7, 33, 0, 12, 59]], lens[[50, 7, 33, 0, 12, 59]])[0]
    np.testing.assert_allclose(rs[0].cpu().numpy(), np.sort(s_ref)[::-1][:4], atol=1e-4, rtol=0)
    ref = r.corpus_embeddings.score(torch.from_numpy(enc.encode(queries[0]).numpy()).to(dev))
    r2 = JinaColBERTRetriever(cfg, encoder=enc)
    r2.load()
    assert r2.corpus_embeddings.ld == 1024
    assert torch.equal(r2.corpus_embeddings.score(torch.from_numpy(enc.encode(queries[0]).numpy()).to(dev)), ref)
