"""GPU: bounded-memory ingest (the reference's index() encodes
the whole corpus at once and torch.saves it, local_rag_complete.py:728-746).

* IndexBuilder (batch by batch into HBM) == the one-shot index, bit for bit,
  for bf16, MXFP8 and fp32-faithful (same tokens, scales, residual, bounds).
* IndexWriter (batches D2H straight into the native file) == ColbertIndex.save.
* JinaColBERTRetriever.index in batches: a small corpus keeps the reference's
  index.pt; a large one (above index_pt_max_docs) is saved as index.cbv2 and
  reloads to the same search results.
* A 1M-doc ingest into HBM through the synthetic encoder keeps host RSS growth
  under 2 GB and the planted positives on top.
"""
import numpy as np
import pytest
import torch

from hybrid_rag_colbertv2_amd import FakeEncoder, RAGConfig, synth
from hybrid_rag_colbertv2_amd.index import ColbertIndex, IndexBuilder, IndexWriter
from hybrid_rag_colbertv2_amd.retriever import JinaColBERTRetriever

pytestmark = pytest.mark.gpu


def _embs(seed, n, ragged=True):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 128, 128, generator=g)
    x = x / x.norm(dim=-1, keepdim=True)
    if not ragged:
        return x
    lens = torch.randint(1, 129, (n,), generator=g)
    return [x[i, : int(lens[i])] for i in range(n)]


@pytest.mark.parametrize("dtype", ["bf16", "fp8", "fp32"])
def test_builder_equals_one_shot(dev, dtype):
    embs = _embs(1, 900)
    ref = ColbertIndex.from_embeddings(embs, device=dev, dtype=dtype)
    b = IndexBuilder(900, dev, dtype)
    for a in range(0, 900, 128):
        b.append(embs[a:a + 128])
    ix = b.finish()
    assert torch.equal(ix.tokens, ref.tokens) and torch.equal(ix.doclens, ref.doclens)
    if dtype == "fp8":
        assert torch.equal(ix.scales, ref.scales)
    if dtype == "fp32":
        assert torch.equal(ix.residual, ref.residual) and ix.bounds == ref.bounds
    Q = torch.randn(20, 32, 128, device=dev)
    s1, i1 = ix.search(Q, 50)
    s0, i0 = ref.search(Q, 50)
    assert torch.equal(i1, i0) and torch.equal(s1, s0)


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_writer_equals_save(dev, tmp_path, dtype):
    embs = _embs(2, 3000, ragged=False)
    ref = ColbertIndex.from_embeddings(embs, device=dev, dtype=dtype, id_base=5)
    ref.save(str(tmp_path / "whole.cbv2"))
    with IndexWriter(str(tmp_path / "streamed.cbv2"), 3000, dtype, id_base=5, device=dev) as w:
        for a in range(0, 3000, 700):
            w.append(embs[a:a + 700].to(dev))
    assert open(tmp_path / "whole.cbv2", "rb").read() == open(tmp_path / "streamed.cbv2", "rb").read()
    with pytest.raises(ValueError):
        w2 = IndexWriter(str(tmp_path / "partial.cbv2"), 10, dtype, device=dev)
        w2.append(embs[:3].to(dev))
        w2.close()


def test_retriever_index_batches_and_persists(dev, tmp_path):
    corpus = [f"document {i} about topic {i % 7} and item {i % 13}" for i in range(600)]
    small = RAGConfig(colbert_index_path=str(tmp_path / "small"), ingest_batch=64)
    r = JinaColBERTRetriever(small, encoder=FakeEncoder())
    r.index(corpus)
    assert (tmp_path / "small" / "index.pt").exists()
    ref = r.search("topic 3 item 5", k=20)
    big = RAGConfig(colbert_index_path=str(tmp_path / "big"), ingest_batch=64, index_pt_max_docs=100)
    r2 = JinaColBERTRetriever(big, encoder=FakeEncoder())
    r2.index(corpus)
    assert not (tmp_path / "big" / "index.pt").exists() and (tmp_path / "big" / "index.cbv2").exists()
    assert r2.search("topic 3 item 5", k=20) == ref
    r3 = JinaColBERTRetriever(big, encoder=FakeEncoder())
    r3.load()                                        # no index.pt: the native file + corpus.json
    assert r3.search("topic 3 item 5", k=20) == ref
    r4 = JinaColBERTRetriever(small, encoder=FakeEncoder())
    r4.load()                                        # the reference's index.pt
    assert r4.search("topic 3 item 5", k=20) == ref


def test_1m_ingest_bounded_host_memory(dev):
    import psutil
    N, B = 1_000_000, 64
    torch.cuda.empty_cache()
    Qf = synth.make_queries(B, 32, seed=1)
    planted = synth.planted_ids(B, N, 10, seed=2)
    enc = synth.SyntheticDocEncoder(Qf, planted, dev)
    proc = psutil.Process()
    rss0 = peak = proc.memory_info().rss
    b = IndexBuilder(N, dev, "bf16")
    for a in range(0, N, 8192):
        b.append(enc.encode(enc.texts(a, min(N, a + 8192))))
        peak = max(peak, proc.memory_info().rss)
    ix = b.finish()
    assert (peak - rss0) < 2 * 2 ** 30, (peak - rss0) / 2 ** 30
    _, ids = ix.search(Qf.to(dev, torch.bfloat16), 100)
    ids = ids.cpu().numpy()
    assert all(set(ids[q, :10]) == set(planted[q]) for q in range(B))
    # the same tokens as the one-shot generator, on a slice
    ref, _ = synth.make_shard(123_456, 123_456 + 3000, Qf, planted, dev)
    assert torch.equal(ix.tokens[123_456:126_456], ref)


def test_reindex_same_directory_serves_latest_format(dev, tmp_path):
    """index() writes ONE persistence format and deletes the other's
    files, so load() after re-indexing never serves an earlier corpus."""
    small = [f"small doc {i} topic {i % 5}" for i in range(40)]
    large = [f"large doc {i} topic {i % 9}" for i in range(300)]
    cfg = RAGConfig(colbert_index_path=str(tmp_path / "ix"), index_pt_max_docs=100, index_dtype="bf16")
    d = tmp_path / "ix"
    for corpus, fmt in ((small, "pt"), (large, "cbv2"), (small, "pt")):
        r = JinaColBERTRetriever(cfg, encoder=FakeEncoder())
        r.index(corpus)
        assert (d / "index.pt").exists() == (fmt == "pt")
        assert (d / "index.cbv2").exists() == (fmt == "cbv2")
        assert (d / "index.corpus.json").exists() == (fmt == "cbv2")
        want = r.search("doc 7 topic 2", k=5)
        r2 = JinaColBERTRetriever(cfg, encoder=FakeEncoder())
        r2.load()
        assert r2.corpus == corpus and r2.search("doc 7 topic 2", k=5) == want
    # the literal scorer always keeps index.pt (its means need the fp32 embeddings)
    lit = RAGConfig(colbert_index_path=str(tmp_path / "lit"), index_pt_max_docs=100, scorer="ref_meanpool_cosine")
    r = JinaColBERTRetriever(lit, encoder=FakeEncoder())
    r.index(large)
    assert (tmp_path / "lit" / "index.pt").exists() and not (tmp_path / "lit" / "index.cbv2").exists()
    r2 = JinaColBERTRetriever(lit, encoder=FakeEncoder())
    r2.load()
    assert r2.search("doc 7 topic 2", k=5) == r.search("doc 7 topic 2", k=5)


def test_faithful_sidecars_never_pair_with_other_tokens(dev, tmp_path):
    """a bf16 save over a faithful file removes its .resid /
    .bounds.json; sidecars copied from another save are refused on load."""
    import shutil
    a = ColbertIndex.from_embeddings(_embs(11, 50, ragged=False), device=dev, dtype="fp32")
    b = ColbertIndex.from_embeddings(_embs(12, 50, ragged=False), device=dev, dtype="fp32")
    p = str(tmp_path / "f.cbv2")
    a.save(p)
    assert ColbertIndex.load(p, device=dev).faithful
    shutil.copy(p + ".resid", tmp_path / "a.resid")
    shutil.copy(p + ".bounds.json", tmp_path / "a.bounds.json")
    b.save(p)
    back = ColbertIndex.load(p, device=dev)
    assert back.faithful and torch.equal(back.residual, b.residual)
    shutil.copy(tmp_path / "a.resid", p + ".resid")
    shutil.copy(tmp_path / "a.bounds.json", p + ".bounds.json")
    with pytest.raises(ValueError, match="not written with"):
        ColbertIndex.load(p, device=dev)
    bf = ColbertIndex.from_embeddings(_embs(13, 50, ragged=False), device=dev, dtype="bf16")
    bf.save(p)
    import os
    assert not os.path.exists(p + ".resid") and not os.path.exists(p + ".bounds.json")
    assert not ColbertIndex.load(p, device=dev).faithful
