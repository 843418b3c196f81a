"""CPU: the Jina-ColBERT encoder module (hybrid-rag-colbertv2_amd/jina_encoder.py,
SURVEY §8 a9/f1) on a tiny config of the same architecture, fp32.  Parity with
the real jina-colbert-v2 weights is unpinned (none offline); these pin the
ColBERT conventions and the masking arithmetic."""
import torch

from hybrid_rag_colbertv2_amd.jina_encoder import (HashTokenizer, JinaColBERTConfig, JinaColBERTEncoder,
                                                   JinaColBERTModel)


def _enc():
    c = JinaColBERTConfig.tiny()
    torch.manual_seed(0)
    return JinaColBERTEncoder(JinaColBERTModel(c), HashTokenizer(c.vocab_size), device="cpu", dtype=torch.float32)


def test_query_augmentation_and_norms():
    e = _enc()
    c = e.config
    ids, mask = e.query_batch([[5, 6, 7]])
    assert ids.shape == (1, c.query_maxlen) and bool(mask.all())
    assert ids[0, :6].tolist() == [c.cls_id, c.query_marker_id, 5, 6, 7, c.sep_id]
    assert (ids[0, 6:] == c.mask_id).all()                        # [MASK] augmentation, attended
    q = e.encode(["what is late interaction", "colbert"], is_query=True)
    assert q.shape == (2, c.query_maxlen, c.colbert_dim)
    torch.testing.assert_close(q.norm(dim=-1), torch.ones(2, c.query_maxlen))
    assert torch.equal(e.encode("colbert", is_query=True), q[1])   # batch-invariant


def test_doc_padding_is_masked():
    """A doc encoded alone equals the same doc padded inside a longer batch."""
    e = _enc()
    short, long = "late interaction retrieval", " ".join(f"w{i}" for i in range(40))
    alone = e.encode([short], is_query=False)[0]
    both = e.encode([short, long], is_query=False)
    assert alone.shape[0] == 3 + 3 and both[1].shape[0] == 43
    torch.testing.assert_close(both[0], alone, atol=1e-5, rtol=1e-5)


def test_doc_truncation():
    e = _enc()
    d = e.encode(" ".join(f"w{i}" for i in range(500)), is_query=False)
    assert d.shape == (e.config.doc_maxlen, e.config.colbert_dim)
