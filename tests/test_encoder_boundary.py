"""CPU: the encoder call at the boundary (LRC:735, 758-761, 782-783).

The reference calls ``model.encode(x, convert_to_tensor=True)``; this package
adds ``is_query`` only for encoders that accept it, so a sentence-transformers
2.x-style ``encode`` (no ``**kwargs``) never sees an unknown keyword."""
import torch

from hybrid_rag_colbertv2_amd.encoder import FakeEncoder, encode


class Strict:
    def __init__(self):
        self.calls = []

    def encode(self, sentences, batch_size=32, show_progress_bar=None, convert_to_tensor=False):
        self.calls.append(dict(convert_to_tensor=convert_to_tensor, show_progress_bar=show_progress_bar))
        return FakeEncoder().encode(sentences, convert_to_tensor=convert_to_tensor)


class Named:
    def __init__(self):
        self.seen = None

    def encode(self, sentences, convert_to_tensor=False, is_query=None):
        self.seen = is_query
        return FakeEncoder().encode(sentences, convert_to_tensor=convert_to_tensor)


class Raises:
    """A TypeError raised INSIDE encode must propagate, not trigger a silent retry."""

    def encode(self, sentences, convert_to_tensor=False, **kw):
        raise TypeError("bad input inside the encoder")


def test_strict_encoder_gets_no_is_query():
    s = Strict()
    out = encode(s, ["a b", "c"], is_query=False, show_progress_bar=False)
    assert isinstance(out, torch.Tensor) and out.shape == (2, 32, 128)
    assert s.calls == [dict(convert_to_tensor=True, show_progress_bar=False)]
    assert torch.equal(encode(s, "a b", is_query=True), FakeEncoder().encode("a b"))


def test_is_query_passed_when_accepted():
    n = Named()
    encode(n, "q", is_query=True)
    assert n.seen is True
    encode(n, ["d"], is_query=False)
    assert n.seen is False


def test_encoder_type_error_propagates():
    import pytest
    with pytest.raises(TypeError, match="inside the encoder"):
        encode(Raises(), "q", is_query=True)
