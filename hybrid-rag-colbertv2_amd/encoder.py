"""Encoders at the retrieval boundary.

The reference builds ``SentenceTransformer("jinaai/jina-colbert-v2",
trust_remote_code=True, device=...)`` (local_rag_complete.py:720-724) and calls
``model.encode(text_or_texts, convert_to_tensor=True)`` (lines 735, 758, 782,
783).  Hub downloads are impossible here, so the path accepts any object with
that ``encode`` method:

* ``FakeEncoder`` — deterministic token-level embeddings derived from a stable
  hash of each word (``zlib.crc32``; never Python ``hash()``, which is salted
  per process).  It stands in for the Jina-ColBERT encoder in tests, golden
  fixtures and the config-1 toy corpus.  Same words → same token vectors, so
  late interaction behaves lexically and results are reproducible bit for bit.
* ``load_local_encoder(path)`` — the Jina-ColBERT-v2 architecture
  (jina_encoder.py, PyTorch-ROCm) from a local ``model.safetensors``, or a
  SentenceTransformer directory if that library is importable (it is not in
  this image); never reaches a hub.
"""
from __future__ import annotations

import re
import zlib
from typing import List, Sequence, Union

import numpy as np
import torch

_WORD = re.compile(r"\w+")


def _token_vector(token: str, dim: int) -> np.ndarray:
    seed = zlib.crc32(token.encode("utf-8"))
    v = np.random.default_rng(seed).standard_normal(dim)
    v /= np.linalg.norm(v)
    return v.astype(np.float32)


class FakeEncoder:
    """SentenceTransformer-compatible stand-in producing ``[maxlen, dim]`` token matrices.

    Every text is lower-cased, split into ``\\w+`` words, truncated to
    ``maxlen`` and padded with position-keyed ``[PAD]<i>`` vectors, so every
    output has exactly ``maxlen`` rows (the reference stacks per-text outputs
    into one dense tensor, local_rag_complete.py:735-739, which requires equal
    lengths).  Each row is an L2-normalised fp32 vector.
    """

    def __init__(self, maxlen: int = 32, dim: int = 128):
        self.maxlen = int(maxlen)
        self.dim = int(dim)
        self._cache = {}

    def _vec(self, token: str) -> np.ndarray:
        v = self._cache.get(token)
        if v is None:
            v = _token_vector(token, self.dim)
            self._cache[token] = v
        return v

    def tokenize(self, text: str) -> List[str]:
        words = _WORD.findall(text.lower())[: self.maxlen]
        return words + [f"[PAD]{i}" for i in range(len(words), self.maxlen)]

    def encode_one(self, text: str) -> np.ndarray:
        return np.stack([self._vec(t) for t in self.tokenize(text)])

    def encode(self, sentences: Union[str, Sequence[str]], convert_to_tensor: bool = True,
               show_progress_bar: bool = False, **_unused):
        if isinstance(sentences, str):
            out = self.encode_one(sentences)
        else:
            out = np.stack([self.encode_one(s) for s in sentences]) if len(sentences) else \
                np.zeros((0, self.maxlen, self.dim), np.float32)
        return torch.from_numpy(out) if convert_to_tensor else out


def _accepts_keyword(fn, name: str) -> bool:
    """True when ``fn`` takes ``name`` as a keyword (explicitly or via **kwargs)."""
    import inspect
    try:
        params = inspect.signature(fn).parameters.values()
    except (TypeError, ValueError):          # builtins / C callables without a signature
        return False
    return any(p.kind is p.VAR_KEYWORD or (p.name == name and p.kind is not p.POSITIONAL_ONLY) for p in params)


def encode(model, texts, is_query: bool, **kw):
    """``model.encode(texts, convert_to_tensor=True, **kw)`` as the reference calls it
    (LRC:735, 758-761, 782-783), adding ``is_query`` only when the encoder's
    ``encode`` accepts it (jina-colbert's remote code and this package's encoders
    do; sentence-transformers 2.x's ``encode`` has no ``**kwargs`` and would raise)."""
    if _accepts_keyword(model.encode, "is_query"):
        kw["is_query"] = is_query
    return model.encode(texts, convert_to_tensor=True, **kw)


def load_local_encoder(path: str, device: str = "cuda"):
    """The Jina-ColBERT encoder from a LOCAL directory on PyTorch-ROCm.

    A directory with ``model.safetensors`` loads into this package's own
    implementation of the architecture (jina_encoder.JinaColBERTEncoder);
    otherwise a SentenceTransformer directory is tried if that library is
    importable (it is not in this image).  Never reaches a hub."""
    import os
    if os.path.exists(os.path.join(path, "model.safetensors")):
        from .jina_encoder import JinaColBERTEncoder
        return JinaColBERTEncoder.from_local(path, device=device)
    try:
        from sentence_transformers import SentenceTransformer  # noqa: WPS433
    except ImportError as e:  # pragma: no cover - not installed in this image
        raise RuntimeError(
            f"no local checkpoint at {path!r} and sentence_transformers is not installed; pass an encoder "
            "object with an encode(texts, convert_to_tensor=True) method (e.g. FakeEncoder) instead") from e
    return SentenceTransformer(path, trust_remote_code=True, device=device, local_files_only=True)
