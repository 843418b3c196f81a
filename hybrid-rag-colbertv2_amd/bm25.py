"""Host-side lexical stage (stage 1 of HybridRetriever.retrieve, LRC:937-950).

The reference uses ``bm25s`` with English stopwords and a Snowball stemmer
(LRC:851-858, 939-945).  Neither bm25s nor PyStemmer is installed in this
image.  This module keeps bm25s' object interface (``tokenize``, ``index``,
``retrieve(query_tokens, k) -> (ids[nq, k], scores[nq, k])``, ``save``/``load``)
and does the scoring natively: text -> term ids here (lower-case ``\\w+``,
scikit-learn's English stopword list, no stemming), then the Lucene BM25
index and multi-threaded search in C++ (csrc/host_bm25.cpp, k1=1.5, b=0.75,
bm25s' defaults).  Parity with bm25s itself is UNPINNED; the C++ scoring is
pinned bit-for-bit by oracle/oracle.py:bm25_topk.
LRC = local_rag_complete.py
"""
from __future__ import annotations

import ctypes
import json
import os
import re
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib

try:  # scikit-learn ships a standard English stopword list
    from sklearn.feature_extraction.text import ENGLISH_STOP_WORDS as _STOP
except Exception:  # pragma: no cover
    _STOP = frozenset("a an and are as at be by for from has he in is it its of on that the to was were will with".split())

_WORD = re.compile(r"\w+")


def to_csr(rows: Sequence[Sequence[int]]) -> Tuple[np.ndarray, np.ndarray]:
    offsets = np.zeros(len(rows) + 1, np.int64)
    offsets[1:] = np.cumsum([len(r) for r in rows])
    flat = np.fromiter((t for r in rows for t in r), dtype=np.int32, count=int(offsets[-1]))
    return flat, offsets


class NativeBM25:
    """Lucene BM25 over term ids (CSR), built and searched in C++.

    ``stats=(n_global, total_global, df_global)`` builds a SHARD of a larger
    corpus (docs [id_base, id_base + n)) with the global statistics, so its
    weights and the merged per-shard results equal the unsharded index's
    (see ``sharded``)."""

    def __init__(self, doc_terms: np.ndarray, doc_offsets: np.ndarray, vocab: int, k1: float = 1.5, b: float = 0.75,
                 id_base: int = 0, stats: Optional[Tuple[int, int, np.ndarray]] = None):
        self.doc_terms = np.ascontiguousarray(doc_terms, np.int32)
        self.doc_offsets = np.ascontiguousarray(doc_offsets, np.int64)
        self.n_docs = len(self.doc_offsets) - 1
        self.vocab, self.k1, self.b, self.id_base = int(vocab), float(k1), float(b), int(id_base)
        h = ctypes.c_void_p()
        if stats is None:
            n_g, tot_g, df_p = 0, 0, None
        else:
            n_g, tot_g, df_g = int(stats[0]), int(stats[1]), np.ascontiguousarray(stats[2], np.int64)
            if df_g.shape != (max(self.vocab, 1),):
                raise ValueError("df_global must have one entry per term")
            df_p = df_g.ctypes.data
        _lib.check(_lib.lib().cbv2_bm25_build_shard(
            self.doc_terms.ctypes.data if self.doc_terms.size else None, self.doc_offsets.ctypes.data,
            self.n_docs, max(self.vocab, 1), self.k1, self.b, self.id_base, n_g, tot_g, df_p, ctypes.byref(h)))
        self._h = h

    @staticmethod
    def doc_freq(doc_terms: np.ndarray, doc_offsets: np.ndarray, vocab: int) -> np.ndarray:
        """Per-term document frequency of a CSR corpus (int64 [vocab])."""
        doc_terms = np.ascontiguousarray(doc_terms, np.int32)
        doc_offsets = np.ascontiguousarray(doc_offsets, np.int64)
        df = np.zeros(max(int(vocab), 1), np.int64)
        _lib.check(_lib.lib().cbv2_bm25_doc_freq(doc_terms.ctypes.data if doc_terms.size else None,
                                                 doc_offsets.ctypes.data, len(doc_offsets) - 1, len(df),
                                                 df.ctypes.data))
        return df

    def __del__(self):
        try:
            if self._h.value:
                _lib.lib().cbv2_bm25_destroy(self._h)
                self._h = ctypes.c_void_p()
        except Exception:
            pass

    def search(self, q_terms: np.ndarray, q_offsets: np.ndarray, k: int, n_threads: int = 0):
        """Queries as CSR of term ids -> (global ids int32 [B, k], scores float32 [B, k])."""
        q_terms = np.ascontiguousarray(q_terms, np.int32)
        q_offsets = np.ascontiguousarray(q_offsets, np.int64)
        B = len(q_offsets) - 1
        ids = np.empty((B, k), np.int32)
        sc = np.empty((B, k), np.float32)
        _lib.check(_lib.lib().cbv2_bm25_search(self._h, q_terms.ctypes.data if q_terms.size else None,
                                               q_offsets.ctypes.data, B, int(k), int(n_threads),
                                               ids.ctypes.data, sc.ctypes.data))
        return ids, sc


def sharded(doc_terms: np.ndarray, doc_offsets: np.ndarray, vocab: int, id_base: int, group=None,
            device=None, k1: float = 1.5, b: float = 0.75) -> NativeBM25:
    """This rank's shard of a doc-sharded BM25 index.

    The global statistics (doc count, token count, per-term df) come from ONE
    all-reduce at build time (on ``device`` for RCCL, host tensors for gloo);
    queries then touch only local postings and the ranks' top-k lists are
    merged with the stage-2 lists (``ShardedSearcher.search_hybrid``)."""
    import torch
    import torch.distributed as dist
    doc_offsets = np.ascontiguousarray(doc_offsets, np.int64)
    n = len(doc_offsets) - 1
    df = NativeBM25.doc_freq(doc_terms, doc_offsets, vocab)
    head = np.array([n, int(doc_offsets[-1] - doc_offsets[0]) if n else 0], np.int64)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        t = torch.from_numpy(np.concatenate([head, df]))
        if device is not None and dist.get_backend(group) == "nccl":
            t = t.to(device)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t = t.cpu().numpy()
        head, df = t[:2], t[2:]
    return NativeBM25(doc_terms, doc_offsets, vocab, k1, b, id_base=id_base,
                      stats=(int(head[0]), int(head[1]), df))


class HostBM25:
    """bm25s-shaped object: tokenize -> index -> retrieve, scoring in C++."""

    def __init__(self, k1: float = 1.5, b: float = 0.75, stopwords: bool = True):
        self.k1, self.b, self.stopwords = k1, b, stopwords
        self.vocab = {}
        self.n_docs = 0
        self._native: Optional[NativeBM25] = None
        self._corpus: Optional[Tuple[np.ndarray, np.ndarray]] = None

    # ---------------------------------------------------------------- text
    def tokenize(self, text: Union[str, Sequence[str]]):
        if isinstance(text, str):
            return [w for w in _WORD.findall(text.lower()) if not (self.stopwords and w in _STOP)]
        return [self.tokenize(t) for t in text]

    def _ids(self, toks: Sequence[str], grow: bool) -> List[int]:
        out = []
        for t in toks:
            v = self.vocab.get(t)
            if v is None and grow:
                v = self.vocab[t] = len(self.vocab)
            if v is not None:
                out.append(v)
        return out

    # ---------------------------------------------------------------- index
    def index(self, corpus_tokens: List[List[str]]) -> None:
        rows = [self._ids(toks, grow=True) for toks in corpus_tokens]
        self._corpus = to_csr(rows)
        self.n_docs = len(rows)
        self._native = NativeBM25(*self._corpus, len(self.vocab), self.k1, self.b)

    def retrieve(self, query_tokens, k: int = 10):
        if query_tokens and isinstance(query_tokens[0], str):
            query_tokens = [query_tokens]
        q, off = to_csr([self._ids(t, grow=False) for t in query_tokens])
        ids, sc = self._native.search(q, off, k)
        return ids.astype(np.int64), sc

    # ---------------------------------------------------------------- persistence
    def save(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        np.savez(os.path.join(path, "bm25_corpus.npz"), terms=self._corpus[0], offsets=self._corpus[1])
        with open(os.path.join(path, "bm25.json"), "w") as f:
            json.dump({"vocab": self.vocab, "n_docs": self.n_docs, "k1": self.k1, "b": self.b,
                       "stopwords": self.stopwords}, f)

    @classmethod
    def load(cls, path: str) -> "HostBM25":
        with open(os.path.join(path, "bm25.json")) as f:
            meta = json.load(f)
        self = cls(meta["k1"], meta["b"], meta["stopwords"])
        self.vocab, self.n_docs = meta["vocab"], meta["n_docs"]
        z = np.load(os.path.join(path, "bm25_corpus.npz"))
        self._corpus = (z["terms"], z["offsets"])
        self._native = NativeBM25(*self._corpus, len(self.vocab), self.k1, self.b)
        return self
