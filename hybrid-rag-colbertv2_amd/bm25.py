r"""Host-side lexical stage (stage 1 of HybridRetriever.retrieve, LRC:937-950).

The reference builds and queries bm25s (LRC:851-858, 939-945):

    tokens = bm25s.tokenize(texts, stopwords="en", stemmer=Stemmer.Stemmer("english"))
    bm25s.BM25().index(tokens);  results, scores = retriever.retrieve(query_tokens, k)

Neither bm25s nor PyStemmer is installed in this image.  This module restates
that pipeline with the same shapes:

  * ``tokenize`` -- bm25s.tokenize's semantics: lower-case, the default token
    pattern ``(?u)\b\w\w+\b`` (Python's own regex engine, so \w is Unicode
    \w exactly), stopwords dropped BEFORE stemming (bm25s' "en" list,
    ``STOPWORDS_EN``), then the UNIQUE tokens stemmed once and mapped to stem
    ids; returns ``Tokenized(ids, vocab)``.
  * ``Stemmer("english")`` -- PyStemmer-shaped (``stemWord``/``stemWords``),
    the Snowball English ("Porter2") algorithm in C++ (csrc/text_en.cpp).
  * ``HostBM25`` -- bm25s.BM25-shaped (``index``/``retrieve``/``save``/``load``);
    the Lucene BM25 index and multi-threaded search are C++
    (csrc/host_bm25.cpp, k1=1.5, b=0.75, bm25s' defaults; a query's score sums
    the postings of every query token, repeats included, as bm25s does).

No fallback exists: a stopword list or stemmer other than these raises.
Parity with bm25s / PyStemmer themselves is UNPINNED (no reference test or
fixture touches BM25); the stemmer is pinned by the published Snowball sample
vocabulary (tests/test_text_en.py) and the C++ scoring bit-for-bit by
oracle/oracle.py:bm25_topk.
LRC = local_rag_complete.py
"""
from __future__ import annotations

import ctypes
import json
import os
import re
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np

from . import _lib

# bm25s.stopwords.STOPWORDS_EN (what bm25s.tokenize(stopwords="en") uses): the
# Lucene / Elasticsearch English stop set.
STOPWORDS_EN = ("a", "an", "and", "are", "as", "at", "be", "but", "by", "for", "if", "in", "into", "is", "it", "no",
                "not", "of", "on", "or", "such", "that", "the", "their", "then", "there", "these", "they", "this",
                "to", "was", "will", "with")
TOKEN_PATTERN = r"(?u)\b\w\w+\b"     # bm25s.tokenize's default


class Stemmer:
    """PyStemmer-shaped Snowball stemmer (``Stemmer.Stemmer("english")``), native."""

    def __init__(self, algorithm: str = "english"):
        if algorithm.lower() not in ("english", "en", "porter2"):
            raise ValueError(f"only the Snowball English stemmer is built (got {algorithm!r})")
        self.algorithm = "english"

    def stemWords(self, words: Sequence[str]) -> List[str]:  # noqa: N802  (PyStemmer's name)
        words = list(words)
        if not words:
            return []
        enc = [w.encode("utf-8") for w in words]
        offs = np.zeros(len(enc) + 1, np.int64)
        offs[1:] = np.cumsum([len(b) for b in enc])
        buf = b"".join(enc)
        out = ctypes.create_string_buffer(max(len(buf), 1))
        out_offs = np.zeros(len(enc) + 1, np.int64)
        src = ctypes.create_string_buffer(buf, max(len(buf), 1))
        _lib.check(_lib.lib().cbv2_stem_en(src, offs.ctypes.data, len(enc), out, len(buf), out_offs.ctypes.data))
        raw = out.raw
        return [raw[out_offs[i]:out_offs[i + 1]].decode("utf-8", errors="surrogateescape") for i in range(len(enc))]

    def stemWord(self, word: str) -> str:  # noqa: N802
        return self.stemWords([word])[0]

    def __call__(self, words):
        return self.stemWords(words)


class Tokenized(NamedTuple):
    """bm25s.tokenization.Tokenized: per-text token ids and the vocabulary."""
    ids: List[List[int]]
    vocab: Dict[str, int]


def _stopword_set(stopwords) -> frozenset:
    if stopwords in (None, False):
        return frozenset()
    if stopwords in ("en", "english", True):
        return frozenset(STOPWORDS_EN)
    if isinstance(stopwords, str):
        raise ValueError(f"only the English stopword list is built (got {stopwords!r})")
    return frozenset(stopwords)


def tokenize(texts: Union[str, Sequence[str]], lower: bool = True, token_pattern: str = TOKEN_PATTERN,
             stopwords="en", stemmer=None, return_ids: bool = True):
    """bm25s.tokenize (the reference's LRC:851-855 / 939-943 call): one row per
    text (an all-stopword or empty text gives an empty row, never a missing one)."""
    if isinstance(texts, str):
        texts = [texts]
    split = re.compile(token_pattern).findall
    stop = _stopword_set(stopwords)
    token_to_index: Dict[str, int] = {}
    rows = []
    for text in texts:
        if lower:
            text = text.lower()
        row = []
        for tok in split(text):
            if tok in stop:
                continue
            tid = token_to_index.get(tok)
            if tid is None:
                tid = token_to_index[tok] = len(token_to_index)
            row.append(tid)
        rows.append(row)
    unique = list(token_to_index)
    if stemmer is not None:
        fn = stemmer.stemWords if hasattr(stemmer, "stemWords") else stemmer
        stems = fn(unique)
        vocab: Dict[str, int] = {}
        remap = []
        for st in stems:
            if st not in vocab:
                vocab[st] = len(vocab)
            remap.append(vocab[st])
        rows = [[remap[t] for t in row] for row in rows]
    else:
        vocab = token_to_index
    if return_ids:
        return Tokenized(rows, vocab)
    inv = {v: k for k, v in vocab.items()}
    return [[inv[t] for t in row] for row in rows]


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
    """bm25s.BM25-shaped host index (LRC:857-861 index/save, 878 load, 945 retrieve):
    ``index(tokenize(corpus, ...))``, ``retrieve(tokenize(query, ...), k)``;
    the BM25 index and search are C++ (NativeBM25)."""

    def __init__(self, k1: float = 1.5, b: float = 0.75, stemmer: Optional[Stemmer] = None, stopwords="en"):
        self.k1, self.b = k1, b
        self.stemmer = stemmer if stemmer is not None else Stemmer("english")
        self.stopwords = stopwords
        self.vocab: Dict[str, int] = {}
        self.n_docs = 0
        self._native: Optional[NativeBM25] = None
        self._corpus: Optional[Tuple[np.ndarray, np.ndarray]] = None

    # ---------------------------------------------------------------- text
    def tokenize(self, texts: Union[str, Sequence[str]]) -> Tokenized:
        """The reference's bm25s.tokenize call: stopwords "en", Snowball English."""
        _stopword_set(self.stopwords)
        return tokenize(texts, stopwords=self.stopwords, stemmer=self.stemmer)

    @staticmethod
    def _rows(tokens) -> List[List[str]]:
        """Tokenized -> token strings per text; a list of strings is ONE text."""
        if isinstance(tokens, Tokenized) or (isinstance(tokens, tuple) and len(tokens) == 2
                                             and isinstance(tokens[1], dict)):
            inv = {v: k for k, v in tokens[1].items()}
            return [[inv[t] for t in row] for row in tokens[0]]
        tokens = list(tokens)
        if not tokens or isinstance(tokens[0], str):
            return [tokens]
        return [list(r) for r in tokens]

    def _ids(self, toks: Sequence[str], grow: bool) -> List[int]:
        out = []
        for t in toks:
            v = self.vocab.get(t)
            if v is None and grow:
                v = self.vocab[t] = len(self.vocab)
            if v is not None:
                out.append(v)          # tokens unknown to the index are dropped (bm25s' get_tokens_ids)
        return out

    # ---------------------------------------------------------------- index
    def index(self, corpus_tokens) -> None:
        self.vocab = {}
        rows = [self._ids(toks, grow=True) for toks in self._rows(corpus_tokens)]
        self._corpus = to_csr(rows)
        self.n_docs = len(rows)
        self._native = NativeBM25(*self._corpus, len(self.vocab), self.k1, self.b)

    def retrieve(self, query_tokens, k: int = 10, n_threads: int = 0):
        """-> (doc ids int64 [n_queries, k], scores float32 [n_queries, k]); rows with no
        scoring term pad with the lowest-id zero-score docs (then -1 past the corpus)."""
        if self._native is None:
            raise RuntimeError("BM25 index not built: call index() or load() first")
        q, off = to_csr([self._ids(t, grow=False) for t in self._rows(query_tokens)])
        ids, sc = self._native.search(q, off, k, n_threads)
        return ids.astype(np.int64), sc

    # ---------------------------------------------------------------- persistence
    FORMAT = 2     # 2: vocabulary of stemmed tokens (bm25s' stopwords + Snowball English)

    def save(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        np.savez(os.path.join(path, "bm25_corpus.npz"), terms=self._corpus[0], offsets=self._corpus[1])
        with open(os.path.join(path, "bm25.json"), "w") as f:
            json.dump({"format": self.FORMAT, "vocab": self.vocab, "n_docs": self.n_docs, "k1": self.k1, "b": self.b,
                       "stopwords": self.stopwords if isinstance(self.stopwords, (str, bool)) or self.stopwords is None
                       else list(self.stopwords), "stemmer": getattr(self.stemmer, "algorithm", "custom")}, f)

    @classmethod
    def load(cls, path: str, stemmer: Optional[Stemmer] = None) -> "HostBM25":
        """Reads what ``save`` wrote.  The query tokens must be stemmed as the
        vocabulary was, so a file without the format/stemmer record (written by
        an older, unstemmed tokenizer) is refused rather than silently matching
        nothing; a "custom" stemmer must be passed in again."""
        with open(os.path.join(path, "bm25.json")) as f:
            meta = json.load(f)
        if meta.get("format") != cls.FORMAT or "stemmer" not in meta:
            raise ValueError(f"{path}/bm25.json has format {meta.get('format')!r} (need {cls.FORMAT}, with its "
                             "stemmer recorded): rebuild the BM25 index")
        if meta["stemmer"] == "custom":
            if stemmer is None:
                raise ValueError(f"{path}/bm25.json was built with a custom stemmer: pass it to load()")
        elif stemmer is None:
            stemmer = Stemmer(meta["stemmer"])
        self = cls(meta["k1"], meta["b"], stemmer=stemmer, stopwords=meta.get("stopwords", "en"))
        self.vocab, self.n_docs = meta["vocab"], meta["n_docs"]
        z = np.load(os.path.join(path, "bm25_corpus.npz"))
        self._corpus = (z["terms"], z["offsets"])
        self._native = NativeBM25(*self._corpus, len(self.vocab), self.k1, self.b)
        return self
