"""Host-side lexical stage (stage 1 of HybridRetriever.retrieve, LRC:937-950).

The reference uses ``bm25s`` with English stopwords and a Snowball stemmer
(LRC:851-858, 939-945).  Neither bm25s nor PyStemmer is installed in this
image, so this is a small Lucene-style BM25 restatement (bm25s' default
``method="lucene"``, k1=1.5, b=0.75) with the same object interface
(``tokenize``, ``index``, ``retrieve(query_tokens, k) -> (ids[1,k], scores[1,k])``,
``save``/``load``).  It runs on the host as SURVEY.md §8 requires; parity with
bm25s is UNPINNED (no stemming; stopword list from scikit-learn).
LRC = local_rag_complete.py
"""
from __future__ import annotations

import json
import os
import re
from typing import List, Sequence, Union

import numpy as np

try:  # scikit-learn ships a standard English stopword list
    from sklearn.feature_extraction.text import ENGLISH_STOP_WORDS as _STOP
except Exception:  # pragma: no cover
    _STOP = frozenset("a an and are as at be by for from has he in is it its of on that the to was were will with".split())

_WORD = re.compile(r"\w+")


class HostBM25:
    def __init__(self, k1: float = 1.5, b: float = 0.75, stopwords: bool = True):
        self.k1, self.b, self.stopwords = k1, b, stopwords
        self.vocab = {}
        self.n_docs = 0

    # ---------------------------------------------------------------- text
    def tokenize(self, text: Union[str, Sequence[str]]):
        if isinstance(text, str):
            return [w for w in _WORD.findall(text.lower()) if not (self.stopwords and w in _STOP)]
        return [self.tokenize(t) for t in text]

    # ---------------------------------------------------------------- index
    def index(self, corpus_tokens: List[List[str]]) -> None:
        self.n_docs = len(corpus_tokens)
        vocab = {}
        rows, cols, tfs = [], [], []
        lens = np.zeros(self.n_docs, np.float64)
        for d, toks in enumerate(corpus_tokens):
            lens[d] = len(toks)
            counts = {}
            for t in toks:
                counts[t] = counts.get(t, 0) + 1
            for t, c in counts.items():
                rows.append(vocab.setdefault(t, len(vocab)))
                cols.append(d)
                tfs.append(c)
        self.vocab = vocab
        V = len(vocab)
        rows = np.asarray(rows, np.int64)
        order = np.argsort(rows, kind="stable")
        self.post_docs = np.asarray(cols, np.int32)[order]
        tf = np.asarray(tfs, np.float64)[order]
        self.post_ptr = np.zeros(V + 1, np.int64)
        np.add.at(self.post_ptr, rows + 1, 1)
        self.post_ptr = np.cumsum(self.post_ptr)
        df = np.diff(self.post_ptr).astype(np.float64)
        avgdl = lens.mean() if self.n_docs else 1.0
        idf = np.log(1.0 + (self.n_docs - df + 0.5) / (df + 0.5))
        # precomputed per-posting BM25 weight (Lucene form)
        norm = tf + self.k1 * (1.0 - self.b + self.b * lens[self.post_docs] / max(avgdl, 1e-9))
        self.post_w = (np.repeat(idf, np.diff(self.post_ptr)) * tf * (self.k1 + 1.0) / norm).astype(np.float32)

    def retrieve(self, query_tokens, k: int = 10):
        if query_tokens and isinstance(query_tokens[0], str):
            query_tokens = [query_tokens]
        out_ids = np.full((len(query_tokens), k), -1, np.int64)
        out_sc = np.zeros((len(query_tokens), k), np.float32)
        for qi, toks in enumerate(query_tokens):
            acc = np.zeros(self.n_docs, np.float32)
            for t in set(toks):
                v = self.vocab.get(t)
                if v is not None:
                    a, b = self.post_ptr[v], self.post_ptr[v + 1]
                    acc[self.post_docs[a:b]] += self.post_w[a:b]
            kk = min(k, self.n_docs)
            order = np.lexsort((np.arange(self.n_docs), -acc))[:kk]
            out_ids[qi, :kk] = order
            out_sc[qi, :kk] = acc[order]
        return out_ids, out_sc

    # ---------------------------------------------------------------- persistence
    def save(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        np.savez(os.path.join(path, "bm25.npz"), post_ptr=self.post_ptr, post_docs=self.post_docs,
                 post_w=self.post_w)
        with open(os.path.join(path, "bm25.json"), "w") as f:
            json.dump({"vocab": self.vocab, "n_docs": self.n_docs, "k1": self.k1, "b": self.b,
                       "stopwords": self.stopwords}, f)

    @classmethod
    def load(cls, path: str) -> "HostBM25":
        with open(os.path.join(path, "bm25.json")) as f:
            meta = json.load(f)
        self = cls(meta["k1"], meta["b"], meta["stopwords"])
        self.vocab, self.n_docs = meta["vocab"], meta["n_docs"]
        z = np.load(os.path.join(path, "bm25.npz"))
        self.post_ptr, self.post_docs, self.post_w = z["post_ptr"], z["post_docs"], z["post_w"]
        return self
