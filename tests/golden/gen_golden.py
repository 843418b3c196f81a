"""Generate golden fixtures from the reference's own retrieval code.

Run ONCE in the build container (the one that has /root/reference mounted):

    python tests/golden/gen_golden.py

It never ships reference source anywhere: it parses
``/root/reference/local_rag_complete.py`` with ``ast``, keeps only the class
definitions ``RAGConfig``, ``JinaColBERTRetriever``, ``DualIndexer`` and
``HybridRetriever`` (local_rag_complete.py:56-86, 715-831, 838-879, 886-1014),
executes them in a private namespace with torch, and records their OUTPUTS on
deterministic inputs as data (``.npz`` / ``.json``) next to this script.
``import local_rag_complete`` itself fails in this image (pymupdf4llm is
missing, then SQLAlchemy 2.x rejects ``Chunk.metadata``: SURVEY.md §0.4), hence
the extraction.

Third-party pieces the reference calls but which are absent offline are
replaced by stand-ins that are recorded in the fixtures:
  * ``SentenceTransformer`` → ``FakeEncoder`` (our package, crc32-keyed words);
  * ``bm25s`` → a recorded lexical ranking (word-overlap count, ties by id),
    because bm25s/PyStemmer are not installed (parity with bm25s: unpinned);
  * the SQLAlchemy session → an in-memory id→chunk table with 0-based ids (the
    reference's 1-based-id lookup bug, SURVEY.md §0.5, is not reproduced).

Fixtures written:
  literal_maxsim.npz — ``_maxsim_score`` (the reference's literal mean-pool
                        cosine) on token-level inputs, 2-D and 3-D queries;
  single_token.npz    — docs of ONE normalised token: there the reference's
                        ranking equals true MaxSim's, so
                        the reference's ``search`` top-k ids pin the MaxSim
                        kernel's ids;
  toy_c1.json         — config 1: 50-chunk toy corpus, 5 queries, the
                        reference's ``search``, ``rerank``,
                        ``_reciprocal_rank_fusion`` and full ``retrieve``;
  rrf_ties.json       — RRF with exact float64 ties;
  exact_grid.npz      — MaxSim known answers on the k/16 grid, computed with
                        exact rational arithmetic (not float), with ties.
"""
from __future__ import annotations

import ast
import contextlib
import io
import json
import os
import sys
import time
import types
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/local_rag_complete.py"
sys.path.insert(0, ROOT)

from hybrid_rag_colbertv2_amd.encoder import FakeEncoder  # noqa: E402

KEEP = ("RAGConfig", "JinaColBERTRetriever", "DualIndexer", "HybridRetriever")


class _Chunk:  # stands in for the ORM class named at local_rag_complete.py:984
    pass


class _Query:
    def __init__(self, table):
        self.table = table
        self._id = None

    def filter_by(self, id):  # noqa: A002 - mirrors the ORM keyword
        self._id = id
        return self

    def first(self):
        return self.table.get(self._id)


class _Session:
    def __init__(self, rows):
        self.table = {r.id: r for r in rows}

    def query(self, _cls):
        return _Query(self.table)


def _lexical_rank(query: str, corpus: List[str], k: int):
    """Recorded BM25 stand-in: word-overlap count, ties broken by lower id."""
    q = set(FakeEncoder().tokenize(query)) - {t for t in FakeEncoder().tokenize("") if t}
    scores = []
    for i, doc in enumerate(corpus):
        words = set(w for w in FakeEncoder(maxlen=10_000).tokenize(doc) if not w.startswith("[PAD]"))
        scores.append((len(q & words), i))
    scores.sort(key=lambda x: (-x[0], x[1]))
    top = scores[:k]
    return [i for _, i in top], [float(s) for s, _ in top]


def extract_reference():
    src = open(REF, encoding="utf-8").read()
    tree = ast.parse(src)
    body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in KEEP]
    assert [n.name for n in body] == list(KEEP), [n.name for n in body]
    mod = ast.Module(body=body, type_ignores=[])
    modobj = types.ModuleType("ref_extract")
    sys.modules["ref_extract"] = modobj  # dataclass() looks its module up here
    ns = modobj.__dict__
    ns.update({
        "torch": torch, "os": os, "time": time, "json": json,
        "List": List, "Dict": Dict, "Tuple": Tuple, "Optional": Optional,
        "dataclass": dataclass, "field": field, "Chunk": _Chunk,
    })
    exec(compile(mod, REF, "exec"), ns)  # noqa: S102 - reference code, study-only, this container
    return ns


def make_retriever(ns, encoder):
    cls = ns["JinaColBERTRetriever"]
    r = cls.__new__(cls)
    r.config = ns["RAGConfig"]()
    r.model = encoder
    r.corpus = None
    r.corpus_embeddings = None
    return r


class _FixedEncoder:
    """encode() returning preset tensors (for literal/single-token cases)."""

    def __init__(self, q):
        self.q = q

    def encode(self, x, convert_to_tensor=True, **_):
        return self.q


def gen_literal(ns):
    rng = np.random.default_rng(1234)
    r = make_retriever(ns, None)
    out = {}
    # case A: 2-D query [Lq, D], docs [N, Ld, D]
    q = rng.standard_normal((32, 128)).astype(np.float32)
    d = rng.standard_normal((64, 16, 128)).astype(np.float32)
    s = r._maxsim_score(torch.from_numpy(q), torch.from_numpy(d))
    out.update(a_q=q, a_docs=d, a_scores=s.numpy())
    # case B: 3-D query [1, Lq, D]
    q = rng.standard_normal((1, 8, 128)).astype(np.float32)
    d = rng.standard_normal((40, 8, 128)).astype(np.float32)
    s = r._maxsim_score(torch.from_numpy(q), torch.from_numpy(d))
    out.update(b_q=q, b_docs=d, b_scores=s.numpy())
    # case C: near-zero mean query (exercises the eps clamp); ragged-looking scale
    q = (rng.standard_normal((4, 128)) * 1e-9).astype(np.float32)
    d = rng.standard_normal((10, 4, 128)).astype(np.float32) * 3.0
    s = r._maxsim_score(torch.from_numpy(q), torch.from_numpy(d))
    out.update(c_q=q, c_docs=d, c_scores=s.numpy())
    np.savez_compressed(os.path.join(HERE, "literal_maxsim.npz"), **out)


def gen_single_token(ns):
    """Docs of ONE unit-norm token: reference ranking == true-MaxSim ranking."""
    # Inputs exactly representable in bf16, docs EXACTLY unit norm (16 entries of
    # +-1/4), so the bf16 device path sees the same numbers as the reference and
    # cosine ranking == MaxSim ranking holds without rounding slack.
    rng = np.random.default_rng(99)
    q = torch.from_numpy(rng.standard_normal((32, 128)).astype(np.float32)).bfloat16().float().numpy()
    d = np.zeros((300, 1, 128), np.float32)
    for i in range(300):
        pos = rng.choice(128, size=16, replace=False)
        d[i, 0, pos] = rng.choice([-0.25, 0.25], size=16)
    r = make_retriever(ns, _FixedEncoder(torch.from_numpy(q)))
    r.corpus_embeddings = torch.from_numpy(d)
    r.corpus = [f"doc{i}" for i in range(len(d))]
    res = r.search("unused", k=25)
    ids = np.array([x["document_id"] for x in res], np.int32)
    scores = np.array([x["score"] for x in res], np.float32)
    np.savez_compressed(os.path.join(HERE, "single_token.npz"), q=q, docs=d, ref_ids=ids, ref_scores=scores)


VOCAB = ("retrieval late interaction token embedding index shard query document chunk "
         "score maxsim rerank fusion lexical semantic vector matrix kernel memory bandwidth "
         "latency throughput batch corpus passage answer model encoder cosine similarity "
         "heading table figure image section paragraph summary context hybrid ranking").split()


def toy_corpus(n=50, nq=5, seed=7):
    rng = np.random.default_rng(seed)
    corpus = [" ".join(rng.choice(VOCAB, size=int(rng.integers(6, 40)))) for _ in range(n)]
    queries = [" ".join(rng.choice(VOCAB, size=int(rng.integers(2, 7)))) for _ in range(nq)]
    return corpus, queries


def gen_toy(ns):
    enc = FakeEncoder(maxlen=32, dim=128)
    corpus, queries = toy_corpus()
    r = make_retriever(ns, enc)
    r.corpus = corpus
    r.corpus_embeddings = enc.encode(corpus, convert_to_tensor=True)
    rows = []
    for i, t in enumerate(corpus):
        c = _Chunk()
        c.id, c.text, c.document_id = i, t, 1 + i // 10
        c.heading_path = f"H{i // 10} > S{i % 10}"
        c.has_images = (i % 7 == 0)
        c.metadata = json.dumps({"pos": i}) if i % 3 else None
        rows.append(c)

    indexer = ns["DualIndexer"].__new__(ns["DualIndexer"])
    indexer.config = r.config
    indexer.colbert_retriever = r
    bm25_lists = {}

    class _BM25:
        def retrieve(self, query_tokens, k):
            ids, sc = _lexical_rank(query_tokens, corpus, k)
            bm25_lists[query_tokens] = (ids, sc)
            return np.array([ids]), np.array([sc])

    indexer.bm25_retriever = _BM25()
    stem = types.SimpleNamespace(Stemmer=types.SimpleNamespace(Stemmer=lambda lang: None))
    ns["bm25s"] = types.SimpleNamespace(tokenize=lambda q, stopwords=None, stemmer=None: q,
                                        stemmer=stem)
    hyb = ns["HybridRetriever"](r.config, indexer, _Session(rows))

    out = {"encoder": {"maxlen": 32, "dim": 128}, "corpus": corpus, "queries": queries,
           "chunks": [{"id": c.id, "document_id": c.document_id, "heading_path": c.heading_path,
                       "has_images": c.has_images, "metadata": c.metadata} for c in rows],
           "search": [], "rerank": [], "retrieve": [], "bm25": [], "rrf": []}
    for q in queries:
        s = r.search(q, k=10)
        out["search"].append([{"document_id": x["document_id"], "score": x["score"]} for x in s])
        docs = [corpus[i] for i in range(0, 50, 3)]
        rr = r.rerank(q, docs, k=5)
        out["rerank"].append({"documents_from": "corpus[0:50:3]",
                              "results": [{"result_index": x["result_index"], "score": x["score"],
                                           "rank": x["rank"]} for x in rr]})
        with contextlib.redirect_stdout(io.StringIO()):
            fin = hyb.retrieve(q)
        out["retrieve"].append([{k: v for k, v in x.items() if k != "text"} for x in fin])
        ids, sc = bm25_lists[q]
        out["bm25"].append({"ids": ids, "scores": sc})
        bm = [{"chunk_id": i, "score": s_, "source": "bm25"} for i, s_ in zip(ids, sc)]
        cb = hyb._colbert_search(q, k=100)
        fused = hyb._reciprocal_rank_fusion(bm, cb)
        out["rrf"].append(fused)
    with open(os.path.join(HERE, "toy_c1.json"), "w") as f:
        json.dump(out, f, indent=1)


def gen_rrf_ties(ns):
    hyb = ns["HybridRetriever"].__new__(ns["HybridRetriever"])
    cases = []
    # ids 3 and 1 tie exactly: (rank 1 in A, rank 2 in B) vs (rank 2 in A, rank 1 in B)
    a = [3, 1, 7, 9, 11]
    b = [1, 3, 5, 7, 2]
    cases.append((a, b))
    rng = np.random.default_rng(5)
    for _ in range(6):
        a = list(rng.permutation(60)[:40])
        b = list(rng.permutation(60)[:40])
        cases.append(([int(x) for x in a], [int(x) for x in b]))
    cases.append(([], [4, 2]))
    cases.append(([4, 2], []))
    cases.append(([5, 5, 6], [6]))  # duplicate ids inside one list
    out = []
    for a, b in cases:
        bm = [{"chunk_id": i, "score": 0.0, "source": "bm25"} for i in a]
        cb = [{"chunk_id": i, "score": 0.0, "source": "colbert"} for i in b]
        out.append({"bm25": a, "colbert": b, "fused": hyb._reciprocal_rank_fusion(bm, cb)})
    with open(os.path.join(HERE, "rrf_ties.json"), "w") as f:
        json.dump(out, f, indent=1)


def _exact_maxsim(q, d, dl):
    """Exact rational MaxSim: q [Lq,D], d [Ld,D] integer numerators over 16."""
    tot = Fraction(0)
    for i in range(q.shape[0]):
        best = None
        for j in range(dl):
            v = Fraction(int(np.dot(q[i].astype(np.int64), d[j].astype(np.int64))), 256)
            best = v if best is None or v > best else best
        tot += best
    return tot


def gen_exact_grid():
    """k/16 grid (k in [-8,8]): exact in bf16/fp8 and in fp32 sums."""
    rng = np.random.default_rng(2024)
    B, N, Lq, Ld, D = 3, 48, 32, 128, 128
    qi = rng.integers(-8, 9, size=(B, Lq, D)).astype(np.int8)
    base = rng.integers(-8, 9, size=(12, Ld, D)).astype(np.int8)
    # duplicate docs to force exact score ties (tie-break: lower id first)
    di = base[rng.integers(0, 12, size=N)]
    doclens = rng.integers(1, Ld + 1, size=N).astype(np.int32)
    doclens[:6] = Ld
    di[::5] = base[0]
    doclens[::5] = Ld
    scores = np.zeros((B, N), np.float64)
    for b in range(B):
        for n in range(N):
            # float64 is exact for these magnitudes; cross-check a subset with Fractions
            s = (qi[b].astype(np.int64) @ di[n, :doclens[n]].astype(np.int64).T).max(axis=1).sum() / 256.0
            scores[b, n] = s
    for b, n in [(0, 0), (1, 7), (2, 13)]:
        assert Fraction(scores[b, n]) == _exact_maxsim(qi[b], di[n], doclens[n])
    # expected top-k by (score desc, id asc)
    order = np.lexsort((np.tile(np.arange(N), (B, 1)), -scores), axis=1)
    n_ties = int(sum(len(np.unique(scores[b])) < N for b in range(B)))
    assert n_ties == B
    np.savez_compressed(os.path.join(HERE, "exact_grid.npz"), q_num=qi, docs_num=di, doclens=doclens,
                        scores=scores, order=order.astype(np.int32))


def main():
    ns = extract_reference()
    gen_literal(ns)
    gen_single_token(ns)
    gen_toy(ns)
    gen_rrf_ties(ns)
    gen_exact_grid()
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
