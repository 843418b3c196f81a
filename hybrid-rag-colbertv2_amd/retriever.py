"""JinaColBERTRetriever — drop-in for local_rag_complete.py:715-831.

Same constructor, methods and result dicts as the reference; the corpus
embeddings live in HBM as a ``ColbertIndex`` and every score / top-k /
rerank runs in the HIP kernels of libcolbert_mi355x.so.

Differences from the reference, all deliberate:
  * ``scorer``: "maxsim" (default) computes true ColBERT MaxSim, which the
    reference's docstring promises (LRC:807-812) but its code does not;
    "ref_meanpool_cosine" reproduces the code as written (LRC:821-829).
  * Ties in top-k / argsort are broken by lower index (the reference's
    torch.topk / argsort order is unspecified).
  * ``search`` works for pooled ([D]) query embeddings as a one-token query;
    the reference raises IndexError there.
  * Added batch entry points for the MI355X path: ``search_embeddings`` and
    ``rerank_ids`` (rerank by gathering precomputed doc tiles by id instead of
    re-encoding 50 chunk texts per query).
LRC = local_rag_complete.py
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence, Union

import torch

from .config import RAGConfig
from .encoder import encode, load_local_encoder
from .index import ColbertIndex, IndexBuilder, select_topk


class JinaColBERTRetriever:
    """ColBERT retrieval over an HBM-resident token index (LRC:715-831)."""

    def __init__(self, config: RAGConfig, encoder=None):
        self.config = config
        dev = config.device if str(config.device).startswith("cuda") else "cuda"
        self.device = torch.device(dev)
        # LRC:720-724 loads the encoder by hub name; here it must be supplied or local.
        self.model = encoder if encoder is not None else load_local_encoder(config.embedding_model, dev)
        self.corpus_embeddings: Optional[ColbertIndex] = None
        self.corpus: Optional[List[str]] = None

    @property
    def scorer(self) -> str:
        return getattr(self.config, "scorer", "maxsim")

    # ------------------------------------------------------------ index / load
    def _build(self, embeddings) -> ColbertIndex:
        return ColbertIndex.from_embeddings(embeddings, device=self.device,
                                            build_means=(self.scorer == "ref_meanpool_cosine"),
                                            dtype=getattr(self.config, "index_dtype", "fp32"))

    def _encode_docs(self, texts: List[str]):
        return encode(self.model, texts, is_query=False, show_progress_bar=False)

    def index(self, corpus: List[str], batch_size: Optional[int] = None) -> None:
        """LRC:728-746: encode the corpus, keep it in HBM, persist it.

        The reference encodes the whole corpus in one call and torch.saves the
        fp32 embeddings (host memory grows with the corpus: 65 GB at 1M docs x
        128 tokens).  Here the corpus is encoded ``config.ingest_batch`` docs at a
        time and each batch goes straight into the HBM index (cast / quantised
        / split on the GPU: ``IndexBuilder``), so host memory stays bounded.
        Persistence: a corpus of at most ``config.index_pt_max_docs`` docs (and
        any corpus of the literal scorer, whose means need the fp32 embeddings)
        is also saved as the reference's ``index.pt`` (its fp32 embeddings, kept
        per batch on the host); a larger one as the native ``index.cbv2``
        (streamed from HBM through pinned buffers) + ``index.corpus.json``.
        Writing one format deletes the other's files from the directory, so
        ``load()`` always serves the latest ``index()``."""
        self.corpus = corpus
        n = len(corpus)
        bs = int(batch_size or getattr(self.config, "ingest_batch", 256))
        # the literal scorer needs the fp32 embeddings back at load(); only index.pt holds them
        keep_pt = n <= int(getattr(self.config, "index_pt_max_docs", 50_000)) or self.scorer == "ref_meanpool_cosine"
        dtype = getattr(self.config, "index_dtype", "fp32")
        print(f"  Encoding {n} documents...")
        if self.scorer == "ref_meanpool_cosine" or n == 0:
            # the literal scorer needs every doc's fp32 means: one pass as the reference does
            embeddings = self._encode_docs(corpus) if n else torch.zeros((0, 1, 128))
            self.corpus_embeddings = self._build(embeddings)
            host = [embeddings.cpu()] if isinstance(embeddings, torch.Tensor) else [[e.cpu() for e in embeddings]]
        else:
            builder = IndexBuilder(n, device=self.device, dtype=dtype)
            host = []
            for a in range(0, n, bs):
                emb = self._encode_docs(corpus[a:a + bs])
                builder.append(emb)
                if keep_pt:
                    host.append(emb.cpu() if isinstance(emb, torch.Tensor) else [e.cpu() for e in emb])
                del emb
            self.corpus_embeddings = builder.finish()
        os.makedirs(self.config.colbert_index_path, exist_ok=True)
        if keep_pt:
            if host and all(isinstance(h, torch.Tensor) for h in host) and \
                    len({tuple(h.shape[1:]) for h in host}) == 1:
                saved = torch.cat(host, 0)
            else:
                saved = [e for h in host for e in (h if isinstance(h, list) else list(h.unbind(0)))]
            torch.save({"embeddings": saved, "corpus": corpus},
                       os.path.join(self.config.colbert_index_path, "index.pt"))
            self._remove_native()
        else:
            self.save_native()
            pt = os.path.join(self.config.colbert_index_path, "index.pt")
            if os.path.exists(pt):      # an earlier, smaller corpus: load() must not serve it
                os.unlink(pt)

    def _remove_native(self) -> None:
        """Delete the native index files an earlier index() left in the index directory."""
        path = self._native_path()
        for f in (path, path + ".resid", path + ".bounds.json", os.path.splitext(path)[0] + ".corpus.json"):
            if os.path.exists(f):
                os.unlink(f)

    def load(self) -> None:
        """LRC:748-753 (reads the reference's own index.pt format; never unpickles code).
        Without an index.pt, the native file written by ``save_native`` is loaded."""
        index_file = os.path.join(self.config.colbert_index_path, "index.pt")
        if not os.path.exists(index_file) and os.path.exists(self._native_path()):
            return self.load_native()
        data = torch.load(index_file, map_location="cpu", weights_only=True)
        self.corpus_embeddings = self._build(data["embeddings"])
        self.corpus = data["corpus"]

    # ------------------------------------------------------------ native index file
    def _native_path(self, path: Optional[str] = None) -> str:
        return path or os.path.join(self.config.colbert_index_path, "index.cbv2")

    def save_native(self, path: Optional[str] = None) -> None:
        """Write the HBM index to the native flat file (+ corpus.json beside it)."""
        path = self._native_path(path)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self.corpus_embeddings.save(path)
        if self.corpus is not None:
            with open(os.path.splitext(path)[0] + ".corpus.json", "w") as f:
                json.dump(self.corpus, f)

    def load_native(self, path: Optional[str] = None, begin: int = 0, end: Optional[int] = None) -> None:
        """Load docs [begin, end) of a native index file straight into HBM (a
        rank's shard: pass shard_range(n, rank, world)); maxsim scorer only."""
        if self.scorer != "maxsim":
            raise ValueError("the native index stores tokens, not the fp32 means the literal scorer needs")
        path = self._native_path(path)
        self.corpus_embeddings = ColbertIndex.load(path, device=self.device, begin=begin, end=end)
        cpath = os.path.splitext(path)[0] + ".corpus.json"
        self.corpus = None
        if os.path.exists(cpath):
            with open(cpath) as f:
                self.corpus = json.load(f)

    def index_embeddings(self, embeddings, corpus: Optional[List[str]] = None) -> None:
        """Install precomputed token embeddings (dense [N, L, D], pooled [N, D] or a list)."""
        self.corpus_embeddings = self._build(embeddings)
        self.corpus = corpus

    # ------------------------------------------------------------ encoding
    def _encode_query(self, query: Union[str, torch.Tensor]) -> torch.Tensor:
        q = query if isinstance(query, torch.Tensor) else encode(self.model, query, is_query=True)
        if q.dim() == 1:
            q = q.unsqueeze(0)
        return q

    # ------------------------------------------------------------ search
    def search(self, query: str, k: int = 10) -> List[Dict]:
        """LRC:755-777: [{'document_id', 'score', 'text'}] best first."""
        ix = self.corpus_embeddings
        if ix is None:
            raise RuntimeError("no index: call index() or load() first")
        q = self._encode_query(query)
        kk = min(k, len(ix))
        if kk <= 0:
            return []
        scores, ids = ix.search(q.unsqueeze(0), kk, scorer=self.scorer)
        scores, ids = scores[0].tolist(), ids[0].tolist()  # one D2H copy each
        return [{"document_id": int(i), "score": float(s), "text": self.corpus[i] if self.corpus else None}
                for s, i in zip(scores, ids)]

    def search_embeddings(self, Q: torch.Tensor, k: int):
        """Batched stage 2: Q [B, lq, D] -> device (scores [B, k], global ids [B, k])."""
        return self.corpus_embeddings.search(Q, k, scorer=self.scorer)

    # ------------------------------------------------------------ rerank
    def rerank(self, query: str, documents: List[str], k: int = 10) -> List[Dict]:
        """LRC:779-800: re-encode query and documents, score, sort, top-k with 1-based rank."""
        if not documents:
            return []
        q = self._encode_query(query)
        d = encode(self.model, documents, is_query=False)
        tmp = self._build(d)
        kk = min(k, len(documents))
        if self.scorer == "maxsim":
            cand = torch.arange(len(documents), dtype=torch.int32, device=self.device).unsqueeze(0)
            scores, _, pos = tmp.rerank(q.unsqueeze(0), cand, kk)
        else:
            raw = tmp.score(q.unsqueeze(0), scorer=self.scorer)
            scores, _, pos = select_topk(raw, kk)
        scores, pos = scores[0].tolist(), pos[0].tolist()
        return [{"result_index": int(p), "score": float(s), "rank": r + 1, "text": documents[p]}
                for r, (s, p) in enumerate(zip(scores, pos))]

    def rerank_ids(self, Q: torch.Tensor, cand: torch.Tensor, k: int):
        """Batched stage 3 on precomputed tiles: -> device (scores, global ids, positions) [B, k]."""
        if self.scorer != "maxsim":
            raise ValueError("rerank_ids gathers token tiles and scores with MaxSim; use rerank() "
                             "for the ref_meanpool_cosine scorer")
        return self.corpus_embeddings.rerank(Q, cand, k)

    # ------------------------------------------------------------ scorer
    def _maxsim_score(self, query_embedding: torch.Tensor, doc_embeddings: torch.Tensor) -> torch.Tensor:
        """LRC:802-831 shape semantics: 2-D inputs gain a leading batch dim; returns .squeeze()."""
        q = query_embedding.unsqueeze(0) if query_embedding.dim() == 2 else query_embedding
        d = doc_embeddings.unsqueeze(0) if doc_embeddings.dim() == 2 else doc_embeddings
        tmp = self._build(d)
        return tmp.score(q, scorer=self.scorer).squeeze()
