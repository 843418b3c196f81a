"""DualIndexer and HybridRetriever — drop-in for local_rag_complete.py:838-1014.

The three-stage flow is the reference's (LRC:894-935): host BM25 top-100,
ColBERT top-100 (HIP scan + top-k), reciprocal rank fusion (host, exact
float64 semantics), ``[:50]`` candidates, ColBERT rerank top-10.  The result
dicts are the reference's (LRC:1004-1013).

MI355X changes:
  * ``_fetch_chunks_from_db`` reads a ``ChunkStore`` (id -> chunk dict) with
    ids equal to index positions; the reference's SQLite lookup treats
    0-based index positions as 1-based primary keys (LRC:984).
  * ``_colbert_rerank`` gathers the candidates' precomputed token tiles from
    HBM by id (``rerank_ids``) instead of re-encoding their texts, and reuses
    the stage-2 query embedding (the reference encodes the query twice).
  * ``retrieve_batch`` runs the same three stages for a batch of query
    embeddings with one device round trip per stage.
LRC = local_rag_complete.py
"""
from __future__ import annotations

import ctypes
import time
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .bm25 import HostBM25, Stemmer, tokenize
from .config import RAGConfig
from .index import LQ_MAX as _LQ_MAX
from .index import _raw_stream
from .index import _stream_ptr as _stream_ptr_fn
from .retriever import JinaColBERTRetriever


# ---------------------------------------------------------------------- fusion
def rrf_fuse(bm25_ids: np.ndarray, colbert_ids: np.ndarray, rrf_k: int = 60, C: int = 50,
             return_scores: bool = False):
    """Batched LRC:960-978 + ``[:C]`` (LRC:916) in native host code.

    bm25_ids [B, kb], colbert_ids [B, kc] int (negative = padding) ->
    fused ids [B, C] int32 (-1 padded) [, float64 scores [B, C], counts [B]].
    """
    bm = np.ascontiguousarray(np.atleast_2d(bm25_ids), dtype=np.int32)
    cb = np.ascontiguousarray(np.atleast_2d(colbert_ids), dtype=np.int32)
    B = max(bm.shape[0], cb.shape[0])
    if bm.shape[0] != B:
        bm = np.ascontiguousarray(np.broadcast_to(bm, (B, bm.shape[1])))
    if cb.shape[0] != B:
        cb = np.ascontiguousarray(np.broadcast_to(cb, (B, cb.shape[1])))
    out = np.empty((B, C), np.int32)
    sc = np.empty((B, C), np.float64)
    cnt = np.empty(B, np.int32)
    _lib.check(_lib.lib().cbv2_rrf_fuse(bm.ctypes.data if bm.size else None, bm.shape[1],
                                        cb.ctypes.data if cb.size else None, cb.shape[1], B, int(rrf_k), C,
                                        out.ctypes.data, sc.ctypes.data, cnt.ctypes.data))
    return (out, sc, cnt) if return_scores else out


# ---------------------------------------------------------------------- chunk store
class ChunkStore:
    """In-memory id -> chunk table (replaces the SQLAlchemy ``Chunk`` lookups, LRC:980-994)."""

    def __init__(self, chunks: Optional[Sequence[Dict]] = None):
        self._rows = {}
        for i, c in enumerate(chunks or []):
            self.add(c.get("chunk_id", c.get("id", i)), c)

    def add(self, chunk_id: int, chunk: Dict) -> None:
        self._rows[int(chunk_id)] = {
            "chunk_id": int(chunk_id),
            "text": chunk.get("text", ""),
            "document_id": chunk.get("document_id"),
            "heading_path": chunk.get("heading_path", ""),
            "has_images": chunk.get("has_images", False),
            "metadata": chunk.get("metadata") or {},
        }

    @classmethod
    def from_corpus(cls, corpus: Sequence[str]) -> "ChunkStore":
        return cls([{"chunk_id": i, "text": t} for i, t in enumerate(corpus)])

    def get(self, chunk_id: int) -> Optional[Dict]:
        return self._rows.get(int(chunk_id))

    def __len__(self):
        return len(self._rows)


# ---------------------------------------------------------------------- indexer
class DualIndexer:
    """LRC:838-879: holds the BM25 and ColBERT retrievers (the drop-in seam)."""

    def __init__(self, config: RAGConfig, encoder=None):
        self.config = config
        self.bm25_retriever: Optional[HostBM25] = None
        self.colbert_retriever = JinaColBERTRetriever(config, encoder=encoder)

    def build_bm25_index(self, corpus: List[str]) -> None:
        """LRC:846-864: bm25s.tokenize(corpus, stopwords="en", stemmer=Stemmer("english")) -> index -> save."""
        print("\n[BM25s] Building lexical search index...", end=" ")
        start = time.time()
        corpus_tokens = tokenize(corpus, stopwords="en", stemmer=Stemmer("english"))
        self.bm25_retriever = HostBM25()
        self.bm25_retriever.index(corpus_tokens)
        self.bm25_retriever.save(self.config.bm25_index_path)
        print(f"✓ {time.time() - start:.2f}s")

    def build_colbert_index(self, corpus: List[str]) -> None:
        print("\n[ColBERT] Building semantic search index...")
        start = time.time()
        self.colbert_retriever.index(corpus)
        print(f"  ✓ {time.time() - start:.2f}s")

    def load_indexes(self) -> None:
        self.bm25_retriever = HostBM25.load(self.config.bm25_index_path)
        self.colbert_retriever.load()


# ---------------------------------------------------------------------- hybrid
class HybridRetriever:
    """Three-stage retrieval: BM25 + ColBERT + ColBERT reranking (LRC:886-1014)."""

    def __init__(self, config: RAGConfig, indexer: DualIndexer, db_session=None, verbose: bool = True):
        self.config = config
        self.indexer = indexer
        self.db_session = db_session
        self.verbose = verbose

    def _log(self, msg: str):
        if self.verbose:
            print(msg)

    def retrieve(self, query: str, top_k_final: int = None) -> List[Dict]:
        """LRC:894-935, same stages, cut-offs and per-stage timing prints."""
        if top_k_final is None:
            top_k_final = self.config.final_top_k
        self._log("\n🔍 Retrieving relevant chunks...")

        start = time.time()
        bm25_results = self._bm25_search(query, k=self.config.bm25_top_k)
        bm25_time = time.time() - start
        self._log(f"   • BM25s: {bm25_time:.3f}s")

        start = time.time()
        q_emb = self.indexer.colbert_retriever._encode_query(query)
        colbert_results = self._colbert_search(q_emb, k=self.config.colbert_top_k)
        colbert_time = time.time() - start
        self._log(f"   • ColBERT: {colbert_time:.3f}s")

        start = time.time()
        fused_results = self._reciprocal_rank_fusion(bm25_results, colbert_results, k=self.config.rrf_k)
        candidates = fused_results[: self.config.fused_candidates]
        fusion_time = time.time() - start
        self._log(f"   • Fusion: {fusion_time:.3f}s")

        start = time.time()
        candidate_chunks = self._fetch_chunks_from_db([r["chunk_id"] for r in candidates])
        fetch_time = time.time() - start
        self._log(f"   • Fetch: {fetch_time:.3f}s")

        start = time.time()
        reranked_results = self._colbert_rerank(q_emb, candidate_chunks, top_k=top_k_final)
        rerank_time = time.time() - start
        self._log(f"   • Rerank: {rerank_time:.3f}s")

        total = bm25_time + colbert_time + fusion_time + fetch_time + rerank_time
        self._log(f"   ✓ Total retrieval: {total:.3f}s")
        return reranked_results

    def _bm25_search(self, query: str, k: int) -> List[Dict]:
        """LRC:937-950 against the host BM25."""
        bm = self.indexer.bm25_retriever
        if bm is None:
            return []
        # the reference's bm25s.tokenize(query, stopwords="en", stemmer=english) (LRC:939-943):
        # one Tokenized row per query, even when every word is a stopword; a
        # retriever with its own tokenize() (HostBM25, test stand-ins) supplies it
        tok = getattr(bm, "tokenize", None)
        query_tokens = tok(query) if callable(tok) else tokenize(query, stopwords="en", stemmer=Stemmer("english"))
        results, scores = bm.retrieve(query_tokens, k=k)
        return [{"chunk_id": int(results[0][i]), "score": float(scores[0][i]), "source": "bm25"}
                for i in range(len(results[0])) if results[0][i] >= 0]

    def _colbert_search(self, query, k: int) -> List[Dict]:
        """LRC:952-958."""
        results = self.indexer.colbert_retriever.search(query=query, k=k)
        return [{"chunk_id": r["document_id"], "score": r["score"], "source": "colbert"} for r in results]

    def _reciprocal_rank_fusion(self, bm25_results: List[Dict], colbert_results: List[Dict],
                                k: int = 60) -> List[Dict]:
        """LRC:960-978 (native, same float64 arithmetic and stable tie order)."""
        bm = np.array([[r["chunk_id"] for r in bm25_results]], np.int32).reshape(1, -1)
        cb = np.array([[r["chunk_id"] for r in colbert_results]], np.int32).reshape(1, -1)
        C = max(1, bm.shape[1] + cb.shape[1])
        ids, sc, cnt = rrf_fuse(bm, cb, rrf_k=k, C=C, return_scores=True)
        n = int(cnt[0])
        return [{"chunk_id": int(ids[0, j]), "rrf_score": float(sc[0, j])} for j in range(n)]

    def _fetch_chunks_from_db(self, chunk_ids: List[int]) -> List[Dict]:
        """LRC:980-994 against a ChunkStore (0-based ids = index positions)."""
        store = self.db_session
        if store is None:
            corpus = self.indexer.colbert_retriever.corpus or []
            return [{"chunk_id": int(i), "text": corpus[i] if i < len(corpus) else "", "document_id": None,
                     "heading_path": "", "has_images": False, "metadata": {}} for i in chunk_ids]
        out = []
        for cid in chunk_ids:
            c = store.get(cid)
            if c:
                out.append(dict(c))
        return out

    def _colbert_rerank(self, query, chunks: List[Dict], top_k: int) -> List[Dict]:
        """LRC:996-1014; scores gathered tiles by chunk id (no re-encode)."""
        if not chunks:
            return []
        retr = self.indexer.colbert_retriever
        if retr.scorer == "maxsim" and not isinstance(query, str):
            q = query if query.dim() == 3 else query.unsqueeze(0)
            cand = torch.tensor([[c["chunk_id"] for c in chunks]], dtype=torch.int32, device=retr.device)
            kk = min(top_k, len(chunks))
            scores, _, pos = retr.rerank_ids(q, cand, kk)
            reranked = [{"result_index": int(p), "score": float(s), "rank": r + 1}
                        for r, (s, p) in enumerate(zip(scores[0].tolist(), pos[0].tolist()))]
        else:
            documents = [c["text"] for c in chunks]
            reranked = retr.rerank(query=query, documents=documents, k=top_k)
        final = []
        for result in reranked:
            original = chunks[result["result_index"]]
            final.append({
                "chunk_id": original["chunk_id"],
                "text": original["text"],
                "document_id": original["document_id"],
                "heading_path": original.get("heading_path", ""),
                "has_images": original.get("has_images", False),
                "metadata": original["metadata"],
                "score": result["score"],
                "rank": result["rank"],
            })
        return final

    # ------------------------------------------------------------------ batched path
    def retrieve_batch(self, Q: torch.Tensor, bm25_ids: np.ndarray, top_k_final: Optional[int] = None):
        """All three stages for B query embeddings at once (the benchmark step).

        Q [B, lq, D] device; bm25_ids [B, kb] host int (stage-1 output) ->
        device (scores [B, k], global ids [B, k]).
        """
        k_final = top_k_final or self.config.final_top_k
        retr = self.indexer.colbert_retriever
        if retr.scorer == "maxsim":       # one host round trip (cbv2_retrieve_begin / _finish), same results
            key = (id(retr.corpus_embeddings), self.config.colbert_top_k, self.config.fused_candidates, k_final,
                   self.config.rrf_k)
            if getattr(self, "_one_key", None) != key:
                self._one = OneTripRetriever(retr.corpus_embeddings, colbert_k=self.config.colbert_top_k,
                                             fused=self.config.fused_candidates, final_k=k_final,
                                             rrf_k=self.config.rrf_k)
                self._one_key = key
            s, i, _ = self._one(Q, np.ascontiguousarray(bm25_ids, np.int32))
            return s, i
        _, ids = retr.search_embeddings(Q, self.config.colbert_top_k)
        ids_h = ids.cpu().numpy()
        cand = rrf_fuse(bm25_ids, ids_h, rrf_k=self.config.rrf_k, C=self.config.fused_candidates)
        cand_d = torch.from_numpy(cand).pin_memory().to(retr.device, non_blocking=True)
        s, i, _ = retr.rerank_ids(Q, cand_d, k_final)
        return s, i


# ---------------------------------------------------------------------- pipelined batches
class PipelinedRetriever:
    """Software-pipelined three-stage retrieval over a stream of query batches.

    The host steps of the path -- stage-1 BM25 (LRC:937-950) and RRF fusion
    (LRC:960-978) -- would otherwise idle the GPU once per batch.  Here batch
    j+1's stage-2 scan is enqueued, and its BM25 runs on the host while the
    GPU scans, BEFORE the host fuses batch j:

        GPU stream:  scan(j) D2H(j) | scan(j+1) D2H(j+1) | rerank(j) | scan(j+2) ...
        host:        bm25(j)        | bm25(j+1), fuse(j) -> H2D cand(j) | ...

    ``searcher`` is a ``ColbertIndex`` (one shard) or a
    ``distributed.ShardedSearcher``; with several ranks each one runs BM25
    over its own doc shard and the lists ride the stage-2 all-gather (the
    collectives are issued in the same order on every rank).  Results per
    batch are exactly those of the unpipelined path.
    """

    def __init__(self, searcher, device, colbert_k: int = 100, fused: int = 50, final_k: int = 10,
                 rrf_k: int = 60):
        from .distributed import ShardedSearcher
        if not hasattr(searcher, "search_hybrid"):
            searcher = ShardedSearcher(searcher, world=1)     # a bare index: one shard
        self.searcher, self.device = searcher, torch.device(device)
        self.k, self.fused, self.final_k, self.rrf_k = colbert_k, fused, final_k, rrf_k
        self._ids_h = [None, None]   # pinned, one per in-flight batch
        self._lex_h = [None, None]
        self._cand_h = [None, None]

    @staticmethod
    def _pinned(buf, rows: int, cols: int):
        if buf is None or buf.shape[0] < rows or buf.shape[1] != cols:
            buf = torch.empty((rows, cols), dtype=torch.int32, pin_memory=True)
        return buf

    def _stage12(self, Q, lex, slot: int):
        """Enqueue stage 2 (+ the D2H of its ids, on the same stream, so the
        copy runs right after the scan and not starved behind the next one);
        run (or take) stage 1 on the host meanwhile."""
        pool = None   # sharded: the gathered lists stage 3 looks its scores up in (no collective)
        if callable(lex):
            _, ids, bm, pool = self.searcher.search_hybrid(Q, self.k, lex, return_pool=True)
        else:
            _, ids = self.searcher.search(Q, self.k)
            bm = np.ascontiguousarray(lex, np.int32)
        B = ids.shape[0]
        self._ids_h[slot] = self._pinned(self._ids_h[slot], B, self.k)
        ids_h = self._ids_h[slot][:B]
        ids_h.copy_(ids, non_blocking=True)
        if isinstance(bm, torch.Tensor):                           # merged across ranks on the device
            self._lex_h[slot] = self._pinned(self._lex_h[slot], B, bm.shape[1])
            lex_h = self._lex_h[slot][:B]
            lex_h.copy_(bm, non_blocking=True)
            bm = lex_h
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        return ids_h, bm, ev, pool

    def run(self, batches):
        """batches: sequence of (Q [B, lq, D] device, lexical), where lexical is
        either the stage-1 ids [B, kb] (host) or a callable returning this
        rank's BM25 top-kb (ids, scores) -- called on the host while the GPU
        scans (see ShardedSearcher.search_hybrid).  Returns [(scores, ids)]."""
        batches = list(batches)
        if not batches:
            return []
        out = []
        cur = self._stage12(*batches[0], slot=0)
        for j, (Q, _) in enumerate(batches):
            B = Q.shape[0]
            # the GPU scans batch j+1 while the host runs its BM25 and fuses batch j
            nxt = self._stage12(*batches[j + 1], slot=(j + 1) & 1) if j + 1 < len(batches) else None
            ids_h, bm, ev, pool = cur
            ev.synchronize()
            bm_h = bm.numpy() if isinstance(bm, torch.Tensor) else bm
            self._cand_h[j & 1] = self._pinned(self._cand_h[j & 1], B, self.fused)
            cand = self._cand_h[j & 1][:B]
            cand.numpy()[:] = rrf_fuse(bm_h, ids_h.numpy(), rrf_k=self.rrf_k, C=self.fused)
            cand_d = cand.to(self.device, non_blocking=True)
            s, i, _ = self.searcher.rerank(Q, cand_d, self.final_k, pool=pool)
            out.append((s, i))
            cur = nxt
        return out


# ---------------------------------------------------------------------- one host round trip
class OneTripRetriever:
    """``retrieve_batch`` (stages 2 -> RRF -> 3, LRC:894-935) with ONE host
    round trip and no Python between the stages: ``cbv2_retrieve_begin``
    enqueues the scan + top-k, stage 1 (``lexical``) runs on the host while
    the GPU scans, and ``cbv2_retrieve_finish`` does the rest in C++ -- the
    ColBERT top-k to the host, the native RRF + ``[:C]`` cut (LRC:960-978,
    :916), the candidates back and the rerank + select (include/
    colbert_mi355x.h).  The latency path: the same results as ``step``-style
    code built from ``search_hybrid`` / ``rrf_fuse`` / ``rerank`` bit for bit,
    without the per-stage Python hops.

    ``searcher``: a ``ColbertIndex`` (one shard), or a
    ``distributed.ShardedSearcher`` built with ``native=True`` or a
    ``distributed.NativeExchange`` (the exchange inside the C ABI; bf16 /
    MXFP8 shards).  ``lexical`` per call: a callable
    returning (ids [B, kb] int32, scores [B, kb] float32) of this rank's BM25
    (host), or a host id array [B, kb] (one shard only), or None (no stage 1).
    Returns device (scores [B, final_k], ids [B, final_k], positions [B, final_k]);
    with ``host=True`` the same three as numpy arrays, on the host when the
    call returns (``cbv2_retrieve_finish_host``: one shard reads them from the
    final select's host words, no copy or stream wait -- the reference's
    ``retrieve`` returns host results, LRC:935)."""

    def __init__(self, searcher, colbert_k: int = 100, fused: int = 50, final_k: int = 10, rrf_k: int = 60,
                 lexical_k: int = 100):
        from .distributed import NativeExchange, ShardedSearcher
        comm = None
        index = searcher
        if isinstance(searcher, NativeExchange):
            index, comm = searcher.index, searcher._h
        elif isinstance(searcher, ShardedSearcher):
            index = searcher.local
            if searcher._nx is not None:
                comm = searcher._nx._h
            elif searcher.world > 1:
                raise ValueError("OneTripRetriever over several ranks needs ShardedSearcher(native=True)")
        self.index, self.comm = index, comm
        self._owner = searcher            # keeps the comm handle alive (NativeExchange frees it on __del__)
        self.k, self.C, self.final_k, self.rrf_k = int(colbert_k), int(fused), int(final_k), int(rrf_k)
        self.lexical_k = int(lexical_k)
        self.device = index.device
        self._dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._ws = None
        self._host = None
        self._sized = None        # (B, lq, kb) -> (ws pointer, bytes): the sizes of the last call
        self.record_marks = False   # latency lab: host timestamps of the last call in self.marks
        self.marks = None
        self._dev_out = None        # host=True: (B, device scores, ids, positions), reused call to call

    def _buffers(self, B: int, lq: int, kb: int):
        if self._sized is not None and self._sized[0] == (B, lq, kb):
            return self._sized[1]           # the latency path: no size queries per call
        L = _lib.lib()
        need = int(L.cbv2_retrieve_workspace_bytes(self.index._h, self.comm, B, lq, self.k, kb, self.C))
        if need == 0:
            raise ValueError(f"cbv2_retrieve_workspace_bytes: bad sizes (B {B}, lq {lq}, k {self.k}, kb {kb})")
        if self._ws is None or self._ws.numel() < need + 256:
            self._ws = torch.empty((need + 256,), dtype=torch.uint8, device=self.device)
        hneed = int(L.cbv2_retrieve_host_bytes(B, self.k, kb, self.C))
        if self._host is None or self._host.numel() < hneed:
            if self._host is not None:
                # the previous finish's candidate upload reads the old pinned block
                # through a raw pointer (no allocator event): wait for it before
                # the block can go back to torch's pinned-memory cache
                torch.cuda.current_stream(self.device).synchronize()
            self._host = torch.empty((hneed,), dtype=torch.uint8, pin_memory=True)
        off = (-self._ws.data_ptr()) % 256                 # 256-B aligned start
        out = (self._ws.data_ptr() + off, self._ws.numel() - off)
        self._sized = ((B, lq, kb), out)
        return out

    def __call__(self, Q: torch.Tensor, lexical=None, host: bool = False):
        t_enter = time.monotonic_ns() if self.record_marks else 0
        L = _lib.lib()
        shape = Q.shape
        if len(shape) == 3 and shape[1] > _LQ_MAX and self.comm is None:
            out = self._stages(Q, lexical)      # long queries: the index sums blocks of <= 32 tokens
            return tuple(x.cpu().numpy() for x in out) if host else out
        if (len(shape) == 3 and 1 <= shape[1] <= _LQ_MAX and shape[2] == 128 and Q.dtype == self._qdtype()
                and Q.is_cuda and Q.get_device() == self._dev_index
                and Q.is_contiguous()):   # the index's query layout: no conversion
            _keep, qptr, qdt, B, lq = Q, Q.data_ptr(), self._qabi, int(Q.shape[0]), int(Q.shape[1])
        else:
            _keep, qptr, qdt, B, lq = self.index._prep_query(Q, "maxsim")
        kb_cap = self.lexical_k if callable(lexical) else (0 if lexical is None else int(np.shape(lexical)[1]))
        ws, wsb = self._buffers(B, lq, kb_cap)
        st = _raw_stream(self._dev_index) if _raw_stream is not None else _stream_ptr_fn(self.device)
        t_prep = time.monotonic_ns() if self.record_marks else 0
        _lib.check(L.cbv2_retrieve_begin(self.index._h, self.comm, qptr, qdt, B, lq, self.k, kb_cap, self.C,
                                         ws, wsb, st))
        t_begun = time.monotonic_ns() if self.record_marks else 0
        try:
            return self._finish(L, Q, lexical, qptr, qdt, B, lq, kb_cap, ws, wsb, st, t_enter, t_prep, t_begun, host)
        except BaseException:
            L.cbv2_retrieve_cancel(self.index._h, ws, st)   # begin's host buffer back to its pool
            raise

    def _finish(self, L, Q, lexical, qptr, qdt, B, lq, kb_cap, ws, wsb, st, t_enter, t_prep, t_begun, host=False):
        lex_i = lex_s = None
        kb = 0
        if lexical is not None:       # stage 1 on the host while the GPU scans
            if callable(lexical):
                lex_i, lex_s = lexical()
                lex_s = np.ascontiguousarray(lex_s, np.float32)
            else:
                lex_i = lexical
                if self.comm is not None:
                    raise ValueError("a sharded retrieve needs the BM25 scores too: pass a callable")
            lex_i = np.ascontiguousarray(lex_i, np.int32)
            kb = int(lex_i.shape[1])
            if lex_i.shape[0] != B or kb > kb_cap:
                raise ValueError(f"stage-1 lists must be [B, <= {kb_cap}] (got {lex_i.shape})")
        lex_ip = lex_i.ctypes.data if kb else None
        lex_sp = lex_s.ctypes.data if (kb and lex_s is not None) else None
        if host:   # device outputs as call-to-call scratch; the results come back as host arrays
            if self._dev_out is None or self._dev_out[0] != B:
                self._dev_out = (B,) + tuple(torch.empty((B, self.final_k), dtype=dt, device=self.device)
                                             for dt in (torch.float32, torch.int32, torch.int32))
            _, out_s, out_i, out_p = self._dev_out
            hs = np.empty((B, self.final_k), np.float32)
            hi = np.empty((B, self.final_k), np.int32)
            hp = np.empty((B, self.final_k), np.int32)
            _lib.check(L.cbv2_retrieve_finish_host(
                self.index._h, self.comm, qptr, qdt, B, lq, self.k, lex_ip, lex_sp, kb,
                self.rrf_k, self.C, self.final_k, ws, wsb, self._host.data_ptr(), self._host.numel(),
                out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(), hs.ctypes.data, hi.ctypes.data, hp.ctypes.data,
                st))
            out = (hs, hi, hp)
        else:
            out_s = torch.empty((B, self.final_k), dtype=torch.float32, device=self.device)
            out_i = torch.empty((B, self.final_k), dtype=torch.int32, device=self.device)
            out_p = torch.empty((B, self.final_k), dtype=torch.int32, device=self.device)
            _lib.check(L.cbv2_retrieve_finish(
                self.index._h, self.comm, qptr, qdt, B, lq, self.k, lex_ip, lex_sp, kb,
                self.rrf_k, self.C, self.final_k, ws, wsb, self._host.data_ptr(), self._host.numel(),
                out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(), st))
            out = (out_s, out_i, out_p)
        if self.record_marks:
            c_marks = (ctypes.c_int64 * 6)()
            L.cbv2_retrieve_host_marks(c_marks, 6)
            self.marks = {"enter": t_enter, "prep": t_prep, "begun": t_begun, "finish": list(c_marks),
                          "exit": time.monotonic_ns()}
        return out

    def _qdtype(self):
        """The torch dtype a query of this index is passed as without conversion
        (None for MXFP8: quantised per call)."""
        if getattr(self, "_qdt_cache", None) is None:
            ix = self.index
            self._qdt_cache = (torch.float32 if ix.faithful else None if ix.fp8 else torch.bfloat16,)
            self._qabi = _lib.DTYPE_F32 if ix.faithful else _lib.DTYPE_BF16
        return self._qdt_cache[0]

    def _stages(self, Q: torch.Tensor, lexical):
        """The same stages called one by one (queries of more than 32 tokens)."""
        _, ids = self.index.search(Q, self.k)
        B = ids.shape[0]
        if lexical is None:
            bm = np.zeros((B, 0), np.int32)
        else:
            bm = np.ascontiguousarray(lexical()[0] if callable(lexical) else lexical, np.int32)
        cand = rrf_fuse(bm, ids.cpu().numpy(), rrf_k=self.rrf_k, C=self.C)
        return self.index.rerank(Q, torch.from_numpy(cand).to(self.device), self.final_k)
