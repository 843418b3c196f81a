"""MI355X-native ColBERT late-interaction retrieval path.

Drop-in for the retrieval classes of techmum21p/hybrid-rag-ColBERTv2
(local_rag_complete.py): ``RAGConfig``, ``JinaColBERTRetriever``,
``DualIndexer``, ``HybridRetriever``.  Scoring, top-k, rerank and the
cross-shard merge run in hand-written HIP kernels (libcolbert_mi355x.so);
BM25 and RRF fusion run on the host.
"""
from .config import RAGConfig  # noqa: F401
from .encoder import FakeEncoder  # noqa: F401


def __getattr__(name):  # lazy: importing the package never touches the GPU
    if name in ("JinaColBERTRetriever",):
        from .retriever import JinaColBERTRetriever
        return JinaColBERTRetriever
    if name in ("DualIndexer", "HybridRetriever", "ChunkStore", "rrf_fuse"):
        from . import hybrid
        return getattr(hybrid, name)
    if name in ("ColbertIndex",):
        from .index import ColbertIndex
        return ColbertIndex
    if name in ("ShardedSearcher",):
        from .distributed import ShardedSearcher
        return ShardedSearcher
    raise AttributeError(name)
