"""RAGConfig — the retrieval-path subset of the reference's configuration.

Mirrors ``RAGConfig`` (local_rag_complete.py:56-86): same field names and
defaults for every field the ColBERT / hybrid retrieval path reads
(``bm25_top_k``, ``colbert_top_k``, ``final_top_k``, ``embedding_model``,
``bm25_index_path``, ``colbert_index_path``, ``device``).  Ingestion, chat and
Ollama fields are kept as inert placeholders so reference call sites that
construct ``RAGConfig(...)`` with them keep working.

Added fields (no reference counterpart):
  * ``scorer``         — "maxsim" (true ColBERT late interaction, the
                          north-star contract) or "ref_meanpool_cosine" (the
                          literal arithmetic of local_rag_complete.py:814-831).
  * ``fused_candidates`` — the ``[:50]`` hard-coded at local_rag_complete.py:916.
  * ``rrf_k``          — the ``k=60`` default at local_rag_complete.py:964.
  * ``doc_maxlen`` / ``query_maxlen`` / ``dim`` — index geometry.
  * ``index_dtype``    — "fp32" (default: fp32-faithful, the reference's fp32
                          scores within ~1e-5 and their exact top-k, as the
                          north star's 1e-3 contract requires for an encoder
                          that returns fp32 embeddings),
                          "bf16" (~3 % more queries/s; scores within ~5e-3 of
                          fp32 on fp32 embeddings, exact on bf16-valued ones)
                          or "fp8" (MXFP8, config 5).
  * ``ingest_batch`` / ``index_pt_max_docs`` — batched, bounded-memory
                          indexing (JinaColBERTRetriever.index).
"""
from dataclasses import dataclass


@dataclass
class RAGConfig:
    # Database (out of scope; kept for constructor compatibility)
    db_path: str = "rag_local.db"

    # Chunking (out of scope)
    min_chunk_size: int = 256
    max_chunk_size: int = 1024
    chunk_overlap: int = 128

    # Retrieval (local_rag_complete.py:68-70)
    bm25_top_k: int = 100
    colbert_top_k: int = 100
    final_top_k: int = 10

    # Models (local_rag_complete.py:73-75)
    chat_model: str = "llama3.2:3b"
    vision_model: str = "llava:7b"
    embedding_model: str = "jinaai/jina-colbert-v2"

    ollama_url: str = "http://localhost:11434"

    # Paths (local_rag_complete.py:81-83)
    bm25_index_path: str = "indexes/bm25s"
    colbert_index_path: str = "indexes/colbert"
    images_dir: str = "extracted_images"

    # Device: the reference picks "mps"/"cpu" (local_rag_complete.py:86); the
    # MI355X path always scores on a ROCm device ("cuda" is HIP under PyTorch-ROCm).
    device: str = "cuda"

    # MI355X additions
    scorer: str = "maxsim"
    fused_candidates: int = 50
    rrf_k: int = 60
    doc_maxlen: int = 128
    query_maxlen: int = 32
    dim: int = 128
    index_dtype: str = "fp32"
    ingest_batch: int = 256            # docs encoded and indexed per batch (bounded host memory)
    index_pt_max_docs: int = 50_000    # larger corpora persist as index.cbv2, not the fp32 index.pt
