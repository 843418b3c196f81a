"""MI355X-native ColBERT late-interaction retrieval path (drop-in for the
reference's JinaColBERTRetriever / DualIndexer / HybridRetriever)."""
from .config import RAGConfig  # noqa: F401
from .encoder import FakeEncoder  # noqa: F401
