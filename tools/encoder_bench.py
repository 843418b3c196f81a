#!/usr/bin/env python3
"""Jina-ColBERT-v2 encoder throughput on PyTorch-ROCm (SURVEY §8 f1 measurement):
the full architecture (24 x 1024, random bf16 weights — none offline) on
synthetic token ids.  Queries: B x 32 tokens, eager and HIP-graph replay;
documents: B x 128 tokens (index ingest)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hybrid_rag_colbertv2_amd.jina_encoder import JinaColBERTConfig, JinaColBERTEncoder  # noqa: E402


def timed(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


c = JinaColBERTConfig()
enc = JinaColBERTEncoder.random(c, device="cuda")
params = sum(p.numel() for p in enc.model.parameters())
out = {"params": params}
for B in (1, 32, 256):
    ids = torch.randint(3, c.vocab_size - 10, (B, c.query_maxlen))
    ids, mask = enc.query_batch(ids.tolist())
    t_eager = timed(lambda: enc.encode_ids(ids, mask))
    enc.capture_queries(B)
    t_graph = timed(lambda: enc.encode_ids(ids, mask))
    flop = 2 * (params - c.vocab_size * c.hidden) * B * c.query_maxlen
    out[f"query_B{B}"] = {"eager_ms": round(t_eager * 1e3, 3), "graph_ms": round(t_graph * 1e3, 3),
                          "qps": round(B / t_graph, 1), "TFLOPs": round(flop / t_graph / 1e12, 1)}
B = 64
ids = torch.randint(3, c.vocab_size - 10, (B, c.doc_maxlen - 3))
dids, dmask = enc.doc_batch(ids.tolist())
t = timed(lambda: enc.encode_ids(dids, dmask), iters=5)
out["docs_B64_L128"] = {"ms": round(t * 1e3, 3), "docs_per_s": round(B / t, 1)}
print(json.dumps(out))
