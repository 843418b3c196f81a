"""Jina-ColBERT-v2 query/document encoder on PyTorch-ROCm.

The reference loads ``SentenceTransformer("jinaai/jina-colbert-v2",
trust_remote_code=True)`` by hub name (local_rag_complete.py:720-724) and calls
``encode`` on queries (LRC:758, 782) and chunks (LRC:735, 783).  Neither the
weights nor sentence-transformers exist offline here, so this module builds the
architecture itself and loads weights only from a LOCAL directory:

  backbone  XLM-RoBERTa-large layout as in Jina's flash implementation:
            word + token-type embeddings (no absolute positions), LayerNorm,
            24 post-LN blocks of [fused-QKV self-attention with rotary
            position embeddings (base 20000) -> out proj] and [fc1 -> GELU ->
            fc2], hidden 1024, 16 heads, FFN 4096, vocab 250002;
  head      ColBERT linear 1024 -> 128 (no bias), L2-normalised per token;
  queries   "[QueryMarker]" prefix, padded to query_maxlen (32) with [MASK]
            tokens that are attended (ColBERT query augmentation);
  documents "[DocumentMarker]" prefix, truncated to doc_maxlen (128 here: the
            index tile height), padding dropped.

Compute is bf16 on the GPU; attention is ``F.scaled_dot_product_attention``
(flash / memory-efficient kernels on ROCm).  The encoder is PyTorch by the
north star's contract ("the Jina-ColBERT encoder runs on PyTorch-ROCm"); the
MaxSim path after it is the HIP library.

Parity: UNPINNED.  No weights, tokenizer or reference outputs exist offline,
so the checkpoint key map (``_KEYMAP``) follows the published layout of
jinaai/xlm-roberta-flash-implementation and fails loudly on any missing key;
tests pin only the arithmetic (bf16 GPU forward vs an fp32 CPU forward of the
same weights) and the ColBERT conventions (marker, augmentation, norms).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Union

import torch
import torch.nn as nn
import torch.nn.functional as F


@dataclass
class JinaColBERTConfig:
    vocab_size: int = 250002
    hidden: int = 1024
    layers: int = 24
    heads: int = 16
    ffn: int = 4096
    type_vocab: int = 1
    rotary_base: float = 20000.0
    ln_eps: float = 1e-5
    colbert_dim: int = 128
    query_maxlen: int = 32
    doc_maxlen: int = 128
    pad_id: int = 1
    cls_id: int = 0
    sep_id: int = 2
    mask_id: int = 250001
    query_marker_id: int = 250002 - 2   # "[QueryMarker]" (added token; overridden by a local tokenizer)
    doc_marker_id: int = 250002 - 3     # "[DocumentMarker]"

    @classmethod
    def tiny(cls) -> "JinaColBERTConfig":
        """A small config of the same architecture for tests."""
        return cls(vocab_size=1000, hidden=64, layers=2, heads=4, ffn=128, mask_id=999,
                   query_marker_id=998, doc_marker_id=997)


def _rotary(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor) -> torch.Tensor:
    """Non-interleaved rotary embedding on the head dim: x [B, H, L, Dh]."""
    d = x.shape[-1] // 2
    x1, x2 = x[..., :d], x[..., d:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


class _Block(nn.Module):
    def __init__(self, c: JinaColBERTConfig):
        super().__init__()
        self.heads = c.heads
        self.Wqkv = nn.Linear(c.hidden, 3 * c.hidden)
        self.out_proj = nn.Linear(c.hidden, c.hidden)
        self.norm1 = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.fc1 = nn.Linear(c.hidden, c.ffn)
        self.fc2 = nn.Linear(c.ffn, c.hidden)
        self.norm2 = nn.LayerNorm(c.hidden, eps=c.ln_eps)

    def forward(self, x, cos, sin, attn_mask):
        B, L, D = x.shape
        qkv = self.Wqkv(x).view(B, L, 3, self.heads, D // self.heads).permute(2, 0, 3, 1, 4)
        q, k, v = _rotary(qkv[0], cos, sin), _rotary(qkv[1], cos, sin), qkv[2]
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=attn_mask)
        x = self.norm1(x + self.out_proj(a.transpose(1, 2).reshape(B, L, D)))
        return self.norm2(x + self.fc2(F.gelu(self.fc1(x))))


class JinaColBERTModel(nn.Module):
    """Backbone + ColBERT head: token ids [B, L] -> L2-normalised [B, L, 128]."""

    def __init__(self, c: JinaColBERTConfig):
        super().__init__()
        self.config = c
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden)
        self.token_type_embeddings = nn.Embedding(c.type_vocab, c.hidden)
        self.emb_ln = nn.LayerNorm(c.hidden, eps=c.ln_eps)
        self.layers = nn.ModuleList([_Block(c) for _ in range(c.layers)])
        self.linear = nn.Linear(c.hidden, c.colbert_dim, bias=False)

    def _rope(self, L: int, device, dtype):
        dh = self.config.hidden // self.config.heads
        inv = 1.0 / (self.config.rotary_base ** (torch.arange(0, dh, 2, device=device, dtype=torch.float32) / dh))
        ang = torch.arange(L, device=device, dtype=torch.float32)[:, None] * inv[None, :]
        return ang.cos().to(dtype), ang.sin().to(dtype)

    def forward(self, ids: torch.Tensor, attention_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
        """attention_mask None = every token attended (queries): SDPA keeps its
        flash path and the forward is capturable in a HIP graph."""
        x = self.word_embeddings(ids) + self.token_type_embeddings(torch.zeros_like(ids))
        x = self.emb_ln(x)
        cos, sin = self._rope(ids.shape[1], ids.device, x.dtype)
        bias = None          # additive key mask [B, 1, 1, L]: padding keys are never attended
        if attention_mask is not None:
            bias = torch.zeros(attention_mask.shape, dtype=x.dtype, device=x.device)
            bias = bias.masked_fill(attention_mask == 0, float("-inf"))[:, None, None, :]
        for blk in self.layers:
            x = blk(x, cos, sin, bias)
        return F.normalize(self.linear(x).float(), dim=-1)


# checkpoint key (jinaai/jina-colbert-v2 model.safetensors, flash implementation) -> module key
_KEYMAP = {
    "roberta.embeddings.word_embeddings.weight": "word_embeddings.weight",
    "roberta.embeddings.token_type_embeddings.weight": "token_type_embeddings.weight",
    "roberta.emb_ln.weight": "emb_ln.weight",
    "roberta.emb_ln.bias": "emb_ln.bias",
    "linear.weight": "linear.weight",
}
_LAYER_KEYS = {
    "mixer.Wqkv.weight": "Wqkv.weight", "mixer.Wqkv.bias": "Wqkv.bias",
    "mixer.out_proj.weight": "out_proj.weight", "mixer.out_proj.bias": "out_proj.bias",
    "norm1.weight": "norm1.weight", "norm1.bias": "norm1.bias",
    "mlp.fc1.weight": "fc1.weight", "mlp.fc1.bias": "fc1.bias",
    "mlp.fc2.weight": "fc2.weight", "mlp.fc2.bias": "fc2.bias",
    "norm2.weight": "norm2.weight", "norm2.bias": "norm2.bias",
}


class HashTokenizer:
    r"""Stand-in tokenizer (no tokenizer.json offline): lower-case ``\w+`` words
    mapped to ids by crc32 into [3, vocab - 4).  Same ``encode(text).ids`` API
    as ``tokenizers.Tokenizer``; for tests and demos only."""

    class _Enc:
        def __init__(self, ids):
            self.ids = ids

    def __init__(self, vocab_size: int):
        self.span = vocab_size - 7

    def encode(self, text: str, add_special_tokens: bool = False):
        import re
        import zlib
        return self._Enc([3 + zlib.crc32(w.encode()) % self.span for w in re.findall(r"\w+", text.lower())])


class JinaColBERTEncoder:
    """``encode(texts, convert_to_tensor=True, is_query=...)`` like the
    SentenceTransformer object the reference holds, producing ColBERT token
    matrices: queries [B, 32, 128] (augmented), documents [B, <=128, 128]."""

    def __init__(self, model: JinaColBERTModel, tokenizer=None, device="cuda", dtype=torch.bfloat16):
        self.config = model.config
        self.device = torch.device(device)
        self.dtype = dtype
        self.model = model.to(device=self.device, dtype=dtype).eval()
        self.tokenizer = tokenizer
        self._graphs = {}

    # ------------------------------------------------------------ construction
    @classmethod
    def random(cls, config: Optional[JinaColBERTConfig] = None, seed: int = 0, device="cuda",
               dtype=torch.bfloat16) -> "JinaColBERTEncoder":
        """Random-init weights of the real architecture (benchmarks; there are no weights offline)."""
        torch.manual_seed(seed)
        return cls(JinaColBERTModel(config or JinaColBERTConfig()), None, device, dtype)

    @classmethod
    def from_local(cls, path: str, device="cuda", dtype=torch.bfloat16) -> "JinaColBERTEncoder":
        """config.json + model.safetensors (+ tokenizer.json) from a LOCAL directory."""
        from safetensors.torch import load_file
        c = JinaColBERTConfig()
        cfg_path = os.path.join(path, "config.json")
        if os.path.exists(cfg_path):
            with open(cfg_path) as f:
                hf = json.load(f)
            c.vocab_size = hf.get("vocab_size", c.vocab_size)
            c.hidden = hf.get("hidden_size", c.hidden)
            c.layers = hf.get("num_hidden_layers", c.layers)
            c.heads = hf.get("num_attention_heads", c.heads)
            c.ffn = hf.get("intermediate_size", c.ffn)
            c.rotary_base = hf.get("rotary_emb_base", c.rotary_base)
            c.ln_eps = hf.get("layer_norm_eps", c.ln_eps)
        state = load_file(os.path.join(path, "model.safetensors"))
        model = JinaColBERTModel(c)
        want = {}
        for src, dst in _KEYMAP.items():
            want[dst] = src
        for i in range(c.layers):
            for src, dst in _LAYER_KEYS.items():
                want[f"layers.{i}.{dst}"] = f"roberta.encoder.layers.{i}.{src}"
        missing = [s for s in want.values() if s not in state]
        if missing:
            raise KeyError(f"{len(missing)} checkpoint tensors missing, e.g. {missing[:3]}")
        model.load_state_dict({d: state[s] for d, s in want.items()}, strict=True)
        tok = None
        tok_path = os.path.join(path, "tokenizer.json")
        if os.path.exists(tok_path):
            from tokenizers import Tokenizer
            tok = Tokenizer.from_file(tok_path)
            for name, attr in (("[QueryMarker]", "query_marker_id"), ("[DocumentMarker]", "doc_marker_id"),
                               ("<mask>", "mask_id"), ("<pad>", "pad_id")):
                tid = tok.token_to_id(name)
                if tid is not None:
                    setattr(c, attr, tid)
        return cls(model, tok, device, dtype)

    # ------------------------------------------------------------ token ids
    def _ids(self, text: str) -> List[int]:
        if self.tokenizer is None:
            raise RuntimeError("no tokenizer: pass token ids (encode_ids) or load a local tokenizer.json")
        return self.tokenizer.encode(text, add_special_tokens=False).ids

    def query_batch(self, rows: Sequence[Sequence[int]]):
        """[CLS] [QueryMarker] ids... [SEP] padded with attended [MASK] to query_maxlen."""
        c = self.config
        L = c.query_maxlen
        ids = torch.full((len(rows), L), c.mask_id, dtype=torch.long)
        for b, r in enumerate(rows):
            seq = [c.cls_id, c.query_marker_id] + list(r)[: L - 3] + [c.sep_id]
            ids[b, : len(seq)] = torch.tensor(seq)
        return ids, torch.ones_like(ids)

    def doc_batch(self, rows: Sequence[Sequence[int]]):
        """[CLS] [DocumentMarker] ids... [SEP], truncated to doc_maxlen, padding masked."""
        c = self.config
        seqs = [[c.cls_id, c.doc_marker_id] + list(r)[: c.doc_maxlen - 3] + [c.sep_id] for r in rows]
        L = max(len(s) for s in seqs) if seqs else 1
        ids = torch.full((len(seqs), L), c.pad_id, dtype=torch.long)
        mask = torch.zeros((len(seqs), L), dtype=torch.long)
        for b, s in enumerate(seqs):
            ids[b, : len(s)] = torch.tensor(s)
            mask[b, : len(s)] = 1
        return ids, mask

    @torch.no_grad()
    def encode_ids(self, ids: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
        """Token ids [B, L] (+ attention mask) -> fp32 [B, L, 128] unit token vectors."""
        full = bool(mask.bool().all())                      # host-side check (no sync in a capture)
        g = self._graphs.get(tuple(ids.shape)) if full else None
        if g is not None:                                   # replay the captured query graph
            graph, static_ids, static_out = g
            static_ids.copy_(ids.to(self.device), non_blocking=True)
            graph.replay()
            return static_out.clone()
        return self.model(ids.to(self.device), None if full else mask.to(self.device))

    @torch.no_grad()
    def capture_queries(self, B: int) -> None:
        """Capture the fixed-shape query forward [B, query_maxlen] in a HIP graph
        (the launch-bound 24-layer stack replays as one graph launch)."""
        L = self.config.query_maxlen
        static_ids = torch.full((B, L), self.config.mask_id, dtype=torch.long, device=self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):                              # warm the allocator / kernel selection
                self.model(static_ids)
        torch.cuda.current_stream(self.device).wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static_out = self.model(static_ids)
        self._graphs[(B, L)] = (graph, static_ids, static_out)

    def encode(self, sentences: Union[str, Sequence[str]], convert_to_tensor: bool = True,
               is_query: bool = True, show_progress_bar: bool = False, batch_size: int = 64, **_unused):
        single = isinstance(sentences, str)
        texts = [sentences] if single else list(sentences)
        outs = []
        for i in range(0, len(texts), batch_size):
            rows = [self._ids(t) for t in texts[i:i + batch_size]]
            ids, mask = self.query_batch(rows) if is_query else self.doc_batch(rows)
            emb = self.encode_ids(ids, mask)
            if is_query:
                outs.extend(emb)
            else:   # padding rows are not document tokens
                outs.extend(e[: int(m.sum())] for e, m in zip(emb, mask))
        if is_query:
            out = torch.stack(outs) if outs else torch.zeros((0, self.config.query_maxlen, self.config.colbert_dim))
            return out[0] if single else out
        return outs[0] if single else outs
