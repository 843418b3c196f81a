"""Multi-GPU path: the corpus sharded by contiguous id range, one process per GPU.

No reference counterpart (the reference is single-process); this
is the §8(e) design:

  stage 2  every rank scans its shard (HIP scan + top-k) -> [B, k] (score,
           global id) -> ONE all-gather over RCCL/xGMI of the packed pairs
           [G, B, k, 2] -> HIP merge with the (score desc, id asc) rule.
           Every rank ends with the identical global top-k.
  stage 3  NO collective: every fused candidate is in a stage-2 list or a
           stage-1 list, and both carry the rerank's score of the doc -- a
           rank's local top-k scores are the rerank's bits (the same MaxSim
           arithmetic), and each rank prescores its own BM25 top-kb with the
           rerank before the stage-2 all-gather, where the prescores ride -- so
           every rank looks the candidates' scores up in the gathered lists
           and selects the top-k (``rerank(..., pool=...)``).  Candidates from
           anywhere else take the collective form: every rank scores the
           candidates it owns (-inf for the rest) -> all-reduce(MAX) over
           [B, C] -> HIP top-k select (each id has exactly one owner).

Stage 1 (host BM25) is doc-sharded the same way (bm25.sharded: global
statistics from one build-time all-reduce), and its per-rank top-kb lists
ride the stage-2 all-gather (search_hybrid), so a query costs each rank only
its shard's postings and the whole exchange stays ONE collective per stage.

Messages are tiny (B=256, k=100, kb=100: 400 KiB per rank), so the exchange
is latency-bound; it is ONE collective per query batch (fp32-faithful shards:
one more, the global band bound).  torch.distributed's "nccl"
backend IS RCCL on ROCm.  The same code runs on "gloo" for CPU tests, where
the caller injects CPU ``local``/``ops`` objects (tests only).
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .encoder import encode


def shard_range(n_total: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [begin, end) of global ids owned by ``rank`` (sizes differ by <= 1)."""
    base, rem = divmod(n_total, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def encode_queries_sharded(encoder, queries, device=None, dtype=torch.bfloat16,
                           group: Optional[dist.ProcessGroup] = None) -> torch.Tensor:
    """Query embeddings ``[B, Lq, D]`` for a batch of query strings, the
    encoder's work split over the ranks instead of replicated on each.

    The reference encodes every query in-process before scoring
    (local_rag_complete.py:758 ``search``, :782 ``rerank``).  With the corpus
    sharded, every rank needs the whole batch's embeddings, so each rank
    encodes its contiguous slice ``shard_range(B, rank, G)`` (``is_query=True``:
    the ColBERT query augmentation pads to Lq) and ONE all-gather of
    ``[G, ceil(B/G), Lq, D]`` (2 MiB at B=256 in bf16) rebuilds the batch on
    every rank, in query order.  The result equals ``encoder.encode(queries)``
    on one process cast to ``dtype`` (gloo-tested at world size 2).  Without an
    initialised process group this is that single encode."""
    queries = [queries] if isinstance(queries, str) else list(queries)
    B = len(queries)

    def enc(rows):
        out = encode(encoder, rows, is_query=True)
        out = out if isinstance(out, torch.Tensor) else torch.as_tensor(np.asarray(out))
        return out.to(device=device, dtype=dtype) if device is not None else out.to(dtype)

    if not (dist.is_available() and dist.is_initialized()) or B == 0:
        return enc(queries)
    G, r = dist.get_world_size(group), dist.get_rank(group)
    per = (B + G - 1) // G
    b0, b1 = shard_range(B, r, G)
    nccl = dist.get_backend(group) == "nccl"
    # the collectives' device: RCCL needs device tensors, gloo takes host ones
    dev = torch.device(device) if device is not None else (
        torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu"))
    mine = enc(queries[b0:b1]).to(dev) if b1 > b0 else None
    # every rank must learn Lq and D even when its slice is empty
    shape = torch.tensor(list(mine.shape[1:]) if mine is not None else [0, 0], dtype=torch.int64, device=dev)
    dist.all_reduce(shape, op=dist.ReduceOp.MAX, group=group)
    lq, d = int(shape[0]), int(shape[1])
    send = torch.zeros((per, lq, d), dtype=dtype, device=dev)
    if mine is not None:   # an encoder that does not pad to Lq: zero rows add 0 to every MaxSim sum
        send[: b1 - b0, : mine.shape[1], : mine.shape[2]].copy_(mine)
    out = torch.empty((G, per, lq, d), dtype=dtype, device=dev)
    if nccl:
        dist.all_gather_into_tensor(out, send, group=group)
    else:
        dist.all_gather(list(out.unbind(0)), send, group=group)
    parts = [out[g, : shard_range(B, g, G)[1] - shard_range(B, g, G)[0]] for g in range(G)]
    return torch.cat(parts, 0)


class _DeviceOps:
    """HIP merge / select (libcolbert_mi355x.so)."""

    @staticmethod
    def merge(S: torch.Tensor, I: torch.Tensor, k: int):
        from .index import merge_topk
        return merge_topk(S, I, k)

    @staticmethod
    def select(scores: torch.Tensor, k: int, ids: torch.Tensor):
        from .index import select_topk
        return select_topk(scores, k, ids=ids)


class _PinnedStage:
    """Host -> device uploads that do not block the host.

    ``torch.from_numpy(x).to(dev)`` from pageable memory synchronises the
    stream, i.e. waits for the scan queued ahead of it -- in the pipelined path
    that stalls the host until batch j+1's scan ends before it can fuse batch j
    and leaves the GPU idle for the host steps.  Here the array is copied into
    a pinned buffer and uploaded with ``non_blocking=True``; buffers rotate
    over ``slots`` calls, and each slot's upload is followed by an event that
    the host waits on before it overwrites that slot again (a caller that loops
    faster than the stream drains never corrupts a pending upload)."""

    def __init__(self, slots: int = 2):
        self._bufs = [None] * slots
        self._events = [None] * slots
        self._next = 0

    def upload(self, arr: np.ndarray, device) -> torch.Tensor:
        device = torch.device(device)
        src = torch.from_numpy(np.ascontiguousarray(arr))
        if device.type != "cuda":
            return src.clone()
        k = self._next
        self._next = (k + 1) % len(self._bufs)
        if self._events[k] is not None:
            self._events[k].synchronize()          # the slot's previous upload has been consumed
        buf = self._bufs[k]
        if buf is None or buf.numel() < src.numel() * src.element_size():
            buf = torch.empty((src.numel() * src.element_size(),), dtype=torch.uint8, pin_memory=True)
            self._bufs[k] = buf
        h = buf[: src.numel() * src.element_size()].view(src.dtype).view(src.shape)
        h.copy_(src)
        out = h.to(device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        self._events[k] = ev
        return out


def loopback_comms(G: int):
    """TEST-ONLY: ``G`` ``cbv2_comm*`` handles forming one in-process loopback
    group on the current device (include/colbert_mi355x.h
    cbv2_comm_loopback_init).  Drive rank r from its own thread and stream
    (``NativeExchange(shard_r, comm=handles[r])``); the handle is freed by the
    NativeExchange that adopts it."""
    import ctypes

    from . import _lib
    arr = (ctypes.c_void_p * G)()
    _lib.check(_lib.lib().cbv2_comm_loopback_init(G, arr))
    return [ctypes.c_void_p(arr[r]) for r in range(G)]


class NativeExchange:
    """The exchange inside libcolbert_mi355x.so (include/colbert_mi355x.h:
    cbv2_search_sharded_local/_exchange, cbv2_rerank_sharded) over the RCCL
    communicator torch.distributed's "nccl" backend already holds: scan,
    all-gather and merges are all enqueued by C++ on the current stream, with
    no Python between them.  An fp32-faithful shard takes the same calls: the
    global k-th bound (``ShardedSearcher._global_kth`` in Python) is one more
    all-gather inside ``cbv2_search_sharded_local``."""

    def __init__(self, index, group: Optional[dist.ProcessGroup] = None, lexical_k: int = 100, comm=None):
        """``comm``: an existing ``cbv2_comm*`` handle to adopt (e.g. one rank of
        ``loopback_comms``, test-only); default: wrap torch's RCCL communicator."""
        import ctypes
        import os

        from . import _lib
        self.index, self.dev, self.lexical_k = index, index.device, int(lexical_k)
        self._lib = _lib
        if comm is not None:
            h = comm
        else:
            pg = group if group is not None else dist.distributed_c10d._get_default_group()
            if dist.get_backend(pg) != "nccl":
                raise RuntimeError("the native exchange needs the RCCL ('nccl') backend")
            warm = torch.zeros(1, device=self.dev)
            dist.all_reduce(warm, group=group)                 # the communicator exists after one collective
            torch.cuda.synchronize(self.dev)
            comm_ptr = pg._get_backend(self.dev)._comm_ptr()
            rccl = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
            h = ctypes.c_void_p()
            _lib.check(_lib.lib().cbv2_comm_init(comm_ptr, rccl.encode() if os.path.exists(rccl) else None,
                                                 ctypes.byref(h)))
        self._h = h
        self._stage = _PinnedStage(slots=4)               # ids + scores per call
        self.world = int(_lib.lib().cbv2_comm_size(h))
        self.rank = int(_lib.lib().cbv2_comm_rank(h))
        # two search workspaces, used in turn: a pipelined caller's stage 3 of
        # batch j reads batch j's gathered blocks (its pool) after batch j+1's
        # exchange was enqueued; + one for the collective rerank's scratch
        self._ws = [None, None, None]
        self._turn = 0

    def __del__(self):
        try:
            self._lib.lib().cbv2_comm_destroy(self._h)
        except Exception:
            pass

    def _workspace(self, B: int, k: int, kb: int, C: int, slot: int = 2) -> torch.Tensor:
        need = int(self._lib.lib().cbv2_sharded_workspace_bytes(self.index._h, self._h, B, k, kb, C))
        if self._ws[slot] is None or self._ws[slot].numel() < need:
            self._ws[slot] = torch.empty((need,), dtype=torch.uint8, device=self.dev)
        return self._ws[slot]

    def comm_stats(self):
        """(all-gathers, all-reduces) issued on this handle so far."""
        import ctypes
        out = (ctypes.c_int64 * 2)()
        self._lib.check(self._lib.lib().cbv2_comm_stats(self._h, out))
        return int(out[0]), int(out[1])

    def search(self, Q: torch.Tensor, k: int, lexical=None, return_pool: bool = False):
        """(scores, ids, merged BM25 ids or None)[, pool]: the pool names this
        call's gathered blocks for ``rerank(..., pool=pool)`` (stage 3 without
        a collective); it stays valid until the next-but-one search."""
        from .index import _stream_ptr
        L = self._lib.lib()
        _keep, qptr, qdt, B, lq = self.index._prep_query(Q, "maxsim")
        st = _stream_ptr(self.dev)
        # the local scan is enqueued BEFORE stage 1 runs on the host, so the
        # workspace is sized for up to ``lexical_k`` stage-1 ids per query
        kb_cap = self.lexical_k if lexical is not None else 0
        slot, self._turn = self._turn, self._turn ^ 1
        ws = self._workspace(B, k, kb_cap, 0, slot)
        self._lib.check(L.cbv2_search_sharded_local(self.index._h, self._h, self._lib.SCORERS["maxsim"], qptr, qdt,
                                                    B, lq, int(k), kb_cap, ws.data_ptr(), ws.numel(), st))
        kb = 0
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.dev)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.dev)
        li = ls = out_li = None
        if lexical is not None:
            lex_i, lex_s = lexical()
            kb = int(lex_i.shape[1])
            if lex_i.shape[0] != B or not 1 <= kb <= kb_cap:
                raise ValueError(f"stage-1 lists must be [B, <= {kb_cap}] (got {lex_i.shape})")
            li = self._stage.upload(np.ascontiguousarray(lex_i, np.int32), self.dev)
            ls = self._stage.upload(np.ascontiguousarray(lex_s, np.float32), self.dev)
            out_li = torch.empty((B, kb), dtype=torch.int32, device=self.dev)
        # (Q: this rank's BM25 top-kb prescored with the rerank before the all-gather)
        self._lib.check(L.cbv2_search_sharded_exchange(
            self.index._h, self._h, qptr, qdt, lq, B, int(k), li.data_ptr() if li is not None else None,
            ls.data_ptr() if ls is not None else None, kb, ws.data_ptr(), ws.numel(), out_s.data_ptr(),
            out_i.data_ptr(), out_li.data_ptr() if out_li is not None else None, st))
        if return_pool:
            return out_s, out_i, out_li, _NativePool(ws, B, int(k), kb)
        return out_s, out_i, out_li

    def rerank(self, Q: torch.Tensor, cand: torch.Tensor, k: int, pool=None, misses: torch.Tensor = None):
        """Stage 3.  pool (from ``search(..., return_pool=True)`` of the batch
        whose lists the candidates were fused from): the scores are looked up
        in that exchange's gathered blocks, no collective
        (cbv2_rerank_sharded_prescored; ``misses``: optional device int32 [1]
        that counts candidates found in no list).  Otherwise every rank scores
        its own candidates and one all-reduce(MAX) combines them."""
        from .index import _stream_ptr
        cand = cand.to(device=self.dev, dtype=torch.int32).contiguous()
        B, C = int(cand.shape[0]), int(cand.shape[1])
        if pool is not None and pool.B == B and C <= 1024:
            out_s = torch.empty((B, k), dtype=torch.float32, device=self.dev)
            out_i = torch.empty((B, k), dtype=torch.int32, device=self.dev)
            out_p = torch.empty((B, k), dtype=torch.int32, device=self.dev)
            self._lib.check(self._lib.lib().cbv2_rerank_sharded_prescored(
                self.index._h, self._h, B, pool.k, pool.kb, cand.data_ptr(), C, int(k), pool.ws.data_ptr(),
                pool.ws.numel(), out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(),
                misses.data_ptr() if misses is not None else None, _stream_ptr(self.dev)))
            return out_s, out_i, out_p
        _keep, qptr, _, B, lq = self.index._prep_query(Q, "maxsim")
        ws = self._workspace(B, 1, 0, C)
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.dev)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.dev)
        out_p = torch.empty((B, k), dtype=torch.int32, device=self.dev)
        self._lib.check(self._lib.lib().cbv2_rerank_sharded(
            self.index._h, self._h, qptr, B, lq, cand.data_ptr(), C, int(k), ws.data_ptr(), ws.numel(),
            out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(), _stream_ptr(self.dev)))
        return out_s, out_i, out_p


class _NativePool:
    """The gathered blocks of one NativeExchange search (its workspace)."""

    def __init__(self, ws, B, k, kb):
        self.ws, self.B, self.k, self.kb = ws, B, k, kb


class _TorchPool:
    """Every rank's stage-2 top-k and prescored stage-1 list of one
    ShardedSearcher.search_hybrid call: [B, M] (id, rerank score) pairs."""

    def __init__(self, ids, scores):
        self.ids, self.scores = ids, scores


def pool_scores(cand: torch.Tensor, ids: torch.Tensor, scores: torch.Tensor):
    """raw [B, C]: each candidate's score in its row of (ids, scores) [B, M]
    (-inf for a negative id, as the rerank scores one; -inf for an id found
    nowhere, counted in misses).  Returns (raw, misses: a 0-d tensor on the
    candidates' device -- read it only where a sync is harmless)."""
    eq = (cand[:, :, None] == ids[:, None, :]) & (cand[:, :, None] >= 0)
    hit = eq.any(-1)
    idx = eq.to(torch.int8).argmax(-1)
    raw = torch.where(hit, scores.gather(1, idx), torch.full_like(cand, float("-inf"), dtype=torch.float32))
    return raw, ((cand >= 0) & ~hit).sum()


class ShardedSearcher:
    """Global search / rerank over a corpus whose shards live on the ranks of ``group``.

    ``local`` is this rank's shard (a ``ColbertIndex``: ``search(Q, k)`` and
    ``rerank(Q, cand, 0)``); ``ops`` provides ``merge`` and ``select``.
    """

    def __init__(self, local, group: Optional[dist.ProcessGroup] = None, ops=None, world: Optional[int] = None,
                 native: bool = False, lexical_k: int = 100):
        self.local = local
        self.group = group
        self._stage = _PinnedStage()
        self.ops = ops if ops is not None else _DeviceOps()
        if world is None:
            world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.world = world
        # native=True: the whole exchange runs inside the C ABI (NativeExchange)
        self._nx = NativeExchange(local, group, lexical_k) if native else None
        self._coll = None          # collective timing record (time_collectives)
        self.last_pool_misses = None   # the last pooled rerank's count of candidates in no list (tensor)

    # ------------------------------------------------------------ measurement
    def time_collectives(self, enable: bool) -> None:
        """Record every collective this searcher issues from now on: HIP events on
        the current stream around it (device time, for RCCL) and the host wall
        time of the call (for gloo, whose collectives block the host)."""
        self._coll = [] if enable else None

    def collective_times(self) -> dict:
        """{name: {"calls", "device_ms", "host_ms"}} summed over the recorded calls
        (synchronises); the record is cleared."""
        rec, self._coll = self._coll or [], None
        out = {}
        for name, e0, e1, host_ms in rec:
            if e1 is not None:
                e1.synchronize()
            d = out.setdefault(name, {"calls": 0, "device_ms": 0.0, "host_ms": 0.0})
            d["calls"] += 1
            d["device_ms"] += e0.elapsed_time(e1) if e0 is not None else 0.0
            d["host_ms"] += host_ms
        return out

    def _collective(self, name: str, fn, device):
        if self._coll is None:
            return fn()
        import time
        cuda = torch.device(device).type == "cuda"
        e0 = e1 = None
        if cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        t0 = time.perf_counter()
        r = fn()
        host_ms = (time.perf_counter() - t0) * 1e3
        if cuda:
            e1.record()
        self._coll.append((name, e0, e1, host_ms))
        return r

    def _all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.world,) + tuple(t.shape), dtype=t.dtype, device=t.device)
        if dist.get_backend(self.group) == "nccl":
            self._collective("all_gather", lambda: dist.all_gather_into_tensor(out, t.contiguous(), group=self.group),
                             t.device)
        else:
            self._collective("all_gather", lambda: dist.all_gather(list(out.unbind(0)), t.contiguous(),
                                                                   group=self.group), t.device)
        return out

    def _local_search(self, Q: torch.Tensor, k: int):
        """This rank's top-k.  An fp32-faithful shard bounds its band by the
        GLOBAL k-th score: every rank's exact faithful scores of its bf16 top-k
        ([B, k] f32, one all-gather) give k docs per rank whose scores are
        known, and the k-th largest of all of them is a lower bound of the
        global k-th score; each rank then rescores only the docs that can reach
        the global top-k rather than its own (cbv2_search_f32_begin / _finish).
        The merge of the per-rank lists is the exact global top-k."""
        if self.world > 1 and getattr(self.local, "faithful", False):
            return self.local.search(Q, k, lb_reduce=lambda fk: self._global_kth(fk, k))
        return self.local.search(Q, k)

    def _global_kth(self, fk: torch.Tensor, k: int) -> torch.Tensor:
        allf = self._all_gather(fk)                                                  # [G, B, k]
        B = fk.shape[0]
        union = allf.permute(1, 0, 2).reshape(B, self.world * k).contiguous()        # [B, G*k]
        s, _, _ = self.ops.select(union, k, None)                                    # HIP select, desc
        return s[:, k - 1].contiguous()

    def search(self, Q: torch.Tensor, k: int):
        if self._nx is not None:
            return self._nx.search(Q, k)[:2]
        s, i = self._local_search(Q, k)
        if self.world == 1:
            return s, i
        return self.search_exchange(s, i, k)

    def search_hybrid(self, Q: torch.Tensor, k: int, lexical=None, return_pool: bool = False):
        """Stage 2 plus this rank's stage-1 lists in the SAME collective.

        ``lexical()`` runs on the host AFTER the scan is enqueued (so it
        overlaps the GPU) and returns this rank's BM25 top-kb (global ids int32
        [B, kb], scores float32 [B, kb]) over its doc shard (``bm25.sharded``).
        Returns (scores, ids, bm25_ids): with one rank bm25_ids is that host
        array; otherwise both lists ride one all-gather and are merged with the
        same (score desc, id asc) rule, which reproduces the unsharded stage 1
        exactly because the shards were built with global statistics.
        With several ranks the rank's BM25 ids are first prescored with the
        rerank (raw MaxSim of its own docs) and the prescores ride the same
        all-gather: ``return_pool=True`` appends the pool that lets
        ``rerank(..., pool=pool)`` run stage 3 with no collective (None with
        one rank).
        """
        if self._nx is not None:
            return self._nx.search(Q, k, lexical, return_pool=return_pool)
        s, i = self._local_search(Q, k)
        if lexical is None:
            if self.world == 1:
                return (s, i, None, None) if return_pool else (s, i, None)
            allp = self._all_gather(torch.stack([s.contiguous().view(torch.int32), i.to(torch.int32)], dim=-1))
            S, I = self.ops.merge(allp[..., 0].contiguous().view(torch.float32), allp[..., 1].contiguous(), k)
            pool = self._pool(allp, k, 0)
            return (S, I, None, pool) if return_pool else (S, I, None)
        lex_i, lex_s = lexical()
        if self.world == 1:
            bm = np.ascontiguousarray(lex_i, np.int32)
            return (s, i, bm, None) if return_pool else (s, i, bm)
        kb = lex_i.shape[1]
        lex_i = np.ascontiguousarray(lex_i, np.int32)
        lex_d = self._stage.upload(lex_i, i.device)
        pre = self.local.rerank(Q, lex_d, 0)                     # this rank's own BM25 docs, rerank arithmetic
        lex = self._stage.upload(np.stack([np.ascontiguousarray(lex_s, np.float32).view(np.int32), lex_i],
                                          axis=-1), i.device)
        packed = torch.cat([torch.stack([s.contiguous().view(torch.int32), i.to(torch.int32)], dim=-1), lex,
                            torch.stack([pre.contiguous().view(torch.int32), lex_d], dim=-1)], dim=1)
        allp = self._all_gather(packed)                                                    # [G, B, k+2kb, 2]
        S, I = self.ops.merge(allp[:, :, :k, 0].contiguous().view(torch.float32), allp[:, :, :k, 1].contiguous(), k)
        _, LI = self.ops.merge(allp[:, :, k:k + kb, 0].contiguous().view(torch.float32),
                               allp[:, :, k:k + kb, 1].contiguous(), kb)
        pool = self._pool(allp, k, kb)
        return (S, I, LI, pool) if return_pool else (S, I, LI)

    @staticmethod
    def _pool(allp: torch.Tensor, k: int, kb: int) -> _TorchPool:
        """[B, G*(k+kb)] (id, score) pairs: every rank's local top-k and its
        prescored stage-1 list (allp [G, B, k + 2kb, 2])."""
        parts = allp[:, :, :k] if kb == 0 else torch.cat([allp[:, :, :k], allp[:, :, k + kb:]], dim=2)
        G, B = parts.shape[0], parts.shape[1]
        flat = parts.permute(1, 0, 2, 3).reshape(B, -1, 2)
        return _TorchPool(flat[..., 1].contiguous(), flat[..., 0].contiguous().view(torch.float32))

    def search_exchange(self, s: torch.Tensor, i: torch.Tensor, k: int):
        packed = torch.stack([s.contiguous().view(torch.int32), i.to(torch.int32)], dim=-1)  # [B, k, 2]
        allp = self._all_gather(packed)                                                    # [G, B, k, 2]
        S = allp[..., 0].contiguous().view(torch.float32)
        I = allp[..., 1].contiguous()
        return self.ops.merge(S, I, k)

    def rerank(self, Q: torch.Tensor, cand: torch.Tensor, k: int, pool=None):
        """Stage 3.  pool: from ``search_hybrid(..., return_pool=True)`` of the
        batch whose lists ``cand`` was fused from -- the candidates' scores are
        looked up in it (no collective; ``last_pool_misses`` counts
        candidates found in none of its lists, which score -inf: fused from
        other lists, pass no pool).  Without a pool: every rank scores its own
        candidates, one all-reduce(MAX)."""
        if self._nx is not None:
            return self._nx.rerank(Q, cand, k, pool=pool)
        if self.world == 1:
            return self.local.rerank(Q, cand, k)                                           # fused select
        if pool is not None:
            cand_d = cand.to(device=pool.ids.device, dtype=torch.int32)
            raw, self.last_pool_misses = pool_scores(cand_d, pool.ids, pool.scores)
            return self.ops.select(raw, k, ids=cand_d)
        raw = self.local.rerank(Q, cand, 0)                                                # [B, C]
        self._collective("all_reduce_max", lambda: dist.all_reduce(raw, op=dist.ReduceOp.MAX, group=self.group),
                         raw.device)
        return self.ops.select(raw, k, ids=cand)
