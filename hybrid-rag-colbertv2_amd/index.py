"""HBM-resident ColBERT index shard and its device calls.

Replaces the reference's ``self.corpus_embeddings`` tensor
(local_rag_complete.py:725, 735-739, 751-752), which holds whatever
``SentenceTransformer.encode`` returned, fp32, on "mps"/"cpu".  Here a shard
is a contiguous id range ``[id_base, id_base + n)`` of the corpus laid out for
the MI355X scan kernel:

    tokens   bf16 [n, ld, 128]   (ld = 128 token slots: 32 KiB per doc; long
                                  documents: ld = 256 / 512 / 1024;
                                  rows >= doclen are padding)
    doclens  int32 [n]
    means    f32  [n, 128]       (optional: literal-reference scorer only)
    residual bf16 [n, ld, 128]   (optional: fp32-faithful index, lo = bf16(x - tokens))

All compute goes through libcolbert_mi355x.so (``_lib``); the tensors are
owned here and borrowed by the C handle.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Iterable, List, Optional, Sequence, Tuple, Union

import torch

from . import _lib

LD = 128
LONG_LDS = (128, 256, 512, 1024)   # token slots per doc an index can hold (long documents)
DIM = 128
LQ_MAX = 32
BAND_CAP = 16384   # fp32-faithful search: largest band rescored per query


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream_ptr(device: torch.device) -> int:
    """The device's current stream as a raw hipStream_t (torch's C accessor:
    no Stream object per call -- the latency path pays for every microsecond)."""
    if _raw_stream is not None:
        return _raw_stream(device.index if device.index is not None else torch.cuda.current_device())
    return torch.cuda.current_stream(device).cuda_stream


_HBM_MIN_BYTES = 64 << 20   # buffers below this stay in torch's caching allocator


class _HbmBlock:
    """Device memory from ``cbv2_hbm_alloc`` -- physically contiguous when the
    driver can provide it (the streaming scans' translation is then one
    contiguous range: the B=1 scan over 1M docs ran 4.63-4.67 ms vs 4.75-4.99
    from plain hipMalloc, tools/probes/alloc_probe.cpp) -- exposed to torch
    through ``__cuda_array_interface__`` (torch keeps a reference for as long
    as a tensor views it) and freed by ``cbv2_hbm_free`` with the last one."""

    def __init__(self, device: torch.device, nbytes: int):
        self.device = device.index if device.index is not None else torch.cuda.current_device()
        h, c = ctypes.c_void_p(), ctypes.c_int32(0)
        _lib.check(_lib.lib().cbv2_hbm_alloc(self.device, int(nbytes), ctypes.byref(h), ctypes.byref(c)))
        self.ptr, self.nbytes, self.contiguous = int(h.value or 0), int(nbytes), bool(c.value)
        self.__cuda_array_interface__ = {"shape": (int(nbytes),), "typestr": "|u1", "data": (self.ptr, False),
                                         "version": 3, "strides": None, "stream": None}

    def __del__(self):
        try:
            if self.ptr:
                _HBM_BLOCKS.pop(self.ptr, None)
                _lib.lib().cbv2_hbm_free(self.device, ctypes.c_void_p(self.ptr))
                self.ptr = 0
        except Exception:
            pass


def hbm_empty(shape, dtype: torch.dtype, device) -> torch.Tensor:
    """An uninitialised device tensor for an index array: at least
    ``_HBM_MIN_BYTES`` -> ``cbv2_hbm_alloc`` (physically contiguous HBM when
    available), smaller -> torch's allocator.  ``hbm_placement(t)`` tells which."""
    device = torch.device(device)
    shape = tuple(int(x) for x in shape)
    numel = 1
    for x in shape:
        numel *= x
    nbytes = numel * torch.empty((), dtype=dtype).element_size()
    if device.type != "cuda" or nbytes < _HBM_MIN_BYTES:
        return torch.empty(shape, dtype=dtype, device=device)
    blk = _HbmBlock(device, nbytes)
    raw = torch.as_tensor(blk, device=device)
    if raw.data_ptr() != blk.ptr or raw.numel() != nbytes:
        raise RuntimeError("torch.as_tensor did not alias the HBM block")
    t = raw.view(dtype).view(shape)
    _HBM_BLOCKS[t.data_ptr()] = blk.contiguous
    return t


_HBM_BLOCKS: dict = {}


def hbm_zeros(shape, dtype: torch.dtype, device) -> torch.Tensor:
    return hbm_empty(shape, dtype, device).zero_()


def hbm_placement(t: torch.Tensor) -> str:
    """"contiguous" / "hipMalloc" for a tensor from ``hbm_empty`` (its first
    byte), "torch" otherwise."""
    c = _HBM_BLOCKS.get(t.data_ptr())
    return "torch" if c is None else ("contiguous" if c else "hipMalloc")


def _require_cuda(t: torch.Tensor, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a ROCm device tensor (got {t.device})")


def long_ld(max_len: int) -> int:
    """Token slots for docs of up to ``max_len`` tokens: the smallest of LONG_LDS."""
    for ld in LONG_LDS:
        if max_len <= ld:
            return ld
    raise ValueError(f"documents of up to {LONG_LDS[-1]} tokens are supported (got {max_len})")


def pack_tokens(embs: Union[torch.Tensor, Sequence[torch.Tensor]], device,
                ld: int = LD, dtype: torch.dtype = torch.bfloat16) -> Tuple[torch.Tensor, torch.Tensor]:
    """Token matrices -> (``dtype`` [n, ld, 128] padded with zeros, int32 doclens [n]).

    Accepts a dense ``[n, L, D]`` tensor (every doc has L tokens, as the
    reference's stacked encode output), a pooled ``[n, D]`` tensor (one token
    per doc: the shape ``encode`` returns by default), or a list of ``[L_i, D]``.
    ``ld=None``: the smallest supported slot count that holds the longest doc
    (128, or 256 / 512 / 1024 for long documents).
    """
    if ld is None:
        if isinstance(embs, torch.Tensor):
            L = 1 if embs.dim() == 2 else int(embs.shape[1])
        else:
            embs = list(embs)
            L = max([1] + [1 if e.dim() == 1 else int(e.shape[0]) for e in embs])
        ld = long_ld(L)
    if isinstance(embs, torch.Tensor):
        if embs.dim() == 2:
            embs = embs.unsqueeze(1)
        if embs.dim() != 3:
            raise ValueError(f"expected [n, L, {DIM}] or [n, {DIM}] embeddings, got {tuple(embs.shape)}")
        n, L, D = embs.shape
        if D != DIM or L > ld:
            raise ValueError(f"doc embeddings must be [n, L<={ld}, {DIM}] (got {tuple(embs.shape)})")
        tokens = hbm_zeros((n, ld, DIM), dtype, device)
        tokens[:, :L] = embs.to(device=device, dtype=dtype)
        doclens = torch.full((n,), L, dtype=torch.int32, device=device)
        return tokens, doclens
    embs = list(embs)
    n = len(embs)
    tokens = hbm_zeros((n, ld, DIM), dtype, device)
    lens = []
    for i, e in enumerate(embs):
        e = e if e.dim() == 2 else e.unsqueeze(0)
        if e.shape[-1] != DIM or e.shape[0] > ld:
            raise ValueError(f"doc {i}: expected [L<={ld}, {DIM}] tokens, got {tuple(e.shape)}")
        tokens[i, : e.shape[0]] = e.to(device=device, dtype=dtype)
        lens.append(e.shape[0])
    doclens = torch.tensor(lens, dtype=torch.int32, device=device)
    return tokens, doclens


def quantize_mxfp8(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """[..., 128] bf16/f32 device tensor -> (e4m3 bytes uint8 [..., 128], E8M0 scales uint8 [..., 2])."""
    _require_cuda(x, "x")
    if x.shape[-1] != DIM:
        raise ValueError(f"last dim must be {DIM}")
    dt = {torch.bfloat16: _lib.DTYPE_BF16, torch.float32: _lib.DTYPE_F32}.get(x.dtype)
    if dt is None:
        x, dt = x.float(), _lib.DTYPE_F32
    x = x.contiguous()
    rows = x.numel() // DIM
    buf = hbm_empty((rows * (DIM + 2),), torch.uint8, x.device)
    q, sc = buf[: rows * DIM], buf[rows * DIM:]
    _lib.check(_lib.lib().cbv2_quantize_mxfp8(x.data_ptr(), dt, rows, q.data_ptr(), sc.data_ptr(),
                                              _stream_ptr(x.device)))
    return q.view(*x.shape[:-1], DIM), sc.view(*x.shape[:-1], 2)


class ColbertIndex:
    """One shard of the corpus resident in HBM, with a C handle borrowing it.

    bf16 tokens (default; [n, ld, 128] with ld = 128, or 256 / 512 / 1024 for
    long documents), or MXFP8 (``tokens`` uint8 e4m3 [n, ld, 128] plus
    ``scales`` uint8 E8M0 [n, ld, 2]; see ``ColbertIndex.mxfp8``)."""

    def __init__(self, tokens: torch.Tensor, doclens: torch.Tensor, id_base: int = 0,
                 scales: Optional[torch.Tensor] = None, residual: Optional[torch.Tensor] = None,
                 bounds: Optional[Tuple[float, float]] = None):
        _require_cuda(tokens, "tokens")
        _require_cuda(doclens, "doclens")
        self.fp8 = tokens.dtype == torch.uint8
        want = torch.uint8 if self.fp8 else torch.bfloat16
        if tokens.dtype != want or tokens.dim() != 3 or tokens.shape[2] != DIM or tokens.shape[1] not in LONG_LDS:
            raise ValueError(f"tokens must be bf16 or MXFP8 uint8 [n, ld, {DIM}] (ld in {LONG_LDS}) "
                             f"(got {tokens.dtype} {tuple(tokens.shape)})")
        self.ld = int(tokens.shape[1])
        if doclens.dtype != torch.int32 or doclens.shape != (tokens.shape[0],):
            raise ValueError("doclens must be int32 [n]")
        if self.fp8 and (scales is None or scales.dtype != torch.uint8
                         or tuple(scales.shape) != (tokens.shape[0], tokens.shape[1], 2)):
            raise ValueError("an MXFP8 index needs uint8 scales [n, ld, 2]")
        self.tokens = tokens.contiguous()
        self.scales = scales.contiguous() if self.fp8 else None
        self.doclens = doclens.contiguous()
        self.device = tokens.device
        self.n = int(tokens.shape[0])
        self.id_base = int(id_base)
        self.means: Optional[torch.Tensor] = None
        self._ws: Optional[torch.Tensor] = None
        self._rr_ws: Optional[torch.Tensor] = None      # cbv2_rerank_ws workspace (small batches)
        h = ctypes.c_void_p()
        dev = self.device.index if self.device.index is not None else torch.cuda.current_device()
        if self.fp8:
            _lib.check(_lib.lib().cbv2_index_create_mxfp8(
                dev, self.tokens.data_ptr(), self.scales.data_ptr(), self.n, self.ld, DIM, self.doclens.data_ptr(),
                self.id_base, ctypes.byref(h)))
        else:
            _lib.check(_lib.lib().cbv2_index_create(
                dev, self.tokens.data_ptr(), _lib.DTYPE_BF16, self.n, self.ld, DIM, self.doclens.data_ptr(),
                self.id_base, ctypes.byref(h)))
        self._h = h
        # docs filling >= 98 % of their 16-token tiles: B <= 2 streams every
        # slot (CBV2_OPT_DENSE_DOCS); one small reduction at build time
        self.dense_docs = False
        if self.ld == 128 and self.n > 0:
            tiles = int(((self.doclens.clamp(0, self.ld) + 15) // 16).sum().item())
            self.dense_docs = tiles >= 0.98 * self.n * (self.ld // 16)
            if self.dense_docs:
                self.set_option(_lib.OPT_DENSE_DOCS, 1)
        self.residual: Optional[torch.Tensor] = None
        self.bounds: Optional[Tuple[float, float]] = None
        if residual is not None:
            if self.fp8 or residual.dtype != torch.bfloat16 or residual.shape != self.tokens.shape \
                    or residual.device != self.device or bounds is None:
                raise ValueError("a residual is bf16 [n, ld, 128] like the tokens, on the index device, "
                                 "with (resid_max, norm_max)")
            self.residual = residual.contiguous()
            self.bounds = (float(bounds[0]), float(bounds[1]))
            _lib.check(_lib.lib().cbv2_index_attach_residual(self._h, self.residual.data_ptr(), self.bounds[0],
                                                             self.bounds[1]))

    @property
    def faithful(self) -> bool:
        """fp32-faithful index (built by ``ColbertIndex.faithful_f32``)."""
        return self.residual is not None

    @classmethod
    def faithful_f32(cls, tokens_f32: torch.Tensor, doclens: torch.Tensor, id_base: int = 0) -> "ColbertIndex":
        """Index fp32 [n, ld, 128] device tokens (as the reference stores them; ld =
        128, or 256 / 512 / 1024 for long documents) so that scores match fp32
        arithmetic within ~1e-5: hi = bf16(x) is scanned, lo = bf16(x - hi) is
        gathered for the candidates (cbv2_split_f32, HIP)."""
        _require_cuda(tokens_f32, "tokens_f32")
        if tokens_f32.dtype != torch.float32 or tokens_f32.dim() != 3 or tokens_f32.shape[2] != DIM \
                or tokens_f32.shape[1] not in LONG_LDS:
            raise ValueError(f"tokens_f32 must be f32 [n, ld, {DIM}], ld in {LONG_LDS} (got {tokens_f32.dtype} "
                             f"{tuple(tokens_f32.shape)})")
        x = tokens_f32.contiguous()
        hi = hbm_empty(x.shape, torch.bfloat16, x.device)     # the array every scan streams
        lo = hbm_empty(x.shape, torch.bfloat16, x.device)
        bounds = torch.zeros(2, dtype=torch.float32, device=x.device)
        _require_cuda(doclens, "doclens")
        if doclens.dtype != torch.int32 or doclens.shape != (x.shape[0],):
            raise ValueError("doclens must be int32 [n]")
        doclens = doclens.contiguous()
        _lib.check(_lib.lib().cbv2_split_f32(x.data_ptr(), x.numel() // DIM, x.shape[1], doclens.data_ptr(),
                                             hi.data_ptr(), lo.data_ptr(), bounds.data_ptr(), _stream_ptr(x.device)))
        b = bounds.tolist()  # synchronises: x may be freed after this
        return cls(hi, doclens, id_base=id_base, residual=lo, bounds=(b[0], b[1]))

    def _f32_ws(self, op: int, B: int, lq: int, cap: int) -> torch.Tensor:
        need = int(_lib.lib().cbv2_f32_workspace_bytes(self._h, op, B, lq, cap))
        if self._ws is None or self._ws.numel() * 4 < need:
            self._ws = torch.empty(((need + 3) // 4,), dtype=torch.float32, device=self.device)
        return self._ws

    @classmethod
    def mxfp8(cls, tokens: torch.Tensor, doclens: torch.Tensor, id_base: int = 0) -> "ColbertIndex":
        """Quantize bf16/f32 [n, ld, 128] device tokens to MXFP8 (HIP kernel) and index them."""
        q, sc = quantize_mxfp8(tokens)
        return cls(q, doclens, id_base=id_base, scales=sc)

    @classmethod
    def from_embeddings(cls, embs, device="cuda", id_base: int = 0, build_means: bool = False,
                        dtype: str = "bf16"):
        """Index encoder output.  dtype: "bf16" (default), "fp8" (MXFP8, HIP
        quantizer) or "fp32" (fp32-faithful: scores as fp32 arithmetic gives them)."""
        device = torch.device(device)
        if dtype not in ("bf16", "fp8", "fp32"):
            raise ValueError(f"index dtype must be bf16, fp8 or fp32 (got {dtype!r})")
        # long documents: the smallest ld of 256 / 512 / 1024 that holds the longest doc
        tokens, doclens = pack_tokens(embs, device, ld=None,
                                      dtype=torch.float32 if dtype == "fp32" else torch.bfloat16)
        if dtype == "fp32":
            ix = cls.faithful_f32(tokens, doclens, id_base=id_base)
        elif dtype == "fp8":
            ix = cls.mxfp8(tokens, doclens, id_base=id_base)
        else:
            ix = cls(tokens, doclens, id_base=id_base)
        del tokens
        if build_means:
            if isinstance(embs, torch.Tensor):
                f32 = embs if embs.dim() == 3 else embs.unsqueeze(1)
                f32 = f32.to(device=device, dtype=torch.float32).contiguous()
            else:
                f32 = torch.zeros((ix.n, ix.ld, DIM), dtype=torch.float32, device=device)
                for i, e in enumerate(embs):
                    e = e if e.dim() == 2 else e.unsqueeze(0)
                    f32[i, : e.shape[0]] = e.to(device=device, dtype=torch.float32)
            ix.build_means(f32)
        return ix

    # ----------------------------------------------------------------- native file
    def save(self, path: str) -> None:
        """Write this shard to the native index file (include/colbert_mi355x.h).

        An fp32-faithful index is two bf16 files of the same layout -- ``path``
        (hi, the tokens every scan reads) and ``path + ".resid"`` (lo) -- plus
        ``path + ".bounds.json"`` (the split's bounds), so a rank loads its doc
        range of both exactly as for a bf16 index.  Long-document indexes keep
        their ld (the file header records it)."""
        dt = _lib.DTYPE_MXFP8 if self.fp8 else _lib.DTYPE_BF16
        torch.cuda.current_stream(self.device).synchronize()
        for side in (path + ".bounds.json", path + ".resid"):   # sidecars of an earlier save at this path
            if os.path.exists(side):
                os.unlink(side)
        _lib.check(_lib.lib().cbv2_index_file_write_ld(
            os.fsencode(path), dt, self.n, self.ld, self.tokens.data_ptr(),
            self.scales.data_ptr() if self.fp8 else None, self.doclens.data_ptr(), self.id_base,
            _stream_ptr(self.device)))
        if self.faithful:
            _lib.check(_lib.lib().cbv2_index_file_write_ld(
                os.fsencode(path + ".resid"), _lib.DTYPE_BF16, self.n, self.ld, self.residual.data_ptr(), None,
                self.doclens.data_ptr(), self.id_base, _stream_ptr(self.device)))
            # written last: the bounds name the exact hi / residual files they belong to
            with open(path + ".bounds.json", "w") as f:
                json.dump({"resid_max": self.bounds[0], "norm_max": self.bounds[1],
                           "hi": file_fingerprint(path), "resid": file_fingerprint(path + ".resid")}, f)

    @classmethod
    def load(cls, path: str, device="cuda", begin: int = 0, end: Optional[int] = None) -> "ColbertIndex":
        """Load docs [begin, end) of a native index file straight into HBM
        (a rank's shard); global ids start at the file's id_base + begin."""
        device = torch.device(device)
        dt, n, id_base, ld = index_file_layout(path)
        end = n if end is None else int(end)
        begin = int(begin)
        m = end - begin
        if begin < 0 or m < 0 or end > n:
            raise ValueError(f"doc range [{begin}, {end}) outside [0, {n})")
        fp8 = dt == _lib.DTYPE_MXFP8
        tokens = hbm_empty((m, ld, DIM), torch.uint8 if fp8 else torch.bfloat16, device)
        scales = hbm_empty((m, ld, 2), torch.uint8, device) if fp8 else None
        doclens = torch.empty((m,), dtype=torch.int32, device=device)
        with torch.cuda.device(device):
            _lib.check(_lib.lib().cbv2_index_file_read(
                os.fsencode(path), begin, end, tokens.data_ptr() if m else None,
                scales.data_ptr() if (fp8 and m) else None, doclens.data_ptr() if m else None,
                _stream_ptr(device)))
        if not fp8 and os.path.exists(path + ".resid") and os.path.exists(path + ".bounds.json"):
            # fp32-faithful: the residual file's same doc range, and the split's bounds
            with open(path + ".bounds.json") as f:
                b = json.load(f)
            if index_file_layout(path + ".resid")[1:] != (n, id_base, ld) or \
                    b.get("hi") != file_fingerprint(path) or b.get("resid") != file_fingerprint(path + ".resid"):
                raise ValueError(f"{path}.resid / .bounds.json were not written with {path}")
            resid = hbm_empty((m, ld, DIM), torch.bfloat16, device)
            dl2 = torch.empty((m,), dtype=torch.int32, device=device)
            with torch.cuda.device(device):
                _lib.check(_lib.lib().cbv2_index_file_read(
                    os.fsencode(path + ".resid"), begin, end, resid.data_ptr() if m else None, None,
                    dl2.data_ptr() if m else None, _stream_ptr(device)))
            if not torch.equal(dl2, doclens):
                raise ValueError(f"{path}.resid does not match {path}")
            return cls(tokens, doclens, id_base=id_base + begin, residual=resid,
                       bounds=(float(b["resid_max"]), float(b["norm_max"])))
        return cls(tokens, doclens, id_base=id_base + begin, scales=scales)

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.lib().cbv2_index_destroy(self._h)
            self._h = ctypes.c_void_p()

    # ------------------------------------------------------------ options / measurement
    def set_option(self, option: int, value: int) -> None:
        """cbv2_index_set_option: _lib.OPT_FUSED_TOPK / OPT_DYNAMIC_TAIL / OPT_BAND_DOC_MAJOR (A/B and tests)."""
        _lib.check(_lib.lib().cbv2_index_set_option(self._h, int(option), int(value)))

    def fused_topk_slots(self, B: int, k: int, scorer: str = "maxsim") -> int:
        """Per-query workgroup lists a search of (B, k) keeps when the top-k is fused
        into the scan (0: the unfused path; cbv2_search_fused_slots)."""
        return int(_lib.lib().cbv2_search_fused_slots(self._h, int(B), int(k), self._scorer(scorer)))

    def last_scan_plan(self) -> dict:
        """Work split of this handle's latest scan launch (cbv2_index_last_scan_plan)."""
        buf = (ctypes.c_int64 * 4)()
        _lib.check(_lib.lib().cbv2_index_last_scan_plan(self._h, buf))
        return {"workgroups": int(buf[0]), "chunk_docs": int(buf[1]), "static_docs": int(buf[2]),
                "dynamic_tail": bool(buf[3])}

    def time_scans(self, enable: bool, clock: bool = False) -> None:
        """Bracket every following MaxSim scan launch of this index with HIP
        events on its own stream (cbv2_index_time_scans); enable clears the
        previous record.  clock: also the doc-interleaved scans' clock probe
        (``scan_clock``)."""
        _lib.check(_lib.lib().cbv2_index_time_scans(self._h, (2 if clock else 1) if enable else 0))

    def scan_clock(self, reset: bool = False):
        """The clock probe's sums since ``time_scans(True, clock=True)`` or the
        last reset (cbv2_index_scan_clock; synchronizes the device): dict with
        the held clock in GHz (run-time weighted over the probed scans'
        workgroups; None when no probed scan ran) and the raw sums."""
        out = (ctypes.c_int64 * 4)()
        _lib.check(_lib.lib().cbv2_index_scan_clock(self._h, out, 1 if reset else 0))
        cyc, ticks, started, ended = (int(x) for x in out)
        ghz = cyc / ticks * 0.1 if ticks > 0 and started == ended and started > 0 else None
        return {"clock_ghz": ghz, "cycles": cyc, "ticks": ticks, "workgroups": ended,
                "complete": started == ended}

    def scan_times(self, max_launches: int = 4096) -> List[float]:
        """Durations (ms) of the scans recorded since ``time_scans(True)``;
        disables timing first, then clears the record.  Waits for the recorded
        launches to finish."""
        self.time_scans(False)
        ms = (ctypes.c_float * max_launches)()
        cnt = ctypes.c_int32(0)
        _lib.check(_lib.lib().cbv2_index_scan_times(self._h, ms, int(max_launches), ctypes.byref(cnt)))
        return [float(ms[i]) for i in range(min(cnt.value, max_launches))]

    def band_times(self, max_searches: int = 4096) -> List[float]:
        """Durations (ms) of the fp32-faithful searches' band work recorded since
        ``time_scans(True)`` (from the end of the bf16 top-k to the end of the
        band select; cbv2_index_band_times); disables timing first, then clears
        the record.  Read after ``scan_times`` or before it: both disable."""
        self.time_scans(False)
        ms = (ctypes.c_float * max_searches)()
        cnt = ctypes.c_int32(0)
        _lib.check(_lib.lib().cbv2_index_band_times(self._h, ms, int(max_searches), ctypes.byref(cnt)))
        return [float(ms[i]) for i in range(min(cnt.value, max_searches))]

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __len__(self):
        return self.n

    # ----------------------------------------------------------------- build
    def build_means(self, tokens_f32: torch.Tensor):
        """Per-doc normalised token means for the literal reference scorer."""
        _require_cuda(tokens_f32, "tokens_f32")
        if tokens_f32.dtype != torch.float32 or tokens_f32.dim() != 3 or tokens_f32.shape[0] != self.n \
                or tokens_f32.shape[2] != DIM:
            raise ValueError(f"tokens_f32 must be f32 [n, L, {DIM}]")
        tokens_f32 = tokens_f32.contiguous()
        means = torch.empty((self.n, DIM), dtype=torch.float32, device=self.device)
        _lib.check(_lib.lib().cbv2_index_build_means(self._h, tokens_f32.data_ptr(), tokens_f32.shape[1],
                                                     means.data_ptr(), _stream_ptr(self.device)))
        self.means = means
        self._means_src = tokens_f32  # kept alive until the kernel has run
        torch.cuda.current_stream(self.device).synchronize()
        self._means_src = None

    # ----------------------------------------------------------------- query prep
    def _prep_query(self, Q: torch.Tensor, scorer: str):
        """-> (buffer kept alive, pointer, ABI dtype, B, lq) in the layout the scorer takes."""
        if Q.dim() == 2:
            Q = Q.unsqueeze(0)
        if Q.dim() != 3 or Q.shape[2] != DIM:
            raise ValueError(f"queries must be [B, lq, {DIM}] (got {tuple(Q.shape)})")
        B, lq = int(Q.shape[0]), int(Q.shape[1])
        Q = Q.to(self.device)
        if scorer == "maxsim" and self.faithful:
            if lq > LQ_MAX:
                raise ValueError(f"maxsim takes at most {LQ_MAX} query tokens (got {lq})")
            Qd = Q.to(torch.float32).contiguous()
            return Qd, Qd.data_ptr(), _lib.DTYPE_F32, B, lq
        if scorer == "maxsim" and self.fp8:
            if lq > LQ_MAX:
                raise ValueError(f"maxsim takes at most {LQ_MAX} query tokens (got {lq})")
            q, _ = quantize_mxfp8(Q)                   # one buffer: B*lq*128 bytes, then B*lq*2 scales
            return q, q.data_ptr(), _lib.DTYPE_MXFP8, B, lq
        if scorer == "maxsim":
            Qd = Q.to(torch.bfloat16).contiguous()
            return Qd, Qd.data_ptr(), _lib.DTYPE_BF16, B, lq
        Qd = Q.to(torch.float32).contiguous()
        return Qd, Qd.data_ptr(), _lib.DTYPE_F32, B, lq

    def _scorer(self, scorer: str) -> int:
        try:
            return _lib.SCORERS[scorer]
        except KeyError:
            raise ValueError(f"unknown scorer {scorer!r}; expected one of {sorted(_lib.SCORERS)}") from None

    # ----------------------------------------------------------------- long queries
    @staticmethod
    def _query_blocks(Q: torch.Tensor, scorer: str):
        """MaxSim queries of more than 32 tokens -> blocks of <= 32 tokens (None
        otherwise).  MaxSim is a sum over query tokens (LRC:807-812), so the
        score of a long query is the sum of its blocks' scores, each block one
        pass of the kernels (which hold 32 query tokens per MFMA column pair)."""
        if scorer != "maxsim":
            return None
        if Q.dim() == 2:
            Q = Q.unsqueeze(0)
        if Q.dim() != 3 or Q.shape[1] <= LQ_MAX:
            return None
        return [Q[:, a:a + LQ_MAX].contiguous() for a in range(0, Q.shape[1], LQ_MAX)]

    # ----------------------------------------------------------------- compute
    def score(self, Q: torch.Tensor, scorer: str = "maxsim") -> torch.Tensor:
        """f32 [B, n] scores of every doc of the shard (the reference's _maxsim_score)."""
        blocks = self._query_blocks(Q, scorer)
        if blocks is not None:     # long queries: the blocks' scores summed in block order
            out = self.score(blocks[0], scorer).clone()
            for q in blocks[1:]:
                out += self.score(q, scorer)
            return out
        sid = self._scorer(scorer)
        _keep, qptr, qdt, B, lq = self._prep_query(Q, scorer)
        out = torch.empty((B, max(self.n, 1)), dtype=torch.float32, device=self.device)
        if self.faithful and scorer == "maxsim":
            ws = self._f32_ws(_lib.F32_SCORE, B, lq, 0)
            _lib.check(_lib.lib().cbv2_score_f32(self._h, qptr, B, lq, ws.data_ptr(), ws.numel() * 4,
                                                 out.data_ptr(), out.shape[1], _stream_ptr(self.device)))
            return out[:, : self.n]
        _lib.check(_lib.lib().cbv2_score(self._h, sid, qptr, qdt, B, lq, out.data_ptr(),
                                         out.shape[1], _stream_ptr(self.device)))
        return out[:, : self.n]

    def search(self, Q: torch.Tensor, k: int, scorer: str = "maxsim",
               lb_reduce=None) -> Tuple[torch.Tensor, torch.Tensor]:
        """Top-k over the shard: (f32 [B, k] scores, int32 [B, k] global ids), -inf/-1 padded.

        ``lb_reduce`` (fp32-faithful index, sharded corpus): called with the
        exact faithful scores of this shard's bf16 top-k (device f32 [B, k]);
        returns a per-row lower bound of the GLOBAL k-th faithful score (device
        f32 [B]: the k-th largest of every shard's lists).  The shard then
        rescores only the docs that can reach the global top-k and returns its
        part of it, which the merge completes (cbv2_search_f32_begin /
        _finish)."""
        if self._query_blocks(Q, scorer) is not None:   # long queries: summed block scores + radix top-k
            return topk_rows(self.score(Q, scorer), int(k), id_base=self.id_base)
        sid = self._scorer(scorer)
        _keep, qptr, qdt, B, lq = self._prep_query(Q, scorer)
        if self.faithful and scorer == "maxsim":
            if lb_reduce is not None:
                return self._search_f32_global(_keep, B, lq, k, lb_reduce)
            return self._search_f32(_keep, B, lq, k)
        L = _lib.lib()
        need = int(L.cbv2_search_workspace_size(self._h, B, int(k), sid))
        if self._ws is None or self._ws.numel() * 4 < need:
            self._ws = torch.empty(((need + 3) // 4,), dtype=torch.float32, device=self.device)
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.device)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.device)
        _lib.check(L.cbv2_search(self._h, sid, qptr, qdt, B, lq, int(k), self._ws.data_ptr(),
                                 self._ws.numel() * 4, out_s.data_ptr(), out_i.data_ptr(),
                                 _stream_ptr(self.device)))
        return out_s, out_i

    def _search_f32(self, Qd: torch.Tensor, B: int, lq: int, k: int, cap: int = BAND_CAP):
        """Faithful search (cbv2_search_f32, asynchronous): rows whose band
        overflowed ``cap`` (``last_band`` -1) are recomputed on the device by
        the full faithful scan; ``last_band`` holds each row's band size."""
        cap = max(int(cap), int(k))
        ws = self._f32_ws(_lib.F32_SEARCH, B, lq, cap)
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.device)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.device)
        status = torch.empty((B,), dtype=torch.int32, device=self.device)
        _lib.check(_lib.lib().cbv2_search_f32(self._h, Qd.data_ptr(), B, lq, int(k), cap, ws.data_ptr(),
                                              ws.numel() * 4, out_s.data_ptr(), out_i.data_ptr(),
                                              status.data_ptr(), _stream_ptr(self.device)))
        self.last_band = status
        return out_s, out_i

    def _search_f32_global(self, Qd: torch.Tensor, B: int, lq: int, k: int, lb_reduce, cap: int = BAND_CAP):
        """Faithful search of one shard against the global k-th bound (see
        ``search``): begin -> lb = lb_reduce(fk) -> finish, asynchronous."""
        cap = max(int(cap), int(k))
        ws = self._f32_ws(_lib.F32_SEARCH, B, lq, cap)
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.device)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.device)
        status = torch.empty((B,), dtype=torch.int32, device=self.device)
        fk = torch.empty((B, k), dtype=torch.float32, device=self.device)
        L = _lib.lib()
        _lib.check(L.cbv2_search_f32_begin(self._h, Qd.data_ptr(), B, lq, int(k), cap, ws.data_ptr(),
                                           ws.numel() * 4, fk.data_ptr(), out_s.data_ptr(), out_i.data_ptr(),
                                           status.data_ptr(), _stream_ptr(self.device)))
        lb = lb_reduce(fk).to(device=self.device, dtype=torch.float32).contiguous()
        if tuple(lb.shape) != (B,):
            raise ValueError(f"lb_reduce must return f32 [{B}] (got {tuple(lb.shape)})")
        _lib.check(L.cbv2_search_f32_finish(self._h, B, lq, int(k), cap, ws.data_ptr(), ws.numel() * 4,
                                            lb.data_ptr(), out_s.data_ptr(), out_i.data_ptr(), status.data_ptr(),
                                            _stream_ptr(self.device)))
        self.last_band = status
        return out_s, out_i

    def rerank(self, Q: torch.Tensor, cand: torch.Tensor, k: int):
        """Gather candidates by global id and MaxSim-rank them.

        k > 0: (scores [B, k], ids [B, k], positions [B, k]); k == 0: raw scores [B, C].
        """
        blocks = self._query_blocks(Q, "maxsim")
        if blocks is not None:     # long queries: the blocks' raw candidate scores summed, then selected
            raw = self.rerank(blocks[0], cand, 0).clone()
            for q in blocks[1:]:
                raw += self.rerank(q, cand, 0)
            if k == 0:
                return raw
            cand = cand.to(device=self.device, dtype=torch.int32)
            return select_topk(raw, int(k), ids=cand if cand.dim() == 2 else cand.unsqueeze(0))
        _keep, qptr, _, Bq, lq = self._prep_query(Q, "maxsim")
        cand = cand.to(device=self.device, dtype=torch.int32).contiguous()
        if cand.dim() == 1:
            cand = cand.unsqueeze(0)
        B, C = int(cand.shape[0]), int(cand.shape[1])
        if Bq != B:
            raise ValueError(f"{Bq} queries but {B} candidate rows")
        if self.faithful:
            ws = self._f32_ws(_lib.F32_RERANK, B, lq, C)
            out_s = torch.empty((B, C if k == 0 else k), dtype=torch.float32, device=self.device)
            out_i = torch.empty((B, k), dtype=torch.int32, device=self.device) if k else None
            out_p = torch.empty((B, k), dtype=torch.int32, device=self.device) if k else None
            _lib.check(_lib.lib().cbv2_rerank_f32(
                self._h, _keep.data_ptr(), B, lq, cand.data_ptr(), C, int(k), ws.data_ptr(), ws.numel() * 4,
                out_s.data_ptr(), out_i.data_ptr() if k else None, out_p.data_ptr() if k else None,
                _stream_ptr(self.device)))
            return out_s if k == 0 else (out_s, out_i, out_p)
        if k == 0:
            out_s = torch.empty((B, C), dtype=torch.float32, device=self.device)
            _lib.check(_lib.lib().cbv2_rerank(self._h, qptr, B, lq, cand.data_ptr(), C, 0,
                                              out_s.data_ptr(), None, None, _stream_ptr(self.device)))
            return out_s
        out_s = torch.empty((B, k), dtype=torch.float32, device=self.device)
        out_i = torch.empty((B, k), dtype=torch.int32, device=self.device)
        out_p = torch.empty((B, k), dtype=torch.int32, device=self.device)
        L = _lib.lib()
        need = int(L.cbv2_rerank_workspace_bytes(B, C))   # small batches: candidate-parallel scores
        if self._rr_ws is None or self._rr_ws.numel() < need:
            self._rr_ws = torch.empty((need,), dtype=torch.uint8, device=self.device)
        _lib.check(L.cbv2_rerank_ws(self._h, qptr, B, lq, cand.data_ptr(), C, int(k), self._rr_ws.data_ptr(),
                                    self._rr_ws.numel(), out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(),
                                    _stream_ptr(self.device)))
        return out_s, out_i, out_p


# --------------------------------------------------------------------- bounded-memory ingest
def _as_batch(embs, device, dtype, ld=LD):
    """Encoder output of one batch -> (tokens ``dtype`` [m, ld, 128], int32 doclens [m]) on ``device``
    (ld=None: the smallest of LONG_LDS that holds the batch's longest doc)."""
    return pack_tokens(embs, device, ld=ld, dtype=dtype)


class IndexBuilder:
    """Builds an HBM-resident index batch by batch, so ingest never holds the
    corpus's embeddings on the host (the reference encodes the whole corpus in
    one ``model.encode`` call and keeps it, fp32, LRC:735-739).  Each batch of
    encoder output is packed on the GPU and written into preallocated shard
    tensors: cast to bf16, quantised to MXFP8 by the HIP quantizer, or split
    into bf16 hi/lo by cbv2_split_f32 (fp32-faithful; the residual bounds
    accumulate over the batches).  ``finish()`` returns the ColbertIndex.

    Long documents: with ``ld=None`` the slot count starts at 128 and grows to
    256 / 512 / 1024 when a batch holds a longer doc (the docs so far are
    re-laid on the GPU); a fixed ``ld`` rejects longer docs."""

    def __init__(self, n: int, device="cuda", dtype: str = "bf16", id_base: int = 0, ld: Optional[int] = None):
        if dtype not in ("bf16", "fp8", "fp32"):
            raise ValueError(f"index dtype must be bf16, fp8 or fp32 (got {dtype!r})")
        if ld is not None and ld not in LONG_LDS:
            raise ValueError(f"ld must be one of {LONG_LDS} (got {ld})")
        self.n, self.dtype, self.id_base = int(n), dtype, int(id_base)
        self.grow = ld is None
        self.ld = LD if ld is None else int(ld)
        self.device = torch.device(device)
        self.pos = 0
        self.doclens = torch.zeros((self.n,), dtype=torch.int32, device=self.device)
        if dtype == "fp8":     # padding rows: e4m3 zeros, scale 2^0 (never scored)
            self.tokens = hbm_zeros((self.n, self.ld, DIM), torch.uint8, self.device)
            self.scales = hbm_empty((self.n, self.ld, 2), torch.uint8, self.device).fill_(127)
        else:
            self.tokens = hbm_zeros((self.n, self.ld, DIM), torch.bfloat16, self.device)
            self.scales = None
        if dtype == "fp32":
            self.residual = hbm_zeros((self.n, self.ld, DIM), torch.bfloat16, self.device)
            self.bounds = torch.zeros(2, dtype=torch.float32, device=self.device)

    def _relayout(self, ld: int) -> None:
        """Grow every doc to ld token slots (padding rows zero, never scored)."""
        def grown(x, fill=0):
            y = hbm_empty((self.n, ld, x.shape[2]), x.dtype, self.device).fill_(fill)
            y[: self.pos, : self.ld] = x[: self.pos]
            return y
        self.tokens = grown(self.tokens)
        if self.dtype == "fp32":
            self.residual = grown(self.residual)
        if self.dtype == "fp8":
            self.scales = grown(self.scales, 127)
        self.ld = ld

    def append(self, embs) -> int:
        """Add the next batch of encoder output (dense [m, L, D], pooled [m, D] or a list
        of [L_i, D]); returns the number of docs added."""
        t, dl = _as_batch(embs, self.device, torch.float32 if self.dtype == "fp32" else torch.bfloat16,
                          ld=None if self.grow else self.ld)
        m = int(t.shape[0])
        if self.pos + m > self.n:
            raise ValueError(f"batch of {m} docs past the declared {self.n} (have {self.pos})")
        if int(t.shape[1]) > self.ld:
            self._relayout(int(t.shape[1]))
        if int(t.shape[1]) < self.ld:     # a batch of shorter docs: pad to the index's slots
            t = torch.nn.functional.pad(t, (0, 0, 0, self.ld - int(t.shape[1])))
        a, b = self.pos, self.pos + m
        self.doclens[a:b] = dl
        if self.dtype == "fp8":
            q, sc = quantize_mxfp8(t)
            self.tokens[a:b] = q
            self.scales[a:b] = sc
        elif self.dtype == "fp32":
            t = t.contiguous()
            hi, lo = self.tokens[a:b], self.residual[a:b]
            _lib.check(_lib.lib().cbv2_split_f32(t.data_ptr(), m * self.ld, self.ld, self.doclens[a:b].data_ptr(),
                                                 hi.data_ptr(), lo.data_ptr(), self.bounds.data_ptr(),
                                                 _stream_ptr(self.device)))
        else:
            self.tokens[a:b] = t
        del t
        self.pos = b
        return m

    def finish(self) -> "ColbertIndex":
        if self.pos != self.n:
            raise ValueError(f"{self.pos} of {self.n} declared docs were appended")
        if self.dtype == "fp32":
            b = self.bounds.tolist()        # synchronises
            return ColbertIndex(self.tokens, self.doclens, id_base=self.id_base, residual=self.residual,
                                bounds=(b[0], b[1]))
        return ColbertIndex(self.tokens, self.doclens, id_base=self.id_base, scales=self.scales)


class IndexWriter:
    """Streams batches straight into the native index file (cbv2_index_writer_*)
    for corpora larger than HBM: each batch is cast (bf16) or quantised
    (MXFP8, HIP) on the GPU and written through two 64 MiB pinned buffers, so
    host memory does not grow with the corpus.  The file is valid only after
    ``close()`` with every declared doc written.  ``ld``: token slots per doc
    (fixed up front, as the file's layout depends on it; long documents 256 /
    512 / 1024)."""

    def __init__(self, path: str, n: int, dtype: str = "bf16", id_base: int = 0, device="cuda", ld: int = LD):
        if dtype not in ("bf16", "fp8"):
            raise ValueError("the native file holds bf16 or MXFP8 tokens")
        if ld not in LONG_LDS:
            raise ValueError(f"ld must be one of {LONG_LDS} (got {ld})")
        self.path, self.n, self.dtype, self.ld = path, int(n), dtype, int(ld)
        self.device = torch.device(device)
        h = ctypes.c_void_p()
        _lib.check(_lib.lib().cbv2_index_writer_open_ld(os.fsencode(path), _lib.DTYPE_MXFP8 if dtype == "fp8"
                                                        else _lib.DTYPE_BF16, self.n, self.ld, int(id_base),
                                                        ctypes.byref(h)))
        self._h = h

    @property
    def written(self) -> int:
        return int(_lib.lib().cbv2_index_writer_count(self._h))

    def append(self, embs) -> int:
        t, dl = _as_batch(embs, self.device, torch.bfloat16, ld=self.ld)
        m = int(t.shape[0])
        sc = None
        if self.dtype == "fp8":
            t, sc = quantize_mxfp8(t)
        t, dl = t.contiguous(), dl.contiguous()
        _lib.check(_lib.lib().cbv2_index_writer_append(self._h, m, t.data_ptr(), sc.data_ptr() if sc is not None
                                                       else None, dl.data_ptr(), 1, _stream_ptr(self.device)))
        return m

    def close(self) -> None:
        if self._h is not None and self._h.value:
            h, self._h = self._h, None
            _lib.check(_lib.lib().cbv2_index_writer_close(h))

    def __enter__(self):
        return self

    def __exit__(self, et, ev, tb):
        if et is None:
            self.close()
        else:                      # keep the original error; the file stays without a header
            try:
                self.close()
            except Exception:
                pass
        return False


# --------------------------------------------------------------------- free functions
def file_fingerprint(path: str, span: int = 4 << 20) -> str:
    """Identity of a native index file as written: its size and a CRC-32 of its
    first and last ``span`` bytes (the header, the doclens and the edge docs'
    tokens).  An fp32-faithful save records the hi and residual files'
    fingerprints in ``.bounds.json``, so a load never pairs a residual with
    another save's tokens."""
    import zlib
    size = os.path.getsize(path)
    with open(path, "rb") as f:
        crc = zlib.crc32(f.read(span))
        if size > span:
            f.seek(max(span, size - span))
            crc = zlib.crc32(f.read(span), crc)
    return f"{size}:{crc:08x}"


def index_file_info(path: str):
    """(ABI dtype, doc count, id_base) of a native index file."""
    dt, n, base = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib().cbv2_index_file_info(os.fsencode(path), ctypes.byref(dt), ctypes.byref(n),
                                               ctypes.byref(base)))
    return int(dt.value), int(n.value), int(base.value)


def index_file_layout(path: str):
    """(ABI dtype, doc count, id_base, token slots per doc) of a native index file."""
    dt, n, base, ld = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int32()
    _lib.check(_lib.lib().cbv2_index_file_info_ld(os.fsencode(path), ctypes.byref(dt), ctypes.byref(n),
                                                  ctypes.byref(base), ctypes.byref(ld)))
    return int(dt.value), int(n.value), int(base.value), int(ld.value)


def select_topk(scores: torch.Tensor, k: int, ids: Optional[torch.Tensor] = None):
    """Top-k of each row of a [B, C] score matrix (any C, any k); ties -> lower position."""
    _require_cuda(scores, "scores")
    scores = scores.to(torch.float32).contiguous()
    if scores.dim() == 1:
        scores = scores.unsqueeze(0)
    B, C = scores.shape
    dev = scores.device
    if ids is not None:
        ids = ids.to(device=dev, dtype=torch.int32).contiguous()
    out_s = torch.empty((B, k), dtype=torch.float32, device=dev)
    out_i = torch.empty((B, k), dtype=torch.int32, device=dev)
    out_p = torch.empty((B, k), dtype=torch.int32, device=dev)
    _lib.check(_lib.lib().cbv2_select_topk(scores.data_ptr(), ids.data_ptr() if ids is not None else None, B, C,
                                           int(k), out_s.data_ptr(), out_i.data_ptr(), out_p.data_ptr(),
                                           _stream_ptr(dev)))
    return out_s, out_i, out_p


def topk_rows(scores: torch.Tensor, k: int, id_base: int = 0, sampled: bool = True):
    """Top-k of each row of a [B, n] score matrix (exact; ties -> lower index).

    ``sampled`` lets long rows use the threshold-filter path (same result)."""
    _require_cuda(scores, "scores")
    if scores.dim() == 1:
        scores = scores.unsqueeze(0)
    scores = scores.to(torch.float32)
    if scores.stride(1) != 1:
        scores = scores.contiguous()
    B, n = scores.shape
    dev = scores.device
    out_s = torch.empty((B, k), dtype=torch.float32, device=dev)
    out_i = torch.empty((B, k), dtype=torch.int32, device=dev)
    need = int(_lib.lib().cbv2_topk_workspace_bytes(B, n)) if sampled else 0
    ws = torch.empty((max(need, 1),), dtype=torch.uint8, device=dev)
    _lib.check(_lib.lib().cbv2_topk_rows(scores.data_ptr(), B, n, scores.stride(0), int(k), int(id_base),
                                         ws.data_ptr() if need else None, need, out_s.data_ptr(),
                                         out_i.data_ptr(), _stream_ptr(dev)))
    return out_s, out_i


def merge_topk(scores: torch.Tensor, ids: torch.Tensor, k: int):
    """Merge [G, B, k] sorted per-shard lists into the global [B, k]."""
    _require_cuda(scores, "scores")
    scores = scores.to(torch.float32).contiguous()
    ids = ids.to(device=scores.device, dtype=torch.int32).contiguous()
    G, B, kk = scores.shape
    if kk != k:
        raise ValueError("per-shard lists must have length k")
    out_s = torch.empty((B, k), dtype=torch.float32, device=scores.device)
    out_i = torch.empty((B, k), dtype=torch.int32, device=scores.device)
    _lib.check(_lib.lib().cbv2_merge_topk(scores.data_ptr(), ids.data_ptr(), G, B, int(k), out_s.data_ptr(),
                                          out_i.data_ptr(), _stream_ptr(scores.device)))
    return out_s, out_i
