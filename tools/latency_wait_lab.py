"""Lab: the bench's B=1 latency loop (no sleep; call + torch.cuda.synchronize,
as bench.latency) on the one-trip path over a fp32-faithful shard, the
round-trip wait of cbv2_retrieve_finish interleaved in one process: poll
hipStreamQuery (mode 1, the default) vs record an event and poll it (mode 0,
round 4's), and the rerank launched after the fusion vs pre-armed (launched
before the wait, polling its tagged candidates).  Round 5's first run had a
third dimension, a poll after finish
(cbv2_stream_wait, removed: +8 to +18 us) -- profiles/r05/latency_wait_ab.jsonl.

  python3 tools/latency_wait_lab.py [docs]"""
import json, statistics, sys, time, ctypes, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from hybrid_rag_colbertv2_amd import _lib, synth, bm25 as bm25_mod
from hybrid_rag_colbertv2_amd.hybrid import OneTripRetriever
from hybrid_rag_colbertv2_amd.index import ColbertIndex
L = _lib.lib()
L.cbv2_set_wait_mode.argtypes = [ctypes.c_int32]
L.cbv2_set_prearm.argtypes = [ctypes.c_int32]
dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
Qf = synth.make_queries(256, 32, seed=1)
planted = synth.planted_ids(256, n, 10, seed=2)
terms, off, V = synth.bm25_shard(0, n, planted)
lex = bm25_mod.sharded(terms, off, V, id_base=0, device=dev)
qt, qo = synth.bm25_queries(256)
bm_one = lambda: lex.search(qt[:qo[1]], qo[:2], 100)
tokens, doclens = synth.make_shard(0, n, Qf, planted, dev, seed=0, dtype=torch.float32)
ix = ColbertIndex.faithful_f32(tokens, doclens)
del tokens
one = OneTripRetriever(ix)
Q1 = Qf[:1].to(dev).contiguous()
variants = [(1, 0), (1, 1), (0, 1)]   # (wait mode, pre-armed rerank)
lat = {v: [] for v in variants}
for it in range(40):
    for (m, s) in variants:
        L.cbv2_set_wait_mode(m)
        L.cbv2_set_prearm(s)
        for _ in range(5):
            torch.cuda.synchronize()
            t = time.perf_counter()
            one(Q1, bm_one)
            torch.cuda.synchronize()
            if it >= 2:
                lat[(m, s)].append((time.perf_counter() - t) * 1e6)
for (m, s), v in lat.items():
    print(json.dumps({"docs": n, "wait_mode": ["event poll", "stream query"][m], "prearm": bool(s),
                      "p50_us": round(statistics.median(v), 1), "p10_us": round(sorted(v)[len(v) // 10], 1)}))
