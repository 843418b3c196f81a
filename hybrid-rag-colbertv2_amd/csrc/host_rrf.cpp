// host_rrf.cpp — HybridRetriever._reciprocal_rank_fusion (local_rag_complete.py:960-978)
// for a batch of queries, host-side as the north star requires (HOST pointers,
// no GPU), plus the `[:50]` cut of :916.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);  // colbert_mi355x.hip

extern "C" {

// Host-side reciprocal rank fusion (HOST pointers).  Restates
// HybridRetriever._reciprocal_rank_fusion (local_rag_complete.py:960-978):
// score[id] += 1.0 / (rrf_k + rank) over the BM25 list, then the ColBERT list
// (rank 1-based, float64, same operation order as the Python), then a STABLE
// sort by score descending, so ties keep first-insertion order.  ids < 0 are
// padding and skipped.  Writes the first C fused ids/scores per query (-1 / 0
// padded); out_count (nullable) receives the number of distinct ids.
int cbv2_rrf_fuse(const int32_t* bm25_ids, int32_t kb, const int32_t* colbert_ids, int32_t kc, int32_t B,
                  int32_t rrf_k, int32_t C, int32_t* out_ids, double* out_scores, int32_t* out_count) {
  if (!(B >= 1 && C >= 1 && kb >= 0 && kc >= 0)) return cbv2_set_error(CBV2_EINVAL, "bad sizes");
  if (!((kb == 0 || bm25_ids) && (kc == 0 || colbert_ids) && out_ids)) return cbv2_set_error(CBV2_EINVAL, "null pointer");
  // per-thread scratch, reused across calls (the B = 1 latency path fuses
  // 200 ids per call: allocation would be most of its cost)
  thread_local std::vector<int32_t> ids, slot;
  thread_local std::vector<double> sc;
  struct Entry {
    double s;
    int32_t j;   // insertion position
  };
  thread_local std::vector<Entry> order;
  thread_local std::vector<uint32_t> used;
  // 1 / (rrf_k + rank) for ranks 1 .. max(kb, kc): the same division, once
  // per call instead of once per list entry
  thread_local std::vector<double> inv;
  thread_local int32_t inv_k = -1;
  const int32_t rmax = std::max(kb, kc);
  if (inv_k != rrf_k || (int32_t)inv.size() < rmax + 1) {
    inv.resize((size_t)rmax + 1);
    for (int32_t r = 1; r <= rmax; ++r) inv[r] = 1.0 / (double)(rrf_k + r);
    inv_k = rrf_k;
  }
  ids.clear();
  sc.clear();
  ids.reserve(kb + kc);
  sc.reserve(kb + kc);
  // id -> position in `ids` by open addressing (a power of two >= 2 (kb + kc)
  // slots, multiplicative hash, linear probing): O(1) per add instead of the
  // reference dict's semantics restated as a linear search (the fused order
  // and values are unchanged: first insertion decides the position, float64
  // sums in list order)
  int bits = 4;
  while ((1 << bits) < 2 * (kb + kc)) ++bits;
  const uint32_t mask = (1u << bits) - 1;
  slot.assign(mask + 1, -1);
  used.clear();
  used.reserve(kb + kc);
  for (int32_t b = 0; b < B; ++b) {
    ids.clear();
    sc.clear();
    for (uint32_t h : used) slot[h] = -1;
    used.clear();
    auto add = [&](int32_t id, int32_t rank) {
      const double inc = inv[rank];
      uint32_t h = ((uint32_t)id * 2654435761u) >> (32 - bits);
      for (;; h = (h + 1) & mask) {
        const int32_t j = slot[h];
        if (j < 0) break;
        if (ids[j] == id) { sc[j] = sc[j] + inc; return; }
      }
      slot[h] = (int32_t)ids.size();
      used.push_back(h);
      ids.push_back(id);
      sc.push_back(0.0 + inc);
    };
    for (int32_t r = 0; r < kb; ++r) {
      const int32_t id = bm25_ids[(size_t)b * kb + r];
      if (id >= 0) add(id, r + 1);
    }
    for (int32_t r = 0; r < kc; ++r) {
      const int32_t id = colbert_ids[(size_t)b * kc + r];
      if (id >= 0) add(id, r + 1);
    }
    order.resize(ids.size());
    for (size_t j = 0; j < ids.size(); ++j) order[j] = Entry{sc[j], (int32_t)j};
    // the first C of the STABLE descending sort: (score desc, insertion order
    // asc) is a strict total order, so a partial sort on it yields exactly the
    // stable sort's prefix
    const size_t m = std::min<size_t>((size_t)C, order.size());
    const auto before = [](const Entry& a, const Entry& c) { return a.s > c.s || (a.s == c.s && a.j < c.j); };
    if (m < order.size()) std::nth_element(order.begin(), order.begin() + m, order.end(), before);
    std::sort(order.begin(), order.begin() + m, before);
    for (int32_t j = 0; j < C; ++j) {
      const bool ok = j < (int32_t)m;
      out_ids[(size_t)b * C + j] = ok ? ids[order[j].j] : -1;
      if (out_scores) out_scores[(size_t)b * C + j] = ok ? order[j].s : 0.0;
    }
    if (out_count) out_count[b] = (int32_t)ids.size();
  }
  return CBV2_OK;
}

}  // extern "C"
