// host_bm25.cpp — stage 1 of HybridRetriever.retrieve (local_rag_complete.py:937-950),
// host-side as the north star requires, native for throughput at thousands of qps.
//
// The reference calls bm25s (English stopwords + Snowball stemmer, Lucene BM25;
// LRC:851-858, 939-945).  bm25s is not installed here, so its published scoring
// is restated over TERM IDS (tokenisation/stopwords stay in Python, bm25.py):
//   idf(t)   = ln(1 + (N - df + 0.5) / (df + 0.5))
//   w(t, d)  = idf * tf * (k1 + 1) / (tf + k1 * (1 - b + b * |d| / avgdl))
//   score(q, d) = sum over the query's terms IN QUERY ORDER, repeats included,
//                 of w(t, d)   (bm25s sums the postings of every query token id:
//                 its get_scores_from_ids -> _compute_relevance_from_scores;
//                 round 1 summed distinct terms, which differs on repeated words)
// Weights are computed in double and stored as float; scores accumulate in
// float in posting order, so oracle/oracle.py:bm25_topk reproduces every bit.
// Ranking: score descending, then doc id ascending; rows are padded with the
// lowest-id zero-score docs (as a full sort of all docs would), then -1.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "colbert_mi355x.h"

struct cbv2_bm25 {
  int64_t n_docs = 0;
  int32_t vocab = 0;
  int32_t id_base = 0;        // global id of local doc 0 (sharded index)
  std::vector<int64_t> ptr;   // [vocab + 1] posting offsets per term
  std::vector<int32_t> docs;  // posting doc ids (ascending within a term)
  std::vector<float> w;       // posting weights
};

extern "C" int cbv2_set_error(int code, const char* msg);  // defined in colbert_mi355x.hip

// (doc_terms may be null when the docs hold no token at all: a shard of empty
// chunks builds an index that matches nothing)
static int check_corpus(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int32_t vocab) {
  if (n_docs < 0 || vocab < 1 || (n_docs > 0 && !doc_offsets))
    return cbv2_set_error(CBV2_EINVAL, "bad bm25 corpus arguments");
  if (n_docs > 0x7fffffffLL) return cbv2_set_error(CBV2_EINVAL, "too many docs for int32 ids");
  for (int64_t d = 0; d < n_docs; ++d)
    if (doc_offsets[d + 1] < doc_offsets[d]) return cbv2_set_error(CBV2_EINVAL, "doc_offsets not ascending");
  const int64_t total = n_docs ? doc_offsets[n_docs] - doc_offsets[0] : 0;
  if (total > 0 && !doc_terms) return cbv2_set_error(CBV2_EINVAL, "bad bm25 corpus arguments (null terms)");
  const int32_t* t = total > 0 ? doc_terms + doc_offsets[0] : nullptr;
  for (int64_t i = 0; i < total; ++i)
    if (t[i] < 0 || t[i] >= vocab) return cbv2_set_error(CBV2_EINVAL, "term id out of range");
  return CBV2_OK;
}

// df of the distinct terms of each doc (sorting a scratch copy per doc)
static void doc_freq(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int64_t* df) {
  if (doc_terms == nullptr) return;   // no tokens (check_corpus)
  std::vector<int32_t> scratch;
  for (int64_t d = 0; d < n_docs; ++d) {
    scratch.assign(doc_terms + doc_offsets[d], doc_terms + doc_offsets[d + 1]);
    std::sort(scratch.begin(), scratch.end());
    for (size_t j = 0; j < scratch.size(); ++j)
      if (j == 0 || scratch[j] != scratch[j - 1]) ++df[scratch[j]];
  }
}

extern "C" int cbv2_bm25_doc_freq(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs,
                                  int32_t vocab, int64_t* df_out) {
  if (!df_out) return cbv2_set_error(CBV2_EINVAL, "null df_out");
  if (int rc = check_corpus(doc_terms, doc_offsets, n_docs, vocab)) return rc;
  std::fill(df_out, df_out + vocab, (int64_t)0);
  doc_freq(doc_terms, doc_offsets, n_docs, df_out);
  return CBV2_OK;
}

extern "C" int cbv2_bm25_build_shard(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs,
                                     int32_t vocab, float k1, float b, int64_t id_base, int64_t n_global,
                                     int64_t total_global, const int64_t* df_global, cbv2_bm25** out) {
  if (!out) return cbv2_set_error(CBV2_EINVAL, "null output handle pointer");
  *out = nullptr;
  if (int rc = check_corpus(doc_terms, doc_offsets, n_docs, vocab)) return rc;
  const bool local = df_global == nullptr;
  if (!local && (id_base < 0 || n_global < id_base + n_docs || total_global < 0))
    return cbv2_set_error(CBV2_EINVAL, "bad global statistics");
  if (id_base + n_docs > 0x7fffffffLL) return cbv2_set_error(CBV2_EINVAL, "global ids exceed int32");
  auto* ix = new cbv2_bm25;
  ix->n_docs = n_docs;
  ix->vocab = vocab;
  ix->id_base = (int32_t)id_base;
  std::vector<int64_t> df(vocab, 0);  // local df sizes the postings
  doc_freq(doc_terms, doc_offsets, n_docs, df.data());
  ix->ptr.assign(vocab + 1, 0);
  for (int32_t t = 0; t < vocab; ++t) ix->ptr[t + 1] = ix->ptr[t] + df[t];
  ix->docs.resize(ix->ptr[vocab]);
  ix->w.resize(ix->ptr[vocab]);
  const int64_t total_local = n_docs ? doc_offsets[n_docs] - doc_offsets[0] : 0;
  const double N = local ? (double)n_docs : (double)n_global;
  const int64_t total = local ? total_local : total_global;
  const double avgdl = N > 0 ? (double)total / N : 1.0;
  const int64_t* dfg = local ? df.data() : df_global;
  std::vector<double> idf(vocab);
  for (int32_t t = 0; t < vocab; ++t) idf[t] = std::log(1.0 + (N - (double)dfg[t] + 0.5) / ((double)dfg[t] + 0.5));
  // postings in doc order
  std::vector<int64_t> fill(ix->ptr.begin(), ix->ptr.end() - 1);
  std::vector<int32_t> scratch;
  for (int64_t d = 0; d < n_docs && doc_terms != nullptr; ++d) {   // (no tokens: no postings)
    scratch.assign(doc_terms + doc_offsets[d], doc_terms + doc_offsets[d + 1]);
    std::sort(scratch.begin(), scratch.end());
    const double dl = (double)scratch.size();
    for (size_t j = 0; j < scratch.size();) {
      size_t e = j;
      while (e < scratch.size() && scratch[e] == scratch[j]) ++e;
      const int32_t t = scratch[j];
      const double tf = (double)(e - j);
      const double norm = tf + (double)k1 * (1.0 - (double)b + (double)b * dl / avgdl);
      const int64_t pos = fill[t]++;
      ix->docs[pos] = (int32_t)d;
      ix->w[pos] = (float)(idf[t] * tf * ((double)k1 + 1.0) / norm);
      j = e;
    }
  }
  *out = ix;
  return CBV2_OK;
}

extern "C" int cbv2_bm25_build(const int32_t* doc_terms, const int64_t* doc_offsets, int64_t n_docs, int32_t vocab,
                               float k1, float b, cbv2_bm25** out) {
  return cbv2_bm25_build_shard(doc_terms, doc_offsets, n_docs, vocab, k1, b, 0, 0, 0, nullptr, out);
}

extern "C" int cbv2_bm25_destroy(cbv2_bm25* ix) {
  delete ix;
  return CBV2_OK;
}

static void search_range(const cbv2_bm25* ix, const int32_t* q_terms, const int64_t* q_offsets, int32_t b0,
                         int32_t b1, int32_t k, int32_t* out_ids, float* out_scores) {
  std::vector<float> acc((size_t)ix->n_docs, 0.0f);
  std::vector<int32_t> touched, terms, order;
  for (int32_t b = b0; b < b1; ++b) {
    terms.assign(q_terms + q_offsets[b], q_terms + q_offsets[b + 1]);
    touched.clear();
    for (int32_t t : terms) {
      if (t < 0 || t >= ix->vocab) continue;
      for (int64_t p = ix->ptr[t]; p < ix->ptr[t + 1]; ++p) {
        const int32_t d = ix->docs[p];
        if (acc[d] == 0.0f) touched.push_back(d);
        acc[d] += ix->w[p];
      }
    }
    const int32_t kk = (int32_t)std::min<int64_t>(k, (int64_t)touched.size());
    auto better = [&](int32_t x, int32_t y) { return acc[x] > acc[y] || (acc[x] == acc[y] && x < y); };
    std::partial_sort(touched.begin(), touched.begin() + kk, touched.end(), better);
    int32_t* oi = out_ids + (size_t)b * k;
    float* os = out_scores ? out_scores + (size_t)b * k : nullptr;
    for (int32_t j = 0; j < kk; ++j) {
      oi[j] = touched[j] + ix->id_base;
      if (os) os[j] = acc[touched[j]];
    }
    // pad with the lowest-id docs that scored 0 (a full sort's order), then -1
    int32_t j = kk;
    if (j < k) {
      std::vector<int32_t> hit(touched.begin(), touched.end());
      std::sort(hit.begin(), hit.end());
      size_t h = 0;
      for (int64_t d = 0; d < ix->n_docs && j < k; ++d) {
        while (h < hit.size() && hit[h] < d) ++h;
        if (h < hit.size() && hit[h] == d) continue;
        oi[j] = (int32_t)d + ix->id_base;
        if (os) os[j] = 0.0f;
        ++j;
      }
    }
    for (; j < k; ++j) {
      oi[j] = -1;
      if (os) os[j] = 0.0f;
    }
    for (int32_t d : touched) acc[d] = 0.0f;
  }
}

extern "C" int cbv2_bm25_search(const cbv2_bm25* ix, const int32_t* q_terms, const int64_t* q_offsets, int32_t B,
                                int32_t k, int32_t n_threads, int32_t* out_ids, float* out_scores) {
  if (!ix) return cbv2_set_error(CBV2_EINVAL, "null bm25 index");
  if (B < 0 || k < 1 || (B > 0 && (!q_offsets || !out_ids))) return cbv2_set_error(CBV2_EINVAL, "bad search arguments");
  if (B == 0) return CBV2_OK;
  int32_t T = n_threads > 0 ? n_threads : (int32_t)std::min<unsigned>(16u, std::max(1u, std::thread::hardware_concurrency()));
  if (T > B) T = B;
  if (T <= 1) {
    search_range(ix, q_terms, q_offsets, 0, B, k, out_ids, out_scores);
    return CBV2_OK;
  }
  std::vector<std::thread> pool;
  const int32_t per = (B + T - 1) / T;
  for (int32_t t = 0; t < T; ++t) {
    const int32_t b0 = t * per, b1 = std::min(B, b0 + per);
    if (b0 >= b1) break;
    pool.emplace_back(search_range, ix, q_terms, q_offsets, b0, b1, k, out_ids, out_scores);
  }
  for (auto& th : pool) th.join();
  return CBV2_OK;
}

extern "C" int64_t cbv2_bm25_num_docs(const cbv2_bm25* ix) { return ix ? ix->n_docs : -1; }
