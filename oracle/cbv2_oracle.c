/*
 * cbv2_oracle.c — plain-C CPU restatement of the ColBERT hot path.
 * TEST INFRASTRUCTURE ONLY: linked by tests/ and timed as bench.py's
 * cpu_baseline leg; the product never calls it.
 *
 *   oracle_maxsim_bf16  S[b,n] = sum_{q<lq} max_{t<len_n} <Q[b,q], D_n[t]>, the
 *                       north-star form of _maxsim_score (LRC:802-831; the
 *                       reference's docstring at LRC:807-812 describes it, its
 *                       code mean-pools instead — see oracle.py), on bf16 bit
 *                       patterns, exact products, double accumulation.
 *   oracle_topk         torch.topk (LRC:767) with ties -> lower index.
 *   oracle_codebook_topk the same MaxSim + top-k for corpora whose tokens are
 *                       rows of a small codebook (exact k/16-grid test corpora
 *                       up to the 1M-doc headline size).
 *
 * LRC = /root/reference/local_rag_complete.py
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static inline double bf16_to_double(uint16_t b) {
  uint32_t u = (uint32_t)b << 16;
  float f;
  memcpy(&f, &u, 4);
  return (double)f;
}

void oracle_maxsim_bf16(const uint16_t* q, int B, int lq, const uint16_t* docs, const int32_t* doclens, int64_t n,
                        int ld, double* out) {
  const int D = 128;
  double* qd = (double*)malloc(sizeof(double) * (size_t)lq * D);
  double* dd = (double*)malloc(sizeof(double) * (size_t)ld * D);
  for (int b = 0; b < B; ++b) {
    for (int i = 0; i < lq * D; ++i) qd[i] = bf16_to_double(q[(size_t)b * lq * D + i]);
    for (int64_t d = 0; d < n; ++d) {
      int len = doclens[d];
      if (len > ld) len = ld;
      if (len <= 0) {
        out[(size_t)b * n + d] = -INFINITY;
        continue;
      }
      for (int i = 0; i < len * D; ++i) dd[i] = bf16_to_double(docs[(size_t)d * ld * D + i]);
      double total = 0.0;
      for (int i = 0; i < lq; ++i) {
        double best = -INFINITY;
        for (int t = 0; t < len; ++t) {
          double s = 0.0;
          for (int c = 0; c < D; ++c) s += qd[i * D + c] * dd[t * D + c];
          if (s > best) best = s;
        }
        total += best;
      }
      out[(size_t)b * n + d] = total;
    }
  }
  free(qd);
  free(dd);
}

/* Insertion of (s, i) into a descending top-k list of cnt entries; indices
 * arrive in ascending order, so an equal score keeps the earlier index first. */
static inline void topk_insert(double s, int64_t i, int k, int* cnt, double* vals, int64_t* ids) {
  if (*cnt == k && !(s > vals[k - 1])) return;
  int pos = *cnt < k ? *cnt : k - 1;
  while (pos > 0 && s > vals[pos - 1]) {
    vals[pos] = vals[pos - 1];
    ids[pos] = ids[pos - 1];
    --pos;
  }
  vals[pos] = s;
  ids[pos] = i;
  if (*cnt < k) ++*cnt;
}

static inline void topk_pad(int cnt, int k, double* vals, int64_t* ids) {
  for (int j = cnt; j < k; ++j) {
    vals[j] = -INFINITY;
    ids[j] = -1;
  }
}

/* torch.topk (LRC:767) with ties -> lower index. */
void oracle_topk(const double* scores, int64_t n, int k, double* out_vals, int64_t* out_ids) {
  int cnt = 0;
  for (int64_t i = 0; i < n; ++i) topk_insert(scores[i], i, k, &cnt, out_vals, out_ids);
  topk_pad(cnt, k, out_vals, out_ids);
}

/* MaxSim + top-k over a CODEBOOK corpus (the exact-arithmetic test corpora of
 * tests/test_gpu_grid_exact.py).  Every scoring token of a codebook doc is a
 * row of a K-row codebook (K <= 32), so max_{t < len} <q, d_t> depends only on
 * the SET of codes among its scoring rows, and the north-star MaxSim
 * (LRC:807-812) is
 *     S[b, n] = sum_{q < lq} max_{c in set(n)} T[b][q][c],   T = <Q[b, q], code_c>.
 * The sets come deduplicated: umask[u] (bit c = code c present; 0 = empty doc,
 * scores -inf) and inv[n] = doc n's entry.  Docs with over_idx[n] >= 0 (planted
 * docs whose tokens are not codebook rows) take the caller's score
 * over_scores[b * n_over + over_idx[n]].  Output: the top-k of every query,
 * ties -> lower index, as oracle_topk; sums in double (exact on k/16 grids). */
void oracle_codebook_topk(const double* T, int B, int lq, int K, const uint32_t* umask, int64_t n_umask,
                          const int32_t* inv, const int32_t* over_idx, const double* over_scores, int64_t n_over,
                          int64_t n, int k, double* out_vals, int64_t* out_ids) {
  double* ms = (double*)malloc(sizeof(double) * (size_t)(n_umask > 0 ? n_umask : 1));
  double* Tt = (double*)malloc(sizeof(double) * (size_t)K * lq); /* [K][lq]: one code's column contiguous */
  double* best = (double*)malloc(sizeof(double) * (size_t)lq);
  for (int b = 0; b < B; ++b) {
    const double* Tb = T + (size_t)b * lq * K;
    for (int q = 0; q < lq; ++q)
      for (int c = 0; c < K; ++c) Tt[(size_t)c * lq + q] = Tb[(size_t)q * K + c];
    for (int64_t u = 0; u < n_umask; ++u) {
      uint32_t m = umask[u];
      if (!m) {
        ms[u] = -INFINITY;
        continue;
      }
      for (int q = 0; q < lq; ++q) best[q] = -INFINITY;
      for (; m; m &= m - 1) { /* the set bits = the codes present */
        const double* col = Tt + (size_t)__builtin_ctz(m) * lq;
        for (int q = 0; q < lq; ++q) best[q] = col[q] > best[q] ? col[q] : best[q];
      }
      double total = 0.0;
      for (int q = 0; q < lq; ++q) total += best[q];
      ms[u] = total;
    }
    int cnt = 0;
    double* vals = out_vals + (size_t)b * k;
    int64_t* ids = out_ids + (size_t)b * k;
    for (int64_t i = 0; i < n; ++i) {
      const double s = over_idx[i] >= 0 ? over_scores[(size_t)b * n_over + over_idx[i]] : ms[inv[i]];
      topk_insert(s, i, k, &cnt, vals, ids);
    }
    topk_pad(cnt, k, vals, ids);
  }
  free(ms);
  free(Tt);
  free(best);
}
