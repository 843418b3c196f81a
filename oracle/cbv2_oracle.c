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

/* Insertion into a descending top-k list; (score desc, index asc). */
void oracle_topk(const double* scores, int64_t n, int k, double* out_vals, int64_t* out_ids) {
  int cnt = 0;
  for (int64_t i = 0; i < n; ++i) {
    double s = scores[i];
    if (cnt == k && !(s > out_vals[k - 1])) continue; /* equal score: the earlier index stays */
    int pos = cnt < k ? cnt : k - 1;
    while (pos > 0 && s > out_vals[pos - 1]) {
      out_vals[pos] = out_vals[pos - 1];
      out_ids[pos] = out_ids[pos - 1];
      --pos;
    }
    out_vals[pos] = s;
    out_ids[pos] = i;
    if (cnt < k) ++cnt;
  }
  for (int j = cnt; j < k; ++j) {
    out_vals[j] = -INFINITY;
    out_ids[j] = -1;
  }
}
