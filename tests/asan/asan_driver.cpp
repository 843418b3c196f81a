// AddressSanitizer / UBSan driver for the HOST C++ of libcolbert_mi355x.so
// ("a -fsanitize=address host build"): host BM25 (build, sharded
// statistics, threaded search, edge cases), RRF, the Snowball stemmer on
// random and malformed UTF-8, and the native index file's host entry points
// including the streaming writer.  Built by tests/test_asan_host.py with g++
// -fsanitize=address,undefined; test infrastructure only (no GPU code).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg) {
  (void)msg;
  return code;
}

static int fails = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                    \
    }                                                             \
  } while (0)

static void bm25_cases(std::mt19937& rng) {
  for (int rep = 0; rep < 20; ++rep) {
    const int N = 1 + rng() % 300, V = 1 + rng() % 50;
    std::vector<int64_t> off(N + 1, 0);
    std::vector<int32_t> terms;
    for (int d = 0; d < N; ++d) {
      const int len = rng() % 40;
      for (int t = 0; t < len; ++t) terms.push_back(rng() % V);
      off[d + 1] = (int64_t)terms.size();
    }
    cbv2_bm25* ix = nullptr;
    CHECK(cbv2_bm25_build(terms.empty() ? nullptr : terms.data(), off.data(), N, V, 1.5f, 0.75f, &ix) == CBV2_OK);
    const int B = 1 + rng() % 9, k = 1 + rng() % (N + 5);
    std::vector<int64_t> qo(B + 1, 0);
    std::vector<int32_t> qt;
    for (int b = 0; b < B; ++b) {
      const int ql = rng() % 7;
      for (int j = 0; j < ql; ++j) qt.push_back((int32_t)(rng() % (V + 4)) - 2);   // out-of-range ids too
      qo[b + 1] = (int64_t)qt.size();
    }
    std::vector<int32_t> ids((size_t)B * k);
    std::vector<float> sc((size_t)B * k);
    CHECK(cbv2_bm25_search(ix, qt.empty() ? nullptr : qt.data(), qo.data(), B, k, 1 + rep % 4, ids.data(),
                           sc.data()) == CBV2_OK);
    // sharded build of the second half with the global statistics
    std::vector<int64_t> df(V);
    CHECK(cbv2_bm25_doc_freq(terms.empty() ? nullptr : terms.data(), off.data(), N, V, df.data()) == CBV2_OK);
    const int h = N / 2;
    std::vector<int64_t> off2(off.begin() + h, off.end());
    cbv2_bm25* sh = nullptr;
    CHECK(cbv2_bm25_build_shard(terms.empty() ? nullptr : terms.data(), off2.data(), N - h, V, 1.5f, 0.75f, h, N,
                                off[N], df.data(), &sh) == CBV2_OK);
    CHECK(cbv2_bm25_search(sh, qt.empty() ? nullptr : qt.data(), qo.data(), B, k, 2, ids.data(), nullptr) == CBV2_OK);
    cbv2_bm25_destroy(sh);
    cbv2_bm25_destroy(ix);
  }
  cbv2_bm25* bad = nullptr;
  int32_t t[2] = {0, 99};
  int64_t o[2] = {0, 2};
  CHECK(cbv2_bm25_build(t, o, 1, 10, 1.5f, 0.75f, &bad) == CBV2_EINVAL && bad == nullptr);
}

static void rrf_cases(std::mt19937& rng) {
  for (int rep = 0; rep < 50; ++rep) {
    const int B = 1 + rng() % 5, kb = rng() % 120, kc = rng() % 120, C = 1 + rng() % 80;
    std::vector<int32_t> bm((size_t)B * kb + 1), cb((size_t)B * kc + 1), out((size_t)B * C);
    std::vector<double> sc((size_t)B * C);
    std::vector<int32_t> cnt(B);
    for (auto& x : bm) x = (int32_t)(rng() % 150) - 5;
    for (auto& x : cb) x = (int32_t)(rng() % 150) - 5;
    CHECK(cbv2_rrf_fuse(bm.data(), kb, cb.data(), kc, B, 60, C, out.data(), sc.data(), cnt.data()) == CBV2_OK);
  }
  int32_t o[1];
  CHECK(cbv2_rrf_fuse(nullptr, 3, nullptr, 0, 1, 60, 1, o, nullptr, nullptr) == CBV2_EINVAL);
}

static void stem_cases(std::mt19937& rng) {
  const char* words[] = {"generously", "knackeries", "'tis", "dog's", "sayings", "naïve", "über", "", "a", "yy",
                         "\xff\xfe", "\xe2\x82", "ies", "sses", "eedly", "ingly", "ational"};
  for (int rep = 0; rep < 400; ++rep) {
    std::string buf;
    std::vector<int64_t> off(1, 0);
    const int n = 1 + rng() % 20;
    for (int i = 0; i < n; ++i) {
      if (rng() % 3 == 0) {
        buf += words[rng() % (sizeof(words) / sizeof(words[0]))];
      } else {
        const int len = rng() % 14;
        for (int c = 0; c < len; ++c) buf += (char)(rng() % 4 == 0 ? (rng() % 256) : "aeiouybcdlmnstY'"[rng() % 16]);
      }
      off.push_back((int64_t)buf.size());
    }
    std::vector<char> out(buf.size() + 1);
    std::vector<int64_t> oo(n + 1);
    CHECK(cbv2_stem_en(buf.data(), off.data(), n, out.data(), (int64_t)buf.size(), oo.data()) == CBV2_OK);
    for (int i = 0; i < n; ++i) CHECK(oo[i + 1] - oo[i] <= off[i + 1] - off[i]);   // stems never grow
  }
}

static void file_cases(const char* dir, std::mt19937& rng) {
  for (int fp8 = 0; fp8 < 2; ++fp8) {
    const int n = 1 + rng() % 17;
    const size_t per = fp8 ? 16384 : 32768;
    std::vector<uint8_t> tok(per * n), sc(256 * (size_t)n);
    std::vector<int32_t> dl(n);
    for (auto& x : tok) x = (uint8_t)rng();
    for (auto& x : sc) x = (uint8_t)rng();
    for (auto& x : dl) x = rng() % 129;
    const int32_t dt = fp8 ? CBV2_DTYPE_MXFP8 : CBV2_DTYPE_BF16;
    std::string p = std::string(dir) + (fp8 ? "/a8.cbv2" : "/a16.cbv2");
    CHECK(cbv2_index_file_write_host(p.c_str(), dt, n, tok.data(), sc.data(), dl.data(), 3) == CBV2_OK);
    std::vector<uint8_t> tok2(per * n), sc2(256 * (size_t)n);
    std::vector<int32_t> dl2(n);
    CHECK(cbv2_index_file_read_host(p.c_str(), 0, n, tok2.data(), sc2.data(), dl2.data()) == CBV2_OK);
    CHECK(tok == tok2 && dl == dl2 && (!fp8 || sc == sc2));
    CHECK(cbv2_index_file_read_host(p.c_str(), 0, n + 1, tok2.data(), sc2.data(), dl2.data()) == CBV2_EINVAL);
    std::string q = std::string(dir) + "/w.cbv2";
    cbv2_index_writer* w = nullptr;
    CHECK(cbv2_index_writer_open(q.c_str(), dt, n, 3, &w) == CBV2_OK);
    for (int a = 0; a < n;) {
      const int m = 1 + rng() % (n - a);
      CHECK(cbv2_index_writer_append(w, m, tok.data() + per * a, sc.data() + 256 * a, dl.data() + a, 0, nullptr) ==
            CBV2_OK);
      a += m;
    }
    CHECK(cbv2_index_writer_append(w, 1, tok.data(), sc.data(), dl.data(), 0, nullptr) == CBV2_EINVAL);
    CHECK(cbv2_index_writer_close(w) == CBV2_OK);
    int32_t d2;
    int64_t n2, b2;
    CHECK(cbv2_index_file_info(q.c_str(), &d2, &n2, &b2) == CBV2_OK && d2 == dt && n2 == n && b2 == 3);
    cbv2_index_writer* w2 = nullptr;
    CHECK(cbv2_index_writer_open(q.c_str(), dt, n + 2, 0, &w2) == CBV2_OK);
    CHECK(cbv2_index_writer_close(w2) == CBV2_EINVAL);    // incomplete: no header
    CHECK(cbv2_index_file_info(q.c_str(), &d2, &n2, &b2) == CBV2_EINVAL);
  }
}

int main(int argc, char** argv) {
  std::mt19937 rng(12345);
  bm25_cases(rng);
  rrf_cases(rng);
  stem_cases(rng);
  file_cases(argc > 1 ? argv[1] : "/tmp", rng);
  printf("asan driver: %d failed checks\n", fails);
  return fails ? 1 : 0;
}
