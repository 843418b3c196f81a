// text_en.cpp — the English text analysis of stage 1 (HybridRetriever._bm25_search,
// local_rag_complete.py:937-945, and DualIndexer.build_bm25_index, :851-855):
// the reference calls bm25s.tokenize(..., stopwords="en",
// stemmer=Stemmer.Stemmer("english")), i.e. PyStemmer's Snowball English
// stemmer.  Neither PyStemmer nor bm25s is installed here, so the stemmer is
// restated from the published Snowball English ("Porter2") algorithm
// (snowballstem.org/algorithms/english/stemmer.html, english.sbl): exception
// list 1, prelude (initial apostrophe, y -> Y), regions R1/R2 with the
// gener/commun/arsen prefixes, steps 1a, exception list 2, 1b, 1c, 2, 3, 4, 5,
// postlude.  It works on Unicode code points decoded from UTF-8, as
// libstemmer does: only a e i o u y are vowels, every other character is a
// non-vowel.  Tokenisation (lower-case + bm25s' (?u)\b\w\w+\b pattern, Python's
// own regex semantics) and the stopword filter stay in bm25.py, which calls
// the batch entry point here for the unique tokens (as bm25s stems its
// vocabulary once).  Parity with PyStemmer is pinned only by the published
// sample vocabulary restated in tests/test_text_en.py.
#include <cstdint>
#include <cstring>
#include <string>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);  // colbert_mi355x.hip

namespace {
using W = std::u32string;

bool is_v(char32_t c) { return c == 'a' || c == 'e' || c == 'i' || c == 'o' || c == 'u' || c == 'y'; }
bool is_double(const W& w, size_t n) {
  if (n < 2 || w[n - 1] != w[n - 2]) return false;
  switch (w[n - 1]) {
    case 'b': case 'd': case 'f': case 'g': case 'm': case 'n': case 'p': case 'r': case 't': return true;
    default: return false;
  }
}
bool valid_li(char32_t c) {
  switch (c) {
    case 'c': case 'd': case 'e': case 'g': case 'h': case 'k': case 'm': case 'n': case 'r': case 't': return true;
    default: return false;
  }
}
bool ends(const W& w, const char* suf) {
  const size_t m = strlen(suf);
  if (w.size() < m) return false;
  for (size_t i = 0; i < m; ++i)
    if (w[w.size() - m + i] != (char32_t)(unsigned char)suf[i]) return false;
  return true;
}
bool equals(const W& w, const char* s) { return w.size() == strlen(s) && ends(w, s); }
bool starts(const W& w, const char* pre) {
  const size_t m = strlen(pre);
  if (w.size() < m) return false;
  for (size_t i = 0; i < m; ++i)
    if (w[i] != (char32_t)(unsigned char)pre[i]) return false;
  return true;
}
void set_suffix(W& w, size_t m, const char* rep) {  // replace the last m characters
  w.resize(w.size() - m);
  for (const char* p = rep; *p; ++p) w.push_back((char32_t)(unsigned char)*p);
}
W from(const char* s) {
  W w;
  for (const char* p = s; *p; ++p) w.push_back((char32_t)(unsigned char)*p);
  return w;
}
bool has_vowel(const W& w, size_t end) {
  for (size_t i = 0; i < end; ++i)
    if (is_v(w[i])) return true;
  return false;
}
// A short syllable ends the first m characters: non-vowel, vowel, non-vowel
// other than w, x, Y; or (m == 2) vowel, non-vowel at the start of the word.
bool shortv(const W& w, size_t m) {
  if (m >= 3 && !is_v(w[m - 1]) && w[m - 1] != 'w' && w[m - 1] != 'x' && w[m - 1] != 'Y' && is_v(w[m - 2]) &&
      !is_v(w[m - 3]))
    return true;
  return m == 2 && !is_v(w[1]) && is_v(w[0]);
}
// Longest suffix of w among `list` (nullptr-terminated); -1 if none.
int longest(const W& w, const char* const* list) {
  int best = -1;
  size_t blen = 0;
  for (int i = 0; list[i]; ++i) {
    const size_t m = strlen(list[i]);
    if ((best < 0 || m > blen) && ends(w, list[i])) best = i, blen = m;
  }
  return best;
}

struct Ex {
  const char* word;
  const char* stem;
};
const Ex kException1[] = {{"skis", "ski"},     {"skies", "sky"},     {"dying", "die"},   {"lying", "lie"},
                          {"tying", "tie"},    {"idly", "idl"},      {"gently", "gentl"}, {"ugly", "ugli"},
                          {"early", "earli"},  {"only", "onli"},     {"singly", "singl"}, {"sky", "sky"},
                          {"news", "news"},    {"howe", "howe"},     {"atlas", "atlas"}, {"cosmos", "cosmos"},
                          {"bias", "bias"},    {"andes", "andes"},   {nullptr, nullptr}};
const char* const kException2[] = {"inning", "outing", "canning", "herring", "earring",
                                   "proceed", "exceed", "succeed", nullptr};

W stem(W w) {
  for (int i = 0; kException1[i].word; ++i)
    if (equals(w, kException1[i].word)) return from(kException1[i].stem);
  if (w.size() < 3) return w;
  // prelude
  if (!w.empty() && w[0] == '\'') w.erase(0, 1);
  bool y_found = false;
  if (!w.empty() && w[0] == 'y') w[0] = 'Y', y_found = true;
  for (size_t i = 1; i < w.size(); ++i)
    if (w[i] == 'y' && is_v(w[i - 1])) w[i] = 'Y', y_found = true;
  // regions
  const size_t n0 = w.size();
  size_t p1 = n0, p2 = n0;
  {
    auto after_vnv = [&](size_t from) -> size_t {  // gopast v, gopast non-v
      size_t i = from;
      while (i < n0 && !is_v(w[i])) ++i;
      if (i >= n0) return n0 + 1;
      ++i;
      while (i < n0 && is_v(w[i])) ++i;
      if (i >= n0) return n0 + 1;
      return i + 1;
    };
    size_t r1;
    if (starts(w, "gener")) r1 = 5;
    else if (starts(w, "commun")) r1 = 6;
    else if (starts(w, "arsen")) r1 = 5;
    else r1 = after_vnv(0);
    if (r1 <= n0) {
      p1 = r1;
      const size_t r2 = after_vnv(p1);
      if (r2 <= n0) p2 = r2;
    }
  }
  // Step 1a
  {
    static const char* const apos[] = {"'s'", "'s", "'", nullptr};
    const int a = longest(w, apos);
    if (a >= 0) w.resize(w.size() - strlen(apos[a]));
    static const char* const l1a[] = {"sses", "ied", "ies", "s", "us", "ss", nullptr};
    const int j = longest(w, l1a);
    if (j == 0) {
      set_suffix(w, 4, "ss");
    } else if (j == 1 || j == 2) {
      set_suffix(w, 3, w.size() - 3 >= 2 ? "i" : "ie");
    } else if (j == 3) {
      // next (skip the letter before s), then a vowel somewhere before it
      if (w.size() >= 2 && has_vowel(w, w.size() - 2)) w.resize(w.size() - 1);
    }
  }
  for (int i = 0; kException2[i]; ++i)
    if (equals(w, kException2[i])) goto postlude;
  // Step 1b
  {
    static const char* const l1b[] = {"eed", "eedly", "ed", "edly", "ing", "ingly", nullptr};
    const int j = longest(w, l1b);
    if (j == 0 || j == 1) {
      const size_t m = strlen(l1b[j]);
      if (w.size() - m >= p1) set_suffix(w, m, "ee");
    } else if (j >= 2) {
      const size_t m = strlen(l1b[j]);
      if (has_vowel(w, w.size() - m)) {
        w.resize(w.size() - m);
        if (ends(w, "at") || ends(w, "bl") || ends(w, "iz"))
          w.push_back('e');
        else if (is_double(w, w.size()))
          w.pop_back();
        else if (w.size() == p1 && shortv(w, w.size()))
          w.push_back('e');
      }
    }
  }
  // Step 1c
  if (w.size() >= 3 && (w.back() == 'y' || w.back() == 'Y') && !is_v(w[w.size() - 2])) w.back() = 'i';
  // Step 2
  {
    static const char* const l2[] = {"tional", "enci",    "anci",  "abli",  "entli",   "izer",    "ization",
                                     "ational", "ation",  "ator",  "alism", "aliti",   "alli",    "fulness",
                                     "ousli",  "ousness", "iveness", "iviti", "biliti", "bli",    "ogi",
                                     "fulli",  "lessli",  "li",    nullptr};
    static const char* const r2[] = {"tion", "ence", "ance", "able", "ent", "ize", "ize", "ate", "ate", "ate",
                                     "al",   "al",   "al",   "ful",  "ous", "ous", "ive", "ive", "ble", "ble",
                                     "og",   "ful",  "less", "",     nullptr};
    const int j = longest(w, l2);
    if (j >= 0) {
      const size_t m = strlen(l2[j]);
      const size_t s = w.size() - m;
      if (s >= p1) {
        if (!strcmp(l2[j], "ogi")) {
          if (s >= 1 && w[s - 1] == 'l') set_suffix(w, m, r2[j]);
        } else if (!strcmp(l2[j], "li")) {
          if (s >= 1 && valid_li(w[s - 1])) set_suffix(w, m, r2[j]);
        } else {
          set_suffix(w, m, r2[j]);
        }
      }
    }
  }
  // Step 3
  {
    static const char* const l3[] = {"tional", "ational", "alize", "icate", "iciti", "ical", "ful", "ness", "ative",
                                     nullptr};
    static const char* const r3[] = {"tion", "ate", "al", "ic", "ic", "ic", "", "", "", nullptr};
    const int j = longest(w, l3);
    if (j >= 0) {
      const size_t m = strlen(l3[j]);
      const size_t s = w.size() - m;
      if (s >= p1 && (strcmp(l3[j], "ative") != 0 || s >= p2)) set_suffix(w, m, r3[j]);
    }
  }
  // Step 4
  {
    static const char* const l4[] = {"al",  "ance", "ence", "er",  "ic",  "able", "ible", "ant", "ement", "ment",
                                     "ent", "ism",  "ate",  "iti", "ous", "ive",  "ize",  "ion", nullptr};
    const int j = longest(w, l4);
    if (j >= 0) {
      const size_t m = strlen(l4[j]);
      const size_t s = w.size() - m;
      if (s >= p2) {
        if (!strcmp(l4[j], "ion")) {
          if (s >= 1 && (w[s - 1] == 's' || w[s - 1] == 't')) w.resize(s);
        } else {
          w.resize(s);
        }
      }
    }
  }
  // Step 5
  if (!w.empty() && w.back() == 'e') {
    const size_t s = w.size() - 1;
    if (s >= p2 || (s >= p1 && !shortv(w, s))) w.resize(s);
  } else if (!w.empty() && w.back() == 'l') {
    const size_t s = w.size() - 1;
    if (s >= p2 && s >= 1 && w[s - 1] == 'l') w.resize(s);
  }
postlude:
  if (y_found)
    for (auto& c : w)
      if (c == 'Y') c = 'y';
  return w;
}

// UTF-8 <-> code points.  A byte that does not start a valid sequence (or
// starts one encoding a surrogate) becomes U+DC00 + byte, a non-vowel, and is
// written back as that single byte (Python's "surrogateescape"), so no stem
// is ever longer in bytes than its word.
W decode(const char* s, size_t n) {
  W w;
  w.reserve(n);
  for (size_t i = 0; i < n;) {
    const unsigned char c = (unsigned char)s[i];
    int len = c < 0x80 ? 1 : (c >> 5) == 6 ? 2 : (c >> 4) == 14 ? 3 : (c >> 3) == 30 ? 4 : 0;
    char32_t cp = 0;
    bool ok = len > 0 && i + len <= n;
    if (ok) {
      cp = len == 1 ? c : len == 2 ? (c & 0x1f) : len == 3 ? (c & 0x0f) : (c & 0x07);
      for (int k = 1; k < len && ok; ++k) {
        const unsigned char d = (unsigned char)s[i + k];
        ok = (d >> 6) == 2;
        cp = (cp << 6) | (d & 0x3f);
      }
      ok = ok && !(cp >= 0xD800 && cp <= 0xDFFF) && cp <= 0x10FFFF;
    }
    if (!ok) {
      w.push_back(0xDC00 + c);
      ++i;
      continue;
    }
    w.push_back(cp);
    i += len;
  }
  return w;
}
void encode(const W& w, std::string& out) {
  for (char32_t cp : w) {
    if (cp >= 0xDC80 && cp <= 0xDCFF) {   // an escaped raw byte
      out.push_back((char)(cp - 0xDC00));
    } else if (cp < 0x80) {
      out.push_back((char)cp);
    } else if (cp < 0x800) {
      out.push_back((char)(0xc0 | (cp >> 6)));
      out.push_back((char)(0x80 | (cp & 0x3f)));
    } else if (cp < 0x10000) {
      out.push_back((char)(0xe0 | (cp >> 12)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
      out.push_back((char)(0x80 | (cp & 0x3f)));
    } else {
      out.push_back((char)(0xf0 | (cp >> 18)));
      out.push_back((char)(0x80 | ((cp >> 12) & 0x3f)));
      out.push_back((char)(0x80 | ((cp >> 6) & 0x3f)));
      out.push_back((char)(0x80 | (cp & 0x3f)));
    }
  }
}
}  // namespace

extern "C" int cbv2_stem_en(const char* words, const int64_t* offsets, int64_t n, char* out, int64_t out_cap,
                            int64_t* out_offsets) {
  if (n < 0 || (n > 0 && (!words || !offsets || !out_offsets)) || out_cap < 0 || (out_cap > 0 && !out))
    return cbv2_set_error(CBV2_EINVAL, "bad stem arguments");
  std::string buf;
  int64_t pos = 0;
  if (n > 0) out_offsets[0] = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t a = offsets[i], b = offsets[i + 1];
    if (b < a) return cbv2_set_error(CBV2_EINVAL, "offsets not ascending");
    buf.clear();
    encode(stem(decode(words + a, (size_t)(b - a))), buf);
    if (pos + (int64_t)buf.size() > out_cap) return cbv2_set_error(CBV2_EINVAL, "stem output buffer too small");
    memcpy(out + pos, buf.data(), buf.size());
    pos += (int64_t)buf.size();
    out_offsets[i + 1] = pos;
  }
  return CBV2_OK;
}
