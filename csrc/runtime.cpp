// Host runtime: scikit-learn CountVectorizer-compatible tokenisation, vocabulary
// building and CSR vectorisation, multithreaded.
//
// Reference behaviour (client.py:369-374, server.py:270-288, main.py:148-152): every
// client's local vocabulary is CountVectorizer(lowercase=True, stop_words='english')
// .fit(corpus).vocabulary_, the global vocabulary is the sorted union, and each
// client's document-term matrix is CountVectorizer(vocabulary=global).transform.
// The default analyzer lowercases and takes the tokens of r"(?u)\b\w\w+\b", i.e.
// the maximal runs of word characters of length >= 2.  This implementation is
// exact for ASCII text (word characters [A-Za-z0-9_]); the Python wrapper routes
// corpora with non-ASCII bytes to scikit-learn, whose Unicode \w and str.lower
// it does not replicate.
//
// C ABI (ctypes): documents are one concatenated buffer + int64 offsets [n + 1].
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

inline bool is_word(unsigned char c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9') || c == '_';
}
inline char lower(unsigned char c) { return (c >= 'A' && c <= 'Z') ? char(c + 32) : char(c); }

// Calls f(token) for every token of doc[0, n), lowercased into `scratch`.
template <class F>
inline void for_each_token(const char* doc, int64_t n, std::string& scratch, F&& f) {
  int64_t i = 0;
  while (i < n) {
    while (i < n && !is_word((unsigned char)doc[i])) ++i;
    const int64_t s = i;
    while (i < n && is_word((unsigned char)doc[i])) ++i;
    if (i - s >= 2) {
      scratch.resize(size_t(i - s));
      for (int64_t k = s; k < i; ++k) scratch[size_t(k - s)] = lower((unsigned char)doc[k]);
      f(std::string_view(scratch));
    }
  }
}

int pick_threads(int requested, int64_t n_docs) {
  int t = requested > 0 ? requested : int(std::thread::hardware_concurrency());
  if (t < 1) t = 1;
  if (t > 64) t = 64;
  const int64_t cap = std::max<int64_t>(1, n_docs / 64);
  return int(std::min<int64_t>(t, cap));
}

template <class F>
void parallel_ranges(int64_t n, int threads, F&& f) {
  if (threads <= 1) { f(0, int64_t(0), n); return; }
  std::vector<std::thread> pool;
  const int64_t per = (n + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t a = t * per, b = std::min(n, a + per);
    if (a >= b) break;
    pool.emplace_back([&f, t, a, b] { f(t, a, b); });
  }
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

void gfr_free(void* p) { std::free(p); }

// Sorted unique tokens of the documents, minus the stop words, as one '\n'-joined
// malloc'ed buffer (*out, *out_len bytes, *n_terms terms).  Returns 0 on success.
int gfr_vocabulary(const char* buf, const int64_t* offs, int64_t n_docs, const char* stop_buf,
                   const int64_t* stop_offs, int64_t n_stop, int n_threads, char** out,
                   int64_t* out_len, int64_t* n_terms) {
  std::unordered_set<std::string_view> stop;
  for (int64_t i = 0; i < n_stop; ++i)
    stop.emplace(stop_buf + stop_offs[i], size_t(stop_offs[i + 1] - stop_offs[i]));
  const int T = pick_threads(n_threads, n_docs);
  // per thread: the distinct tokens seen, as views into a node-stable arena
  std::vector<std::unordered_set<std::string_view>> part(static_cast<size_t>(T));
  std::vector<std::deque<std::string>> arena(static_cast<size_t>(T));
  parallel_ranges(n_docs, T, [&](int t, int64_t a, int64_t b) {
    std::string scratch;
    auto& mine = part[size_t(t)];
    auto& store = arena[size_t(t)];
    for (int64_t d = a; d < b; ++d)
      for_each_token(buf + offs[d], offs[d + 1] - offs[d], scratch, [&](std::string_view tok) {
        if (mine.find(tok) != mine.end() || stop.find(tok) != stop.end()) return;
        store.emplace_back(tok);
        mine.emplace(store.back());
      });
  });
  std::unordered_set<std::string_view> all;
  for (auto& p : part) all.insert(p.begin(), p.end());
  std::vector<std::string_view> terms(all.begin(), all.end());
  std::sort(terms.begin(), terms.end());
  int64_t bytes = 0;
  for (auto& s : terms) bytes += int64_t(s.size()) + 1;
  char* o = static_cast<char*>(std::malloc(size_t(bytes > 0 ? bytes : 1)));
  if (!o) return -1;
  int64_t p = 0;
  for (auto& s : terms) {
    std::memcpy(o + p, s.data(), s.size());
    p += int64_t(s.size());
    o[p++] = '\n';
  }
  *out = o;
  *out_len = bytes;
  *n_terms = int64_t(terms.size());
  return 0;
}

// Document-term counts over a fixed vocabulary (term i -> column cols[i]) as CSR:
// indptr [n_docs + 1] caller-allocated; *indices (int32) and *data (float32) are
// malloc'ed (free with gfr_free); column indices sorted within each row.
int gfr_vectorize(const char* buf, const int64_t* offs, int64_t n_docs, const char* voc_buf,
                  const int64_t* voc_offs, const int32_t* cols, int64_t n_vocab, int n_threads,
                  int64_t* indptr, int32_t** indices, float** data, int64_t* nnz) {
  std::unordered_map<std::string_view, int32_t> vocab;
  vocab.reserve(size_t(n_vocab) * 2);
  for (int64_t i = 0; i < n_vocab; ++i)
    vocab.emplace(std::string_view(voc_buf + voc_offs[i], size_t(voc_offs[i + 1] - voc_offs[i])),
                  cols[i]);
  const int T = pick_threads(n_threads, n_docs);
  std::vector<std::vector<int32_t>> row_cols(static_cast<size_t>(n_docs));
  std::vector<std::vector<float>> row_vals(static_cast<size_t>(n_docs));
  parallel_ranges(n_docs, T, [&](int, int64_t a, int64_t b) {
    std::string scratch;
    std::vector<int32_t> hits;
    for (int64_t d = a; d < b; ++d) {
      hits.clear();
      for_each_token(buf + offs[d], offs[d + 1] - offs[d], scratch, [&](std::string_view tok) {
        auto it = vocab.find(tok);
        if (it != vocab.end()) hits.push_back(it->second);
      });
      std::sort(hits.begin(), hits.end());
      auto& rc = row_cols[size_t(d)];
      auto& rv = row_vals[size_t(d)];
      for (size_t k = 0; k < hits.size();) {
        size_t e = k;
        while (e < hits.size() && hits[e] == hits[k]) ++e;
        rc.push_back(hits[k]);
        rv.push_back(float(e - k));
        k = e;
      }
    }
  });
  indptr[0] = 0;
  for (int64_t d = 0; d < n_docs; ++d) indptr[d + 1] = indptr[d] + int64_t(row_cols[size_t(d)].size());
  const int64_t total = indptr[n_docs];
  int32_t* ix = static_cast<int32_t*>(std::malloc(size_t(total > 0 ? total : 1) * sizeof(int32_t)));
  float* dv = static_cast<float*>(std::malloc(size_t(total > 0 ? total : 1) * sizeof(float)));
  if (!ix || !dv) { std::free(ix); std::free(dv); return -1; }
  parallel_ranges(n_docs, T, [&](int, int64_t a, int64_t b) {
    for (int64_t d = a; d < b; ++d) {
      const auto& rc = row_cols[size_t(d)];
      const auto& rv = row_vals[size_t(d)];
      std::copy(rc.begin(), rc.end(), ix + indptr[d]);
      std::copy(rv.begin(), rv.end(), dv + indptr[d]);
    }
  });
  *indices = ix;
  *data = dv;
  *nnz = total;
  return 0;
}

}  // extern "C"
