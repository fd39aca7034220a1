// Host-side sanitizer harness for csrc/runtime.cpp (ASan + UBSan), run by
// tests/test_native_runtime.py: random ASCII corpora, empty documents, documents
// without tokens, vocabulary and vectorisation with several thread counts.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

extern "C" {
void gfr_free(void*);
int gfr_vocabulary(const char*, const int64_t*, int64_t, const char*, const int64_t*, int64_t, int,
                   char**, int64_t*, int64_t*);
int gfr_vectorize(const char*, const int64_t*, int64_t, const char*, const int64_t*,
                  const int32_t*, int64_t, int, int64_t*, int32_t**, float**, int64_t*);
}

static void pack(const std::vector<std::string>& v, std::string& buf, std::vector<int64_t>& offs) {
  buf.clear();
  offs.assign(1, 0);
  for (auto& s : v) { buf += s; offs.push_back((int64_t)buf.size()); }
}

int main() {
  std::mt19937 rng(7);
  const char* alphabet = "abcXYZ019_ .,;!-'\n\t";
  for (int round = 0; round < 20; ++round) {
    std::vector<std::string> docs(1 + rng() % 300);
    for (auto& d : docs) {
      const int len = rng() % 200;
      for (int i = 0; i < len; ++i) d.push_back(alphabet[rng() % 19]);
    }
    std::string buf, sbuf;
    std::vector<int64_t> offs, soffs;
    pack(docs, buf, offs);
    pack({"the", "and", "abc"}, sbuf, soffs);
    for (int threads : {1, 3, 8}) {
      char* out = nullptr;
      int64_t out_len = 0, n = 0;
      if (gfr_vocabulary(buf.data(), offs.data(), (int64_t)docs.size(), sbuf.data(), soffs.data(), 3,
                         threads, &out, &out_len, &n)) return 1;
      std::vector<std::string> terms;
      std::string cur;
      for (int64_t i = 0; i < out_len; ++i) {
        if (out[i] == '\n') { terms.push_back(cur); cur.clear(); } else cur.push_back(out[i]);
      }
      gfr_free(out);
      if ((int64_t)terms.size() != n) return 2;
      std::string vbuf;
      std::vector<int64_t> voffs;
      pack(terms, vbuf, voffs);
      std::vector<int32_t> cols(terms.size());
      for (size_t i = 0; i < cols.size(); ++i) cols[i] = (int32_t)i;
      std::vector<int64_t> indptr(docs.size() + 1);
      int32_t* ix = nullptr;
      float* dv = nullptr;
      int64_t nnz = 0;
      if (gfr_vectorize(buf.data(), offs.data(), (int64_t)docs.size(), vbuf.data(), voffs.data(),
                        cols.data(), (int64_t)cols.size(), threads, indptr.data(), &ix, &dv, &nnz))
        return 3;
      if (indptr.back() != nnz) return 4;
      for (size_t d = 0; d < docs.size(); ++d)
        for (int64_t k = indptr[d] + 1; k < indptr[d + 1]; ++k)
          if (ix[k] <= ix[k - 1]) return 5;   // sorted, unique columns
      gfr_free(ix);
      gfr_free(dv);
    }
  }
  std::printf("runtime sanitize ok\n");
  return 0;
}
