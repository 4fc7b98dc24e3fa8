// Host-side sanitizer driver for the native runtime (ASan + UBSan, or TSan):
// every prefix of valid query_range documents (truncation must never read past
// the buffer), deterministic byte mutations, and the threaded count / pack
// entry points.  Built and run by tools/sanitize_host.sh and
// tests/test_native_sanitizers.py.  Exit code 0 = clean.
#include "../promparse.cpp"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static const char* kDocs[] = {
    R"({"status":"success","data":{"resultType":"matrix","result":[{"metric":{"pod":"a-1"},"values":[[1760000000,"1.5"],[1760000060,"2.5e1"],[1760000120,"NaN"]]},{"metric":{},"values":[[1760000000.5,"-3"]]}]}})",
    R"({"status":"success","data":{"resultType":"vector","result":[{"metric":{"app":"x"},"value":[1760000000,"7"]}]}})",
    R"({"status":"error","errorType":"bad_data","error":"parse error"})",
    R"({"status":"success","data":{"resultType":"matrix","result":[]}})",
};

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_rand() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

static int parse_exact(const std::string& s) {
  // heap copy of exactly s.size() bytes: any over-read is an ASan report
  std::vector<char> buf(s.begin(), s.end());
  const char* p = buf.empty() ? nullptr : buf.data();
  int64_t ns = 0, np = 0;
  int rc = fm_prom_count(p, (int64_t)buf.size(), &ns, &np);
  if (rc == 0 && ns >= 0 && np >= 0) {
    std::vector<double> t((size_t)np + 1);
    std::vector<float> v((size_t)np + 1);
    std::vector<int64_t> off((size_t)ns + 1), spans((size_t)ns * 2 + 2);
    int rc2 = fm_prom_fill(p, (int64_t)buf.size(), t.data(), v.data(), off.data(), spans.data());
    if (rc2 != 0) return 100;
    if (off[(size_t)ns] != np) return 101;
  }
  return rc;
}

int main() {
  int checked = 0;
  for (const char* d : kDocs) {
    const std::string s(d);
    for (size_t n = 0; n <= s.size(); ++n) { parse_exact(s.substr(0, n)); ++checked; }
    for (int m = 0; m < 2000; ++m) {
      std::string t = s;
      const int edits = 1 + (int)(next_rand() % 4);
      for (int e = 0; e < edits; ++e) {
        const size_t pos = (size_t)(next_rand() % t.size());
        const char c = "\"[]{},:0123456789.eE-+ aNn\\"[next_rand() % 27];
        switch (next_rand() % 3) {
          case 0: t[pos] = c; break;
          case 1: t.insert(pos, 1, c); break;
          default: t.erase(pos, 1); if (t.empty()) t = "{"; break;
        }
      }
      parse_exact(t);
      ++checked;
    }
  }
  if (parse_exact(kDocs[0]) != 0) { std::fprintf(stderr, "valid document rejected\n"); return 2; }
  // threaded entry points
  std::vector<std::string> docs(64, kDocs[0]);
  std::vector<const char*> ptrs;
  std::vector<int64_t> lens, ns(64), np(64);
  std::vector<int> rc(64);
  for (auto& d : docs) { ptrs.push_back(d.data()); lens.push_back((int64_t)d.size()); }
  fm_prom_count_many(ptrs.data(), lens.data(), 64, ns.data(), np.data(), rc.data(), 8);
  for (int i = 0; i < 64; ++i)
    if (rc[i] != 0 || ns[i] != 2 || np[i] != 4) { std::fprintf(stderr, "count_many mismatch %d\n", i); return 3; }
  std::vector<std::vector<float>> rows(97);
  std::vector<const float*> src;
  std::vector<int64_t> rl;
  for (size_t r = 0; r < rows.size(); ++r) {
    rows[r].resize(r * 3 % 50);
    for (size_t i = 0; i < rows[r].size(); ++i) rows[r][i] = (float)i;
    src.push_back(rows[r].data());
    rl.push_back((int64_t)rows[r].size());
  }
  std::vector<float> dst(97 * 44);
  fm_pack_right(src.data(), rl.data(), 97, dst.data(), 44, 40, 8);
  for (size_t r = 0; r < rows.size(); ++r) {
    const int64_t n = rl[r] < 40 ? rl[r] : 40;
    if (n > 0 && dst[r * 44 + 39] != rows[r].back()) { std::fprintf(stderr, "pack mismatch %zu\n", r); return 4; }
  }
  std::printf("promparse sanitizer driver: %d documents checked, clean\n", checked);
  return 0;
}
