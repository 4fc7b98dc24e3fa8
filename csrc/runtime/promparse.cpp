// Native ingest runtime: Prometheus query_range (matrix) response parser and a
// right-aligned row packer.
//
// The brain fetches one JSON document per (job, metric, category); at fleet
// scale that is ~10^4-10^5 documents per tick, each up to 10,080 samples.
// Parsing them with Python's json module dominates the host side, so this is a
// single-pass scanner that writes (time, value) pairs straight into caller-
// allocated arrays (two calls: count, then fill), plus a multi-threaded batch
// entry point.  Labels ("metric" objects) are returned as byte spans for the
// caller to decode (they are tiny).
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

namespace {

struct Cursor {
  const char* p;
  const char* e;
  bool ok = true;
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p; }
  bool eat(char c) { ws(); if (p < e && *p == c) { ++p; return true; } return false; }
  char peek() { ws(); return p < e ? *p : '\0'; }
};

// skip a JSON string starting at '"'
bool skip_string(Cursor& c) {
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  while (c.p < c.e) {
    if (*c.p == '\\') { c.p += 2; continue; }
    if (*c.p == '"') { ++c.p; return true; }
    ++c.p;
  }
  return false;
}

bool skip_value(Cursor& c);

bool skip_container(Cursor& c, char open, char close) {
  if (!c.eat(open)) return false;
  if (c.eat(close)) return true;
  for (;;) {
    if (open == '{') {
      c.ws();
      if (!skip_string(c)) return false;
      if (!c.eat(':')) return false;
    }
    if (!skip_value(c)) return false;
    if (c.eat(',')) continue;
    return c.eat(close);
  }
}

bool skip_value(Cursor& c) {
  char ch = c.peek();
  if (ch == '"') return skip_string(c);
  if (ch == '{') return skip_container(c, '{', '}');
  if (ch == '[') return skip_container(c, '[', ']');
  while (c.p < c.e && *c.p != ',' && *c.p != '}' && *c.p != ']') ++c.p;  // number / literal
  return true;
}

// read a JSON string's raw contents (no escapes expected in keys/numbers)
bool read_key(Cursor& c, std::string& out) {
  c.ws();
  if (c.p >= c.e || *c.p != '"') return false;
  const char* s = ++c.p;
  while (c.p < c.e && *c.p != '"') { if (*c.p == '\\') ++c.p; ++c.p; }
  if (c.p >= c.e) return false;
  out.assign(s, c.p - s);
  ++c.p;
  return true;
}

double parse_number_token(Cursor& c) {
  // in place: strtod stops at the closing quote / ',' / ']' and understands
  // Prometheus' "NaN", "+Inf", "-Inf" spellings; the document buffer is
  // terminated by its closing brace so strtod cannot run off the end.
  c.ws();
  const bool quoted = c.p < c.e && *c.p == '"';
  if (quoted) ++c.p;
  char* end = nullptr;
  const double v = std::strtod(c.p, &end);
  if (end == c.p || end > c.e) { c.ok = false; return NAN; }
  c.p = end;
  if (quoted) {
    if (c.p < c.e && *c.p == '"') ++c.p; else c.ok = false;
  }
  return v;
}

struct Sink {
  // counting mode when times == nullptr
  double* times = nullptr;
  float* values = nullptr;
  int64_t* offsets = nullptr;     // [nseries + 1]
  int64_t* label_spans = nullptr; // [nseries, 2] (begin, end) byte offsets of the "metric" object
  int64_t nseries = 0, npoints = 0;
};

bool parse_pairs(Cursor& c, Sink& s, bool single) {
  auto pair = [&]() -> bool {
    if (!c.eat('[')) return false;
    double t = parse_number_token(c);
    if (!c.eat(',')) return false;
    double v = parse_number_token(c);
    if (!c.eat(']')) return false;
    if (s.times) { s.times[s.npoints] = t; s.values[s.npoints] = (float)v; }
    ++s.npoints;
    return c.ok;
  };
  if (single) return pair();
  if (!c.eat('[')) return false;
  if (c.eat(']')) return true;
  for (;;) {
    if (!pair()) return false;
    if (c.eat(',')) continue;
    return c.eat(']');
  }
}

bool parse_result_array(Cursor& c, const char* base, Sink& s) {
  if (!c.eat('[')) return false;
  if (c.eat(']')) return true;
  for (;;) {
    if (!c.eat('{')) return false;
    int64_t lb = -1, le = -1;
    if (s.offsets) s.offsets[s.nseries] = s.npoints;
    if (!c.eat('}')) {
      for (;;) {
        std::string k;
        if (!read_key(c, k) || !c.eat(':')) return false;
        if (k == "metric") {
          c.ws();
          lb = c.p - base;
          if (!skip_value(c)) return false;
          le = c.p - base;
        } else if (k == "values") {
          if (!parse_pairs(c, s, false)) return false;
        } else if (k == "value") {
          if (!parse_pairs(c, s, true)) return false;
        } else if (!skip_value(c)) {
          return false;
        }
        if (c.eat(',')) continue;
        if (!c.eat('}')) return false;
        break;
      }
    }
    if (s.label_spans) { s.label_spans[2 * s.nseries] = lb; s.label_spans[2 * s.nseries + 1] = le; }
    ++s.nseries;
    if (s.offsets) s.offsets[s.nseries] = s.npoints;
    if (c.eat(',')) continue;
    return c.eat(']');
  }
}

// returns 0 ok, 1 status != success, 2 malformed
int parse_doc(const char* buf, int64_t len, Sink& s) {
  Cursor c{buf, buf + len};
  if (!c.eat('{')) return 2;
  bool success = false, have_result = false;
  for (;;) {
    std::string k;
    if (!read_key(c, k) || !c.eat(':')) return 2;
    if (k == "status") {
      std::string v;
      if (!read_key(c, v)) return 2;
      success = (v == "success");
    } else if (k == "data") {
      if (!c.eat('{')) return 2;
      if (!c.eat('}')) {
        for (;;) {
          std::string dk;
          if (!read_key(c, dk) || !c.eat(':')) return 2;
          if (dk == "result") {
            if (!parse_result_array(c, buf, s)) return 2;
            have_result = true;
          } else if (!skip_value(c)) {
            return 2;
          }
          if (c.eat(',')) continue;
          if (!c.eat('}')) return 2;
          break;
        }
      }
    } else if (!skip_value(c)) {
      return 2;
    }
    if (c.eat(',')) continue;
    if (!c.eat('}')) return 2;
    break;
  }
  if (!success) return 1;
  (void)have_result;
  return c.ok ? 0 : 2;
}

}  // namespace

FM_API int fm_prom_count(const char* buf, int64_t len, int64_t* nseries, int64_t* npoints) {
  Sink s;
  int rc = parse_doc(buf, len, s);
  *nseries = s.nseries;
  *npoints = s.npoints;
  return rc;
}

FM_API int fm_prom_fill(const char* buf, int64_t len, double* times, float* values, int64_t* offsets,
                        int64_t* label_spans) {
  Sink s;
  s.times = times;
  s.values = values;
  s.offsets = offsets;
  s.label_spans = label_spans;
  if (offsets) offsets[0] = 0;
  return parse_doc(buf, len, s);
}

// Batch: count every document on a thread pool (the caller then allocates and
// fills each document).  rc[i] per document.
FM_API void fm_prom_count_many(const char* const* bufs, const int64_t* lens, int64_t n, int64_t* nseries,
                               int64_t* npoints, int* rc, int threads) {
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t i = next++; i < n; i = next++) rc[i] = fm_prom_count(bufs[i], lens[i], &nseries[i], &npoints[i]);
  };
  int nt = threads > 0 ? threads : (int)std::thread::hardware_concurrency();
  if (nt > 64) nt = 64;
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

// Left-align variable-length rows into a padded [nrows, ld] matrix: the newest
// min(len, ncols) samples of every row start at column 0, NaN after.  The
// resident history store keeps static rows this way so a full row has no
// missing sample inside the scored view (the row-stats fast path).
FM_API void fm_pack_left(const float* const* srcs, const int64_t* lens, int64_t nrows, float* dst, int64_t ld,
                         int64_t ncols, int threads) {
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t r = next++; r < nrows; r = next++) {
      float* d = dst + r * ld;
      const int64_t n = lens[r] < ncols ? lens[r] : ncols;
      if (n > 0) std::memcpy(d, srcs[r] + (lens[r] - n), n * sizeof(float));
      for (int64_t i = n; i < ld; ++i) d[i] = NAN;
    }
  };
  int nt = threads > 0 ? threads : 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

// Right-align variable-length rows into a padded [nrows, ld] matrix: the last
// sample of every source row lands in column ncols-1 (the "now" edge), missing
// leading samples are NaN.  Rows longer than ncols keep their newest ncols.
FM_API void fm_pack_right(const float* const* srcs, const int64_t* lens, int64_t nrows, float* dst, int64_t ld,
                          int64_t ncols, int threads) {
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t r = next++; r < nrows; r = next++) {
      float* d = dst + r * ld;
      const int64_t n = lens[r] < ncols ? lens[r] : ncols;
      const int64_t pad = ncols - n;
      for (int64_t i = 0; i < pad; ++i) d[i] = NAN;
      if (n > 0) std::memcpy(d + pad, srcs[r] + (lens[r] - n), n * sizeof(float));
      for (int64_t i = ncols; i < ld; ++i) d[i] = NAN;
    }
  };
  int nt = threads > 0 ? threads : 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}
