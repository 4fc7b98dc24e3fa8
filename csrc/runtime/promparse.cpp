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
#include <charconv>
#include <system_error>
#include <cmath>
#include <cstdint>
#include <cstdio>
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
  // in place, std::from_chars (no locale, no allocation); Prometheus' "NaN",
  // "+Inf", "-Inf" spellings: from_chars reads "NaN" / "Inf" / "-Inf" but not
  // a leading '+', which is skipped first.
  c.ws();
  const bool quoted = c.p < c.e && *c.p == '"';
  if (quoted) ++c.p;
  const char* s = c.p;
  if (s < c.e && *s == '+') ++s;
  double v = NAN;
  const auto r = std::from_chars(s, c.e, v);
  if (r.ec != std::errc() || r.ptr == s) {
    // a spelling from_chars does not take (e.g. a hex float): strtod, bounded by
    // the document's closing brace
    char* end = nullptr;
    v = std::strtod(c.p, &end);
    if (end == c.p || end > c.e) { c.ok = false; return NAN; }
    c.p = end;
  } else {
    c.p = r.ptr;
  }
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
  // keyed mode: FNV-1a 64 of the decoded value of label `key` per series
  // (0 when the series has no such label)
  const char* key = nullptr;
  int64_t keylen = 0;
  uint64_t* key_hash = nullptr;
};

constexpr uint64_t kFnvBasis = 1469598103934665603ull;
constexpr uint64_t kFnvPrime = 1099511628211ull;

inline uint64_t fnv_byte(uint64_t h, unsigned char b) { return (h ^ b) * kFnvPrime; }

int hexval(char ch) {
  if (ch >= '0' && ch <= '9') return ch - '0';
  if (ch >= 'a' && ch <= 'f') return ch - 'a' + 10;
  if (ch >= 'A' && ch <= 'F') return ch - 'A' + 10;
  return -1;
}

bool read_hex4(Cursor& c, uint32_t& u) {
  if (c.e - c.p < 4) return false;
  u = 0;
  for (int i = 0; i < 4; ++i) {
    const int h = hexval(c.p[i]);
    if (h < 0) return false;
    u = (u << 4) | (uint32_t)h;
  }
  c.p += 4;
  return true;
}

uint64_t fnv_codepoint(uint64_t h, uint32_t cp) {
  if (cp < 0x80) return fnv_byte(h, (unsigned char)cp);
  if (cp < 0x800) {
    h = fnv_byte(h, (unsigned char)(0xC0 | (cp >> 6)));
    return fnv_byte(h, (unsigned char)(0x80 | (cp & 0x3F)));
  }
  if (cp < 0x10000) {
    h = fnv_byte(h, (unsigned char)(0xE0 | (cp >> 12)));
    h = fnv_byte(h, (unsigned char)(0x80 | ((cp >> 6) & 0x3F)));
    return fnv_byte(h, (unsigned char)(0x80 | (cp & 0x3F)));
  }
  h = fnv_byte(h, (unsigned char)(0xF0 | (cp >> 18)));
  h = fnv_byte(h, (unsigned char)(0x80 | ((cp >> 12) & 0x3F)));
  h = fnv_byte(h, (unsigned char)(0x80 | ((cp >> 6) & 0x3F)));
  return fnv_byte(h, (unsigned char)(0x80 | (cp & 0x3F)));
}

// hash the decoded UTF-8 bytes of the JSON string at the cursor (JSON escapes
// incl. \uXXXX surrogate pairs decoded), so the hash equals FNV-1a of the
// label value's UTF-8 encoding on the Python side
bool hash_string(Cursor& c, uint64_t& out) {
  c.ws();
  if (c.p >= c.e || *c.p != '"') return false;
  ++c.p;
  uint64_t h = kFnvBasis;
  while (c.p < c.e) {
    const char ch = *c.p;
    if (ch == '"') { ++c.p; out = h; return true; }
    if (ch != '\\') { h = fnv_byte(h, (unsigned char)ch); ++c.p; continue; }
    if (c.e - c.p < 2) return false;
    const char e = c.p[1];
    c.p += 2;
    switch (e) {
      case '"': h = fnv_byte(h, '"'); break;
      case '\\': h = fnv_byte(h, '\\'); break;
      case '/': h = fnv_byte(h, '/'); break;
      case 'b': h = fnv_byte(h, '\b'); break;
      case 'f': h = fnv_byte(h, '\f'); break;
      case 'n': h = fnv_byte(h, '\n'); break;
      case 'r': h = fnv_byte(h, '\r'); break;
      case 't': h = fnv_byte(h, '\t'); break;
      case 'u': {
        uint32_t u;
        if (!read_hex4(c, u)) return false;
        if (u >= 0xD800 && u < 0xDC00 && c.e - c.p >= 6 && c.p[0] == '\\' && c.p[1] == 'u') {
          Cursor d{c.p + 2, c.e};
          uint32_t lo;
          if (read_hex4(d, lo) && lo >= 0xDC00 && lo < 0xE000) {
            u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
            c.p = d.p;
          }
        }
        h = fnv_codepoint(h, u);
        break;
      }
      default: return false;
    }
  }
  return false;
}

// the "metric" object in keyed mode: hash the value of label s.key
bool parse_metric_keyed(Cursor& c, Sink& s, uint64_t& kh) {
  kh = 0;
  if (!c.eat('{')) return false;
  if (c.eat('}')) return true;
  for (;;) {
    c.ws();
    if (c.p >= c.e || *c.p != '"') return false;
    const char* ks = c.p + 1;
    if (!skip_string(c)) return false;
    const int64_t klen = (c.p - 1) - ks;
    if (!c.eat(':')) return false;
    if (klen == s.keylen && std::memcmp(ks, s.key, (size_t)klen) == 0) {
      if (!hash_string(c, kh)) return false;
    } else if (!skip_value(c)) {
      return false;
    }
    if (c.eat(',')) continue;
    return c.eat('}');
  }
}

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
    uint64_t kh = 0;
    if (s.offsets) s.offsets[s.nseries] = s.npoints;
    if (!c.eat('}')) {
      for (;;) {
        std::string k;
        if (!read_key(c, k) || !c.eat(':')) return false;
        if (k == "metric") {
          c.ws();
          lb = c.p - base;
          if (s.key) {
            if (!parse_metric_keyed(c, s, kh)) return false;
          } else if (!skip_value(c)) {
            return false;
          }
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
    if (s.key_hash) s.key_hash[s.nseries] = kh;
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

// Keyed parse (the brain's batched queries: one response answers many jobs,
// split by the value of one label, e.g. `pod` or `app`).  Count, then fill:
// key_hash[i] = FNV-1a 64 of series i's decoded `key` label value (0: absent).
// The GIL is released by ctypes for the duration of the call, so the fetch
// threads parse their responses in parallel.
FM_API int fm_prom_keyed_count(const char* buf, int64_t len, const char* key, int64_t keylen, int64_t* nseries,
                               int64_t* npoints) {
  Sink s;
  s.key = key;
  s.keylen = keylen;
  int rc = parse_doc(buf, len, s);
  *nseries = s.nseries;
  *npoints = s.npoints;
  return rc;
}

FM_API int fm_prom_keyed_fill(const char* buf, int64_t len, const char* key, int64_t keylen, double* times,
                              float* values, int64_t* offsets, uint64_t* key_hash) {
  Sink s;
  s.key = key;
  s.keylen = keylen;
  s.times = times;
  s.values = values;
  s.offsets = offsets;
  s.key_hash = key_hash;
  if (offsets) offsets[0] = 0;
  return parse_doc(buf, len, s);
}

// FNV-1a 64 of n strings packed in buf at [off[i], off[i+1]) (UTF-8 bytes).
FM_API void fm_fnv1a_many(const char* buf, const int64_t* off, int64_t n, uint64_t* out) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h = kFnvBasis;
    for (int64_t j = off[i]; j < off[i + 1]; ++j) h = fnv_byte(h, (unsigned char)buf[j]);
    out[i] = h;
  }
}

// The other direction (demo/promserver.py, the fake Prometheus the HTTP benches
// and tests talk to): a query_range matrix response from a dense
// [nseries, npts] float32 grid on the times t0 + k*step; NaN samples are left
// out, as Prometheus leaves out steps without a sample.  Series i's "metric"
// object is the pre-rendered JSON at labels[loff[i], loff[i+1]).  Returns the
// bytes written, or -1 when cap is too small (bound: fm_prom_format_bound).
FM_API int64_t fm_prom_format_bound(int64_t nseries, int64_t npts, int64_t label_bytes) {
  return 64 + label_bytes + nseries * 32 + nseries * npts * 48;
}

FM_API int64_t fm_prom_format(int64_t nseries, const char* labels, const int64_t* loff, double t0, double step,
                              int64_t npts, const float* values, char* out, int64_t cap) {
  char* p = out;
  char* const e = out + cap;
  auto put = [&](const char* s, size_t n) -> bool {
    if (e - p < (ptrdiff_t)n) return false;
    std::memcpy(p, s, n);
    p += n;
    return true;
  };
  static const char head[] = "{\"status\":\"success\",\"data\":{\"resultType\":\"matrix\",\"result\":[";
  if (!put(head, sizeof(head) - 1)) return -1;
  for (int64_t i = 0; i < nseries; ++i) {
    if (i && !put(",", 1)) return -1;
    if (!put("{\"metric\":", 10) || !put(labels + loff[i], (size_t)(loff[i + 1] - loff[i])) ||
        !put(",\"values\":[", 11))
      return -1;
    bool first = true;
    const float* row = values + i * npts;
    for (int64_t k = 0; k < npts; ++k) {
      const float v = row[k];
      if (std::isnan(v)) continue;
      if (e - p < 48) return -1;
      if (!first) *p++ = ',';
      first = false;
      *p++ = '[';
      const double t = t0 + step * (double)k;
      const double tr = std::nearbyint(t);
      std::to_chars_result r;
      if (t == tr && std::fabs(t) < 9e15) {
        r = std::to_chars(p, e, (long long)tr);
      } else {
        r = std::to_chars(p, e, t, std::chars_format::fixed, 3);
      }
      if (r.ec != std::errc()) return -1;
      p = r.ptr;
      *p++ = ',';
      *p++ = '"';
      if (std::isinf(v)) {
        const char* s = v > 0 ? "+Inf" : "-Inf";
        std::memcpy(p, s, 4);
        p += 4;
      } else {
        r = std::to_chars(p, e, v);          // shortest text that reads back as this float
        if (r.ec != std::errc()) return -1;
        p = r.ptr;
      }
      *p++ = '"';
      *p++ = ']';
    }
    if (!put("]}", 2)) return -1;
  }
  if (!put("]}}", 3)) return -1;
  return p - out;
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

// Finite values per row of a [R, n] float32 matrix with row stride ld (the
// sliding windows' point counts, one pass instead of numpy's mask + sum).
FM_API void fm_count_finite(const float* a, int64_t R, int64_t n, int64_t ld, int64_t* out) {
  for (int64_t r = 0; r < R; ++r) {
    const float* p = a + r * ld;
    int64_t c = 0;
    for (int64_t i = 0; i < n; ++i) c += std::isfinite(p[i]) ? 1 : 0;
    out[r] = c;
  }
}

// The host half of a sliding-grid write (engine/resident.py
// write_sliding_flat), one pass instead of ~15 numpy passes: samples (row r,
// time t, value v) whose grid column c = round((t - t0) / step) lies in the
// window [ws, e) and whose value is finite go out as (r * width + c, v) into
// out_flat / out_v; per row the finite count gains the samples newer than the
// row's newest column BEFORE this batch (a re-sent sample counts once) and
// last_t becomes the newest time.  Returns the samples written out.
FM_API int64_t fm_sliding_prep(const int64_t* r, const double* t, const float* v, int64_t n, double t0, double step,
                               int64_t ws, int64_t e, int64_t width, double* last_t, int64_t* nfin,
                               int64_t* out_flat, float* out_v, unsigned char* inc) {
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    inc[i] = 0;
    if (!std::isfinite(v[i])) continue;
    const int64_t c = (int64_t)std::nearbyint((t[i] - t0) / step);
    if (c < ws || c >= e) continue;
    const double lt = last_t[r[i]];
    const int64_t prev = std::isfinite(lt) ? (int64_t)std::nearbyint((lt - t0) / step) : -1;
    inc[i] = c > prev ? 2 : 1;                 // 1: in the window, 2: and a new column
    out_flat[k] = r[i] * width + c;
    out_v[k] = v[i];
    ++k;
  }
  for (int64_t i = 0; i < n; ++i) {
    if (!inc[i]) continue;
    if (inc[i] == 2) nfin[r[i]] += 1;
    if (!(last_t[r[i]] >= t[i])) last_t[r[i]] = t[i];
  }
  return k;
}

// Host ring of the newest grid columns of every sliding row
// (engine/fastpath.py _ring_write): clear the slots of the columns
// (top_old, top_new] in every row, then store the samples whose column is
// inside the ring (finite values only).  ring [nrows, width] float32,
// slot = column mod width.
FM_API void fm_ring_write(float* ring, int64_t nrows, int64_t width, int64_t top_old, int64_t top_new,
                          const int64_t* r, const double* t, const float* v, int64_t n, double step) {
  if (top_new > top_old) {
    const int64_t k = top_new - top_old >= width ? width : top_new - top_old;
    for (int64_t row = 0; row < nrows; ++row) {
      float* p = ring + row * width;
      for (int64_t c = top_new - k + 1; c <= top_new; ++c) p[((c % width) + width) % width] = NAN;
    }
  }
  const int64_t lo = top_new - width;
  for (int64_t i = 0; i < n; ++i) {
    if (!std::isfinite(v[i])) continue;
    const int64_t c = (int64_t)std::nearbyint(t[i] / step);
    if (c <= lo || c > top_new) continue;
    ring[r[i] * width + ((c % width) + width) % width] = v[i];
  }
}
