// Prometheus text exposition of the brain's gauge table (engine/exporter.py).
//
// At fleet scale rank 0 publishes ~240k gauges (10k services x 8 metrics x
// upper/lower/anomaly, plus HPA scores); building them as Python objects at
// scrape time took seconds and held the GIL against the brain loop.  Here the
// label part of every sample line is rendered once, when its slot is created
// (``prefix``: `name{namespace="..",app=".."} `), and a scrape only formats
// the values: shortest round-trip decimal (std::to_chars), Prometheus'
// NaN / +Inf / -Inf spellings, one line per slot in the caller's order.  The
// call runs without the GIL (ctypes) on a few threads.
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

namespace {

inline char* put_value(char* o, double v) {
  if (std::isnan(v)) { std::memcpy(o, "NaN", 3); return o + 3; }
  if (std::isinf(v)) { std::memcpy(o, v > 0 ? "+Inf" : "-Inf", 4); return o + 4; }
  auto r = std::to_chars(o, o + 32, v);
  return r.ptr;
}

// Renders lines [lo, hi) of ``order`` into ``o``; returns the end pointer.
char* render_range(const char* prefix, const int64_t* poff, const int64_t* order, int64_t lo, int64_t hi,
                   const double* vals, char* o) {
  for (int64_t i = lo; i < hi; ++i) {
    const int64_t s = order ? order[i] : i;
    const int64_t a = poff[s], b = poff[s + 1];
    std::memcpy(o, prefix + a, static_cast<size_t>(b - a));
    o += b - a;
    o = put_value(o, vals[s]);
    *o++ = '\n';
  }
  return o;
}

}  // namespace

// Upper bound of the rendered size of ``n`` lines (caller allocates).
FM_API int64_t fm_render_bound(const int64_t* poff, const int64_t* order, int64_t n) {
  int64_t tot = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = order ? order[i] : i;
    tot += poff[s + 1] - poff[s] + 33;
  }
  return tot;
}

// Writes `prefix[order[i]] value\n` for i < n into ``out`` (capacity ``cap``,
// at least fm_render_bound); returns the number of bytes written, -1 if
// ``cap`` is too small.
FM_API int64_t fm_render_lines(const char* prefix, const int64_t* poff, const int64_t* order, int64_t n,
                               const double* vals, char* out, int64_t cap, int threads) {
  if (n <= 0) return 0;
  if (cap < fm_render_bound(poff, order, n)) return -1;
  threads = threads < 1 ? 1 : threads;
  if (threads == 1 || n < 2048) {
    return render_range(prefix, poff, order, 0, n, vals, out) - out;
  }
  // each thread formats its chunk in place at the chunk's worst-case offset
  // inside ``out`` (no scratch allocation), then the chunks are slid down
  // back to back
  const int64_t per = (n + threads - 1) / threads;
  std::vector<int64_t> start(threads + 1, 0), used(threads, 0);
  for (int t = 0; t < threads; ++t) {
    const int64_t lo = t * per < n ? t * per : n, hi = lo + per < n ? lo + per : n;
    int64_t bound = 0;
    for (int64_t i = lo; i < hi; ++i) {
      const int64_t s = order ? order[i] : i;
      bound += poff[s + 1] - poff[s] + 33;
    }
    start[t + 1] = start[t] + bound;
  }
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) {
    pool.emplace_back([&, t] {
      const int64_t lo = t * per < n ? t * per : n, hi = lo + per < n ? lo + per : n;
      used[t] = render_range(prefix, poff, order, lo, hi, vals, out + start[t]) - (out + start[t]);
    });
  }
  used[0] = render_range(prefix, poff, order, 0, per < n ? per : n, vals, out) - out;
  for (auto& th : pool) th.join();
  char* o = out + used[0];
  for (int t = 1; t < threads; ++t) {
    if (used[t]) std::memmove(o, out + start[t], static_cast<size_t>(used[t]));
    o += used[t];
  }
  return o - out;
}
