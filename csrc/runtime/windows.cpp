// Window table read-out (engine/ingest.py WindowTable): the brain keeps every
// canary job's current / baseline window as a dense [slots, columns] grid --
// one slot per key series (pod), one column per query step -- filled
// incrementally from batched query_range answers.  Scoring wants, per
// (job, metric) row, the window's samples pod-major and time-minor with the
// missing steps squeezed out (what one per-job query_range returns,
// concatenated), left-aligned and NaN-padded to the group's width: this
// packs any subset of rows straight from the grid, on a few threads.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

FM_API void fm_window_pack(const float* V, int64_t ld, const int64_t* slot0, const int64_t* nslot,
                           const int64_t* ncol, const double* start, const double* step, int64_t R, float* out_v,
                           double* out_t, int64_t n, int64_t* lens, int threads) {
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    for (int64_t r = next.fetch_add(64); r < R; r = next.fetch_add(64)) {
      const int64_t r1 = r + 64 < R ? r + 64 : R;
      for (int64_t i = r; i < r1; ++i) {
        float* ov = out_v + i * n;
        double* ot = out_t ? out_t + i * n : nullptr;
        int64_t k = 0;
        const int64_t s0 = slot0[i];
        if (s0 >= 0) {
          const int64_t nc = ncol[i] < ld ? ncol[i] : ld;
          const double t0 = start[i], dt = step[i];
          for (int64_t s = 0; s < nslot[i] && k < n; ++s) {
            const float* row = V + (s0 + s) * ld;
            for (int64_t c = 0; c < nc && k < n; ++c) {
              const float x = row[c];
              if (std::isnan(x)) continue;
              ov[k] = x;
              if (ot) ot[k] = t0 + dt * (double)c;
              ++k;
            }
          }
        }
        lens[i] = k;
        for (int64_t j = k; j < n; ++j) {
          ov[j] = NAN;
          if (ot) ot[j] = NAN;
        }
      }
    }
  };
  int nt = threads > 0 ? threads : 1;
  if (R < 2048) nt = 1;
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}

// The time of the k[i]-th packed sample of window row i (fm_window_pack's
// order: pods slot by slot, time within a pod, NaNs squeezed out), NaN past
// the row's samples -- what a verdict needs of the packed times, for its
// anomalous points only, instead of a [R, n] float64 time matrix per cycle.
FM_API void fm_window_times(const float* V, int64_t ld, const int64_t* slot0, const int64_t* nslot,
                            const int64_t* ncol, const double* start, const double* step, int64_t m,
                            const int64_t* k, double* out) {
  for (int64_t i = 0; i < m; ++i) {
    double t = NAN;
    const int64_t s0 = slot0[i];
    if (s0 >= 0 && k[i] >= 0) {
      const int64_t nc = ncol[i] < ld ? ncol[i] : ld;
      int64_t seen = 0;
      for (int64_t s = 0; s < nslot[i] && std::isnan(t); ++s) {
        const float* row = V + (s0 + s) * ld;
        for (int64_t c = 0; c < nc; ++c) {
          if (std::isnan(row[c])) continue;
          if (seen++ == k[i]) {
            t = start[i] + step[i] * (double)c;
            break;
          }
        }
      }
    }
    out[i] = t;
  }
}

// Write one fetch round's batched answers into the grid (WindowTable.apply
// for every request at once).  Request r covers the windows
// ws[woff[r] .. woff[r+1]) -- each takes its own grid range [lo, hi] (same
// positions) -- and the answer series [soff[r] .. soff[r+1]) of the
// concatenated keyed answers (key hash kh[s], samples t / v[off[s] ..
// off[s+1])).  A series feeds every slot of the request's windows whose key
// hash it carries; a sample lands in column rint((t - start - toff) / step)
// when it lies in the window's [lo, hi], on its phase and inside the window.
// toff (the sample phase of a window, NaN until seen) is set from the first
// sample a window receives.  A window belongs to one request of a round, so
// requests run in parallel without sharing a row.  dup[w] is set when two
// series of one answer carry the same key value of window w (extra labels:
// the table has one slot per key value, so such a window cannot hold them).
FM_API void fm_window_apply(float* V, int64_t ld, const uint64_t* khash, const double* start, const double* step,
                            double* toff, const int64_t* ncol, const int64_t* slot0, const int64_t* nslot,
                            int64_t R, const int64_t* woff, const int64_t* ws, const double* lo, const double* hi,
                            const int64_t* soff, const uint64_t* kh, const int64_t* off, const double* t,
                            const float* v, uint8_t* dup, int threads) {
  struct Slot {
    uint64_t h;
    int64_t slot;
    int64_t w;    // window id
    int64_t pos;  // position of the window in ws / lo / hi
  };
  std::atomic<int64_t> next{0};
  auto work = [&]() {
    std::vector<Slot> sl;
    for (int64_t r = next++; r < R; r = next++) {
      sl.clear();
      for (int64_t p = woff[r]; p < woff[r + 1]; ++p) {
        const int64_t w = ws[p];
        for (int64_t k = 0; k < nslot[w]; ++k) sl.push_back({khash[slot0[w] + k], slot0[w] + k, w, p});
      }
      std::sort(sl.begin(), sl.end(), [](const Slot& a, const Slot& b) { return a.h < b.h; });
      std::vector<uint8_t> hit(sl.size(), 0);
      for (int64_t s = soff[r]; s < soff[r + 1]; ++s) {
        auto it = std::lower_bound(sl.begin(), sl.end(), kh[s], [](const Slot& a, uint64_t h) { return a.h < h; });
        for (; it != sl.end() && it->h == kh[s]; ++it) {
          const int64_t w = it->w;
          uint8_t& seen = hit[(size_t)(it - sl.begin())];
          if (seen) dup[w] = 1;
          seen = 1;
          const double st = start[w], sp = step[w];
          const double wlo = lo[it->pos] - 1e-6, whi = hi[it->pos] + 1e-6;
          float* row = V + it->slot * ld;
          for (int64_t j = off[s]; j < off[s + 1]; ++j) {
            const double tj = t[j];
            double d = std::fmod(tj - st, sp);
            if (d < 0) d += sp;
            if (sp - d < 1e-3) d = 0.0;
            if (std::isnan(toff[w])) toff[w] = d;
            const double to = toff[w];
            const int64_t c = (int64_t)std::nearbyint((tj - st - to) / sp);
            if (tj >= wlo && tj <= whi && c >= 0 && c < ncol[w] && std::fabs(d - to) < 1e-3) row[c] = v[j];
          }
        }
      }
    }
  };
  const int T = (int)std::max<int64_t>(1, std::min<int64_t>(threads, R));
  std::vector<std::thread> th;
  for (int k = 1; k < T; ++k) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
}
