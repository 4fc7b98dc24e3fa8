// Window table read-out (engine/ingest.py WindowTable): the brain keeps every
// canary job's current / baseline window as a dense [slots, columns] grid --
// one slot per key series (pod), one column per query step -- filled
// incrementally from batched query_range answers.  Scoring wants, per
// (job, metric) row, the window's samples pod-major and time-minor with the
// missing steps squeezed out (what one per-job query_range returns,
// concatenated), left-aligned and NaN-padded to the group's width: this
// packs any subset of rows straight from the grid, on a few threads.
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
