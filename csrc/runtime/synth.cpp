// Inner [keys x times] loop of the synthetic Prometheus-shaped source
// (foremast_amd/engine/sources.py SyntheticSource.many): the fake Prometheus
// server and the staged benchmarks generate every window they answer with it,
// and a 10k-job warm restart asks for ~200M samples in its first cycle -- the
// numpy version spent ~30 element passes per sample.  Here one pass per
// sample, rows split over a few threads.
//
// Per-key terms (level, seasonal amplitudes, phase sines, noise-key hash) and
// per-time terms (seasonal sines, the key-independent part of the counter
// hash) are computed by the caller; the arithmetic below follows the numpy
// expression order (fp64 season, fp32 Box-Muller noise) so both paths give the
// same series up to the libm's last-ulp differences.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <thread>
#include <vector>

#define FM_API extern "C" __attribute__((visibility("default")))

namespace {

inline uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

inline float u01(uint32_t h) { return ((float)(h >> 8) + 1.0f) * (1.0f / 16777216.0f); }

}  // namespace

// out[k, i] for K keys x nt times.  mag: per-key fault multiplier or null;
// fault_after: multiplier applies where t >= fault_after.
FM_API void fm_synth_many(int64_t K, int64_t nt, const double* level, const double* ad, const double* aw,
                          const double* sph, const double* cph, const uint32_t* kh, const double* t,
                          const double* swd, const double* cwd, const double* sww, const double* cww,
                          const uint32_t* inner, uint32_t c2, float noise, const double* mag, double fault_after,
                          float* out, int threads) {
  std::atomic<int64_t> next{0};
  const float two_pi = (float)(2.0 * 3.14159265358979323846);
  auto work = [&]() {
    for (int64_t k = next++; k < K; k = next++) {
      const double lv = level[k], a_d = ad[k], a_w = aw[k], sp = sph[k], cp = cph[k];
      const uint32_t kk = kh[k] * 0x9E3779B1u;
      const double mg = mag ? mag[k] : 1.0;
      float* o = out + k * nt;
      for (int64_t i = 0; i < nt; ++i) {
        const double season = 1.0 + a_d * (swd[i] * cp + cwd[i] * sp) + a_w * (sww[i] * cp + cww[i] * sp);
        const uint32_t h1 = hash_u32(kk ^ inner[i]);
        const uint32_t h2 = hash_u32((h1 * 0x9E3779B1u) ^ c2);
        const float nz = std::sqrt(-2.0f * std::log(u01(h1))) * std::cos(two_pi * u01(h2));
        const float f = 1.0f + noise * nz;
        double v = lv * season * (double)f;
        if (mag && t[i] >= fault_after) v *= mg;
        o[i] = (float)std::max(v, 0.0);
      }
    }
  };
  int nt_ = threads > 0 ? threads : 1;
  if (K < 64) nt_ = 1;
  std::vector<std::thread> pool;
  for (int i = 1; i < nt_; ++i) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
}
