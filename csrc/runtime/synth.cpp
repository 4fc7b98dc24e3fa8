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
#include <climits>
#include <cstring>
#include <string_view>
#include <thread>
#include <unordered_map>
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

// Fault multipliers of the synthetic source: out[i] = product of mags[j] over
// the fault substrings j contained in key i (each counted once, multiplied in
// j order -- the Python loop's `for sub, m in faults.items(): if sub in key`).
// A restart asks for ~800k keys against ~200 faults.  Each substring of 8+
// bytes is indexed by its RAREST 8-byte window among all substrings' windows
// (fault lists share prefixes like `app="svc`), looked up at every key
// position behind a 16-bit filter, then verified; shorter substrings by a
// plain search.
FM_API void fm_fault_mag(const char* kbuf, const int64_t* koff, int64_t n, const char* sbuf, const int64_t* soff,
                         int64_t nsub, const double* mags, double* out) {
  constexpr int64_t W = 8;
  auto win = [](const char* p) {
    uint64_t h;
    std::memcpy(&h, p, (size_t)W);
    return h;
  };
  auto mix = [](uint64_t h) { return (size_t)((h * 0x9E3779B97F4A7C15ull) >> 48); };
  std::unordered_map<uint64_t, int64_t> freq;
  std::vector<int64_t> shorts;
  for (int64_t j = 0; j < nsub; ++j) {
    const int64_t sl = soff[j + 1] - soff[j];
    if (sl < W) {
      shorts.push_back(j);
      continue;
    }
    for (int64_t o = 0; o + W <= sl; ++o) ++freq[win(sbuf + soff[j] + o)];
  }
  struct Cand { int64_t j, o; };
  std::unordered_multimap<uint64_t, Cand> index;
  index.reserve((size_t)nsub * 2);
  std::vector<uint8_t> seen(1 << 16, 0);
  for (int64_t j = 0; j < nsub; ++j) {
    const int64_t sl = soff[j + 1] - soff[j];
    if (sl < W) continue;
    int64_t best = 0, bf = INT64_MAX;
    for (int64_t o = 0; o + W <= sl; ++o) {
      const int64_t f = freq[win(sbuf + soff[j] + o)];
      if (f < bf) { bf = f; best = o; }
    }
    const uint64_t h = win(sbuf + soff[j] + best);
    index.emplace(h, Cand{j, best});
    seen[mix(h)] = 1;
  }
  std::vector<int64_t> hits;
  for (int64_t i = 0; i < n; ++i) {
    const char* k = kbuf + koff[i];
    const int64_t L = koff[i + 1] - koff[i];
    const std::string_view kv(k, (size_t)L);
    hits.clear();
    for (int64_t j : shorts)
      if (kv.find(std::string_view(sbuf + soff[j], (size_t)(soff[j + 1] - soff[j]))) != std::string_view::npos)
        hits.push_back(j);
    if (!index.empty()) {
      for (int64_t p = 0; p + W <= L; ++p) {
        const uint64_t h = win(k + p);
        if (!seen[mix(h)]) continue;
        auto r = index.equal_range(h);
        for (auto it = r.first; it != r.second; ++it) {
          const int64_t j = it->second.j, st = p - it->second.o, sl = soff[j + 1] - soff[j];
          if (st >= 0 && st + sl <= L && std::memcmp(k + st, sbuf + soff[j], (size_t)sl) == 0) hits.push_back(j);
        }
      }
    }
    double m = 1.0;
    if (!hits.empty()) {
      std::sort(hits.begin(), hits.end());
      hits.erase(std::unique(hits.begin(), hits.end()), hits.end());
      for (int64_t j : hits) m *= mags[j];
    }
    out[i] = m;
  }
}
