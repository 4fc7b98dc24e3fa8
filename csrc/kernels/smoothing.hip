// K2: exponential smoothing family (single / double (Holt) / Holt-Winters
// additive and multiplicative) with a batched parameter-grid fit, plus an
// incremental update that advances a cached fitted model over new samples.
//
// Reference: the brain's model zoo lists Exponential Smoothing, Double
// Exponential Smoothing and Holt-Winters (docs/guides/design.md:62-72) and
// caches fitted models between cycles (MAX_CACHE_SIZE, foremast-brain/
// README.md:30); the statistics follow the textbook recursions
// (docs/BRAIN_SPEC.md §3.2).
//
// Mapping: one THREAD per (row, candidate) pair, candidates fastest, so the
// lanes that share a row read the same history sample (one coalesced request).
// The Holt-Winters seasonal state (m values per pair) lives in a global
// scratch laid out [m][pairs]: at step t every lane touches phase t % m of its
// own column, i.e. one coalesced load + store per wave per step.  At the
// BASELINE config-2 shape (40k series x 27 candidates x m=1440) that scratch
// traffic IS the fit's cost (2 x 8,640 steps x 1.08M pairs per fit), so the
// additive grid fit can store it in fp16, scaled per row (indices / mean |x|
// of the first season, saturated to the fp16 range): half the bytes of fp32
// scratch (ops/smoothing.py picks it for the additive model with m >= 1000;
// multiplicative indices, which multiply the level, stay fp32).  The recursion itself runs in
// fp32 registers; only the parked seasonal indices are rounded (relative
// 2^-11 per lap, damped by (1 - gamma) on every later lap).  The incremental
// update of cached models keeps fp32 seasons (es_update_kernel).
//
// Rows are right-aligned with NaN padding on the left (ragged histories), so
// every fit starts at the row's first finite sample and the seasonal
// initialisation averages only finite samples.
#include "fm_common.h"

using namespace fm;

constexpr int kPrefetch = 16;  // season/sample loads issued ahead per chunk (HW fit)
constexpr float kDivEps = 1e-6f;

// kind: 0 = SES, 1 = Holt (double), 2 = Holt-Winters additive, 3 = multiplicative
template <int KIND>
struct EsModel {
  float al, be, ga;
  float lvl, tr;
  // One step on sample xt with seasonal index s (in/out); an observed sample
  // adds its squared one-step error to acc and counts in n.  (Accumulating
  // inside the observed branch keeps the compiler from deferring 16 error
  // terms to the end of a prefetch chunk, which cost ~15 % in VGPRs/VALU.)
  __device__ __forceinline__ void step(float xt, float& s, float& acc, int& n) {
    const float pred = KIND == 3 ? (lvl + tr) * s : lvl + tr + s;
    if (isfinite(xt)) {
      const float e = xt - pred;
      acc += e * e;
      ++n;
      const float lprev = lvl;
      if (KIND == 0) {
        lvl = al * xt + (1.f - al) * lvl;
      } else if (KIND == 1) {
        lvl = al * xt + (1.f - al) * (lvl + tr);
        tr = be * (lvl - lprev) + (1.f - be) * tr;
      } else if (KIND == 2) {
        lvl = al * (xt - s) + (1.f - al) * (lvl + tr);
        tr = be * (lvl - lprev) + (1.f - be) * tr;
        s = ga * (xt - lvl) + (1.f - ga) * s;
      } else {
        const float ds = fabsf(s) > kDivEps ? xt / s : xt;
        lvl = al * ds + (1.f - al) * (lvl + tr);
        tr = be * (lvl - lprev) + (1.f - be) * tr;
        const float dl = fabsf(lvl) > kDivEps ? xt / lvl : 1.f;
        s = ga * dl + (1.f - ga) * s;
      }
    } else {
      lvl = lvl + tr;  // missing sample: propagate the forecast
    }
  }
};

// Seasonal-state storage: fp32 as is, or fp16 scaled by 1/sc (sc = 1 for the
// multiplicative model).
template <typename ST>
struct SeasonIO {
  float sc, isc;
  __device__ __forceinline__ float ld(const ST* p, int64_t i) const {
    if constexpr (sizeof(ST) == 4) return p[i];
    else return (float)p[i] * sc;
  }
  __device__ __forceinline__ void st(ST* p, int64_t i, float v) const {
    if constexpr (sizeof(ST) == 4) p[i] = v;
    else p[i] = (ST)__builtin_amdgcn_fmed3f(v * isc, -65504.f, 65504.f);
  }
};

// Initial seasonal index of a sample one season before (additive: x - s1,
// multiplicative: x / s1; missing -> 0 / 1).
template <int KIND>
struct SeasonInit {
  float s1, inv1;
  bool mul_ok;
  __device__ __forceinline__ float operator()(float v) const {
    const bool ok = isfinite(v);
    return KIND == 3 ? (ok && mul_ok ? v * inv1 : 1.f) : (ok ? v - s1 : 0.f);
  }
};

// Run the recursion over samples [t, T) of row xr.  Seasonal state of this
// (row, candidate) pair is column `col` of season[m][P]; ph = t % m on entry
// and on exit.  `t` and `ph` must be wave-uniform so the season addressing
// stays scalar (SGPR phase, one VGPR column offset); lanes whose own series
// starts later (ragged rows) pass GATED = true and their first sample t_act,
// and skip the steps before it.  err2/n carry the SSE (fp32 partials flushed
// to fp64 every 64 steps) and the observation count.
// LAP1: the first season after the initialisation window, whose seasonal
// indices are computed from the sample one period earlier (x[t - m], shared
// by the row's candidates and L2-resident) instead of being materialised per
// candidate and read back: saves a full write + read pass over the
// [m][R*G] scratch.
// NOSTORE: the tail of the last season, whose updated indices no forecast
// reads (the H-step forecast needs phases T..T+H-1, last written in the
// first H steps of the final season) -- when the caller does not keep the
// fitted state, those stores are skipped.
template <int KIND, bool GATED, bool LAP1 = false, bool NOSTORE = false, typename ST = float>
__device__ __forceinline__ void es_run(EsModel<KIND>& md, const float* __restrict__ xr, int t, int T, int t_act,
                                       int m, ST* __restrict__ season, int64_t P, int64_t col, int& ph,
                                       double& err2, int& n, SeasonInit<KIND> init = {},
                                       SeasonIO<ST> io = {1.f, 1.f}) {
  constexpr bool kSeason = KIND >= 2;
  float acc = 0.f;
  int chunk = 0;
  if (kSeason && m > kPrefetch) {
    // The season slot read at step t was written at step t - m, so the U
    // reads of a chunk never alias the chunk's own writes (U < m): issue all
    // U season + sample loads up front, then run the U dependent steps from
    // registers.  The per-step memory latency of the naive loop (load ->
    // dependent update -> store -> next load) is paid once per chunk.
    for (; t + kPrefetch <= T; t += kPrefetch) {
      float sv[kPrefetch], xv[kPrefetch];
      int64_t si[kPrefetch];
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        int pu = ph + u;
        if (pu >= m) pu -= m;
        si[u] = (int64_t)pu * P + col;
        sv[u] = LAP1 ? xr[t + u - m] : io.ld(season, si[u]);
        xv[u] = xr[t + u];
      }
      ph += kPrefetch;
      if (ph >= m) ph -= m;
      if (LAP1) {
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u) sv[u] = init(sv[u]);
      }
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        if (GATED && t + u < t_act) continue;
        md.step(xv[u], sv[u], acc, n);
      }
      if (!NOSTORE) {
#pragma unroll
        for (int u = 0; u < kPrefetch; ++u) io.st(season, si[u], sv[u]);
      }
      chunk += kPrefetch;
      if (chunk >= 64) { err2 += acc; acc = 0.f; chunk = 0; }
    }
  }
  for (; t < T; ++t) {
    float s = 0.f;
    int64_t sidx = 0;
    if (kSeason) {
      sidx = (int64_t)ph * P + col;
      s = LAP1 ? init(xr[t - m]) : io.ld(season, sidx);
      if (++ph == m) ph = 0;
    }
    if (GATED && t < t_act) continue;
    md.step(xr[t], s, acc, n);
    if (kSeason && !NOSTORE) io.st(season, sidx, s);
    if (++chunk == 64) { err2 += acc; acc = 0.f; chunk = 0; }
  }
  err2 += acc;
}

// fp16 seasonal scratch, blocked [m/8][P][8]: the 8 phases of a block are
// one 16-B vector per pair, so a 16-step chunk of the recursion is 2 vector
// loads + 2 vector stores per lane (1 KB fully coalesced per wave each)
// instead of 16 + 16 two-byte accesses.  Requires m % 8 == 0.
__device__ __forceinline__ int64_t blk_idx(int ph, int64_t P, int64_t col) {
  return ((int64_t)(ph >> 3) * P + col) * 8 + (ph & 7);
}

template <int KIND, bool GATED, bool LAP1 = false, bool NOSTORE = false>
__device__ __forceinline__ void es_run_blk(EsModel<KIND>& md, const float* __restrict__ xr, int t, int T, int t_act,
                                           int m, _Float16* __restrict__ season, int64_t P, int64_t col, int& ph,
                                           double& err2, int& n, SeasonInit<KIND> init, SeasonIO<_Float16> io) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  float acc = 0.f;
  int chunk = 0;
  auto one = [&](int tt) {
    const int64_t si = blk_idx(ph, P, col);
    float s = LAP1 ? init(xr[tt - m]) : io.ld(season, si);
    if (++ph == m) ph = 0;
    if (!(GATED && tt < t_act)) {
      md.step(xr[tt], s, acc, n);
      if (!NOSTORE) io.st(season, si, s);
    }
    if (++chunk >= 64) { err2 += acc; acc = 0.f; chunk = 0; }
  };
  for (; t < T && (ph & 7) != 0; ++t) one(t);            // align the phase to a block
  h8* sv8 = reinterpret_cast<h8*>(season);
  // Software-pipelined: chunk k+1's two season vectors and 16 samples are
  // loaded before chunk k's 16 dependent steps run (the slots read by chunk
  // k+1 were written m >> 32 steps earlier, never by chunk k), so the HBM
  // latency overlaps the recursion instead of preceding it.
  if (t + 16 <= T) {
    h8 na = {}, nb = {};
    float nx[16];
    int64_t nb0, nb1;
    auto issue = [&](int tt, int p0) {
      int p1 = p0 + 8;
      if (p1 >= m) p1 -= m;
      nb0 = (int64_t)(p0 >> 3) * P + col;
      nb1 = (int64_t)(p1 >> 3) * P + col;
      if (!LAP1) {
        na = sv8[nb0];
        nb = sv8[nb1];
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) nx[u] = xr[tt + u];
    };
    issue(t, ph);
    for (; t + 16 <= T; t += 16) {
      const int64_t b0 = nb0, b1 = nb1;
      float sv[16], xv[16];
      if (LAP1) {
#pragma unroll
        for (int u = 0; u < 16; ++u) sv[u] = init(xr[t + u - m]);
      } else {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sv[u] = (float)na[u] * io.sc;
          sv[8 + u] = (float)nb[u] * io.sc;
        }
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) xv[u] = nx[u];
      ph += 16;
      if (ph >= m) ph -= m;
      if (t + 32 <= T) issue(t + 16, ph);
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        if (GATED && t + u < t_act) continue;
        md.step(xv[u], sv[u], acc, n);
      }
      if (!NOSTORE) {
        h8 a, b;
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          a[u] = (_Float16)__builtin_amdgcn_fmed3f(sv[u] * io.isc, -65504.f, 65504.f);
          b[u] = (_Float16)__builtin_amdgcn_fmed3f(sv[8 + u] * io.isc, -65504.f, 65504.f);
        }
        sv8[b0] = a;
        sv8[b1] = b;
      }
      chunk += 16;
      if (chunk >= 64) { err2 += acc; acc = 0.f; chunk = 0; }
    }
  }
  for (; t < T; ++t) one(t);
  err2 += acc;
}

__device__ __forceinline__ int first_finite(const float* __restrict__ xr, int T) {
  int b = 0;
  while (b < T && !isfinite(xr[b])) ++b;
  return b;
}

// Finite-sample mean of xr[lo, hi); sets cnt (and the mean |x| in *mabs).
// Branch-free body so the loads of consecutive iterations are issued back to
// back.
__device__ __forceinline__ float nan_mean(const float* __restrict__ xr, int lo, int hi, int& cnt,
                                          float* mabs = nullptr) {
  float s = 0.f, a = 0.f;
  int c = 0;
#pragma unroll 8
  for (int i = lo; i < hi; ++i) {
    const float v = xr[i];
    const bool f = isfinite(v);
    s += f ? v : 0.f;
    a += f ? fabsf(v) : 0.f;
    c += f;
  }
  cnt = c;
  if (mabs != nullptr) *mabs = c > 0 ? a / c : 0.f;
  return c > 0 ? s / c : 0.f;
}

// Seasonal indices of samples xs[i0, i1) written to consecutive phases from
// sp on (stride P); samples at or past navail are missing.
template <int KIND, typename ST>
__device__ __forceinline__ void season_init(const float* __restrict__ xs, int i0, int i1, int navail,
                                            SeasonInit<KIND> init, ST* __restrict__ sp, int64_t P, SeasonIO<ST> io) {
  const int last = navail > 0 ? navail - 1 : 0;
#pragma unroll 8
  for (int i = i0; i < i1; ++i) {
    const float v = xs[i < last ? i : last];   // unpredicated load, masked below
    io.st(sp, (int64_t)(i - i0) * P, i < navail ? init(v) : init(__builtin_nanf("")));
  }
}

template <int KIND>
__device__ __forceinline__ void season_init_blk(const float* __restrict__ xs, int ph0, int m, int navail,
                                                SeasonInit<KIND> init, _Float16* __restrict__ season, int64_t P,
                                                int64_t col, SeasonIO<_Float16> io) {
  const int last = navail > 0 ? navail - 1 : 0;
  for (int i = 0; i < m; ++i) {
    const float v = xs[i < last ? i : last];
    int ph = ph0 + i;
    if (ph >= m) ph -= m;
    io.st(season, blk_idx(ph, P, col), i < navail ? init(v) : init(__builtin_nanf("")));
  }
}

template <int KIND, typename ST>
__global__ __launch_bounds__(256) void es_fit_kernel(const float* __restrict__ x, int64_t ld, int T, int64_t R,
                                                    const float* __restrict__ cand, int G, int m,
                                                    ST* __restrict__ season /*[m][R*G]*/, float* __restrict__ sse,
                                                    float* __restrict__ state /*[R*G,3]*/, int* __restrict__ nobs,
                                                    int t_store_end, float* __restrict__ sscale /*[R]*/,
                                                    int* __restrict__ nfin /*[R] or null*/) {
  const int64_t P = R * G;
  const int64_t pid_raw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((pid_raw & ~(int64_t)63) >= P) return;      // whole wave past the end
  // tail lanes of the last wave shadow the last pair (the wave-uniform start
  // below needs every lane) and store no results of their own
  const bool live = pid_raw < P;
  const int64_t pid = live ? pid_raw : P - 1;
  const int64_t row = pid / G;
  const int g = (int)(pid - row * G);
  EsModel<KIND> md{cand[3 * g + 0], cand[3 * g + 1], cand[3 * g + 2], 0.f, 0.f};
  const float* xr = x + row * ld;
  const int base = first_finite(xr, T);
  int t0;
  int nf0 = 0;                // finite samples consumed by the initialisation
  SeasonInit<KIND> sinit{0.f, 0.f, false};
  SeasonIO<ST> io{1.f, 1.f};
  if (base >= T) {
    md.lvl = __builtin_nanf("");
    t0 = T;
  } else if (KIND >= 2) {
    // level = mean of the first season, trend = (mean of the second - mean of
    // the first) / m, seasonal indices from the first season (finite samples)
    int c1, c2;
    const int e1 = min(base + m, T), e2 = min(base + 2 * m, T);
    float a1;
    const float s1 = nan_mean(xr, base, e1, c1, &a1);
    if (sizeof(ST) == 2 && KIND == 2) {
      const float sc = a1 > 1e-20f ? a1 : 1.f;
      io = SeasonIO<ST>{sc, 1.f / sc};
    }
    const float s2 = nan_mean(xr, e1, e2, c2);
    md.lvl = s1;
    md.tr = c2 > 0 ? (s2 - s1) / m : 0.f;
    const bool mul_ok = fabsf(s1) > kDivEps;
    sinit = SeasonInit<KIND>{s1, mul_ok ? 1.f / s1 : 0.f, mul_ok};
    t0 = base + m;
    nf0 = c1;
  } else {
    md.lvl = xr[base];
    if (KIND == 1 && base + 1 < T && isfinite(xr[base + 1])) md.tr = xr[base + 1] - xr[base];
    t0 = base + 1;
    nf0 = 1;
  }
  double err2 = 0.0;
  int n = 0;
  // wave-uniform start: all lanes run from the wave's earliest first step
  const int lo = __builtin_amdgcn_readfirstlane(wave_min(t0));
  const int hi = __builtin_amdgcn_readfirstlane(wave_max(t0));
  int ph = KIND >= 2 ? lo % m : 0;
  if (lo == hi && (KIND < 2 || lo + m <= T)) {
    if (KIND >= 2) {
      // seasons written up to t_store_end (T when the fitted state is kept)
      const int ts = max(lo + m, min(t_store_end, T));
      if constexpr (sizeof(ST) == 2) {
        es_run_blk<KIND, false, true, false>(md, xr, lo, lo + m, lo, m, season, P, pid, ph, err2, n, sinit, io);
        es_run_blk<KIND, false, false, false>(md, xr, lo + m, ts, lo, m, season, P, pid, ph, err2, n, {}, io);
        es_run_blk<KIND, false, false, true>(md, xr, ts, T, lo, m, season, P, pid, ph, err2, n, {}, io);
      } else {
        es_run<KIND, false, true, false, ST>(md, xr, lo, lo + m, lo, m, season, P, pid, ph, err2, n, sinit, io);
        es_run<KIND, false, false, false, ST>(md, xr, lo + m, ts, lo, m, season, P, pid, ph, err2, n, {}, io);
        es_run<KIND, false, false, true, ST>(md, xr, ts, T, lo, m, season, P, pid, ph, err2, n, {}, io);
      }
    } else {
      es_run<KIND, false, false, false, float>(md, xr, lo, T, lo, m, (float*)season, P, pid, ph, err2, n);
    }
  } else {
    // ragged rows in this wave: materialise the initial seasons (sample
    // base + i has absolute phase (base + i) % m: phases ph0 .. m-1, then
    // 0 .. ph0-1), then run with per-lane start gating
    if (KIND >= 2 && base < T) {
      const int ph0 = base % m;
      const int navail = min(m, T - base);
      if constexpr (sizeof(ST) == 2) {
        season_init_blk<KIND>(xr + base, ph0, m, navail, sinit, season, P, pid, io);
      } else {
        season_init<KIND, ST>(xr + base, 0, m - ph0, navail, sinit, season + (int64_t)ph0 * P + pid, P, io);
        season_init<KIND, ST>(xr + base, m - ph0, m, navail, sinit, season + pid, P, io);
      }
    }
    if constexpr (sizeof(ST) == 2)
      es_run_blk<KIND, true>(md, xr, lo, T, t0, m, season, P, pid, ph, err2, n, {}, io);
    else
      es_run<KIND, true, false, false, ST>(md, xr, lo, T, t0, m, season, P, pid, ph, err2, n, {}, io);
  }
  // shadow lanes recompute their twin's pair in lockstep (same values, same
  // addresses) and then store no results of their own
  if (!live) return;
  if (g == 0) sscale[row] = io.sc;
  // the row's finite history samples (the MIN_HISTORICAL_DATA_POINT gate),
  // a by-product of the fit: no separate pass over the history
  if (g == 0 && nfin) nfin[row] = nf0 + n;
  sse[pid] = (float)err2;
  state[pid * 3 + 0] = md.lvl;
  state[pid * 3 + 1] = md.tr;
  state[pid * 3 + 2] = (float)(KIND >= 2 ? T % m : 0);
  nobs[pid] = n;
}

// ---------------------------------------------------------------------------
// Additive Holt-Winters grid fit, packed: each THREAD runs TWO candidates of
// one row (g = 2j, 2j+1) as float2 with v_pk_{add,mul,fma}_f32, so the
// recursion costs ~half the VALU instructions per candidate, and the shared
// sample is loaded, scaled and tested once.  The fit runs in row-scaled units
// (x / sc, sc = mean |x| of the first season), so the fp16 seasonal scratch
// is stored without per-access rescaling.  Missing samples are branch-free:
// the sample is replaced by the prediction, which leaves level + trend
// advancing, trend and season unchanged and adds no error (the recursion's
// own missing-sample rule).  Scratch: blocked [m/8][R*GP][2][8] fp16.
// ---------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h8v __attribute__((ext_vector_type(8)));

__device__ __forceinline__ h8v to_h8(const float* v) {
  h8v o;
#pragma unroll
  for (int u = 0; u < 8; ++u) o[u] = (_Float16)__builtin_amdgcn_fmed3f(v[u], -65504.f, 65504.f);
  return o;
}

template <bool GATED, bool LAP1, bool NOSTORE>
__device__ __forceinline__ void hw2_run(f2v& l, f2v& tr, const f2v al, const f2v be, const f2v ga,
                                        const float* __restrict__ xr, float isc, float s1, int t, int T, int t_act,
                                        int m, h8v* __restrict__ sv8, int64_t NT, int64_t tid, int& ph, f2v& acc,
                                        double& ea, double& eb, int& n, int& chunk, bool xal) {
  // Closed forms of the additive recursion in the one-step error e = x - pred:
  //   l' = lt + a e,  t' = t + a b e,  s' = s + g (1 - a) e   (lt = l + t)
  // (algebraically the textbook updates; 3 packed adds + 4 packed FMAs per
  // step instead of 9 + 4, and (l' - l - t) no longer cancels).
  const f2v ab = al * be, gm1 = ga * ((f2v){1.f, 1.f} - al);
  auto step = [&](float xv_raw, f2v& s, bool act) {
    const float xv = xv_raw * isc;
    const bool fin = isfinite(xv);
    const f2v lt = l + tr;
    const f2v pred = lt + s;
    const f2v xe = fin ? (f2v){xv, xv} : pred;
    const f2v e = xe - pred;
    const f2v ln = __builtin_elementwise_fma(al, e, lt);
    const f2v tn = __builtin_elementwise_fma(ab, e, tr);
    const f2v sn = __builtin_elementwise_fma(gm1, e, s);
    if (!GATED || act) {
      acc = __builtin_elementwise_fma(e, e, acc);
      n += fin ? 1 : 0;
      l = ln;
      tr = tn;
      s = sn;
    }
  };
  auto flush = [&](int k) {
    chunk += k;
    if (chunk >= 64) { ea += acc.x; eb += acc.y; acc = (f2v){0.f, 0.f}; chunk = 0; }
  };
  auto one = [&](int tt) {            // single step, scalar phase access
    const int64_t bi = ((int64_t)(ph >> 3) * NT + tid) * 16 + (ph & 7);
    _Float16* sh = reinterpret_cast<_Float16*>(sv8);
    f2v s;
    if (LAP1) {
      const float v = xr[tt - m] * isc;
      s = (f2v){isfinite(v) ? v - s1 : 0.f, isfinite(v) ? v - s1 : 0.f};
    } else {
      s = (f2v){(float)sh[bi], (float)sh[bi + 8]};
    }
    if (++ph == m) ph = 0;
    step(xr[tt], s, !GATED || tt >= t_act);
    if (!NOSTORE && (!GATED || tt >= t_act)) {
      sh[bi] = (_Float16)__builtin_amdgcn_fmed3f(s.x, -65504.f, 65504.f);
      sh[bi + 8] = (_Float16)__builtin_amdgcn_fmed3f(s.y, -65504.f, 65504.f);
    }
    flush(1);
  };
  for (; t < T && (ph & 7) != 0; ++t) one(t);
  for (; t + 8 <= T; t += 8) {
    const int64_t b = ((int64_t)(ph >> 3) * NT + tid) * 2;
    float sa[8], sb[8];
    if (LAP1) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const float v = xr[t + u - m] * isc;
        sa[u] = sb[u] = isfinite(v) ? v - s1 : 0.f;
      }
    } else {
      const h8v a = sv8[b], c = sv8[b + 1];
#pragma unroll
      for (int u = 0; u < 8; ++u) { sa[u] = (float)a[u]; sb[u] = (float)c[u]; }
    }
    float xv[8];
    if (xal && (t & 3) == 0) {        // wave-uniform; xal: x and its row stride are 16-B aligned
      const float4 x0 = *reinterpret_cast<const float4*>(xr + t);
      const float4 x1 = *reinterpret_cast<const float4*>(xr + t + 4);
      xv[0] = x0.x; xv[1] = x0.y; xv[2] = x0.z; xv[3] = x0.w;
      xv[4] = x1.x; xv[5] = x1.y; xv[6] = x1.z; xv[7] = x1.w;
    } else {
#pragma unroll
      for (int u = 0; u < 8; ++u) xv[u] = xr[t + u];
    }
    ph += 8;
    if (ph >= m) ph -= m;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      f2v s = {sa[u], sb[u]};
      step(xv[u], s, !GATED || t + u >= t_act);
      sa[u] = s.x;
      sb[u] = s.y;
    }
    if (!NOSTORE) {
      sv8[b] = to_h8(sa);
      sv8[b + 1] = to_h8(sb);
    }
    flush(8);
  }
  for (; t < T; ++t) one(t);
}

__global__ __launch_bounds__(256) void hw2_fit_kernel(const float* __restrict__ x, int64_t ld, int T, int64_t R,
                                                      const float* __restrict__ cand, int G, int m,
                                                      h8v* __restrict__ season, float* __restrict__ sse,
                                                      float* __restrict__ state, int* __restrict__ nobs,
                                                      int t_store_end, float* __restrict__ sscale,
                                                      int* __restrict__ nfin, int xal) {
  const int GP = (G + 1) >> 1;
  const int64_t NT = R * GP;
  const int64_t tid_raw = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((tid_raw & ~(int64_t)63) >= NT) return;
  const bool live = tid_raw < NT;
  const int64_t tid = live ? tid_raw : NT - 1;
  const int64_t row = tid / GP;
  const int j = (int)(tid - row * GP);
  const int ga_i = 2 * j, gb_i = 2 * j + 1 < G ? 2 * j + 1 : 2 * j;
  const f2v al = {cand[3 * ga_i], cand[3 * gb_i]}, be = {cand[3 * ga_i + 1], cand[3 * gb_i + 1]},
            gm = {cand[3 * ga_i + 2], cand[3 * gb_i + 2]};
  const float* xr = x + row * ld;
  const int base = first_finite(xr, T);
  f2v l = {0.f, 0.f}, tr = {0.f, 0.f};
  float sc = 1.f, s1 = 0.f;
  int t0, nf0 = 0;
  if (base >= T) {
    l = (f2v){__builtin_nanf(""), __builtin_nanf("")};
    t0 = T;
  } else {
    int c1, c2;
    const int e1 = min(base + m, T), e2 = min(base + 2 * m, T);
    float a1;
    const float m1 = nan_mean(xr, base, e1, c1, &a1);
    const float m2 = nan_mean(xr, e1, e2, c2);
    sc = a1 > 1e-20f ? a1 : 1.f;
    s1 = m1 / sc;
    const float trend = c2 > 0 ? (m2 - m1) / sc / m : 0.f;
    l = (f2v){s1, s1};
    tr = (f2v){trend, trend};
    t0 = base + m;
    nf0 = c1;
  }
  const float isc = 1.f / sc;
  f2v acc = {0.f, 0.f};
  double ea = 0.0, eb = 0.0;
  int n = 0, chunk = 0;
  const int lo = __builtin_amdgcn_readfirstlane(wave_min(t0));
  const int hi = __builtin_amdgcn_readfirstlane(wave_max(t0));
  int ph = lo % m;
  if (lo == hi && lo + m <= T) {
    const int ts = max(lo + m, min(t_store_end, T));
    hw2_run<false, true, false>(l, tr, al, be, gm, xr, isc, s1, lo, lo + m, lo, m, season, NT, tid, ph, acc, ea, eb, n,
                                chunk, xal != 0);
    hw2_run<false, false, false>(l, tr, al, be, gm, xr, isc, s1, lo + m, ts, lo, m, season, NT, tid, ph, acc, ea, eb,
                                 n, chunk, xal != 0);
    hw2_run<false, false, true>(l, tr, al, be, gm, xr, isc, s1, ts, T, lo, m, season, NT, tid, ph, acc, ea, eb, n,
                                chunk, xal != 0);
  } else {
    // ragged rows in this wave: materialise each row's initial seasons, then
    // run with per-lane start gating
    if (base < T) {
      _Float16* sh = reinterpret_cast<_Float16*>(season);
      const int navail = min(m, T - base);
      for (int i = 0; i < m; ++i) {
        const float v = i < navail ? xr[base + i] * isc : __builtin_nanf("");
        const float si = isfinite(v) ? v - s1 : 0.f;
        const int p = (base + i) % m;
        const int64_t bi = ((int64_t)(p >> 3) * NT + tid) * 16 + (p & 7);
        sh[bi] = sh[bi + 8] = (_Float16)__builtin_amdgcn_fmed3f(si, -65504.f, 65504.f);
      }
    }
    hw2_run<true, false, false>(l, tr, al, be, gm, xr, isc, s1, lo, T, t0, m, season, NT, tid, ph, acc, ea, eb, n,
                                chunk, xal != 0);
  }
  ea += acc.x;
  eb += acc.y;
  if (!live) return;
  const float s2 = sc * sc;
  const int64_t pa = row * G + ga_i;
  sse[pa] = (float)(ea * s2);
  state[pa * 3 + 0] = l.x * sc;
  state[pa * 3 + 1] = tr.x * sc;
  state[pa * 3 + 2] = (float)(T % m);
  nobs[pa] = n;
  if (2 * j + 1 < G) {
    const int64_t pb = pa + 1;
    sse[pb] = (float)(eb * s2);
    state[pb * 3 + 0] = l.y * sc;
    state[pb * 3 + 1] = tr.y * sc;
    state[pb * 3 + 2] = (float)(T % m);
    nobs[pb] = n;
  }
  if (j == 0) sscale[row] = sc;
  if (j == 0 && nfin) nfin[row] = nf0 + n;
}

__global__ __launch_bounds__(256) void hw2_forecast_kernel(const float* __restrict__ sse,
                                                           const float* __restrict__ state,
                                                           const int* __restrict__ nobs,
                                                           const _Float16* __restrict__ season,
                                                           const float* __restrict__ sscale, int64_t R, int G, int m,
                                                           int H, float* __restrict__ fc, float* __restrict__ sigma,
                                                           int* __restrict__ best) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= R) return;
  const int GP = (G + 1) >> 1;
  const int64_t NT = R * GP;
  int bg = 0;
  float bs = sse[row * G];
  for (int g = 1; g < G; ++g) {
    const float v = sse[row * G + g];
    if (v < bs || !isfinite(bs)) { bs = v; bg = g; }
  }
  const int64_t pid = row * G + bg;
  const int64_t tid = row * GP + (bg >> 1);
  const float lvl = state[pid * 3 + 0], tr = state[pid * 3 + 1], sc = sscale[row];
  const int tph = (int)state[pid * 3 + 2];
  const int n = nobs[pid];
  sigma[row] = n > 1 ? sqrtf(bs / (float)(n - 1)) : 0.f;
  best[row] = bg;
  for (int h = 1; h <= H; ++h) {
    const int p = (tph + h - 1) % m;
    const float sv = (float)season[((int64_t)(p >> 3) * NT + tid) * 16 + (bg & 1) * 8 + (p & 7)] * sc;
    fc[row * H + (h - 1)] = lvl + h * tr + sv;
  }
}

// Incremental update of cached models, in place in the cache's slab: row r
// of x (its new samples x[r, t_new[r] .. T)) advances slot s = slots[r] (or
// r when slots is null) of params/state [C,3] (level, trend, phase of the
// next sample), season [C, m] (row-major per slot), sse/nobs [C], then
// writes the H-step forecast and residual sigma of row r.  One thread per
// row; k is a handful of samples, so the scattered slot accesses are noise.
template <int KIND>
__global__ __launch_bounds__(256) void es_update_kernel(const float* __restrict__ x, int64_t ld, int T, int64_t R,
                                                       const int* __restrict__ t_new,
                                                       const int64_t* __restrict__ slots,
                                                       const float* __restrict__ params, int m,
                                                       float* __restrict__ season, float* __restrict__ sse,
                                                       float* __restrict__ state, int* __restrict__ nobs, int H,
                                                       float* __restrict__ fc, float* __restrict__ sigma) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= R) return;
  const int64_t sl = slots != nullptr ? slots[row] : row;
  EsModel<KIND> md{params[sl * 3 + 0], params[sl * 3 + 1], params[sl * 3 + 2], state[sl * 3 + 0],
                   state[sl * 3 + 1]};
  int ph = KIND >= 2 ? (int)state[sl * 3 + 2] : 0;
  int t0 = t_new[row];
  t0 = t0 < 0 ? 0 : (t0 > T ? T : t0);
  double err2 = sse[sl];
  int n = nobs[sl];
  float* srow = KIND >= 2 ? season + sl * m : season;
  es_run<KIND, false>(md, x + row * ld, t0, T, t0, m, srow, 1, 0, ph, err2, n);
  sse[sl] = (float)err2;
  state[sl * 3 + 0] = md.lvl;
  state[sl * 3 + 1] = md.tr;
  state[sl * 3 + 2] = (float)ph;
  nobs[sl] = n;
  sigma[row] = n > 1 ? sqrtf((float)err2 / (float)(n - 1)) : 0.f;
  int p = ph;
  for (int h = 1; h <= H; ++h) {
    float f = md.lvl + (KIND >= 1 ? h * md.tr : 0.f);
    if (KIND >= 2) {
      const float sv = srow[p];
      f = KIND == 3 ? f * sv : f + sv;
      if (++p == m) p = 0;
    }
    fc[row * H + (h - 1)] = f;
  }
}

// Per row: pick the candidate with the smallest SSE and write the H-step
// forecast + residual sigma.
template <typename ST>
__global__ __launch_bounds__(256) void es_forecast_kernel(const float* __restrict__ sse, const float* __restrict__ state,
                                                          const int* __restrict__ nobs, const ST* __restrict__ season,
                                                          const float* __restrict__ sscale, int64_t R, int G, int m,
                                                          int kind, int H, float* __restrict__ fc /*[R,H]*/,
                                                          float* __restrict__ sigma, int* __restrict__ best) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= R) return;
  const int64_t P = R * G;
  int bg = 0;
  float bs = sse[row * G];
  for (int g = 1; g < G; ++g) {
    const float v = sse[row * G + g];
    if (v < bs || !isfinite(bs)) { bs = v; bg = g; }
  }
  const int64_t pid = row * G + bg;
  const float lvl = state[pid * 3 + 0], tr = state[pid * 3 + 1];
  const int tph = (int)state[pid * 3 + 2];
  const int n = nobs[pid];
  sigma[row] = n > 1 ? sqrtf(bs / (float)(n - 1)) : 0.f;
  best[row] = bg;
  for (int h = 1; h <= H; ++h) {
    float f = lvl + (kind >= 1 ? h * tr : 0.f);
    if (kind >= 2) {
      const int sp = (tph + h - 1) % m;
      const float s = (float)season[sizeof(ST) == 2 ? blk_idx(sp, P, pid) : (int64_t)sp * P + pid] * sscale[row];
      f = kind == 3 ? f * s : f + s;
    }
    fc[row * H + (h - 1)] = f;
  }
}

#define FM_ES_DISPATCH(KERNEL, GRID, ...)                                                           \
  do {                                                                                              \
    if (kind == 0) hipLaunchKernelGGL(KERNEL<0>, GRID, dim3(256), 0, stream, __VA_ARGS__);          \
    else if (kind == 1) hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(256), 0, stream, __VA_ARGS__);     \
    else if (kind == 2) hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(256), 0, stream, __VA_ARGS__);     \
    else hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(256), 0, stream, __VA_ARGS__);                    \
  } while (0)
#define FM_ES_DISPATCH_T(KERNEL, ST, GRID, ...)                                                      \
  do {                                                                                              \
    if (kind == 0) hipLaunchKernelGGL((KERNEL<0, ST>), GRID, dim3(256), 0, stream, __VA_ARGS__);    \
    else if (kind == 1) hipLaunchKernelGGL((KERNEL<1, ST>), GRID, dim3(256), 0, stream, __VA_ARGS__); \
    else if (kind == 2) hipLaunchKernelGGL((KERNEL<2, ST>), GRID, dim3(256), 0, stream, __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<3, ST>), GRID, dim3(256), 0, stream, __VA_ARGS__);              \
  } while (0)

// keep_season = 0: only the seasonal indices the H-step forecast reads are
// guaranteed in `season` afterwards (saves one store pass); 1: all of them
// (the caller extracts the fitted state, e.g. for the model cache).
// season_half = 1 (additive, m % 8 == 0): packed two-candidate kernel with
// an fp16 season scratch blocked [m/8][R*ceil(G/2)][2][8] in row-scaled units
// (the scale written to sscale[R]); 0: fp32 [m][R*G] (sscale[R] = 1).
FM_API int fm_es_fit(const float* x, int64_t ld, int T, int64_t R, const float* cand, int G, int m, int kind,
                     void* season, float* sse, float* state, int* nobs, int H, float* fc, float* sigma, int* best,
                     int keep_season, int season_half, float* sscale, int* nfin, hipStream_t stream) {
  if (R <= 0) return 0;
  if (kind < 0 || kind > 3) return (int)hipErrorInvalidValue;
  if (kind >= 2 && (m < 2 || 2 * m > T)) return (int)hipErrorInvalidValue;
  if (kind < 2 && T < 2) return (int)hipErrorInvalidValue;
  if (season_half && (kind != 2 || m % 8 != 0)) return (int)hipErrorInvalidValue;   // blocked fp16 layout
  if (kind < 2) m = 1;
  const int64_t P = R * G;
  const int t_store_end = keep_season || kind < 2 || H >= m ? T : T - m + H;
  const dim3 gf((unsigned)((P + 255) / 256)), gr((unsigned)((R + 255) / 256));
  if (season_half) {
    // packed two-candidates-per-thread additive fit (hw2_fit_kernel; two
    // pairs per thread measured slower: profiles/hw_pairs_ab_r3.jsonl)
    const int64_t NT = R * ((G + 1) / 2);
    const int xal = ((uintptr_t)x % 16 == 0) && (ld % 4 == 0);
    hipLaunchKernelGGL(hw2_fit_kernel, dim3((unsigned)((NT + 255) / 256)), dim3(256), 0, stream, x, ld, T, R, cand, G,
                       m, (h8v*)season, sse, state, nobs, t_store_end, sscale, nfin, xal);
    FM_LAUNCH_CHECK();
    hipLaunchKernelGGL(hw2_forecast_kernel, gr, dim3(256), 0, stream, sse, state, nobs, (const _Float16*)season,
                       sscale, R, G, m, H, fc, sigma, best);
  } else {
    FM_ES_DISPATCH_T(es_fit_kernel, float, gf, x, ld, T, R, cand, G, m, (float*)season, sse, state, nobs, t_store_end,
                     sscale, nfin);
    FM_LAUNCH_CHECK();
    hipLaunchKernelGGL(es_forecast_kernel<float>, gr, dim3(256), 0, stream, sse, state, nobs, (const float*)season,
                       sscale, R, G, m, kind, H, fc, sigma, best);
  }
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_es_update(const float* x, int64_t ld, int T, int64_t R, const int* t_new, const int64_t* slots,
                        const float* params, int m, int kind, float* season, float* sse, float* state, int* nobs,
                        int H, float* fc, float* sigma, hipStream_t stream) {
  if (R <= 0) return 0;
  if (kind < 0 || kind > 3) return (int)hipErrorInvalidValue;
  if (kind >= 2 && m < 2) return (int)hipErrorInvalidValue;
  if (kind < 2) m = 1;
  FM_ES_DISPATCH(es_update_kernel, dim3((unsigned)((R + 255) / 256)), x, ld, T, R, t_new, slots, params, m, season,
                 sse, state, nobs, H, fc, sigma);
  FM_LAUNCH_CHECK();
  return 0;
}
#undef FM_ES_DISPATCH
#undef FM_ES_DISPATCH_T

// ---------------------------------------------------------------------------
// Model-agnostic band decision: compare current points against per-point
// bands centre +/- thr * sigma (forecasting models: ES/HW, prophet-lite,
// LSTM).  One wave per row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void band_decide_kernel(const float* __restrict__ cur, int64_t ld_c, int n,
                                                          const float* __restrict__ center, int64_t ld_f,
                                                          const float* __restrict__ sigma, int64_t R, int M,
                                                          const float* __restrict__ thr,
                                                          const int* __restrict__ bound,
                                                          const float* __restrict__ minlb,
                                                          const int8_t* __restrict__ diff, float pair_factor,
                                                          float* __restrict__ upper, float* __restrict__ lower,
                                                          unsigned long long* __restrict__ flags, int NW,
                                                          int* __restrict__ count, float* __restrict__ score) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R) return;
  const int lane = lane_id();
  const int m = (int)(row % M);
  float th = thr[m];
  if (diff != nullptr && diff[row]) th *= pair_factor;
  const int bd = bound[m];
  const float sd = sigma[row];
  const float inv = sd > 0.f ? 1.f / sd : 0.f;
  int cnt = 0;
  float best = 0.f;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    if (i < n) {
      const float c = center[row * ld_f + i];
      const float up = c + th * sd;
      float lo = c - th * sd;
      if (lo < minlb[m]) lo = minlb[m];
      upper[row * n + i] = up;
      lower[row * n + i] = lo;
      const float x = cur[row * ld_c + i];
      if (isfinite(x) && isfinite(c)) {
        const bool hi = (bd & 1) && x > up;
        const bool lw = (bd & 2) && x < lo;
        f = hi || lw;
        if (f) {
          ++cnt;
          const float z = sd > 0.f ? (hi ? x - up : lo - x) * inv : 1e30f;
          best = z > best ? z : best;
        }
      }
    }
    const unsigned long long bal = __ballot(f);
    if (lane == 0 && i0 / 64 < NW) flags[row * NW + i0 / 64] = bal;
  }
  cnt = wave_sum(cnt);
  best = wave_max(best);
  if (lane == 0) { count[row] = cnt; score[row] = best; }
}

FM_API int fm_band_decide(const float* cur, int64_t ld_c, int n, const float* center, int64_t ld_f, const float* sigma,
                          int64_t R, int M, const float* thr, const int* bound, const float* minlb, const int8_t* diff,
                          float pair_factor, float* upper, float* lower, unsigned long long* flags, int NW, int* count,
                          float* score, hipStream_t stream) {
  if (R <= 0) return 0;
  if (NW * 64 < n) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(band_decide_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, cur, ld_c, n, center,
                     ld_f, sigma, R, M, thr, bound, minlb, diff, pair_factor, upper, lower, flags, NW, count, score);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// The steady sliding cycle of a forecasting group in ONE launch (VERDICT r4
// #2): advance the cached ES/Holt-Winters models over the samples the window
// gained, judge every current point against the forecast band at its own
// horizon, reduce the verdicts per service and stream-compact the anomalous
// points.  Before this the cycle was gather_cols (materialise the tail) ->
// es_update -> ~40 ATen glue kernels (horizon gather, validity masks, stats
// stack, service reduce, counter reset, compaction).
//
// One workgroup per service, one wave per metric row (M waves):
//   * the row's k new samples are read straight from the resident history
//     grid (row rm[r], dense column c -> grid column c - (shift[r] - dk),
//     valid below lim[r] + dk: the shift-only slide of a polled fleet is the
//     scalar dk, no per-row rewrite) into LDS; lane 0 advances the model in
//     the cache slab (params/state/season/sse/nobs of slot slots[r]);
//   * the forecast at a point's horizon h is lvl + h tr (+|x) season[(ph + h
//     - 1) % m], read per lane -- the season entries lane 0 just rewrote come
//     from LDS (a wave's lanes do not see one lane's global stores ordered);
//   * band / flags / count / score exactly as band_decide_kernel + zoo.band
//     (rows without history, valid bit 0, flag nothing);
//   * stats[r] = (nan, nan, upper, lower) at the row's last finite point;
//   * wave 0 reduces the service (service_reduce_kernel semantics) from LDS;
//   * anomalous points append (row, point, band upper, band lower), value
//     through one atomic per row to ctr[par]; block 0 zeroes ctr[par ^ 1]
//     for the next cycle.  The host takes the total from the per-row counts
//     (their sum), so no counter copy follows the launch.  (A
//     last-workgroup-publishes-the-counter epilogue -- one same-address
//     device atomic per workgroup -- measured 43 -> 327 us at 10k
//     workgroups.)
//   * the current window is row r of cur, or (cur_rm) grid row cur_rm[r] of
//     cur = the grid's first window column: read in place, no gather.
// Host outputs land in one buffer (hostv: packed [S,4] | stats [R,4] | count
// [R] (int) | dead [R] (int) | counters [2] (int, unused)) for a single
// device->host copy.
// ---------------------------------------------------------------------------
constexpr int kStepKMax = 64;      // new samples per row per cycle handled in-kernel
constexpr int kStepMMax = 16;      // metrics per service (waves per workgroup)

template <int KIND>
__global__ __launch_bounds__(1024) void es_band_step_kernel(
    const float* __restrict__ buf, int64_t ld, const int* __restrict__ rm, const int* __restrict__ shift,
    const int* __restrict__ lim, int dk, int T, int kmax, const int* __restrict__ t_new,
    const int64_t* __restrict__ slots, const float* __restrict__ params, int m, float* __restrict__ season,
    float* __restrict__ sse, float* __restrict__ state, int* __restrict__ nobs,
    const float* __restrict__ cur, int64_t ld_c, int n, const int64_t* __restrict__ hor, int H, int64_t S, int M,
    const float* __restrict__ thr, const int* __restrict__ bound, const float* __restrict__ minlb,
    const int8_t* __restrict__ diff, float pair_factor, const int* __restrict__ valid,
    const int64_t* __restrict__ lastk, float* __restrict__ upper, float* __restrict__ lower,
    float* __restrict__ sigma_out, float* __restrict__ fc, int Hf, float* __restrict__ hostv, int cap,
    int* __restrict__ ctr, int par, int* __restrict__ out_idx, float* __restrict__ out_val,
    float* __restrict__ last3, const int* __restrict__ cur_rm) {
  __shared__ float xs[kStepMMax][kStepKMax];
  __shared__ float su[kStepMMax][kStepKMax];
  __shared__ int s_cnt[kStepMMax];
  __shared__ float s_score[kStepMMax];
  __shared__ int s_valid[kStepMMax];
  const int64_t s = blockIdx.x;
  const int mi = wave_id();
  const int lane = lane_id();
  const int64_t R = S * M;
  const int64_t row = s * M + mi;
  // the row's current window: its own row of cur, or (cur_rm) a grid row
  const float* __restrict__ crow = cur + (cur_rm != nullptr ? (int64_t)cur_rm[row] : row) * ld_c;
  if (blockIdx.x == 0 && threadIdx.x == 0) ctr[par ^ 1] = 0;
  float lvl = 0.f, tr = 0.f, sig = 0.f;
  int ph = 0, ph_old = 0, k = 0;
  const float* srow = season;
  if constexpr (KIND >= 0) {
    const int64_t sl = slots[row];
    int k0 = t_new[row];
    k0 = k0 < 0 ? 0 : (k0 > kmax ? kmax : k0);
    // the tail columns [T - kmax, T) of the row, from the grid
    {
      const int64_t g = rm[row];
      const int off = dk - shift[row];
      const int lm = lim[row] + dk;
      if (lane < kmax) {
        const int c = T - kmax + lane + off;
        xs[mi][lane] = (c >= 0 && c < lm) ? buf[g * ld + c] : __builtin_nanf("");
      }
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    k = kmax - k0;
    if (KIND >= 2) srow = season + sl * m;
    if (lane == 0) {
      EsModel<KIND> md{params[sl * 3 + 0], params[sl * 3 + 1], params[sl * 3 + 2], state[sl * 3 + 0],
                       state[sl * 3 + 1]};
      ph = KIND >= 2 ? (int)state[sl * 3 + 2] : 0;
      const int ph0 = ph;
      double err2 = sse[sl];
      int nn = nobs[sl];
      es_run<KIND, false>(md, &xs[mi][0], k0, kmax, k0, m, season + (KIND >= 2 ? sl * m : 0), 1, 0, ph, err2, nn);
      sse[sl] = (float)err2;
      state[sl * 3 + 0] = md.lvl;
      state[sl * 3 + 1] = md.tr;
      state[sl * 3 + 2] = (float)ph;
      nobs[sl] = nn;
      lvl = md.lvl;
      tr = md.tr;
      sig = nn > 1 ? sqrtf((float)err2 / (float)(nn - 1)) : 0.f;
      sigma_out[row] = sig;
      if (KIND >= 2) {
        int p = ph0;
        for (int j = 0; j < k; ++j) {     // this thread's own stores: program order
          su[mi][j] = srow[p];
          if (++p == m) p = 0;
        }
      }
      reinterpret_cast<int*>(hostv)[S * 4 + R * 4 + R + row] = (isfinite(lvl) && isfinite(tr)) ? 0 : 1;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    lvl = __shfl(lvl, 0);
    tr = __shfl(tr, 0);
    sig = __shfl(sig, 0);
    ph = __shfl(ph, 0);
    ph_old = KIND >= 2 ? ((ph - k) % m + m) % m : 0;
  } else {
    // a forecast computed elsewhere (LSTM, Prophet): fc [R, Hf] and sigma are inputs
    sig = sigma_out[row];
    if (lane == 0) reinterpret_cast<int*>(hostv)[S * 4 + R * 4 + R + row] = 0;
  }
  auto fcast = [&](int h) -> float {
    if constexpr (KIND < 0) {
      return fc[row * Hf + (h - 1)];
    } else {
      float f = lvl + (KIND >= 1 ? (float)h * tr : 0.f);
      if (KIND >= 2) {
        const int idx = (ph + h - 1) % m;
        int d = idx - ph_old;
        d = d < 0 ? d + m : d;
        const float sv = d < k ? su[mi][d] : srow[idx];
        f = KIND == 3 ? f * sv : f + sv;
      }
      return f;
    }
  };
  if (KIND >= 0 && fc != nullptr) {
    for (int h = 1 + lane; h <= Hf; h += 64) fc[row * Hf + (h - 1)] = fcast(h);
  }
  // band decision (band_decide_kernel + zoo.band's history gate)
  const int mm = (int)(row % M);
  float th = thr[mm];
  if (diff != nullptr && diff[row]) th *= pair_factor;
  const int bd = bound[mm];
  const float inv = sig > 0.f ? 1.f / sig : 0.f;
  const int vld = valid[row];
  const bool has = (vld & 1) != 0;
  const int lk = (int)lastk[row];
  int cnt = 0;
  float best = 0.f;
  unsigned long long words[4] = {0ull, 0ull, 0ull, 0ull};
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    if (i < n) {
      int h = (int)hor[row * n + i];
      h = h < 1 ? 1 : (h > H ? H : h);
      const float c = fcast(h);
      const float up = c + th * sig;
      float lo = c - th * sig;
      if (lo < minlb[mm]) lo = minlb[mm];
      upper[row * n + i] = up;
      lower[row * n + i] = lo;
      const float x = crow[i];
      if (i == lk) {
        float* st = hostv + S * 4 + row * 4;
        st[0] = __builtin_nanf("");
        st[1] = __builtin_nanf("");
        st[2] = up;
        st[3] = lo;
        if (last3 != nullptr) {       // the newest point and its band, NaN without one (HPA score input)
          const bool okx = isfinite(x);
          last3[row] = x;
          last3[R + row] = okx ? up : __builtin_nanf("");
          last3[2 * R + row] = okx ? lo : __builtin_nanf("");
        }
      }
      if (isfinite(x) && isfinite(c)) {
        const bool hi = (bd & 1) && x > up;
        const bool lw = (bd & 2) && x < lo;
        f = hi || lw;
        if (f) {
          ++cnt;
          const float z = sig > 0.f ? (hi ? x - up : lo - x) * inv : 1e30f;
          best = z > best ? z : best;
        }
      }
    }
    const unsigned long long bal = __ballot(f && has);
    if (i0 / 64 < 4) words[i0 / 64] = bal;
  }
  cnt = has ? wave_sum(cnt) : 0;
  best = wave_max(best);
  // compaction: one atomic per row with anomalies
  if (cnt > 0) {
    int base = 0;
    if (lane == 0) base = atomicAdd(&ctr[par], cnt);
    base = __shfl(base, 0);
    int written = 0;
    for (int w = 0; w < 4 && w * 64 < n; ++w) {
      const unsigned long long word = words[w];
      if (!word) continue;
      const unsigned long long below = lane == 0 ? 0ull : (word & ((1ull << lane) - 1ull));
      const int slot = base + written + __popcll(below);
      if (((word >> lane) & 1ull) && slot < cap) {
        // [row, point, band upper, band lower] (the band at the point read
        // back from this lane's own writes above): a verdict's reasons need
        // no gather of the per-point bands
        const int pt = w * 64 + lane;
        out_idx[4 * slot + 0] = (int)row;
        out_idx[4 * slot + 1] = pt;
        out_idx[4 * slot + 2] = __float_as_int(upper[row * n + pt]);
        out_idx[4 * slot + 3] = __float_as_int(lower[row * n + pt]);
        out_val[slot] = crow[pt];
      }
      written += __popcll(word);
    }
  }
  if (lane == 0) {
    reinterpret_cast<int*>(hostv)[S * 4 + R * 4 + row] = cnt;
    s_cnt[mi] = cnt;
    s_score[mi] = best;
    s_valid[mi] = vld;
  }
  __syncthreads();
  if (mi == 0 && lane == 0) {    // service_reduce_kernel semantics
    int tot = 0, mask = 0;
    bool unknown = false;
    float sb = 0.f;
    for (int j = 0; j < M; ++j) {
      tot += s_cnt[j];
      if (s_cnt[j] > 0) mask |= 1 << j;
      if ((s_valid[j] & 3) != 3) unknown = true;
      sb = s_score[j] > sb ? s_score[j] : sb;
    }
    float* pk = hostv + s * 4;
    pk[0] = (float)(tot > 0 ? 1 : (unknown ? 2 : 0));
    pk[1] = sb;
    pk[2] = (float)mask;
    pk[3] = (float)tot;
  }
}

FM_API int fm_es_band_step(const float* buf, int64_t ld, const int* rm, const int* shift, const int* lim, int dk, int T,
                           int kmax, const int* t_new, const int64_t* slots, const float* params, int m, int kind,
                           float* season, float* sse, float* state, int* nobs, const float* cur, int64_t ld_c, int n,
                           const int64_t* hor, int H, int64_t S, int M, const float* thr, const int* bound,
                           const float* minlb, const int8_t* diff, float pair_factor, const int* valid,
                           const int64_t* lastk, float* upper, float* lower, float* sigma, float* fc, int Hf,
                           float* hostv, int cap, int* ctr, int par, int* out_idx, float* out_val, float* last3,
                           const int* cur_rm, hipStream_t stream) {
  if (S <= 0) return 0;
  // kind -1: the forecast fc [R, Hf] (Hf >= H) and sigma are given (band + reduce + compaction only)
  if (kind < -1 || kind > 3 || M < 1 || M > kStepMMax || n < 1 || n > 256 || H < 1 || (par != 0 && par != 1) ||
      (kind >= 0 && (kmax < 1 || kmax > kStepKMax || kmax > T || (kind >= 2 && m < 2))) ||
      (fc != nullptr && Hf < 1) || (kind < 0 && (fc == nullptr || Hf < H || sigma == nullptr)))
    return (int)hipErrorInvalidValue;
  if (kind < 2) m = 1;
  const dim3 grid((unsigned)S), block((unsigned)(64 * M));
#define FM_EBS(KK)                                                                                               \
  hipLaunchKernelGGL(es_band_step_kernel<KK>, grid, block, 0, stream, buf, ld, rm, shift, lim, dk, T, kmax, t_new, \
                     slots, params, m, season, sse, state, nobs, cur, ld_c, n, hor, H, S, M, thr, bound, minlb, diff, \
                     pair_factor, valid, lastk, upper, lower, sigma, fc, Hf, hostv, cap, ctr, par, out_idx, out_val, \
                     last3, cur_rm)
  if (kind == -1) FM_EBS(-1);
  else if (kind == 0) FM_EBS(0);
  else if (kind == 1) FM_EBS(1);
  else if (kind == 2) FM_EBS(2);
  else FM_EBS(3);
#undef FM_EBS
  FM_LAUNCH_CHECK();
  return 0;
}
