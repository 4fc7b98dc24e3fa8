// K2: exponential smoothing family (single / double (Holt) / Holt-Winters
// additive) with a batched parameter-grid fit.
//
// Reference: the brain's model zoo lists Exponential Smoothing, Double
// Exponential Smoothing and Holt-Winters (docs/guides/design.md:62-72); the
// statistics follow the textbook additive recursions (docs/BRAIN_SPEC.md §3.2).
//
// Mapping: one THREAD per (row, candidate) pair, candidates fastest, so the
// lanes that share a row read the same history sample (one coalesced request).
// The Holt-Winters seasonal state (m floats per pair) lives in a global
// scratch laid out [m][pairs]: at step t every lane touches phase t % m of its
// own column, i.e. one coalesced 256-B load + store per wave per step.  At the
// BASELINE config-2 shape (40k series x 27 candidates x m=1440) that is 6 GB of
// scratch, deliberately spent from the 288 GB of HBM instead of serialising the
// grid.
#include "fm_common.h"

using namespace fm;

struct Cand { float a, b, g; };
constexpr int kPrefetch = 16;  // season/sample loads issued ahead per chunk (HW fit)

// kind: 0 = SES, 1 = Holt (double), 2 = Holt-Winters additive
template <int KIND>
__global__ __launch_bounds__(256) void es_fit_kernel(const float* __restrict__ x, int64_t ld, int T, int64_t R,
                                                    const float* __restrict__ cand, int G, int m,
                                                    float* __restrict__ season /*[m][R*G]*/, float* __restrict__ sse,
                                                    float* __restrict__ state /*[R*G,3]*/, int* __restrict__ nobs) {
  const int64_t pid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t P = R * G;
  if (pid >= P) return;
  const int64_t row = pid / G;
  const int g = (int)(pid - row * G);
  const float al = cand[3 * g + 0], be = cand[3 * g + 1], ga = cand[3 * g + 2];
  const float* xr = x + row * ld;
  float lvl, tr = 0.f;
  int t0;
  if (KIND == 2) {
    // initial level = mean of season 1, trend = (mean season 2 - mean season 1)/m,
    // seasonal indices = x_i - level over season 1
    float s1 = 0.f, s2 = 0.f;
    for (int i = 0; i < m; ++i) { s1 += xr[i]; s2 += xr[m + i]; }
    s1 /= m; s2 /= m;
    lvl = s1;
    tr = (s2 - s1) / m;
    for (int i = 0; i < m; ++i) season[(int64_t)i * P + pid] = xr[i] - s1;
    t0 = m;
  } else if (KIND == 1) {
    lvl = xr[0];
    tr = xr[1] - xr[0];
    t0 = 1;
  } else {
    lvl = xr[0];
    t0 = 1;
  }
  double err2 = 0.0;
  float acc = 0.f;
  int n = 0, chunk = 0;
  int ph = 0;  // t % m, advanced incrementally (no per-step integer modulo)
  int t = t0;
  if (KIND == 2 && m > kPrefetch) {
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
        si[u] = (int64_t)pu * P + pid;
        sv[u] = season[si[u]];
        xv[u] = xr[t + u];
      }
      ph += kPrefetch;
      if (ph >= m) ph -= m;
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) {
        const float xt = xv[u], s_old = sv[u];
        const float pred = lvl + tr + s_old;
        if (isfinite(xt)) {
          const float e = xt - pred;
          acc += e * e;
          ++n;
          const float lprev = lvl;
          lvl = al * (xt - s_old) + (1.f - al) * (lvl + tr);
          tr = be * (lvl - lprev) + (1.f - be) * tr;
          sv[u] = ga * (xt - lvl) + (1.f - ga) * s_old;
        } else {
          lvl = lvl + tr;
        }
      }
#pragma unroll
      for (int u = 0; u < kPrefetch; ++u) season[si[u]] = sv[u];
      chunk += kPrefetch;
      if (chunk >= 64) { err2 += acc; acc = 0.f; chunk = 0; }
    }
  }
  for (; t < T; ++t) {
    const float xt = xr[t];
    float s_old = 0.f;
    int64_t sidx = 0;
    if (KIND == 2) { sidx = (int64_t)ph * P + pid; s_old = season[sidx]; if (++ph == m) ph = 0; }
    const float pred = lvl + tr + s_old;
    if (isfinite(xt)) {
      const float e = xt - pred;
      acc += e * e;
      ++n;
      if (++chunk == 64) { err2 += acc; acc = 0.f; chunk = 0; }
      const float lprev = lvl;
      if (KIND == 0) {
        lvl = al * xt + (1.f - al) * lvl;
      } else if (KIND == 1) {
        lvl = al * xt + (1.f - al) * (lvl + tr);
        tr = be * (lvl - lprev) + (1.f - be) * tr;
      } else {
        lvl = al * (xt - s_old) + (1.f - al) * (lvl + tr);
        tr = be * (lvl - lprev) + (1.f - be) * tr;
        season[sidx] = ga * (xt - lvl) + (1.f - ga) * s_old;
      }
    } else {
      // missing sample: propagate the forecast
      lvl = lvl + tr;
    }
  }
  err2 += acc;
  sse[pid] = (float)err2;
  state[pid * 3 + 0] = lvl;
  state[pid * 3 + 1] = tr;
  state[pid * 3 + 2] = (float)(T % (m > 0 ? m : 1));
  nobs[pid] = n;
}

// Per row: pick the candidate with the smallest SSE and write the H-step
// forecast + residual sigma.
__global__ __launch_bounds__(256) void es_forecast_kernel(const float* __restrict__ sse, const float* __restrict__ state,
                                                          const int* __restrict__ nobs, const float* __restrict__ season,
                                                          int64_t R, int G, int m, int kind, int H,
                                                          float* __restrict__ fc /*[R,H]*/, float* __restrict__ sigma,
                                                          int* __restrict__ best) {
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
    if (kind == 2) f += season[(int64_t)((tph + h - 1) % m) * P + pid];
    fc[row * H + (h - 1)] = f;
  }
}

FM_API int fm_es_fit(const float* x, int64_t ld, int T, int64_t R, const float* cand, int G, int m, int kind,
                     float* season, float* sse, float* state, int* nobs, int H, float* fc, float* sigma, int* best,
                     hipStream_t stream) {
  if (R <= 0) return 0;
  if (kind == 2 && (m < 2 || 2 * m > T)) return (int)hipErrorInvalidValue;
  if (kind < 2 && T < 2) return (int)hipErrorInvalidValue;
  const int64_t P = R * G;
  const dim3 grid((unsigned)((P + 255) / 256)), block(256);
  if (kind == 0)
    hipLaunchKernelGGL(es_fit_kernel<0>, grid, block, 0, stream, x, ld, T, R, cand, G, m, season, sse, state, nobs);
  else if (kind == 1)
    hipLaunchKernelGGL(es_fit_kernel<1>, grid, block, 0, stream, x, ld, T, R, cand, G, m, season, sse, state, nobs);
  else
    hipLaunchKernelGGL(es_fit_kernel<2>, grid, block, 0, stream, x, ld, T, R, cand, G, m, season, sse, state, nobs);
  FM_LAUNCH_CHECK();
  hipLaunchKernelGGL(es_forecast_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, stream, sse, state, nobs,
                     season, R, G, m, kind, H, fc, sigma, best);
  FM_LAUNCH_CHECK();
  return 0;
}

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
