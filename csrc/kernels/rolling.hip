// K1 rolling bands: per-time-point mean / population std of the finite samples
// in a trailing window of w points, for every row of a [R, T] fp32 batch
// (NaN = missing sample).  This is the [S*M, T] band output of SURVEY §2.4 K1
// (the dashboard's metric bands, foremast-dashboard/src/config/metrics.js:21-29,
// over the brain's moving_average window; deploy/foremast/3_brain/
// foremast-brain.yaml:24-25 names the algorithm).
//
// One 256-thread workgroup per row walks it in tiles of 2048 samples (8
// contiguous samples per thread, two 16-B loads).  Per tile: thread-local
// prefix sums of (count, d, d^2) with d = x - c (c = mean of the row's first
// tile, so the squares do not swamp the variance), a wave scan on DPP and a
// 4-entry cross-wave pass, and the tile-local prefixes go to an LDS ring of
// two tiles (counts uint16, sums fp64: 72 KB, two workgroups per CU).  The
// next tile's samples are loaded while this tile's outputs are written.  A window
// sum is then P[t] - P[t - w]: both ends sit in this tile or the previous one
// (w <= 2048), so only the previous tile's totals bridge the two and every
// prefix stays tile-local (no row-long running sum).  The sums are fp64 because
// a fp32 prefix difference over a 2048-sample tile loses ~2048 ulps of the
// tile's sum of squares: for a 1-point window that is a std of 1 % of the
// row's instead of 0.  Outputs are written one sample per thread per
// 256-wide stripe: coalesced.  HBM traffic: the row read once, the two bands
// written once.
#include "fm_common.h"

using namespace fm;

namespace {

constexpr int kTile = 2048;           // samples per tile = 256 threads x 8
constexpr int kRing = 2 * kTile;      // LDS ring: this tile + the previous one

struct Tri {
  float n;
  double s, q;
};

__device__ __forceinline__ Tri tri_add(Tri a, Tri b) { return Tri{a.n + b.n, a.s + b.s, a.q + b.q}; }

// inclusive block scan of one Tri per thread (256 threads); also returns the
// block total.  scratch: 4 Tri in LDS.
__device__ __forceinline__ Tri block_incl_scan(Tri v, Tri* scratch, Tri& total) {
  Tri w{wave_incl_sum(v.n), wave_incl_sum(v.s), wave_incl_sum(v.q)};
  const int wid = wave_id();
  if (lane_id() == 63) scratch[wid] = w;
  __syncthreads();
  Tri off{0.f, 0.0, 0.0};
  for (int i = 0; i < wid; ++i) off = tri_add(off, scratch[i]);
  total = tri_add(tri_add(scratch[0], scratch[1]), tri_add(scratch[2], scratch[3]));
  __syncthreads();   // scratch is reused by the next tile
  return tri_add(w, off);
}

__global__ __launch_bounds__(256) void rolling_stats_kernel(const float* __restrict__ x, int64_t ld_x, int T,
                                                            int w, int min_count, float* __restrict__ mean,
                                                            float* __restrict__ sd, int64_t ld_o) {
  __shared__ unsigned short pn[kRing];
  __shared__ double ps[kRing], pq[kRing];
  __shared__ Tri scratch[4];
  __shared__ double red[4];
  const int64_t row = blockIdx.x;
  const float* __restrict__ xr = x + row * ld_x;
  float* __restrict__ mr = mean + row * ld_o;
  float* __restrict__ sr = sd + row * ld_o;
  const int tid = threadIdx.x;
  const float NaNf = __builtin_nanf("");
  float c = 0.f;
  Tri prev_total{0.f, 0.0, 0.0};
  // 8 contiguous samples per thread
  auto load8 = [&](int tb, float (&v)[8]) {
    const int e0 = tb + 8 * tid;
    if (e0 + 8 <= T) {
      const float4 a = *reinterpret_cast<const float4*>(xr + e0);
      const float4 b = *reinterpret_cast<const float4*>(xr + e0 + 4);
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = e0 + k < T ? xr[e0 + k] : NaNf;
    }
  };
  float nx[8];
  load8(0, nx);
  for (int tb = 0, tile = 0; tb < T; tb += kTile, ++tile) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = nx[k];
    if (tb + kTile < T) load8(tb + kTile, nx);   // in flight while this tile is scanned and written
    if (tile == 0) {
      // shift: mean of the first tile's finite samples
      float ls = 0.f, lc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (isfinite(v[k])) { ls += v[k]; lc += 1.f; }
      const double s = block_sum<256>((double)ls, red);
      const double n = block_sum<256>((double)lc, red);
      c = n > 0 ? (float)(s / n) : 0.f;
    }
    // thread-local inclusive prefixes (8 terms: fp32 is exact enough)
    float ln[8], ls[8], lq[8];
    float an = 0.f, as = 0.f, aq = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool f = isfinite(v[k]);
      const float d = f ? v[k] - c : 0.f;
      an += f ? 1.f : 0.f;
      as += d;
      aq = fmaf(d, d, aq);
      ln[k] = an; ls[k] = as; lq[k] = aq;
    }
    Tri total;
    const Tri incl = block_incl_scan(Tri{an, (double)as, (double)aq}, scratch, total);
    const float en = incl.n - an;
    const double es = incl.s - (double)as, eq = incl.q - (double)aq;
    const int rb = (tile & 1) * kTile;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = rb + 8 * tid + k;
      pn[i] = (unsigned short)(en + ln[k]);
      ps[i] = es + (double)ls[k];
      pq[i] = eq + (double)lq[k];
    }
    __syncthreads();
    // outputs of this tile: one per thread per 256-wide stripe
    const int pb = ((tile + 1) & 1) * kTile;   // ring base of the previous tile
#pragma unroll 2
    for (int j = tid; j < kTile; j += 256) {
      const int t = tb + j;
      if (t >= T) break;
      float n = (float)pn[rb + j];
      double s = ps[rb + j], q = pq[rb + j];
      const int u = j - w;     // t - w, relative to this tile
      if (u >= 0) {
        n -= (float)pn[rb + u]; s -= ps[rb + u]; q -= pq[rb + u];
      } else if (t - w >= 0) {
        // the window starts in the previous tile: its prefix there is
        // P_prev[u + kTile], and the previous tile's total bridges the two
        n += prev_total.n - (float)pn[pb + u + kTile];
        s += prev_total.s - ps[pb + u + kTile];
        q += prev_total.q - pq[pb + u + kTile];
      }   // else t < w: the window is [0, t], whose prefix is already tile 0's
      if (n >= (float)min_count && n > 0.f) {
        const double inv = 1.0 / (double)n;
        const double m = s * inv;
        const double var = fmax(q * inv - m * m, 0.0);
        mr[t] = c + (float)m;
        sr[t] = (float)sqrt(var);
      } else {
        mr[t] = NaNf;
        sr[t] = NaNf;
      }
    }
    prev_total = total;
    // the next tile overwrites the ring half this tile's outputs read as
    // "previous": wait for every output of this tile first
    __syncthreads();
  }
}

}  // namespace

// x [R, ld_x] fp32 (16-B aligned rows), 1 <= w <= 2048; mean / sd [R, ld_o].
FM_API int fm_rolling_stats(const float* x, int64_t ld_x, int T, int64_t R, int w, int min_count, float* mean,
                            float* sd, int64_t ld_o, hipStream_t stream) {
  if (R <= 0 || T <= 0) return 0;
  if (w < 1 || w > kTile || (ld_x & 3) != 0 || (((uintptr_t)x) & 15) != 0 || ld_o < T || ld_x < T)
    return (int)hipErrorInvalidValue;
  if (R > 0x7fffffffLL) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(rolling_stats_kernel, dim3((unsigned)R), dim3(256), 0, stream, x, ld_x, T, w, min_count, mean,
                     sd, ld_o);
  FM_LAUNCH_CHECK();
  return 0;
}
