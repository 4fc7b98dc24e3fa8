// K1 rolling bands: per-time-point mean / population std of the finite samples
// in a trailing window of w points, for every row of a [R, T] fp32 batch
// (NaN = missing sample).  This is the [S*M, T] band output of SURVEY §2.4 K1
// (the dashboard's metric bands, foremast-dashboard/src/config/metrics.js:21-29,
// over the brain's moving_average window; deploy/foremast/3_brain/
// foremast-brain.yaml:24-25 names the algorithm).
//
// One 256-thread workgroup per row walks it in tiles of 2048 samples; thread
// i owns the 8 contiguous samples / outputs [8i, 8i + 8) of a tile (two 16-B
// loads, two 16-B stores per band).  Per tile: the shifted samples d = x - c
// (c = mean of the row's first tile, so squares do not swamp the variance;
// NaN kept for missing samples) go to an LDS ring of two tiles, a block scan
// gives each thread the tile-local exclusive prefix of (count, sum d, sum d^2)
// (sums fp64), and those 256 prefixes go to a second small ring.  A thread's
// first window sum is P(t0) - P(t0 - w): P(t0) is its own prefix, P(t0 - w)
// the owner segment's prefix plus up to 8 ring samples.  Its next 7 windows
// slide in registers (+ own sample, - the sample leaving the window).
// Because t0 is a multiple of 8, the offset (t0 - w) mod 8 = (-w) mod 8 is the
// same for every thread, so the leaving samples are a fixed rotation of two
// ring segments (a switch on a uniform value).  w <= 2048 keeps every window
// inside this tile and the previous one, bridged by the previous tile's
// totals, so prefixes stay tile-local.  LDS 26 KB: several workgroups per CU
// keep enough rows in flight (a first version held full fp64 prefix rings,
// 72 KB, two workgroups per CU: 2.45 TB/s).  HBM traffic: the row read once,
// the two bands written once.
#include "fm_common.h"

using namespace fm;

namespace {

constexpr int kTile = 2048;           // samples per tile = 256 threads x 8
constexpr int kRing = 2 * kTile;      // sample ring: this tile + the previous one

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

// contributions of one (shifted) sample: finite count, d, d^2
__device__ __forceinline__ void contrib(float d, float& n, float& s, float& q) {
  const bool f = isfinite(d);
  n = f ? 1.f : 0.f;
  s = f ? d : 0.f;
  q = s * s;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void rolling_stats_kernel(const float* __restrict__ x, int64_t ld_x, int T,
                                                            int w, int min_count, float* __restrict__ mean,
                                                            float* __restrict__ sd, int64_t ld_o) {
  __shared__ float4 ring4[kRing / 4];              // shifted samples (NaN = missing)
  __shared__ float exn[2 * 256];                    // per-thread exclusive prefixes, two tiles
  __shared__ double exs[2 * 256], exq[2 * 256];
  __shared__ Tri scratch[4];
  __shared__ double red[4];
  const int64_t row = blockIdx.x;
  const float* __restrict__ xr = x + row * ld_x;
  float* __restrict__ mr = mean + row * ld_o;
  float* __restrict__ sr = sd + row * ld_o;
  const int tid = threadIdx.x;
  const float NaNf = __builtin_nanf("");
  const float* ring = reinterpret_cast<const float*>(ring4);
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
  const int r = (-w) & 7;                     // (t0 - w) mod 8, the same for every thread
  const int segback = (w + r) >> 3;           // owner segment of t0 - w is (own segment) - segback
  float c = 0.f;
  Tri prev_total{0.f, 0.0, 0.0};
  float nx[8];
  load8(0, nx);
  for (int tb = 0, tile = 0; tb < T; tb += kTile, ++tile) {
    float d[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] = nx[k];
    if (tb + kTile < T) load8(tb + kTile, nx);   // in flight while this tile is scanned and written
    if (tile == 0) {
      float ls = 0.f, lc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (isfinite(d[k])) { ls += d[k]; lc += 1.f; }
      const double s = block_sum<256>((double)ls, red);
      const double n = block_sum<256>((double)lc, red);
      c = n > 0 ? (float)(s / n) : 0.f;
    }
    float an = 0.f, as = 0.f, aq = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      d[k] = d[k] - c;                        // NaN stays NaN
      float n, s, q;
      contrib(d[k], n, s, q);
      an += n; as += s; aq = fmaf(s, s, aq);
    }
    const int half = tile & 1;
    ring4[half * (kTile / 4) + 2 * tid] = make_float4(d[0], d[1], d[2], d[3]);
    ring4[half * (kTile / 4) + 2 * tid + 1] = make_float4(d[4], d[5], d[6], d[7]);
    Tri total;
    const Tri incl = block_incl_scan(Tri{an, (double)as, (double)aq}, scratch, total);
    const float en = incl.n - an;
    const double es = incl.s - (double)as, eq = incl.q - (double)aq;
    exn[half * 256 + tid] = en;
    exs[half * 256 + tid] = es;
    exq[half * 256 + tid] = eq;
    __syncthreads();
    // P(t0 - w), relative to this tile's carry, and the 8 samples leaving
    // the 8 windows: positions g0 .. g0 + 7 (g0 = t0 - w)
    const int seg = (tb >> 3) + tid - segback;        // global owner segment of g0 (may be < 0)
    float lv[16];
    double pn = 0.0, ps = 0.0, pq = 0.0;
    if (seg + 1 >= 0) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int sg = seg + h;
        float4 a = make_float4(NaNf, NaNf, NaNf, NaNf), b = a;
        if (sg >= 0) {
          const int rbase = ((sg >> 8) & 1) * (kTile / 4) + (sg & 255) * 2;
          a = ring4[rbase];
          b = ring4[rbase + 1];
        }
        lv[8 * h + 0] = a.x; lv[8 * h + 1] = a.y; lv[8 * h + 2] = a.z; lv[8 * h + 3] = a.w;
        lv[8 * h + 4] = b.x; lv[8 * h + 5] = b.y; lv[8 * h + 6] = b.z; lv[8 * h + 7] = b.w;
      }
      if (seg >= 0) {
        const int eh = ((seg >> 8) & 1) * 256 + (seg & 255);
        pn = exn[eh]; ps = exs[eh]; pq = exq[eh];
        float sn = 0.f, ss = 0.f, sq = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float n, s, q;
          contrib(lv[i], n, s, q);
          if (i <= r) { sn += n; ss += s; sq = fmaf(s, s, sq); }
        }
        pn += sn; ps += ss; pq += sq;
        if ((seg >> 8) != tile) { pn -= prev_total.n; ps -= prev_total.s; pq -= prev_total.q; }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) lv[i] = NaNf;
    }
    // leaving sample of window k is lv[r + 1 + k] (k < 7 slides); rotate by the uniform r
    float out[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = lv[k + 8];
    switch (r) {
#define FM_ROT(RR) case RR: _Pragma("unroll") for (int k = 0; k < 8; ++k) out[k] = lv[RR + 1 + k < 16 ? RR + 1 + k : 15]; break;
      FM_ROT(0) FM_ROT(1) FM_ROT(2) FM_ROT(3) FM_ROT(4) FM_ROT(5) FM_ROT(6) FM_ROT(7)
#undef FM_ROT
    }
    // window 0 = P(t0) - P(g0); window k = window k-1 + own d[k] - leaving out[k-1]
    double wn = (double)en - pn, ws = es - ps, wq = eq - pq;
    float om[8], os[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float n, s, q;
      contrib(d[k], n, s, q);
      wn += n; ws += s; wq += q;
      if (k > 0) {
        contrib(out[k - 1], n, s, q);
        wn -= n; ws -= s; wq -= q;
      }
      if (wn >= (double)min_count && wn > 0.5) {
        // wn is an integer <= 2048: a 1-ulp fp32 reciprocal is exact enough,
        // and the moments stay fp64 until the variance is formed (no fp64
        // divide / sqrt sequences per output)
        const double inv = (double)__builtin_amdgcn_rcpf((float)wn);
        const double m = ws * inv;
        om[k] = c + (float)m;
        os[k] = sqrtf((float)fmax(fma(-m, m, wq * inv), 0.0));
      } else {
        om[k] = NaNf;
        os[k] = NaNf;
      }
    }
    const int t0 = tb + 8 * tid;
    if (t0 + 8 <= T && (ld_o & 3) == 0) {
      *reinterpret_cast<float4*>(mr + t0) = make_float4(om[0], om[1], om[2], om[3]);
      *reinterpret_cast<float4*>(mr + t0 + 4) = make_float4(om[4], om[5], om[6], om[7]);
      *reinterpret_cast<float4*>(sr + t0) = make_float4(os[0], os[1], os[2], os[3]);
      *reinterpret_cast<float4*>(sr + t0 + 4) = make_float4(os[4], os[5], os[6], os[7]);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (t0 + k < T) { mr[t0 + k] = om[k]; sr[t0 + k] = os[k]; }
    }
    prev_total = total;
    // the next tile overwrites the ring half this tile read as "previous"
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
