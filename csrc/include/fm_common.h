// Shared device helpers for the foremast_amd CDNA4 (gfx950) kernel library.
//
// Every kernel in csrc/kernels is written for 64-wide wavefronts: reductions,
// scans and sorts are wave-synchronous over 64 lanes, workgroups are multiples
// of 64 threads, and rows of metric data are mapped to whole waves or whole
// workgroups so that loads stay 16-B vectorised and coalesced.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#define FM_WAVE 64

#define FM_API extern "C" __attribute__((visibility("default")))

// Launch-check helper: every host entry point returns a hipError_t as int.
#define FM_LAUNCH_CHECK() do { hipError_t _e = hipGetLastError(); if (_e != hipSuccess) return (int)_e; } while (0)

namespace fm {

__device__ __forceinline__ int lane_id() { return threadIdx.x & (FM_WAVE - 1); }
__device__ __forceinline__ int wave_id() { return threadIdx.x / FM_WAVE; }

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o); v = v > w ? v : w; }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) { T w = __shfl_xor(v, o); v = v < w ? v : w; }
  return v;
}

// Inclusive prefix sum over the 64 lanes of a wave.
template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) { T w = __shfl_up(v, o); if (l >= o) v += w; }
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) { T w = __shfl_up(v, o); if (l >= o) v = v > w ? v : w; }
  return v;
}
// Inclusive suffix min (lane l sees min over lanes l..63).
template <typename T>
__device__ __forceinline__ T wave_incl_suffix_min(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) { T w = __shfl_down(v, o); if (l + o < 64) v = v < w ? v : w; }
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` must hold NT/64 entries.
template <int NT, typename T>
__device__ __forceinline__ T block_sum(T v, T* scratch) {
  v = wave_sum(v);
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  T r = 0;
#pragma unroll
  for (int w = 0; w < NT / FM_WAVE; ++w) r += scratch[w];
  __syncthreads();
  return r;
}
template <int NT, typename T>
__device__ __forceinline__ T block_max(T v, T* scratch) {
  v = wave_max(v);
  if (lane_id() == 0) scratch[wave_id()] = v;
  __syncthreads();
  T r = scratch[0];
#pragma unroll
  for (int w = 1; w < NT / FM_WAVE; ++w) r = r > scratch[w] ? r : scratch[w];
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// Counter-based RNG (integer finaliser hash).  Identical arithmetic is used by
// the numpy oracle in foremast_amd/ops/reference.py so CPU and GPU synthetic
// fleets agree element for element (up to libm sin/cos/log rounding).
__host__ __device__ __forceinline__ uint32_t hash_u32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU;
  x ^= x >> 15; x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
__host__ __device__ __forceinline__ uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  return hash_u32(a * 0x9E3779B1U ^ hash_u32(b * 0x85EBCA77U ^ hash_u32(c + 0x165667B1U)));
}
// uniform in (0, 1]
__host__ __device__ __forceinline__ float u01(uint32_t h) { return ((float)(h >> 8) + 1.0f) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------------------
// Special functions for p-values (double precision; one evaluation per row).
__device__ __forceinline__ double norm_sf(double z) { return 0.5 * erfc(z * 0.70710678118654752440); }

// Regularized lower incomplete gamma P(a,x) / upper Q(a,x).
__device__ inline double gamma_q(double a, double x) {
  if (!(x > 0.0)) return 1.0;
  const double gln = lgamma(a);
  if (x < a + 1.0) {  // series for P
    double ap = a, sum = 1.0 / a, del = sum;
    for (int n = 0; n < 500; ++n) {
      ap += 1.0; del *= x / ap; sum += del;
      if (fabs(del) < fabs(sum) * 1e-15) break;
    }
    double p = sum * exp(-x + a * log(x) - gln);
    return 1.0 - p;
  }
  // continued fraction for Q (modified Lentz)
  const double tiny = 1e-300;
  double b = x + 1.0 - a, c = 1.0 / tiny, d = 1.0 / b, h = d;
  for (int i = 1; i < 500; ++i) {
    double an = -i * (i - a);
    b += 2.0;
    d = an * d + b; if (fabs(d) < tiny) d = tiny;
    c = b + an / c; if (fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    double del = d * c; h *= del;
    if (fabs(del - 1.0) < 1e-15) break;
  }
  return exp(-x + a * log(x) - gln) * h;
}
__device__ __forceinline__ double chi2_sf(double x, double df) { return gamma_q(0.5 * df, 0.5 * x); }

// Continued fraction for the regularized incomplete beta (modified Lentz).
__device__ inline double betacf(double a, double b, double x) {
  const double tiny = 1e-300;
  double qab = a + b, qap = a + 1.0, qam = a - 1.0;
  double c = 1.0, d = 1.0 - qab * x / qap;
  if (fabs(d) < tiny) d = tiny;
  d = 1.0 / d;
  double h = d;
  for (int m = 1; m <= 400; ++m) {
    int m2 = 2 * m;
    double aa = m * (b - m) * x / ((qam + m2) * (a + m2));
    d = 1.0 + aa * d; if (fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c; if (fabs(c) < tiny) c = tiny;
    d = 1.0 / d; h *= d * c;
    aa = -(a + m) * (qab + m) * x / ((a + m2) * (qap + m2));
    d = 1.0 + aa * d; if (fabs(d) < tiny) d = tiny;
    c = 1.0 + aa / c; if (fabs(c) < tiny) c = tiny;
    d = 1.0 / d;
    double del = d * c; h *= del;
    if (fabs(del - 1.0) < 1e-15) break;
  }
  return h;
}
__device__ inline double betainc_reg(double a, double b, double x) {
  if (x <= 0.0) return 0.0;
  if (x >= 1.0) return 1.0;
  double lbt = lgamma(a + b) - lgamma(a) - lgamma(b) + a * log(x) + b * log1p(-x);
  double bt = exp(lbt);
  if (x < (a + 1.0) / (a + b + 2.0)) return bt * betacf(a, b, x) / a;
  return 1.0 - bt * betacf(b, a, 1.0 - x) / b;
}
// Two-sided Student-t p-value.
__device__ __forceinline__ double student_t_2sided(double t, double df) {
  double x = df / (df + t * t);
  return betainc_reg(0.5 * df, 0.5, x);
}
// Asymptotic Kolmogorov survival Q_KS(lambda) = 2 sum (-1)^{k-1} exp(-2 k^2 lambda^2).
__device__ inline double kolmogorov_sf(double lam) {
  if (lam < 0.18) return 1.0;
  if (lam < 1.18) {
    // small-lambda form: 1 - sqrt(2 pi)/lam * sum exp(-(2k-1)^2 pi^2 / (8 lam^2))
    double s = 0.0, f = -(M_PI * M_PI) / (8.0 * lam * lam);
    for (int k = 1; k <= 8; k += 1) { int o = 2 * k - 1; s += exp(f * o * o); }
    double cdf = 2.5066282746310002 / lam * s;
    return 1.0 - cdf;
  }
  double s = 0.0, sign = 1.0;
  for (int k = 1; k <= 100; ++k) {
    double term = exp(-2.0 * k * k * lam * lam);
    s += sign * term; sign = -sign;
    if (term < 1e-17) break;
  }
  double p = 2.0 * s;
  return p < 0.0 ? 0.0 : (p > 1.0 ? 1.0 : p);
}

}  // namespace fm
