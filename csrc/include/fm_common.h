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
// Wave index within the workgroup, as a wave-uniform (SGPR) value: rows and
// addresses derived from it stay scalar instead of being recomputed per lane
// in 64-bit VALU arithmetic.  Block x-dimensions are multiples of 64.
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x / FM_WAVE); }

// ---------------------------------------------------------------------------
// Cross-lane primitives without the LDS crossbar.  __shfl_xor lowers to
// ds_bpermute_b32 (an LDS-pipe round trip per exchange); inside a 16-lane row
// DPP does the same exchange as a VALU operand modifier, and the gfx950
// v_permlane16_swap / v_permlane32_swap move whole rows / half-waves:
//   xor 1, 2  quad_perm [1,0,3,2] / [2,3,0,1]
//   xor 4     row_shl:4 for lanes with bit 2 clear, row_shr:4 otherwise
//   xor 8     row_ror:8 (a rotate by half a row IS the xor)
//   xor 16    permlane16_swap(v, v): rows {r0,r0,r2,r2} / {r1,r1,r3,r3}
//   xor 32    permlane32_swap(v, v): halves {lo,lo} / {hi,hi}
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ unsigned xor_lane_u32(unsigned v) {
  // mov_dpp (no "old" operand): every lane we keep has a valid source, so
  // no v_mov to pre-initialise the destination is needed
  if constexpr (S == 1) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
  } else if constexpr (S == 2) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, true);
  } else if constexpr (S == 4) {
    const unsigned up = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x104, 0xF, 0xF, true);
    const unsigned dn = (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x114, 0xF, 0xF, true);
    return (lane_id() & 4) ? dn : up;
  } else if constexpr (S == 8) {
    return (unsigned)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
  } else if constexpr (S == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    return (lane_id() & 16) ? r[0] : r[1];
  } else {
    static_assert(S == 32, "xor stride must be a power of two < 64");
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return (lane_id() & 32) ? r[0] : r[1];
  }
}

// DPP move with compile-time control; lanes whose source is invalid get `old`.
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_mov(T old, T x) {
  static_assert(sizeof(T) == 4, "32-bit");
  return __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_update_dpp(
      (int)__builtin_bit_cast(unsigned, old), (int)__builtin_bit_cast(unsigned, x), CTRL, 0xF, 0xF, false));
}

template <int S, typename T>
__device__ __forceinline__ T xor_lane(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "32/64-bit lanes only");
  if constexpr (sizeof(T) == 4) {
    return __builtin_bit_cast(T, xor_lane_u32<S>(__builtin_bit_cast(unsigned, v)));
  } else {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = xor_lane_u32<S>((unsigned)u), hi = xor_lane_u32<S>((unsigned)(u >> 32));
    return __builtin_bit_cast(T, ((unsigned long long)hi << 32) | lo);
  }
}

// Runtime-stride form for unrolled loops (the switch folds to one case).
template <typename T>
__device__ __forceinline__ T xor_lane_any(T v, int s) {
  switch (s) {
    case 1: return xor_lane<1>(v);
    case 2: return xor_lane<2>(v);
    case 4: return xor_lane<4>(v);
    case 8: return xor_lane<8>(v);
    case 16: return xor_lane<16>(v);
    default: return xor_lane<32>(v);
  }
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
  v += xor_lane<1>(v); v += xor_lane<2>(v); v += xor_lane<4>(v);
  v += xor_lane<8>(v); v += xor_lane<16>(v); v += xor_lane<32>(v);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
  T w;
  w = xor_lane<1>(v); v = v > w ? v : w;
  w = xor_lane<2>(v); v = v > w ? v : w;
  w = xor_lane<4>(v); v = v > w ? v : w;
  w = xor_lane<8>(v); v = v > w ? v : w;
  w = xor_lane<16>(v); v = v > w ? v : w;
  w = xor_lane<32>(v); v = v > w ? v : w;
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
  T w;
  w = xor_lane<1>(v); v = v < w ? v : w;
  w = xor_lane<2>(v); v = v < w ? v : w;
  w = xor_lane<4>(v); v = v < w ? v : w;
  w = xor_lane<8>(v); v = v < w ? v : w;
  w = xor_lane<16>(v); v = v < w ? v : w;
  w = xor_lane<32>(v); v = v < w ? v : w;
  return v;
}

// Inclusive prefix scans over the 64 lanes (Hillis-Steele: row_shr 1,2,4,8
// inside each 16-lane row, then the row totals carried by permlane swaps).
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan_dpp(T v, T ident, Op op) {
  static_assert(sizeof(T) == 4, "32-bit scans");
  const int l = lane_id();
  v = op(v, dpp_mov<0x111>(ident, v));  // row_shr:1 (lanes with l%16 < 1 read the identity)
  v = op(v, dpp_mov<0x112>(ident, v));
  v = op(v, dpp_mov<0x114>(ident, v));
  v = op(v, dpp_mov<0x118>(ident, v));
  // row r's total sits in lane 16r+15; carry row 0 -> 1 and row 2 -> 3
  const T t15 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 15));
  const T t47 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 47));
  if ((l >> 4) == 1) v = op(v, t15);
  if ((l >> 4) == 3) v = op(v, t47);
  const T t31 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 31));
  if (l >= 32) v = op(v, t31);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_incl_sum(T v) {
  if constexpr (sizeof(T) == 4) {
    return wave_incl_scan_dpp(v, (T)0, [](T a, T b) { return a + b; });
  } else {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) { T w = __shfl_up(v, o); if (l >= o) v += w; }
    return v;
  }
}
template <typename T>
__device__ __forceinline__ T wave_incl_max(T v, T ident) {
  return wave_incl_scan_dpp(v, ident, [](T a, T b) { return a > b ? a : b; });
}
template <typename T>
__device__ __forceinline__ T wave_incl_max(T v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) { T w = __shfl_up(v, o); if (l >= o) v = v > w ? v : w; }
  return v;
}
// Inclusive suffix scan, 32-bit (row_shl 1,2,4,8 inside rows, then row totals
// carried downward through readlane of each row's first lane).
template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_suffix_scan_dpp(T v, T ident, Op op) {
  static_assert(sizeof(T) == 4, "32-bit scans");
  const int l = lane_id();
  v = op(v, dpp_mov<0x101>(ident, v));  // row_shl:1 (lane i reads i+1 inside the row)
  v = op(v, dpp_mov<0x102>(ident, v));
  v = op(v, dpp_mov<0x104>(ident, v));
  v = op(v, dpp_mov<0x108>(ident, v));
  const T t16 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 16));
  const T t48 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 48));
  if ((l >> 4) == 0) v = op(v, t16);
  if ((l >> 4) == 2) v = op(v, t48);
  const T t32 = __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), 32));
  if (l < 32) v = op(v, t32);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_incl_suffix_min(T v, T ident) {
  return wave_incl_suffix_scan_dpp(v, ident, [](T a, T b) { return a < b ? a : b; });
}

// Neighbour lanes across the whole wave (gfx9 DPP wave_shr:1 / wave_shl:1);
// lane 0 (resp. 63) receives `edge`.
template <typename T>
__device__ __forceinline__ T lane_prev(T v, T edge) { return dpp_mov<0x138>(edge, v); }
template <typename T>
__device__ __forceinline__ T lane_next(T v, T edge) { return dpp_mov<0x130>(edge, v); }
template <typename T>
__device__ __forceinline__ T lane_bcast(T v, int lane) {
  static_assert(sizeof(T) == 4, "32-bit");
  return __builtin_bit_cast(T, (unsigned)__builtin_amdgcn_readlane((int)__builtin_bit_cast(unsigned, v), lane));
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

// 1/x from the hardware reciprocal estimate refined by two Newton steps
// (4 dependent FMAs) instead of the IEEE division sequence (div_scale x2,
// rcp, 5 FMAs, div_fmas, div_fixup): relative error ~1 ulp for the normal,
// finite arguments the continued fractions below produce.
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// Continued fraction for the regularized incomplete beta (modified Lentz).
// The recurrence is latency-bound (one row per thread; the Welch t-test is
// the slowest p-value), so its dependent chain is kept short: the partial
// numerators aa(m) do not depend on the recurrence and are computed off the
// chain, and the reciprocals are rcp_nr instead of IEEE divisions.
__device__ inline double betacf(double a, double b, double x) {
  const double tiny = 1e-300;
  const double qab = a + b, qap = a + 1.0, qam = a - 1.0;
  double c = 1.0, d = 1.0 - qab * x / qap;
  if (fabs(d) < tiny) d = tiny;
  d = rcp_nr(d);
  double h = d;
  for (int m = 1; m <= 400; ++m) {
    const double m2 = 2.0 * m, dm = m;
    const double ao = dm * (b - dm) * x * rcp_nr((qam + m2) * (a + m2));
    const double ae = -(a + dm) * (qab + dm) * x * rcp_nr((a + m2) * (qap + m2));
    d = fma(ao, d, 1.0); if (fabs(d) < tiny) d = tiny;
    c = fma(ao, rcp_nr(c), 1.0); if (fabs(c) < tiny) c = tiny;
    d = rcp_nr(d); h *= d * c;
    d = fma(ae, d, 1.0); if (fabs(d) < tiny) d = tiny;
    c = fma(ae, rcp_nr(c), 1.0); if (fabs(c) < tiny) c = tiny;
    d = rcp_nr(d);
    const double del = d * c; h *= del;
    if (fabs(del - 1.0) < 3e-15) break;
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
