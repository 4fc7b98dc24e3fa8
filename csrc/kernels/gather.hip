// Row gather out of the device-resident history (engine/resident.py) for the
// forecasting models of the brain's fast path (engine/fastpath.py).
//
// moving_average_all reads resident rows in place through a row map; the
// forecasters (exponential smoothing / Holt-Winters, Prophet, LSTM,
// bivariate) need each row RIGHT-aligned at the end of its history (the
// forecast horizon of a current point counts from the last history sample),
// while static rows are stored left-aligned.  This kernel copies, for every
// output row r and column j < ncols,
//
//     out[r, j] = src[rm[r], off[r] + j]   if 0 <= off[r] + j < lim[r]
//               = NaN                      otherwise
//
// so one launch builds either the whole right-aligned window (a cold fit) or
// only its last k columns (a cached model advanced over k new samples, an
// LSTM lookback of L samples) -- a steady-state cycle moves rows x k floats,
// not rows x T.
//
// Mapping: one 64-lane wave per output row (row parameters are wave-uniform
// scalars), four rows per 256-thread workgroup, each lane keeping four
// independent loads in flight; the copy is HBM-bound.
#include "fm_common.h"

namespace {

constexpr int kRowsPerBlock = 4;
constexpr int kUnroll = 4;

__global__ __launch_bounds__(256) void gather_cols_kernel(const float* __restrict__ src, int64_t ld,
                                                          const int32_t* __restrict__ rm,
                                                          const int32_t* __restrict__ off,
                                                          const int32_t* __restrict__ lim, int64_t R, int ncols,
                                                          float* __restrict__ out, int64_t ldo) {
  const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + fm::wave_id();
  if (r >= R) return;
  const int lane = fm::lane_id();
  const int64_t row = rm ? (int64_t)__builtin_amdgcn_readfirstlane(rm[r]) : r;
  const int o = __builtin_amdgcn_readfirstlane(off[r]);
  const int l = __builtin_amdgcn_readfirstlane(lim[r]);
  const float* __restrict__ s = src + row * ld;
  float* __restrict__ d = out + r * ldo;
  const float nan = __builtin_nanf("");
  int j = lane;
  for (; j + (kUnroll - 1) * FM_WAVE < ncols; j += kUnroll * FM_WAVE) {
    float v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const int c = o + j + u * FM_WAVE;
      v[u] = (c >= 0 && c < l) ? __builtin_nontemporal_load(s + c) : nan;
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) d[j + u * FM_WAVE] = v[u];
  }
  for (; j < ncols; j += FM_WAVE) {
    const int c = o + j;
    d[j] = (c >= 0 && c < l) ? __builtin_nontemporal_load(s + c) : nan;
  }
}

}  // namespace

// ``rm`` may be null (identity).  Rows are [R, ncols] at stride ``ldo``.
FM_API int fm_gather_cols(const float* src, int64_t ld, const int32_t* rm, const int32_t* off, const int32_t* lim,
                          int64_t R, int ncols, float* out, int64_t ldo, hipStream_t stream) {
  if (R <= 0 || ncols <= 0) return 0;
  const int64_t blocks = (R + kRowsPerBlock - 1) / kRowsPerBlock;
  hipLaunchKernelGGL(gather_cols_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, src, ld, rm, off, lim, R,
                     ncols, out, ldo);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Sliding-grid columns leaving the window (ResidentHistory.advance): per row
// the finite samples in columns [lo, hi) are counted into gone[row] (the
// history gate's finite count drops by them) and the columns are set to NaN,
// in ONE pass -- was isfinite + sum + a device->host copy + a strided fill,
// seven launches per cycle.  One thread per row; a 60-s poll retires one
// column per cycle.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void grid_retire_kernel(float* __restrict__ buf, int64_t ld, int64_t R, int lo,
                                                          int hi, int* __restrict__ gone) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float* row = buf + r * ld;
  int n = 0;
  for (int c = lo; c < hi; ++c) {
    n += isfinite(row[c]) ? 1 : 0;
    row[c] = __builtin_nanf("");
  }
  gone[r] = n;
}

FM_API int fm_grid_retire(float* buf, int64_t ld, int64_t R, int lo, int hi, int* gone, hipStream_t stream) {
  if (R <= 0 || hi <= lo) return 0;
  if (lo < 0 || hi > ld) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(grid_retire_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, stream, buf, ld, R, lo, hi,
                     gone);
  FM_LAUNCH_CHECK();
  return 0;
}
