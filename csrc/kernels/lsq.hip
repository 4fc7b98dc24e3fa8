// K10: batched least-squares projection on f32 MFMA ("prophet-lite": trend +
// changepoint hinges + daily/weekly Fourier seasonality, docs/guides/design.md:72
// lists Prophet).  For every series y (a row of Y) and ONE shared design matrix
// X [T, F=32] the kernel computes z = X^T (y - c) and yy = ||y - c||^2 in a
// single streaming pass, c = the row's first sample (a cheap per-row shift that
// keeps the later SSE = yy - 2 b.z + b'Gb free of catastrophic cancellation).
// The F x F normal matrix G = X^T X is shared by all rows, so the solve is a
// tiny [R,F] x [F,F] product done once on the host side.
//
// MFMA mapping (v_mfma_f32_32x32x2_f32, exact fp32 fmaf chains): one wave owns
// a 32-row x 32-feature output tile.  The reduction index t is permuted so that
// for a 64-sample chunk lane l (row/feature l&31, half h = l>>5) consumes
// samples t0 + 32h + kk at MFMA kk = 0..31: both operands are then 32
// contiguous floats per lane (8 x 16-B loads straight to VGPRs, 128-B lines
// fully used), with X stored transposed [F][T] so it streams exactly like Y.
#include "fm_common.h"

using namespace fm;

typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ __launch_bounds__(256) void lsq_project_kernel(const float* __restrict__ Y, int64_t ld_y, int T, int64_t R,
                                                          const float* __restrict__ XT /*[32][ld_x]*/, int64_t ld_x,
                                                          float* __restrict__ Z /*[R,32]*/, float* __restrict__ yy,
                                                          float* __restrict__ shift, int* __restrict__ nvalid) {
  const int lane = lane_id();
  const int64_t tile = (int64_t)blockIdx.x * 4 + wave_id();
  const int64_t row0 = tile * 32;
  if (row0 >= R) return;
  const int r = lane & 31, h = lane >> 5;
  const int64_t row = row0 + r;
  const bool live = row < R;
  const float* yr = Y + (live ? row : row0) * ld_y;
  const float* xr = XT + (int64_t)r * ld_x;
  float c0 = live ? yr[0] : 0.f;
  if (!isfinite(c0)) c0 = 0.f;
  f32x16 acc = {};
  float sq = 0.f;
  int cnt = 0;
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int tb = t0 + 32 * h;
    float yv[32], xv[32];
    if (tb + 32 <= T) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float4 a = live ? *reinterpret_cast<const float4*>(yr + tb + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 b = *reinterpret_cast<const float4*>(xr + tb + 4 * q);
        yv[4 * q + 0] = a.x; yv[4 * q + 1] = a.y; yv[4 * q + 2] = a.z; yv[4 * q + 3] = a.w;
        xv[4 * q + 0] = b.x; xv[4 * q + 1] = b.y; xv[4 * q + 2] = b.z; xv[4 * q + 3] = b.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int t = tb + q;
        yv[q] = (live && t < T) ? yr[t] : NAN;   // past the end = missing (not a zero sample)
        xv[q] = t < T ? xr[t] : 0.f;
      }
    }
#pragma unroll
    for (int kk = 0; kk < 32; ++kk) {
      float y = yv[kk];
      if (isfinite(y) && live) { y -= c0; ++cnt; } else { y = 0.f; }
      sq += y * y;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(y, xv[kk], acc, 0, 0, 0);
    }
  }
  // rows owned by lane l and l+32 are the same row: combine the halves
  sq += __shfl_xor(sq, 32);
  cnt += __shfl_xor(cnt, 32);
  // C/D map: col = lane & 31 (feature), row = (i & 3) + 8 * (i >> 2) + 4 * h
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int rr = (i & 3) + 8 * (i >> 2) + 4 * h;
    if (row0 + rr < R) Z[(row0 + rr) * 32 + r] = acc[i];
  }
  if (h == 0 && live) { yy[row] = sq; shift[row] = c0; nvalid[row] = cnt; }
}

FM_API int fm_lsq_project(const float* Y, int64_t ld_y, int T, int64_t R, const float* XT, int64_t ld_x, float* Z,
                          float* yy, float* shift, int* nvalid, hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_y & 3) || (ld_x & 3) || (((uintptr_t)Y) & 15) || (((uintptr_t)XT) & 15)) return (int)hipErrorInvalidValue;
  const int64_t tiles = (R + 31) / 32;
  hipLaunchKernelGGL(lsq_project_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, stream, Y, ld_y, T, R, XT,
                     ld_x, Z, yy, shift, nvalid);
  FM_LAUNCH_CHECK();
  return 0;
}
