// K10: batched least-squares projection on f32 MFMA ("prophet-lite": trend +
// changepoint hinges + daily/weekly Fourier seasonality, docs/guides/design.md:72
// lists Prophet).  For every series y (a row of Y) and ONE shared design matrix
// X [T, F=32] the kernel computes z = X^T (y - c) and yy = ||y - c||^2 in a
// single streaming pass, c = the row's first sample.  The design is passed as
// an orthonormal basis U (thin SVD, ops/lsq.py), so the coefficients are z
// itself.  The residual sum of squares is NOT derived as yy - |z|^2 (that
// difference of two large fp32-accumulated sums cancels catastrophically when
// the fit is good); lsq_residual_kernel below re-streams the rows and sums the
// residuals y - c - U z directly (fp32 residuals, fp64 accumulation).
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

// ---------------------------------------------------------------------------
// Residual pass: sse[r] = sum over finite samples t of (y[r,t] - c[r] - yhat[r,t])^2
// with yhat = Z[r,:] U[:,t].  One wave owns 32 rows; per 32-sample chunk the
// fitted tile yhat[32 rows x 32 t] is 16 v_mfma_f32_32x32x2_f32 steps (A = the
// rows' coefficients, B = 32 columns of U^T), then every lane forms the
// residuals of its 16 (row, t) entries (C/D layout: t = lane & 31, row =
// (i & 3) + 8 (i >> 2) + 4 h) and accumulates their squares in fp64.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lsq_residual_kernel(const float* __restrict__ Y, int64_t ld_y, int T, int64_t R,
                                                           const float* __restrict__ XT, int64_t ld_x,
                                                           const float* __restrict__ Z, const float* __restrict__ shift,
                                                           double* __restrict__ sse) {
  const int lane = lane_id();
  const int64_t tile = (int64_t)blockIdx.x * 4 + wave_id();
  const int64_t row0 = tile * 32;
  if (row0 >= R) return;
  const int j = lane & 31, h = lane >> 5;
  // A operand per K-step s: Z[row0 + j][2s + h]
  float za[16];
  {
    const int64_t ar = row0 + j < R ? row0 + j : R - 1;
#pragma unroll
    for (int st = 0; st < 16; ++st) za[st] = Z[ar * 32 + 2 * st + h];
  }
  int64_t rows[16];
  float cr[16];
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int64_t rr = row0 + (i & 3) + 8 * (i >> 2) + 4 * h;
    rows[i] = rr < R ? rr : -1;
    cr[i] = rr < R ? shift[rr] : 0.f;
    acc[i] = 0.0;
  }
  for (int t0 = 0; t0 < T; t0 += 32) {
    const int t = t0 + j;
    f32x16 yh = {};
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const float b = t < T ? XT[(int64_t)(2 * st + h) * ld_x + t] : 0.f;
      yh = __builtin_amdgcn_mfma_f32_32x32x2f32(za[st], b, yh, 0, 0, 0);
    }
    if (t < T) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (rows[i] < 0) continue;
        const float y = Y[rows[i] * ld_y + t];
        if (isfinite(y)) {
          const float r = (y - cr[i]) - yh[i];
          acc[i] += (double)r * (double)r;
        }
      }
    }
  }
  // sum each row's partials over the 32 lanes of its half-wave
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    double v = acc[i];
#pragma unroll
    for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (j == 0 && rows[i] >= 0) sse[rows[i]] = v;
  }
}

FM_API int fm_lsq_residual(const float* Y, int64_t ld_y, int T, int64_t R, const float* XT, int64_t ld_x,
                           const float* Z, const float* shift, double* sse, hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_y & 3) || (ld_x & 3)) return (int)hipErrorInvalidValue;
  const int64_t tiles = (R + 31) / 32;
  hipLaunchKernelGGL(lsq_residual_kernel, dim3((unsigned)((tiles + 3) / 4)), dim3(256), 0, stream, Y, ld_y, T, R, XT,
                     ld_x, Z, shift, sse);
  FM_LAUNCH_CHECK();
  return 0;
}
