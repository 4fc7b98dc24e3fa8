// K3: FFT seasonal analysis.  Real input of length Nr is packed into a
// complex sequence of N = Nr/2 points (z_j = x_2j + i x_2j+1), transformed by a
// mixed-radix Stockham FFT (radices 4,2,9,3,5,7) that lives entirely in LDS
// (one 256-thread workgroup per series; N <= 8192 complex = 64 KB), then
// unpacked to the one-sided real spectrum.  The periodogram peak in a
// [kmin, kmax] band gives the dominant seasonal period (docs/dynamic_autoscaling.md:5-30,
// "Determine TPS seasonality & trend").
//
// 10,080 = 7 days at 60 s (metricsquery.go:93-97) -> N = 5040 = 4*4*9*5*7:
// five passes, no zero padding, so the spectral resolution is exactly 1/week.
#include "fm_common.h"

using namespace fm;

namespace {

template <int R> struct RootTable;
template <> struct RootTable<3> {
  static constexpr float c[3] = {1.00000000000000000e+00f, -4.99999999999999778e-01f, -5.00000000000000444e-01f};
  static constexpr float s[3] = {0.00000000000000000e+00f, 8.66025403784438708e-01f, -8.66025403784438375e-01f};
};
template <> struct RootTable<5> {
  static constexpr float c[5] = {1.00000000000000000e+00f, 3.09016994374947451e-01f, -8.09016994374947340e-01f, -8.09016994374947562e-01f, 3.09016994374947229e-01f};
  static constexpr float s[5] = {0.00000000000000000e+00f, 9.51056516295153531e-01f, 5.87785252292473248e-01f, -5.87785252292473026e-01f, -9.51056516295153642e-01f};
};
template <> struct RootTable<7> {
  static constexpr float c[7] = {1.00000000000000000e+00f, 6.23489801858733594e-01f, -2.22520933956314337e-01f, -9.00968867902419035e-01f, -9.00968867902419146e-01f, -2.22520933956314587e-01f, 6.23489801858733372e-01f};
  static constexpr float s[7] = {0.00000000000000000e+00f, 7.81831482468029804e-01f, 9.74927912181823619e-01f, 4.33883739117558231e-01f, -4.33883739117558009e-01f, -9.74927912181823619e-01f, -7.81831482468029915e-01f};
};
template <> struct RootTable<9> {
  static constexpr float c[9] = {1.00000000000000000e+00f, 7.66044443118978013e-01f, 1.73648177666930414e-01f, -4.99999999999999778e-01f, -9.39692620785908317e-01f, -9.39692620785908428e-01f, -5.00000000000000444e-01f, 1.73648177666929970e-01f, 7.66044443118977791e-01f};
  static constexpr float s[9] = {0.00000000000000000e+00f, 6.42787609686539252e-01f, 9.84807753012208020e-01f, 8.66025403784438708e-01f, 3.42020143325668879e-01f, -3.42020143325668657e-01f, -8.66025403784438375e-01f, -9.84807753012208131e-01f, -6.42787609686539585e-01f};
};

__device__ __forceinline__ float2 cmul(float2 a, float2 b) { return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }

// forward DFT (W = e^{-2 pi i / R}) of R points in registers
template <int R>
__device__ __forceinline__ void dft(float2 (&v)[R]) {
  if constexpr (R == 2) {
    float2 a = v[0], b = v[1];
    v[0] = cadd(a, b); v[1] = csub(a, b);
  } else if constexpr (R == 4) {
    const float2 a0 = v[0], a1 = v[1], a2 = v[2], a3 = v[3];
    const float2 s02 = cadd(a0, a2), d02 = csub(a0, a2), s13 = cadd(a1, a3), d13 = csub(a1, a3);
    v[0] = cadd(s02, s13);
    v[2] = csub(s02, s13);
    v[1] = make_float2(d02.x + d13.y, d02.y - d13.x);   // d02 - i d13
    v[3] = make_float2(d02.x - d13.y, d02.y + d13.x);   // d02 + i d13
  } else {
    float2 o[R];
#pragma unroll
    for (int p = 0; p < R; ++p) {
      float2 acc = v[0];
#pragma unroll
      for (int q = 1; q < R; ++q) {
        const int m = (p * q) % R;
        const float c = RootTable<R>::c[m], s = RootTable<R>::s[m];
        // v[q] * (c - i s)
        acc.x += v[q].x * c + v[q].y * s;
        acc.y += v[q].y * c - v[q].x * s;
      }
      o[p] = acc;
    }
#pragma unroll
    for (int p = 0; p < R; ++p) v[p] = o[p];
  }
}

constexpr int kMaxN = 8192;
constexpr int kThreads = 256;

// j / Ns and j % Ns by a multiply-high with a per-pass magic number (exact
// for j, Ns < 2^13: the 32-bit reciprocal's error times j stays below one
// part in 2^19, less than the smallest fractional part 1/Ns).
__device__ __forceinline__ int div_magic(int j, unsigned magic) { return (int)__umulhi((unsigned)j, magic); }

// Twiddle w^q, q = 1..R-1, for w = exp(-2 pi i m / N): w from the hardware
// sine / cosine (v_sin_f32 / v_cos_f32 take revolutions, so the argument is
// the exact fraction m / N), the powers by complex products (R <= 9: a few
// ulps) instead of R-1 gathers from a global table.
template <int R>
__device__ __forceinline__ void twiddles(int m, float invN, float2 (&w)[R]) {
  const float r = -(float)m * invN;
  w[0] = make_float2(1.f, 0.f);
  w[1] = make_float2(__builtin_amdgcn_cosf(r), __builtin_amdgcn_sinf(r));
#pragma unroll
  for (int q = 2; q < R; ++q) w[q] = cmul(w[q - 1], w[1]);
}

template <int R, int MAXN>
__device__ __forceinline__ void stockham_pass(float2* buf, int N, int Ns, float invN) {
  constexpr int MAXB = (MAXN / R + kThreads - 1) / kThreads;
  const int nb = N / R;
  const int step = N / (Ns * R);
  const unsigned magic = 0xFFFFFFFFu / (unsigned)Ns + 1u;   // scalar
  float2 v[MAXB][R];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = threadIdx.x + b * kThreads;
    if (j < nb) {
      const int k = Ns == 1 ? 0 : j - div_magic(j, magic) * Ns;
#pragma unroll
      for (int q = 0; q < R; ++q) v[b][q] = buf[j + q * nb];
      if (k > 0) {
        float2 w[R];
        twiddles<R>(k * step, invN, w);
#pragma unroll
        for (int q = 1; q < R; ++q) v[b][q] = cmul(v[b][q], w[q]);
      }
      dft<R>(v[b]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = threadIdx.x + b * kThreads;
    if (j < nb) {
      const int g = Ns == 1 ? j : div_magic(j, magic);
      const int k = j - g * Ns;
      const int base = g * Ns * R + k;
#pragma unroll
      for (int p = 0; p < R; ++p) buf[base + p * Ns] = v[b][p];
    }
  }
  __syncthreads();
}

}  // namespace

struct FftPlan {
  int n_pass;
  int radix[16];
};

// MAXN: compile-time bound on N (register arrays are sized by it; the
// 7-day series has N = 5040 and runs the 5120 variant at 4 workgroups/CU).
template <int MAXN>
__global__ __launch_bounds__(kThreads) void fft_seasonal_kernel(
    const float* __restrict__ x, int64_t ld, int Nr, int64_t R, const float2* __restrict__ tw,
    const float2* __restrict__ tw2, FftPlan plan, int kmin, int kmax, float* __restrict__ power, int64_t ld_p,
    float2* __restrict__ spec, int64_t ld_s, int* __restrict__ period_bin, float* __restrict__ strength,
    float* __restrict__ mean_out, float* __restrict__ slope_out) {
  extern __shared__ __attribute__((aligned(16))) float2 buf[];
  (void)tw;   // twiddles are computed in-kernel (kept in the C ABI)
  __shared__ float redf[8];
  __shared__ int redi[8];
  const int64_t row = blockIdx.x;
  const int N = Nr >> 1;
  const float* xr = x + row * ld;
  const int tid = threadIdx.x;
  // The row is read ONCE: its complex pairs z_j = (x_2j, x_2j+1) go to
  // registers (all loads issued up front), the least-squares linear detrend
  // sums over finite samples are taken from there, and the detrended values
  // are written to LDS.  (NaN -> trend line, so a slow trend does not leak
  // into the low-frequency bins.)
  constexpr int NPT = MAXN / kThreads;        // complex values per thread
  float2 z[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int j = tid + i * kThreads;
    z[i] = j < N ? reinterpret_cast<const float2*>(xr)[j] : make_float2(__builtin_nanf(""), __builtin_nanf(""));
  }
  double s = 0.0, st = 0.0, stt = 0.0, sx = 0.0, c = 0.0;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const double t0 = 2.0 * (tid + i * kThreads);
    if (isfinite(z[i].x)) { s += z[i].x; st += t0; stt += t0 * t0; sx += t0 * z[i].x; c += 1.0; }
    if (isfinite(z[i].y)) { const double t1 = t0 + 1.0; s += z[i].y; st += t1; stt += t1 * t1; sx += t1 * z[i].y; c += 1.0; }
  }
  // the five block sums in one LDS round trip
  __shared__ double red5[5][kThreads / 64];
  s = wave_sum(s); st = wave_sum(st); stt = wave_sum(stt); sx = wave_sum(sx); c = wave_sum(c);
  if (lane_id() == 0) {
    red5[0][wave_id()] = s; red5[1][wave_id()] = st; red5[2][wave_id()] = stt; red5[3][wave_id()] = sx;
    red5[4][wave_id()] = c;
  }
  __syncthreads();
  s = st = stt = sx = c = 0.0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    s += red5[0][w]; st += red5[1][w]; stt += red5[2][w]; sx += red5[3][w]; c += red5[4][w];
  }
  const double dc = c > 0 ? c : 1.0;
  const double tbar = st / dc, xbar = s / dc;
  const double vt = stt / dc - tbar * tbar;
  const double slope_d = vt > 0 ? (sx / dc - tbar * xbar) / vt : 0.0;
  const float mu = c > 0 ? (float)xbar : 0.f;
  const float slope = (float)slope_d, tb = (float)tbar;
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int j = tid + i * kThreads;
    if (j < N) {
      const float t0 = (float)(2 * j) - tb;
      buf[j] = make_float2(isfinite(z[i].x) ? z[i].x - mu - slope * t0 : 0.f,
                           isfinite(z[i].y) ? z[i].y - mu - slope * (t0 + 1.f) : 0.f);
    }
  }
  __syncthreads();
  const float invN = 1.f / (float)N;
  int Ns = 1;
  for (int ps = 0; ps < plan.n_pass; ++ps) {
    const int r = plan.radix[ps];
    switch (r) {
      case 2: stockham_pass<2, MAXN>(buf, N, Ns, invN); break;
      case 3: stockham_pass<3, MAXN>(buf, N, Ns, invN); break;
      case 4: stockham_pass<4, MAXN>(buf, N, Ns, invN); break;
      case 5: stockham_pass<5, MAXN>(buf, N, Ns, invN); break;
      case 7: stockham_pass<7, MAXN>(buf, N, Ns, invN); break;
      case 9: stockham_pass<9, MAXN>(buf, N, Ns, invN); break;
      default: break;
    }
    Ns *= r;
  }
  // unpack the real spectrum X[k], k = 0..N
  float best = -1.f;
  int bk = 0;
  float tot = 0.f;
  for (int k = tid; k <= N; k += kThreads) {
    const float2 zk = buf[k == N ? 0 : k];
    const float2 zn = buf[k == 0 ? 0 : N - k];
    const float2 zc = make_float2(zn.x, -zn.y);
    const float2 e = make_float2(0.5f * (zk.x + zc.x), 0.5f * (zk.y + zc.y));
    const float2 d = make_float2(0.5f * (zk.x - zc.x), 0.5f * (zk.y - zc.y));
    const float2 o = make_float2(d.y, -d.x);  // -i * d
    const float2 X = cadd(e, cmul(tw2[k], o));
    const float pw = X.x * X.x + X.y * X.y;
    if (power) power[row * ld_p + k] = pw;
    if (spec) spec[row * ld_s + k] = X;
    if (k >= 1) tot += pw;
    if (k >= kmin && k <= kmax && pw > best) { best = pw; bk = k; }
  }
  // block argmax (value, index) and total
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o);
    const int ok = __shfl_xor(bk, o);
    if (ob > best || (ob == best && ok < bk)) { best = ob; bk = ok; }
    tot += __shfl_xor(tot, o);
  }
  if (lane_id() == 0) { redf[wave_id()] = best; redi[wave_id()] = bk; redf[4 + wave_id()] = tot; }
  __syncthreads();
  if (tid == 0) {
    float b = redf[0]; int k = redi[0]; float t = redf[4];
    for (int w = 1; w < kThreads / 64; ++w) {
      if (redf[w] > b || (redf[w] == b && redi[w] < k)) { b = redf[w]; k = redi[w]; }
      t += redf[4 + w];
    }
    period_bin[row] = k;
    strength[row] = t > 0.f ? b / t : 0.f;
    mean_out[row] = mu;
    slope_out[row] = slope;
  }
}

FM_API int fm_fft_seasonal(const float* x, int64_t ld, int Nr, int64_t R, const float2* tw, const float2* tw2,
                           const int* radices, int n_pass, int kmin, int kmax, float* power, int64_t ld_p,
                           float2* spec, int64_t ld_s, int* period_bin, float* strength, float* mean_out, float* slope_out,
                           hipStream_t stream) {
  if (R <= 0) return 0;
  if ((Nr & 1) || Nr / 2 > kMaxN || n_pass > 16 || (ld & 1) || (((uintptr_t)x) & 7)) return (int)hipErrorInvalidValue;
  FftPlan plan;
  plan.n_pass = n_pass;
  int prod = 1;
  for (int i = 0; i < n_pass; ++i) { plan.radix[i] = radices[i]; prod *= radices[i]; }
  if (prod != Nr / 2) return (int)hipErrorInvalidValue;
  const size_t lds = (size_t)(Nr / 2) * sizeof(float2);
#define FM_FFT(MN)                                                                                            \
  hipLaunchKernelGGL(fft_seasonal_kernel<MN>, dim3((unsigned)R), dim3(kThreads), lds, stream, x, ld, Nr, R, tw, tw2, \
                     plan, kmin, kmax, power, ld_p, spec, ld_s, period_bin, strength, mean_out, slope_out)
  if (Nr / 2 <= 2048) FM_FFT(2048);
  else if (Nr / 2 <= 5120) FM_FFT(5120);
  else FM_FFT(kMaxN);
#undef FM_FFT
  FM_LAUNCH_CHECK();
  return 0;
}

// Seasonal profile: mean of the (mean-removed) series at each phase of a
// per-row period (phase-averaging over complete cycles), one workgroup per
// row, LDS accumulation.
__global__ __launch_bounds__(256) void phase_profile_kernel(const float* __restrict__ x, int64_t ld, int T,
                                                            const int* __restrict__ period, int maxp,
                                                            const float* __restrict__ mean, const float* __restrict__ slope,
                                                            float* __restrict__ out /*[R, maxp]*/) {
  extern __shared__ __attribute__((aligned(16))) float acc[];  // 2 * maxp
  const int64_t row = blockIdx.x;
  const int p = period[row];
  float* sum = acc;
  float* cnt = acc + maxp;
  for (int i = threadIdx.x; i < 2 * maxp; i += blockDim.x) acc[i] = 0.f;
  __syncthreads();
  const float mu = mean[row], sl = slope[row], tb = 0.5f * (float)(T - 1);
  const float* xr = x + row * ld;
  if (p > 0 && p <= maxp) {
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
      const float v = xr[t];
      if (isfinite(v)) { atomicAdd(&sum[t % p], v - mu - sl * ((float)t - tb)); atomicAdd(&cnt[t % p], 1.f); }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < maxp; i += blockDim.x)
    out[row * maxp + i] = (i < p && cnt[i] > 0.f) ? sum[i] / cnt[i] : 0.f;
}

FM_API int fm_phase_profile(const float* x, int64_t ld, int T, int64_t R, const int* period, int maxp,
                            const float* mean, const float* slope, float* out, hipStream_t stream) {
  if (R <= 0) return 0;
  if (maxp <= 0 || maxp > 16384) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(phase_profile_kernel, dim3((unsigned)R), dim3(256), (size_t)(2 * maxp) * sizeof(float), stream,
                     x, ld, T, period, maxp, mean, slope, out);
  FM_LAUNCH_CHECK();
  return 0;
}
