// K3: FFT seasonal analysis.  Real input of length Nr is packed into a
// complex sequence of N = Nr/2 points (z_j = x_2j + i x_2j+1), transformed by a
// mixed-radix Stockham FFT (radices 2,3,4,5,7,9) that lives entirely in LDS
// (one 256-thread workgroup per series; N <= 8192 complex = 64 KB), then
// unpacked to the one-sided real spectrum.  The periodogram peak in a
// [kmin, kmax] band gives the dominant seasonal period (docs/dynamic_autoscaling.md:5-30,
// "Determine TPS seasonality & trend").
//
// 10,080 = 7 days at 60 s (metricsquery.go:93-97) -> N = 5040 = 7*4*9*4*5:
// five passes, no zero padding, so the spectral resolution is exactly 1/week.
//
// CDNA4 shape of the work (r2):
//   * the common lengths (N = 5040 / 1008 / 720: 7 days at 1 min / 5 min,
//     1 day at 1 min) run a compile-time plan: every pass's stride, butterfly
//     count and the j / Ns division are constants, no per-pass dispatch;
//   * the radix order starts with an odd radix, then alternates 4 with the
//     rest (7,4,9,4,5): the self-sorting writes of an early radix-4 pass are
//     8-dword strided (4-way LDS bank conflicts on ds_write_b64), an odd
//     stride spreads over all banks -- a bank model of every pass puts the
//     order at 1.10x the conflict-free LDS cycles, vs 1.57x for 4,4,9,5,7;
//   * butterflies are packed-fp32 (float2 ext vectors -> v_pk_fma/add/mul_f32)
//     and odd radices use the conjugate-pair form (outputs p and R-p share
//     one set of products): a radix-7 butterfly is ~33 packed ops, not the
//     168 scalar FMAs of the textbook O(R^2) sum;
//   * the total power for the strength ratio comes from Parseval over the
//     detrended samples (sum e^2, X_0, X_N, accumulated while the row is
//     written to LDS), so only the [kmin, kmax] band is unpacked unless the
//     caller asked for the whole periodogram.
#include "fm_common.h"

using namespace fm;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

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

// The half-swapped, half-negated operands of complex arithmetic folded into
// the VOP3P source modifiers (op_sel / op_sel_hi pick the half feeding each
// result lane, neg_lo / neg_hi negate it): one v_pk_* each.  Written out
// because the compiler builds (b.y, -b.x) with a v_mov + v_xor pair per use.
__device__ __forceinline__ f2 cmul(f2 a, f2 b) {   // a * b
  f2 t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ f2 add_negi(f2 a, f2 b) {   // a - i b = (a.x + b.y, a.y - b.x)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 add_posi(f2 a, f2 b) {   // a + i b = (a.x - b.y, a.y + b.x)
  f2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f2 neg_i(f2 a) { return (f2){a.y, -a.x}; }   // -i a

// forward DFT (W = e^{-2 pi i / R}) of R points in registers
template <int R>
__device__ __forceinline__ void dft(f2 (&v)[R]) {
  if constexpr (R == 2) {
    const f2 a = v[0], b = v[1];
    v[0] = a + b;
    v[1] = a - b;
  } else if constexpr (R == 4) {
    const f2 s02 = v[0] + v[2], d02 = v[0] - v[2], s13 = v[1] + v[3], d13 = v[1] - v[3];
    v[0] = s02 + s13;
    v[2] = s02 - s13;
    v[1] = add_negi(d02, d13);
    v[3] = add_posi(d02, d13);
  } else {
    // conjugate pairs: X_p = v0 + sum_q c_pq S_q - i sum_q s_pq D_q,
    // X_{R-p} = v0 + sum_q c_pq S_q + i sum_q s_pq D_q  (q = 1..(R-1)/2)
    constexpr int H = (R - 1) / 2;
    f2 S[H], D[H];
    f2 x0 = v[0];
#pragma unroll
    for (int q = 1; q <= H; ++q) {
      S[q - 1] = v[q] + v[R - q];
      D[q - 1] = v[q] - v[R - q];
      x0 += S[q - 1];
    }
    f2 o[R];
    o[0] = x0;
#pragma unroll
    for (int p = 1; p <= H; ++p) {
      f2 A = v[0], B = (f2){0.f, 0.f};
#pragma unroll
      for (int q = 1; q <= H; ++q) {
        const int m = (p * q) % R;
        A += RootTable<R>::c[m] * S[q - 1];
        B += RootTable<R>::s[m] * D[q - 1];
      }
      o[p] = add_negi(A, B);
      o[R - p] = add_posi(A, B);
    }
#pragma unroll
    for (int p = 0; p < R; ++p) v[p] = o[p];
  }
}

constexpr int kMaxN = 8192;
constexpr int kThreads = 256;

// Twiddles w^q, q = 0..R-1, for w = exp(2 pi i r), r in revolutions (v_sin_f32
// / v_cos_f32 take revolutions, so r is the exact fraction -m / N); the
// powers by complex products (R <= 9: a few ulps) instead of R-1 gathers.
template <int R>
__device__ __forceinline__ void twiddles(float r, f2 (&w)[R]) {
  w[0] = (f2){1.f, 0.f};
  // in asm with the trailing wait states: the hazard recognizer does not see
  // the transcendental-result -> VALU-use hazard when the user is inline asm
  // (cmul below), so the asm block carries its own s_nop
  f2 w1;
  asm("v_cos_f32 %0, %2\n\tv_sin_f32 %1, %2\n\ts_nop 1" : "=&v"(w1.x), "=&v"(w1.y) : "v"(r));
  w[1] = w1;
#pragma unroll
  for (int q = 2; q < R; ++q) w[q] = cmul(w[q - 1], w[1]);
}

// One Stockham pass, compile-time N / R / Ns.
template <int N, int R, int Ns>
__device__ __forceinline__ void pass_ct(f2* buf) {
  constexpr int nb = N / R;
  constexpr int MAXB = (nb + kThreads - 1) / kThreads;
  constexpr float inv = -1.f / (float)(Ns * R);
  f2 v[MAXB][R];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = threadIdx.x + b * kThreads;
    if ((b + 1) * kThreads <= nb || j < nb) {
#pragma unroll
      for (int q = 0; q < R; ++q) v[b][q] = buf[j + q * nb];
      if constexpr (Ns > 1) {
        f2 w[R];
        twiddles<R>((float)(j % Ns) * inv, w);
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
    if ((b + 1) * kThreads <= nb || j < nb) {
      const int g = j / Ns, k = j - g * Ns;
      const int base = g * Ns * R + k;
#pragma unroll
      for (int p = 0; p < R; ++p) buf[base + p * Ns] = v[b][p];
    }
  }
  __syncthreads();
}

template <int N, int Ns, int R, int... Rest>
__device__ __forceinline__ void passes_ct(f2* buf) {
  pass_ct<N, R, Ns>(buf);
  if constexpr (sizeof...(Rest) > 0) passes_ct<N, Ns * R, Rest...>(buf);
}

// j / Ns and j % Ns by a multiply-high with a per-pass magic number (exact
// for j, Ns < 2^13: the 32-bit reciprocal's error times j stays below one
// part in 2^19, less than the smallest fractional part 1/Ns).
__device__ __forceinline__ int div_magic(int j, unsigned magic) { return (int)__umulhi((unsigned)j, magic); }

// One Stockham pass with a run-time plan (lengths without a fixed plan).
template <int R, int MAXN>
__device__ __forceinline__ void stockham_pass(f2* buf, int N, int Ns) {
  constexpr int MAXB = (MAXN / R + kThreads - 1) / kThreads;
  const int nb = N / R;
  const float inv = -1.f / (float)(Ns * R);
  const unsigned magic = 0xFFFFFFFFu / (unsigned)Ns + 1u;   // scalar
  f2 v[MAXB][R];
#pragma unroll
  for (int b = 0; b < MAXB; ++b) {
    const int j = threadIdx.x + b * kThreads;
    if (j < nb) {
      const int k = Ns == 1 ? 0 : j - div_magic(j, magic) * Ns;
#pragma unroll
      for (int q = 0; q < R; ++q) v[b][q] = buf[j + q * nb];
      if (k > 0) {
        f2 w[R];
        twiddles<R>((float)k * inv, w);
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

// Fixed plans: the first radix R1 (its pass is fused with the row load:
// the butterflies read their inputs straight from the detrended registers)
// and the remaining passes, which start at Ns = R1.
template <int FN> struct FixedPlan { static constexpr bool ok = false; static constexpr int R1 = 1; };
template <> struct FixedPlan<5040> {
  static constexpr bool ok = true;
  static constexpr int R1 = 7;
  static __device__ __forceinline__ void run_rest(f2* b) { passes_ct<5040, 7, 4, 9, 4, 5>(b); }
};
template <> struct FixedPlan<1008> {
  static constexpr bool ok = true;
  static constexpr int R1 = 7;
  static __device__ __forceinline__ void run_rest(f2* b) { passes_ct<1008, 7, 4, 9, 4>(b); }
};
template <> struct FixedPlan<720> {
  static constexpr bool ok = true;
  static constexpr int R1 = 5;
  static __device__ __forceinline__ void run_rest(f2* b) { passes_ct<720, 5, 4, 9, 4>(b); }
};

}  // namespace

struct FftPlan {
  int n_pass;
  int radix[16];
};

// MAXN: compile-time bound on N (register arrays are sized by it); FN: the
// compile-time N of a fixed plan (0: the run-time plan in `plan`).
template <int MAXN, int FN>
__global__ __launch_bounds__(kThreads) void fft_seasonal_kernel(
    const float* __restrict__ x, int64_t ld, int Nr, int64_t R, const float2* __restrict__ tw,
    const float2* __restrict__ tw2, FftPlan plan, int kmin, int kmax, float* __restrict__ power, int64_t ld_p,
    float2* __restrict__ spec, int64_t ld_s, int* __restrict__ period_bin, float* __restrict__ strength,
    float* __restrict__ mean_out, float* __restrict__ slope_out) {
  extern __shared__ __attribute__((aligned(16))) f2 buf[];
  (void)tw;   // twiddles are computed in-kernel (kept in the C ABI)
  __shared__ float redf[6][kThreads / 64];
  __shared__ int redi[kThreads / 64];
  __shared__ float red5[5][kThreads / 64];
  const int64_t row = blockIdx.x;
  const int N = FN > 0 ? FN : Nr >> 1;
  const float* xr = x + row * ld;
  const int tid = threadIdx.x, wv = wave_id();
  // The row is read ONCE: its complex pairs z_j = (x_2j, x_2j+1) go to
  // registers (all loads issued up front), the least-squares linear detrend
  // sums over finite samples are taken from there, and the detrended values
  // feed the transform.  (NaN -> trend line, so a slow trend does not leak
  // into the low-frequency bins.)  Time is centred (tc = t - (Nr-1)/2), so
  // sum tc and sum tc^2 over ALL samples are closed forms and only the
  // missing samples' terms are accumulated (a branch no wave takes on a
  // complete row); the sample sums are packed (x, y) fp32 per thread, the
  // cross-lane sums fp64.  Branch-free: a wave of 40 divergent if-blocks
  // per row cost more than the butterflies of a pass.
  // Element e of a thread: fixed plans load in the first pass's order
  // (butterfly jb = tid + 256 (e / R1), input q = e % R1 at jb + q N/R1), so
  // that pass runs on the registers -- no LDS write + read of the row and
  // one barrier fewer; the run-time plan loads z_j, j = tid + 256 e.
  constexpr bool FIX = FN > 0;
  constexpr int R1 = FIX ? FixedPlan<FN>::R1 : 1;
  constexpr int NB1 = FIX ? FN / R1 : 1;                          // first-pass butterflies
  constexpr int MB = FIX ? (NB1 + kThreads - 1) / kThreads : 1;   // butterflies per thread
  constexpr int NE = FIX ? MB * R1 : MAXN / kThreads;             // elements per thread
  auto eidx = [&](int e) -> int {
    return FIX ? tid + kThreads * (e / R1) + (e % R1) * NB1 : tid + kThreads * e;
  };
  auto evalid = [&](int e) -> bool {
    if constexpr (FIX) return (e / R1 + 1) * kThreads <= NB1 || tid + kThreads * (e / R1) < NB1;
    else return tid + kThreads * e < N;
  };
  f2 z[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) z[e] = evalid(e) ? reinterpret_cast<const f2*>(xr)[eidx(e)] : (f2){0.f, 0.f};
  const float tmid = 0.5f * (float)(Nr - 1);
  auto etime = [&](int e) -> f2 {
    const float t = (float)(2 * eidx(e)) - tmid;
    return (f2){t, t + 1.f};
  };
  f2 s2 = (f2){0.f, 0.f}, sx2 = (f2){0.f, 0.f};
  bool bad = false;
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const f2 t2 = etime(e);
    const bool okx = isfinite(z[e].x), oky = isfinite(z[e].y);
    const f2 xv = (f2){okx ? z[e].x : 0.f, oky ? z[e].y : 0.f};
    s2 += xv;
    sx2 += t2 * xv;
    bad |= !(okx && oky);
  }
  // wave partials in fp32 (64 per-thread partials of 40 samples each), the
  // block combine in fp64; the missing-sample terms only in a wave that has one
  float cn = 0.f, stn = 0.f, sttn = 0.f;      // missing samples: count, sum tc, sum tc^2
  if (__any(bad)) {
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const f2 t2 = etime(e);
      const bool inb = evalid(e);
      const float mx = (inb && !isfinite(z[e].x)) ? 1.f : 0.f, my = (inb && !isfinite(z[e].y)) ? 1.f : 0.f;
      cn += mx + my;
      stn += mx * t2.x + my * t2.y;
      sttn += mx * t2.x * t2.x + my * t2.y * t2.y;
    }
    cn = wave_sum(cn);
    stn = wave_sum(stn);
    sttn = wave_sum(sttn);
  }
  const float ws = wave_sum(s2.x + s2.y), wsx = wave_sum(sx2.x + sx2.y);
  if (lane_id() == 0) { red5[0][wv] = ws; red5[1][wv] = wsx; red5[2][wv] = cn; red5[3][wv] = stn; red5[4][wv] = sttn; }
  __syncthreads();
  double ds = 0.0, dsx = 0.0, dcn = 0.0, dstn = 0.0, dsttn = 0.0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) {
    ds += red5[0][w]; dsx += red5[1][w]; dcn += red5[2][w]; dstn += red5[3][w]; dsttn += red5[4][w];
  }
  const double nr = (double)Nr;
  const double dc = nr - dcn;                                     // finite samples
  const double dst = -dstn;                                       // sum tc over all = 0
  const double dstt = nr * (nr * nr - 1.0) / 12.0 - dsttn;        // sum tc^2 over all
  const double cnt = dc > 0 ? dc : 1.0;
  const double tbar = dst / cnt, xbar = ds / cnt;
  const double vt = dstt / cnt - tbar * tbar;
  const double slope_d = vt > 0 ? (dsx / cnt - tbar * xbar) / vt : 0.0;
  const float mu = dc > 0 ? (float)xbar : 0.f;
  const float slope = (float)slope_d;
  // e = x - mu - slope (tc - tbar) = x - c0 - slope tc
  const float c0 = (float)((dc > 0 ? xbar : 0.0) - slope_d * tbar);
  // detrended samples (in place), with the Parseval terms: sum e^2, and
  // ex = (sum e_even, sum e_odd): X_0 = ex.x + ex.y, X_N = ex.x - ex.y
  f2 e2v = (f2){0.f, 0.f}, ex = (f2){0.f, 0.f};
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    if (evalid(e)) {
      f2 v = (z[e] - c0) - slope * etime(e);
      v.x = isfinite(z[e].x) ? v.x : 0.f;
      v.y = isfinite(z[e].y) ? v.y : 0.f;
      z[e] = v;
      e2v += v * v;
      ex += v;
    }
  }
  float e2 = e2v.x + e2v.y, x0 = ex.x + ex.y, xn = ex.x - ex.y;
  if constexpr (FIX) {
    // first pass (Ns = 1: no twiddles) on the registers, outputs to LDS
#pragma unroll
    for (int bb = 0; bb < MB; ++bb) {
      if (evalid(bb * R1)) {
        f2 v[R1];
#pragma unroll
        for (int q = 0; q < R1; ++q) v[q] = z[bb * R1 + q];
        dft<R1>(v);
        const int jb = tid + kThreads * bb;
#pragma unroll
        for (int p = 0; p < R1; ++p) buf[jb * R1 + p] = v[p];
      }
    }
    __syncthreads();
    FixedPlan<FN>::run_rest(buf);
  } else {
#pragma unroll
    for (int e = 0; e < NE; ++e)
      if (evalid(e)) buf[eidx(e)] = z[e];
    __syncthreads();
    int Ns = 1;
    for (int ps = 0; ps < plan.n_pass; ++ps) {
      const int r = plan.radix[ps];
      switch (r) {
        case 2: stockham_pass<2, MAXN>(buf, N, Ns); break;
        case 3: stockham_pass<3, MAXN>(buf, N, Ns); break;
        case 4: stockham_pass<4, MAXN>(buf, N, Ns); break;
        case 5: stockham_pass<5, MAXN>(buf, N, Ns); break;
        case 7: stockham_pass<7, MAXN>(buf, N, Ns); break;
        case 9: stockham_pass<9, MAXN>(buf, N, Ns); break;
        default: break;
      }
      Ns *= r;
    }
  }
  // unpack the real spectrum X[k]: the search band, or k = 0..N when the
  // periodogram / spectrum is wanted
  const bool full = power != nullptr || spec != nullptr;
  const int k0 = full ? 0 : kmin, k1 = full ? N : kmax;
  float best = -1.f;
  int bk = 0;
  for (int k = k0 + tid; k <= k1; k += kThreads) {
    const f2 zk = buf[k == N ? 0 : k];
    const f2 zn = buf[k == 0 ? 0 : N - k];
    const f2 zc = (f2){zn.x, -zn.y};
    const f2 e = 0.5f * (zk + zc);
    const f2 o = neg_i(0.5f * (zk - zc));
    const float2 t2 = tw2[k];
    const f2 X = e + cmul(o, (f2){t2.x, t2.y});
    const float pw = X.x * X.x + X.y * X.y;
    if (power) power[row * ld_p + k] = pw;
    if (spec) spec[row * ld_s + k] = make_float2(X.x, X.y);
    if (k >= kmin && k <= kmax && pw > best) { best = pw; bk = k; }
  }
  // block argmax (value, index) and the Parseval sums
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o);
    const int ok = __shfl_xor(bk, o);
    if (ob > best || (ob == best && ok < bk)) { best = ob; bk = ok; }
  }
  e2 = wave_sum(e2);
  x0 = wave_sum(x0);
  xn = wave_sum(xn);
  if (lane_id() == 0) { redf[0][wv] = best; redi[wv] = bk; redf[1][wv] = e2; redf[2][wv] = x0; redf[3][wv] = xn; }
  __syncthreads();
  if (tid == 0) {
    float b = redf[0][0], se = redf[1][0], s0 = redf[2][0], sn = redf[3][0];
    int k = redi[0];
    for (int w = 1; w < kThreads / 64; ++w) {
      if (redf[0][w] > b || (redf[0][w] == b && redi[w] < k)) { b = redf[0][w]; k = redi[w]; }
      se += redf[1][w]; s0 += redf[2][w]; sn += redf[3][w];
    }
    // sum_{k=1..N} |X_k|^2 = (Nr sum e^2 - X_0^2 + X_N^2) / 2 (Parseval, real input)
    const float t = 0.5f * ((float)Nr * se - s0 * s0 + sn * sn);
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
  if (kmin < 0 || kmax > Nr / 2) return (int)hipErrorInvalidValue;
  FftPlan plan;
  plan.n_pass = n_pass;
  int prod = 1;
  for (int i = 0; i < n_pass; ++i) { plan.radix[i] = radices[i]; prod *= radices[i]; }
  if (prod != Nr / 2) return (int)hipErrorInvalidValue;
  const int N = Nr / 2;
  const size_t lds = (size_t)N * sizeof(float2);
#define FM_FFT(MN, FN)                                                                                        \
  hipLaunchKernelGGL((fft_seasonal_kernel<MN, FN>), dim3((unsigned)R), dim3(kThreads), lds, stream, x, ld, Nr, R, \
                     tw, tw2, plan, kmin, kmax, power, ld_p, spec, ld_s, period_bin, strength, mean_out, slope_out)
  if (N == 5040) FM_FFT(5120, 5040);
  else if (N == 1008) FM_FFT(1024, 1008);
  else if (N == 720) FM_FFT(768, 720);
  else if (N <= 2048) FM_FFT(2048, 0);
  else if (N <= 5120) FM_FFT(5120, 0);
  else FM_FFT(kMaxN, 0);
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
