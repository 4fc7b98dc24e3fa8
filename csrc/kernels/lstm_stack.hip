// K6 at full spec: H up to 256, 1-2 stacked layers, multivariate input, on
// bf16 MFMA (v_mfma_f32_32x32x16_bf16, fp32 accumulate).  Reference intent:
// the brain's LSTM forecasts "3+ metrics" jointly (docs/guides/design.md:81-85)
// for HPA / ClusterAutoScaler prediction (README.md:58-59, BASELINE config 4).
//
// Why a second kernel (lstm.hip keeps every weight in registers): at H = 256
// one layer's [W_hh | W_ih | b] is 4H x (H + 16) bf16 = 544 KB, more than a
// CU's whole register file (512 KB) and 3.4x its LDS; two layers are 1.6 MB.
// So the weights stream from L2 every step (one fleet-wide copy, 1.6 MB per
// XCD's 4 MB L2) and everything per-sequence stays on chip:
//
//   * one workgroup owns BT = 32 NCT sequences for all L steps;
//   * wave w owns RT row tiles of 32 gate rows = 8 RT hidden units
//     ([i f g o] x 8 units per tile, the layout of lstm.hip), so the cell
//     update is lane-local and c (both layers) lives in fp32 registers;
//   * h of both layers is double-buffered in LDS as bf16 [BT][H + 8] images
//     (row pad: conflict-free ds_read_b128 of the B operand);
//   * per step: layer 0 gates = [W_hh0 | W_ih0 | b0] x [h0_{t-1}; x_t; 1],
//     cell -> h0_t (LDS), barrier; layer 1 gates = [W_hh1 | W_ih1 | b1] x
//     [h1_{t-1}; h0_t; 1], cell -> h1_t (LDS), barrier.  Layer 1 consumes
//     layer 0's h from LDS in the same step: h0 never goes to HBM.
//   * the A fragments of each k-step are loaded (16 B per lane, L2 hits) one
//     k-step ahead of the MFMAs that use them.
#include "fm_common.h"

using namespace fm;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kExpClamp = 29.f;

__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  const __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ float exp2_clamped(float x) {
  return __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(x, -kExpClamp, kExpClamp));
}
// fused-fraction cell (same algebra as lstm.hip: 5 exp + 2 rcp per unit-step)
__device__ __forceinline__ void cell(float ai, float af, float ag, float ao, float& c, float& h) {
  const float pi = 1.f + exp2_clamped(ai * -kLog2e);
  const float pf = 1.f + exp2_clamped(af * -kLog2e);
  const float eg = exp2_clamped(ag * (-2.f * kLog2e));
  const float pg = 1.f + eg;
  const float pig = pi * pg;
  const float cn = (c * pig + (1.f - eg) * pf) * __builtin_amdgcn_rcpf(pf * pig);
  c = cn;
  const float po = 1.f + exp2_clamped(ao * -kLog2e);
  const float ec = exp2_clamped(cn * (-2.f * kLog2e));
  h = (1.f - ec) * __builtin_amdgcn_rcpf(po * (1.f + ec));
}

union Frag {
  bf16x8 v;
  uint4 u;
};

}  // namespace

// W0: [NW][RT][KS0][64] x 16 B, KS0 = H/16 + 1 (last k-step: x_t and the bias)
// W1: [NW][RT][KS1][64] x 16 B, KS1 = 2H/16 + 1 (h1_{t-1}, h0_t, bias)
// xa: [B, L, 16] bf16 (features at k < I, 1.0 at k = I)
template <int H, int RT, int NCT, int LAYERS>
__global__ __launch_bounds__(64 * H / (8 * RT)) void lstm_stack_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out /*[B,H] top layer*/, float* __restrict__ c_out /*[B,H]*/) {
  constexpr int NW = H / (8 * RT);     // waves
  constexpr int KH = H / 16;           // k-steps over one hidden vector
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 32 * NCT;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                          // [2][BT][HP]
  unsigned short* h1b = lds + 2 * BT * HP;            // [2][BT][HP] (LAYERS == 2)
  const int lane = lane_id(), w = wave_id();
  const int hf = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  for (int i = threadIdx.x; i < LAYERS * 2 * BT * HP; i += 64 * NW) lds[i] = 0;   // h_{-1} = 0
  float c0[RT][NCT][4], c1[RT][NCT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) c0[rt][ct][j] = c1[rt][ct][j] = 0.f;
  __syncthreads();

  const uint4* xp[NCT];
  bool inb[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    int64_t bb = b0 + 32 * ct + col;
    inb[ct] = bb < B;
    bb = bb < B ? bb : B - 1;
    xp[ct] = xa + (bb * L) * 2 + hf;
  }
  const uint4* W0w = W0 + (int64_t)w * RT * KS0 * 64 + lane;
  const uint4* W1w = W1 + (int64_t)w * RT * KS1 * 64 + lane;
  Frag ones;                                          // layer-1 bias step: B = [1, 0, ..., 0]
  ones.u = make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);

  // gates[rt][ct] = sum_ks A[rt][ks] B[ks][ct]; B of k-step ks from `bsrc`
  auto gemm = [&](const uint4* Ww, int KS, auto bsrc, f32x16 (&acc)[RT][NCT]) {
    Frag a[RT], an[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[rt].u = Ww[(rt * KS + 0) * 64];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = (f32x16){};
    // not unrolled: unrolling lets the scheduler hoist every k-step's A
    // fragments (33 x RT x 16 B per lane at H = 256) and spill; one k-step of
    // lookahead is what the L2 latency needs with 2 waves per SIMD (at 4 x 2
    // tiling the lookahead costs 65 spilled VGPRs and still wins: without it
    // config 4 at H = 256 x 2 layers runs 10.1 instead of 9.0 ms)
#pragma unroll 1
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) an[rt].u = Ww[(rt * KS + ks + 1) * 64];
      }
      Frag bf[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) bf[ct].u = bsrc(ks, ct);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt].v, bf[ct].v, acc[rt][ct], 0, 0, 0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) a[rt] = an[rt];
    }
  };
  // lane-local cell update; regs j, 4+j, 8+j, 12+j = i, f, g, o of unit u0 + j
  auto update = [&](f32x16 (&acc)[RT][NCT], float (&c)[RT][NCT][4], unsigned short* hdst, bool last) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        float hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          cell(acc[rt][ct][j], acc[rt][ct][4 + j], acc[rt][ct][8 + j], acc[rt][ct][12 + j], c[rt][ct][j], hv[j]);
        const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
        uint2 pk;
        pk.x = pack_bf2(hv[0], hv[1]);
        pk.y = pack_bf2(hv[2], hv[3]);
        *reinterpret_cast<uint2*>(&hdst[(32 * ct + col) * HP + u0]) = pk;
        if (last && inb[ct]) {
          const int64_t bb = b0 + 32 * ct + col;
          *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          *reinterpret_cast<float4*>(&c_out[bb * H + u0]) =
              make_float4(c[rt][ct][0], c[rt][ct][1], c[rt][ct][2], c[rt][ct][3]);
        }
      }
  };

  uint4 xn[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) xn[ct] = xp[ct][0];
  for (int t = 0; t < L; ++t) {
    const int cur = t & 1, prv = cur ^ 1;
    const bool last = t == L - 1;
    uint4 xt[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      xt[ct] = xn[ct];
      if (!last) xn[ct] = xp[ct][(t + 1) * 2];
    }
    f32x16 acc[RT][NCT];
    const unsigned short* h0p = h0b + prv * BT * HP;
    gemm(W0w, KS0,
         [&](int ks, int ct) -> uint4 {
           return ks < KH ? *reinterpret_cast<const uint4*>(&h0p[(32 * ct + col) * HP + 16 * ks + 8 * hf]) : xt[ct];
         },
         acc);
    update(acc, c0, h0b + cur * BT * HP, last && LAYERS == 1);
    __syncthreads();
    if (LAYERS == 2) {
      const unsigned short* h1p = h1b + prv * BT * HP;
      const unsigned short* h0c = h0b + cur * BT * HP;
      gemm(W1w, KS1,
           [&](int ks, int ct) -> uint4 {
             if (ks < KH) return *reinterpret_cast<const uint4*>(&h1p[(32 * ct + col) * HP + 16 * ks + 8 * hf]);
             if (ks < 2 * KH)
               return *reinterpret_cast<const uint4*>(&h0c[(32 * ct + col) * HP + 16 * (ks - KH) + 8 * hf]);
             return ones.u;
           },
           acc);
      update(acc, c1, h1b + cur * BT * HP, last);
      __syncthreads();
    }
  }
}

template <int H, int RT, int NCT, int LAYERS>
static int launch_stack(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out, float* c_out,
                        hipStream_t stream) {
  constexpr int NW = H / (8 * RT);
  constexpr int BT = 32 * NCT;
  const size_t lds = (size_t)LAYERS * 2 * BT * (H + 8) * sizeof(unsigned short);
  auto k = lstm_stack_kernel<H, RT, NCT, LAYERS>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + BT - 1) / BT)), dim3(64 * NW), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
}

// Row tiles per wave / column tiles per workgroup (see ops/lstm.py STACK_TILING):
// H=256: 4 x 2 (8 waves, 64 sequences share every streamed weight fragment:
// half the L2 weight traffic of 4 x 1, which wins despite 65 spilled VGPRs
// and half the workgroups -- config 4 at 2 layers 10.8 -> 9.0 ms,
// profiles/lstm_tile_ab_r2.txt); H<=128: 2 x 2 (H/16 waves, 64 sequences).
// rt / nct = 0 pick that default; the other H = 256 tilings (4 x 1, 2 x 2,
// 2 x 1) stay instantiated for the A/B (ops/lstm.py FM_LSTM_STACK_TILING)
// and need weights packed with the same RT.
FM_API int fm_lstm_stack(const void* xa, int64_t B, int L, int H, int layers, const void* W0, const void* W1,
                         float* h_out, float* c_out, int rt, int nct, hipStream_t stream) {
  if (B <= 0 || L <= 0) return 0;
  if (layers != 1 && layers != 2) return (int)hipErrorInvalidValue;
  if (layers == 2 && W1 == nullptr) return (int)hipErrorInvalidValue;
#define FM_STK(HH, RTT, NCC)                                                                              \
  return layers == 2 ? launch_stack<HH, RTT, NCC, 2>(xa, B, L, W0, W1, h_out, c_out, stream)            \
                     : launch_stack<HH, RTT, NCC, 1>(xa, B, L, W0, W1, h_out, c_out, stream)
  switch (H) {
    case 256:
      if (rt == 0 || (rt == 4 && nct == 2)) FM_STK(256, 4, 2);
      if (rt == 4 && nct == 1) FM_STK(256, 4, 1);
      if (rt == 2 && nct == 2) FM_STK(256, 2, 2);
      if (rt == 2 && nct == 1) FM_STK(256, 2, 1);
      return (int)hipErrorInvalidValue;
    case 128: if (rt == 0 || (rt == 2 && nct == 2)) FM_STK(128, 2, 2); return (int)hipErrorInvalidValue;
    case 64: if (rt == 0 || (rt == 2 && nct == 2)) FM_STK(64, 2, 2); return (int)hipErrorInvalidValue;
    case 32: if (rt == 0 || (rt == 2 && nct == 2)) FM_STK(32, 2, 2); return (int)hipErrorInvalidValue;
    default: return (int)hipErrorInvalidValue;
  }
#undef FM_STK
}

// Multivariate forecaster features, one row per SERVICE: the last L samples of
// its M metric series (rows s*M .. s*M+M-1 of the packed history), each
// z-scored over its own window's finite samples (missing -> 0), then the daily
// phase sin / cos, then 1.0 (bias) -> [S, L, 16] bf16.  Needs M + 3 <= 16.
// One wave per (service, metric) for the moments, then the interleave.
__global__ __launch_bounds__(256) void lstm_features_mv_kernel(const float* __restrict__ hist, int64_t ld, int T,
                                                               int64_t S, int M, int L, float period,
                                                               unsigned short* __restrict__ xa,
                                                               float* __restrict__ mu_out,
                                                               float* __restrict__ sd_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + wave_id();      // series row s*M + m
  if (r >= S * M) return;
  const int lane = lane_id();
  const float* hr = hist + r * ld + (T - L);
  float s = 0.f;
  int n = 0;
  for (int i = lane; i < L; i += 64) {
    const float v = hr[i];
    if (isfinite(v)) { s += v; ++n; }
  }
  s = wave_sum(s);
  n = wave_sum(n);
  const float mu = s / (float)(n > 0 ? n : 1);
  float q = 0.f;
  for (int i = lane; i < L; i += 64) {
    const float v = hr[i];
    if (isfinite(v)) { const float d = v - mu; q += d * d; }
  }
  q = wave_sum(q);
  float sd = sqrtf(q / (float)(n > 0 ? n : 1));
  sd = sd > 1e-6f ? sd : 1e-6f;
  const float inv = 1.f / sd;
  const int64_t svc = r / M;
  const int m = (int)(r - svc * M);
  const float w0 = 6.283185307179586f / period;
  unsigned short* xs = xa + svc * L * 16;
  for (int i = lane; i < L; i += 64) {
    const float v = hr[i];
    xs[i * 16 + m] = f2bf(isfinite(v) ? (v - mu) * inv : 0.f);
    if (m == 0) {                                   // one wave per service writes the shared columns
      const float ph = w0 * (float)(T - L + i);
      xs[i * 16 + M] = f2bf(sinf(ph));
      xs[i * 16 + M + 1] = f2bf(cosf(ph));
      xs[i * 16 + M + 2] = f2bf(1.f);
      for (int k = M + 3; k < 16; ++k) xs[i * 16 + k] = 0;
    }
  }
  if (lane == 0) { mu_out[r] = mu; sd_out[r] = sd; }
}

FM_API int fm_lstm_features_mv(const float* hist, int64_t ld, int T, int64_t S, int M, int L, float period, void* xa,
                               float* mu, float* sd, hipStream_t stream) {
  if (S <= 0) return 0;
  if (L <= 0 || L > T || M <= 0 || M + 3 > 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(lstm_features_mv_kernel, dim3((unsigned)((S * M + 3) / 4)), dim3(256), 0, stream, hist, ld, T, S,
                     M, L, period, (unsigned short*)xa, mu, sd);
  FM_LAUNCH_CHECK();
  return 0;
}
