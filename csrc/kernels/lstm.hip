// K6: LSTM forecaster cell on bf16 MFMA (v_mfma_f32_32x32x16_bf16, fp32
// accumulate).  Reference: the brain's deep model is an LSTM on Keras/MXNet
// (docs/guides/design.md:81-85, foremast-brain/faq.md:10), used for HPA /
// ClusterAutoScaler prediction (README.md:58-59; BASELINE config 4).
//
// Persistent-over-time structure: one workgroup owns a tile of Bt = 64
// sequences for all L steps; wave w (H/16 waves) owns hidden units
// [16w, 16w+16).  The recurrent AND input weights are register-resident for
// the whole sequence: the input projection and bias are folded into the GEMM
// by augmenting K with one extra 16-wide k-step, B = [h_{t-1}; x_t; 1; 0..]
// and A = [W_hh | W_ih | b | 0].  Gate rows inside a 32-row tile are ordered
// [i(8 units) f(8) g(8) o(8)], so with the 32x32 C/D map (row = (reg&3) +
// 8(reg>>2) + 4(lane>>5)) every lane holds i, f, g, o of the same 4 units and
// one batch column: the cell update is lane-local, c stays in fp32 registers,
// and only h (bf16) crosses LDS, read back as the next step's B operand with
// ds_read_b128 from a [batch][H + 8] image (row pad -> conflict-free).
#include "fm_common.h"

using namespace fm;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// RNE float -> bf16 on the hardware converter (v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ unsigned short f2bf(float f) {
  const __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
// Gate nonlinearities on the transcendental unit, 2 transcendentals each:
//   sigm(x) = 1 / (1 + 2^(-x log2 e))          v_mul, v_exp, v_add, v_rcp
//   tanh(x) = 2 sigm(2x) - 1                    (+1 fma; saturates correctly
//                                                 through exp -> inf/0)
// A correctly rounded '/' would expand to a ~10-instruction
// div_scale/div_fmas/div_fixup sequence; the cell update does 5 per unit per step.
constexpr float kLog2e = 1.4426950408889634f;
__device__ __forceinline__ float sigm(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * -kLog2e));
}
__device__ __forceinline__ float tanh_f(float x) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * (-2.f * kLog2e))) - 1.f;
}

union Frag {
  bf16x8 v;
  unsigned short s[8];
  uint4 u;
};

// Wpack: [H/16 waves][2 rt][KS k-steps][64 lanes] x 8 bf16, pre-swizzled on the
// host so each lane loads its A fragment with one 16-B load.
template <int H>
__global__ __launch_bounds__(H * 4) void lstm_fwd_kernel(const float* __restrict__ x /*[B, L, I]*/, int64_t B, int L,
                                                         int I, const uint4* __restrict__ Wpack,
                                                         const float* __restrict__ h0, const float* __restrict__ c0,
                                                         float* __restrict__ h_out /*[B,H]*/,
                                                         float* __restrict__ c_out /*[B,H]*/,
                                                         unsigned short* __restrict__ hseq /*[B,L,H] bf16 or null*/) {
  constexpr int KS = H / 16 + 1;  // k-steps: H/16 recurrent + 1 augmented (x, 1)
  constexpr int HP = H + 8;       // padded LDS row (bf16)
  constexpr int BT = 64;
  __shared__ __attribute__((aligned(16))) unsigned short hbuf[2][BT * HP];
  const int lane = lane_id(), w = wave_id();
  const int h = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  // register-resident A fragments
  Frag A[2][KS];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) A[rt][ks].u = Wpack[(((int64_t)w * 2 + rt) * KS + ks) * 64 + lane];

  // initial state: this lane's units u = 16w + 8rt + 4h + j, batch = b0 + 32ct + col
  float c[2][2][4];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = 16 * w + 8 * rt + 4 * h + j;
        const int64_t bb = b0 + 32 * ct + col;
        c[rt][ct][j] = (c0 != nullptr && bb < B) ? c0[bb * H + u] : 0.f;
        const float hv = (h0 != nullptr && bb < B) ? h0[bb * H + u] : 0.f;
        hbuf[0][(32 * ct + col) * HP + u] = f2bf(hv);
      }
  __syncthreads();

  // x_t of this lane's features (h == 0 lanes: k = 0..7; h == 1: k = 8..15) is
  // loaded one step ahead so the global-memory latency hides behind the
  // previous step's MFMAs instead of stalling the head of every step.
  float xn[2][8];
  auto load_x = [&](int tt) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const int64_t bb = b0 + 32 * ct + col;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * h + j;
        xn[ct][j] = (k < I && bb < B && tt < L) ? x[(bb * L + tt) * I + k] : 0.f;
      }
    }
  };
  load_x(0);
  int cur = 0;
  for (int t = 0; t < L; ++t) {
    // augmented operand: x_t features, bias "1" at k = I
    Frag xb[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int j = 0; j < 8; ++j) xb[ct].s[j] = f2bf(8 * h + j == I ? 1.f : xn[ct][j]);
    load_x(t + 1);
    f32x16 acc[2][2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) acc[rt][ct] = (f32x16){};
#pragma unroll
    for (int ks = 0; ks < KS - 1; ++ks) {
      Frag bfr[2];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        bfr[ct].u = *reinterpret_cast<const uint4*>(&hbuf[cur][(32 * ct + col) * HP + 16 * ks + 8 * h]);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][ks].v, bfr[ct].v, acc[rt][ct], 0, 0, 0);
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct)
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][KS - 1].v, xb[ct].v, acc[rt][ct], 0, 0, 0);

    // lane-local cell update; regs j, 4+j, 8+j, 12+j = i, f, g, o of unit 16w+8rt+4h+j
    const int nxt = cur ^ 1;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        float hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float ig = sigm(acc[rt][ct][j]);
          const float fg = sigm(acc[rt][ct][4 + j]);
          const float gg = tanh_f(acc[rt][ct][8 + j]);
          const float og = sigm(acc[rt][ct][12 + j]);
          const float cc = fg * c[rt][ct][j] + ig * gg;
          c[rt][ct][j] = cc;
          const float hh = og * tanh_f(cc);
          hv[j] = hh;
          if (t == L - 1) {
            const int64_t bb = b0 + 32 * ct + col;
            const int u = 16 * w + 8 * rt + 4 * h + j;
            if (bb < B) { h_out[bb * H + u] = hh; c_out[bb * H + u] = cc; }
          }
        }
        const int u0 = 16 * w + 8 * rt + 4 * h;
        uint2 pk;
        pk.x = pack_bf2(hv[0], hv[1]);
        pk.y = pack_bf2(hv[2], hv[3]);
        *reinterpret_cast<uint2*>(&hbuf[nxt][(32 * ct + col) * HP + u0]) = pk;
        if (hseq != nullptr) {
          const int64_t bb = b0 + 32 * ct + col;
          if (bb < B) *reinterpret_cast<uint2*>(&hseq[(bb * L + t) * H + u0]) = pk;
        }
      }
    __syncthreads();
    cur = nxt;
  }
}

FM_API int fm_lstm_forward(const float* x, int64_t B, int L, int I, int H, const void* Wpack, const float* h0,
                           const float* c0, float* h_out, float* c_out, unsigned short* hseq, hipStream_t stream) {
  if (B <= 0 || L <= 0) return 0;
  if (I < 0 || I > 15) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((B + 63) / 64));
  if (H == 128)
    hipLaunchKernelGGL(lstm_fwd_kernel<128>, grid, dim3(512), 0, stream, x, B, L, I, (const uint4*)Wpack, h0, c0,
                       h_out, c_out, hseq);
  else if (H == 64)
    hipLaunchKernelGGL(lstm_fwd_kernel<64>, grid, dim3(256), 0, stream, x, B, L, I, (const uint4*)Wpack, h0, c0,
                       h_out, c_out, hseq);
  else if (H == 32)
    hipLaunchKernelGGL(lstm_fwd_kernel<32>, grid, dim3(128), 0, stream, x, B, L, I, (const uint4*)Wpack, h0, c0,
                       h_out, c_out, hseq);
  else
    return (int)hipErrorInvalidValue;
  FM_LAUNCH_CHECK();
  return 0;
}
