// fm-hipcc-flags: -fno-slp-vectorize
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
#include "fm_lstm_cell.h"

#include <type_traits>

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
// The cell update (fm_lstm_cell.h): the packed weights carry the gate
// scales (i, f, o rows by -log2 e, g rows by -2 log2 e) and c is kept scaled
// (cs = -2 log2(e) c) -- 14 VALU + 8 transcendental issues per unit-step.
union Frag {
  bf16x8 v;
  unsigned short s[8];
  uint4 u;
};

// Wpack: [H/16 waves][2 rt][KS k-steps][64 lanes] x 8 bf16, pre-swizzled on the
// host so each lane loads its A fragment with one 16-B load.
//
// Input xa: [B, L, 16] bf16, the augmented K step already laid out
// (features at k < I, 1.0 at k = I for the bias, zeros above): lane half h
// reads its 8 values of step t with ONE 16-B load, no conversion and no
// per-feature branches (fm_lstm_features writes it straight from the history).
template <int H, int NCT, int CELL>
__global__ __launch_bounds__(H * 4) void lstm_fwd_kernel(const uint4* __restrict__ xa /*[B, L, 2] x 16 B*/,
                                                         int64_t B, int L, const uint4* __restrict__ Wpack,
                                                         const float* __restrict__ h0, const float* __restrict__ c0,
                                                         float* __restrict__ h_out /*[B,H]*/,
                                                         float* __restrict__ c_out /*[B,H]*/,
                                                         unsigned short* __restrict__ hseq /*[B,L,H] bf16 or null*/) {
  constexpr int KS = H / 16 + 1;  // k-steps: H/16 recurrent + 1 augmented (x, 1)
  constexpr int HP = H + 8;       // padded LDS row (bf16)
  constexpr int BT = 32 * NCT;     // batch columns per workgroup (NCT 32-wide MFMA column tiles)
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
  float c[2][NCT][4];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = 16 * w + 8 * rt + 4 * h + j;
        const int64_t bb = b0 + 32 * ct + col;
        c[rt][ct][j] = (c0 != nullptr && bb < B) ? kLstmK * c0[bb * H + u] : 0.f;
        const float hv = (h0 != nullptr && bb < B) ? h0[bb * H + u] : 0.f;
        hbuf[0][(32 * ct + col) * HP + u] = f2bf(hv);
      }
  __syncthreads();

  // per-lane input streams (rows past B clamp to B-1: loaded, never stored)
  const uint4* xp[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    int64_t bb = b0 + 32 * ct + col;
    bb = bb < B ? bb : B - 1;
    xp[ct] = xa + (bb * L) * 2 + h;
  }
  // x_{t+1} is loaded while step t computes
  uint4 xn[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) xn[ct] = xp[ct][0];
  int cur = 0;

  auto step = [&](int t, auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
    Frag xb[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      xb[ct].u = xn[ct];
      if (!LAST) xn[ct] = xp[ct][(t + 1) * 2];
    }
    f32x16 acc[2][NCT];
    {
      Frag bfr[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        bfr[ct].u = *reinterpret_cast<const uint4*>(&hbuf[cur][(32 * ct + col) * HP + 8 * h]);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][0].v, bfr[ct].v, (f32x16){}, 0, 0, 0);
    }
#pragma unroll
    for (int ks = 1; ks < KS - 1; ++ks) {
      Frag bfr[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        bfr[ct].u = *reinterpret_cast<const uint4*>(&hbuf[cur][(32 * ct + col) * HP + 16 * ks + 8 * h]);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][ks].v, bfr[ct].v, acc[rt][ct], 0, 0, 0);
    }
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct)
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][KS - 1].v, xb[ct].v, acc[rt][ct], 0, 0, 0);

    // lane-local cell update; regs j, 4+j, 8+j, 12+j = i, f, g, o of unit 16w+8rt+4h+j
    const int nxt = cur ^ 1;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        float hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (CELL == 1)
            lstm_cell(acc[rt][ct][j], acc[rt][ct][4 + j], acc[rt][ct][8 + j], acc[rt][ct][12 + j], c[rt][ct][j], hv[j]);
          else
            lstm_cell_separate(acc[rt][ct][j], acc[rt][ct][4 + j], acc[rt][ct][8 + j], acc[rt][ct][12 + j],
                               c[rt][ct][j], hv[j]);
        }
        const int u0 = 16 * w + 8 * rt + 4 * h;
        const int64_t bb = b0 + 32 * ct + col;
        uint2 pk;
        pk.x = pack_bf2(hv[0], hv[1]);
        pk.y = pack_bf2(hv[2], hv[3]);
        if (LAST) {
          if (bb < B) {
            *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
            *reinterpret_cast<float4*>(&c_out[bb * H + u0]) =
                make_float4(c[rt][ct][0] * kLstmInvK, c[rt][ct][1] * kLstmInvK, c[rt][ct][2] * kLstmInvK,
                            c[rt][ct][3] * kLstmInvK);
          }
        } else {
          *reinterpret_cast<uint2*>(&hbuf[nxt][(32 * ct + col) * HP + u0]) = pk;
        }
        if (hseq != nullptr && bb < B) *reinterpret_cast<uint2*>(&hseq[(bb * L + t) * H + u0]) = pk;
      }
    if (!LAST) {
      __syncthreads();
      cur = nxt;
    }
  };
  for (int t = 0; t < L - 1; ++t) step(t, std::false_type{});
  step(L - 1, std::true_type{});
}

// ---------------------------------------------------------------------------
// Column-tile pipelined form (2 tiles of 32 sequences per workgroup).  The
// kernel above does, per step, all MFMAs (both tiles) and then the cell
// update that consumes them, so the matrix pipe and the VALU/transcendental
// pipes take turns (PMC: MFMA busy 32 %, co-exec cycles ~30 % of MFMA
// cycles).  Here a step is two half-steps, each pairing the MFMAs of one tile
// with the cell update of the OTHER tile, whose accumulators were produced in
// the previous half-step:
//     A(t): MFMA tile1(t)   ||  cell tile0(t) -> h tile0(t)   ; barrier
//     B(t): MFMA tile0(t+1) ||  cell tile1(t) -> h tile1(t)   ; barrier
// The two instruction streams of a half-step are independent, so a wave
// issues VALU while its own MFMAs occupy the matrix pipe.  Each tile's h is
// single-buffered in LDS: it is rewritten one half-step after its last
// reader, with a barrier in between.
// ---------------------------------------------------------------------------
// x sources of the pipelined kernel: fetch(ct, t) issues the load of step t
// of column tile ct (one step ahead of its use), make(ct, t, raw) turns it
// into this lane's 16-B half of the augmented K step.
struct XaSource {            // the augmented bf16 input [B, L, 16] (fm_lstm_features)
  using Raw = uint4;
  const uint4* xp[2];
  __device__ void setup(const uint4* xa, int64_t b0, int64_t B, int L, int col, int h) {
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      int64_t bb = b0 + 32 * ct + col;
      bb = bb < B ? bb : B - 1;
      xp[ct] = xa + (bb * L) * 2 + h;
    }
  }
  __device__ __forceinline__ Raw fetch(int ct, int t) const { return xp[ct][t * 2]; }
  __device__ __forceinline__ uint4 make(int, int, const Raw& r) const { return r; }
};

// The forecaster's features computed in the kernel from the history rows
// themselves (a resident grid row through rm / shift / lim, or a plain
// [B, ld] matrix): per sequence the last L samples z-scored over their finite
// values (population std, >= 1e-6, missing -> 0), then sin / cos of the daily
// phase 2 pi c / period of the dense column c, 1.0 at k = I -- the layout
// fm_lstm_features writes, without its [B, L, 16] bf16 round trip through HBM.
struct HistSource {
  using Raw = float;
  const float* row[2];
  int off[2], lim[2];
  float mu[2], inv[2];
  int c0;                    // dense column of step 0 (T - L)
  float p, ip;               // period and 1 / period
  int I;
  bool lo_half;              // lane holds k = 0..7 (the features), else k = 8..15 (zeros)
  // per step t: {f1, bits of pack_bf2(f2, f3)} -- the phase features are the
  // same for every sequence, built once per workgroup in LDS (null: L too
  // long for the table, computed per lane)
  const float2* tab;
  __device__ __forceinline__ Raw fetch(int ct, int t) const {
    const int bc = c0 + t + off[ct];
    return (lo_half && bc >= 0 && bc < lim[ct]) ? row[ct][bc] : __builtin_nanf("");
  }
  __device__ __forceinline__ uint4 make(int ct, int t, const Raw& v) const {
    if (!lo_half) return make_uint4(0u, 0u, 0u, 0u);
    const float z = isfinite(v) ? (v - mu[ct]) * inv[ct] : 0.f;
    if (tab != nullptr) {
      const float2 e = tab[t];
      return make_uint4(pack_bf2(I > 0 ? z : 1.f, e.x), __float_as_uint(e.y), 0u, 0u);
    }
    const float c = (float)(c0 + t);
    const float q = floorf(c * ip);
    const float fr = __builtin_fmaf(-q, p, c) * ip;          // phase in revolutions, [0, 1)
    const float sn = __builtin_amdgcn_sinf(fr), cs = __builtin_amdgcn_cosf(fr);
    // [z, sin, cos][:I], 1.0 at k = I, zeros above (I <= 3)
    const float f0 = I > 0 ? z : 1.f;
    const float f1 = I > 1 ? sn : (I == 1 ? 1.f : 0.f);
    const float f2 = I > 2 ? cs : (I == 2 ? 1.f : 0.f);
    const float f3 = I == 3 ? 1.f : 0.f;
    return make_uint4(pack_bf2(f0, f1), pack_bf2(f2, f3), 0u, 0u);
  }
  // the table entry of step t (what make() computes per lane without it)
  __device__ __forceinline__ float2 phase_entry(int t) const {
    const float c = (float)(c0 + t);
    const float q = floorf(c * ip);
    const float fr = __builtin_fmaf(-q, p, c) * ip;
    const float sn = __builtin_amdgcn_sinf(fr), cs = __builtin_amdgcn_cosf(fr);
    const float f1 = I > 1 ? sn : (I == 1 ? 1.f : 0.f);
    const float f2 = I > 2 ? cs : (I == 2 ? 1.f : 0.f);
    const float f3 = I == 3 ? 1.f : 0.f;
    return make_float2(f1, __uint_as_float(pack_bf2(f2, f3)));
  }
};

constexpr int kLstmPhaseTab = 2048;     // steps of the LDS phase table (16 KB)

template <int H, bool HSEQ, typename XS>
__device__ __forceinline__ void lstm_pipe_body(const XS& xs, int64_t B, int L, const uint4* __restrict__ Wpack,
                                               const float* __restrict__ h0, const float* __restrict__ c0,
                                               float* __restrict__ h_out, float* __restrict__ c_out,
                                               unsigned short* __restrict__ hseq, unsigned short* hbuf) {
  constexpr int KS = H / 16 + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 64;
  const int lane = lane_id(), w = wave_id();
  const int h = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  Frag A[2][KS];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) A[rt][ks].u = Wpack[(((int64_t)w * 2 + rt) * KS + ks) * 64 + lane];

  float c[2][2][4];   // [tile][rt][j]
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int u = 16 * w + 8 * rt + 4 * h + j;
        const int64_t bb = b0 + 32 * ct + col;
        c[ct][rt][j] = (c0 != nullptr && bb < B) ? kLstmK * c0[bb * H + u] : 0.f;
        const float hv = (h0 != nullptr && bb < B) ? h0[bb * H + u] : 0.f;
        hbuf[(32 * ct + col) * HP + u] = f2bf(hv);
      }
  __syncthreads();

  bool inb[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) inb[ct] = b0 + 32 * ct + col < B;

  // MFMAs of one tile for one step: h_{t-1} of the tile from LDS, x_t from xv
  auto gates = [&](int ct, const uint4& xv, f32x16 (&acc)[2]) {
    const unsigned short* hb = &hbuf[(32 * ct + col) * HP + 8 * h];
    Frag bfr[KS - 1];
#pragma unroll
    for (int ks = 0; ks < KS - 1; ++ks) bfr[ks].u = *reinterpret_cast<const uint4*>(hb + 16 * ks);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][0].v, bfr[0].v,
                                                                                    (f32x16){}, 0, 0, 0);
#pragma unroll
    for (int ks = 1; ks < KS - 1; ++ks)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][ks].v, bfr[ks].v, acc[rt], 0, 0, 0);
    Frag xb;
    xb.u = xv;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
      acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][KS - 1].v, xb.v, acc[rt], 0, 0, 0);
  };
  // cell update of one tile; writes h_t to LDS (or the final state)
  auto cell = [&](int ct, int t, const f32x16 (&acc)[2], bool last) {
    const int64_t bb = b0 + 32 * ct + col;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      float hv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) lstm_cell(acc[rt][j], acc[rt][4 + j], acc[rt][8 + j], acc[rt][12 + j], c[ct][rt][j], hv[j]);
      const int u0 = 16 * w + 8 * rt + 4 * h;
      uint2 pk;
      pk.x = pack_bf2(hv[0], hv[1]);
      pk.y = pack_bf2(hv[2], hv[3]);
      if (last) {
        if (inb[ct]) {
          *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          *reinterpret_cast<float4*>(&c_out[bb * H + u0]) =
              make_float4(c[ct][rt][0] * kLstmInvK, c[ct][rt][1] * kLstmInvK, c[ct][rt][2] * kLstmInvK,
                          c[ct][rt][3] * kLstmInvK);
        }
      } else {
        *reinterpret_cast<uint2*>(&hbuf[(32 * ct + col) * HP + u0]) = pk;
      }
      if (HSEQ && inb[ct]) *reinterpret_cast<uint2*>(&hseq[(bb * L + t) * H + u0]) = pk;
    }
  };

  f32x16 acc0[2], acc1[2];
  typename XS::Raw x0n = xs.fetch(0, 0), x1n = xs.fetch(1, 0);
  gates(0, xs.make(0, 0, x0n), acc0);                // tile 0, step 0
  if (L > 1) x0n = xs.fetch(0, 1);                   // x_1 of tile 0
  __syncthreads();                                   // tile-0 h_{-1} read by all before A(0) rewrites it
  for (int t = 0; t < L; ++t) {
    const bool last = t == L - 1;
    // A(t): tile-1 MFMAs for step t || tile-0 cell of step t
    const typename XS::Raw x1 = x1n;
    if (!last) x1n = xs.fetch(1, t + 1);
    gates(1, xs.make(1, t, x1), acc1);
    cell(0, t, acc0, last);
    __syncthreads();
    // B(t): tile-0 MFMAs for step t+1 || tile-1 cell of step t
    if (!last) {
      const typename XS::Raw x0 = x0n;
      if (t + 2 < L) x0n = xs.fetch(0, t + 2);
      gates(0, xs.make(0, t + 1, x0), acc0);
    }
    cell(1, t, acc1, last);
    if (!last) __syncthreads();
  }
}

template <int H, bool HSEQ>
__global__ __launch_bounds__(H * 4) void lstm_fwd_pipe_kernel(const uint4* __restrict__ xa /*[B, L, 2] x 16 B*/,
                                                              int64_t B, int L, const uint4* __restrict__ Wpack,
                                                              const float* __restrict__ h0,
                                                              const float* __restrict__ c0,
                                                              float* __restrict__ h_out, float* __restrict__ c_out,
                                                              unsigned short* __restrict__ hseq) {
  __shared__ __attribute__((aligned(16))) unsigned short hbuf[64 * (H + 8)];
  XaSource xs;
  xs.setup(xa, (int64_t)blockIdx.x * 64, B, L, lane_id() & 31, lane_id() >> 5);
  lstm_pipe_body<H, HSEQ>(xs, B, L, Wpack, h0, c0, h_out, c_out, hseq, hbuf);
}

// The univariate forecaster straight from the history: sequence b is row
// rm[b] (or b) of hist [., ld], dense columns [T - L, T) read at grid column
// c - (shift[b] - dk) below lim[b] + dk (shift / lim null: the row as is, T
// columns).  The workgroup's 64 sequences are z-scored in a prologue (mu /
// sd also written out for the forecast's de-normalisation).
template <int H>
__global__ __launch_bounds__(H * 4) void lstm_fwd_hist_kernel(const float* __restrict__ hist, int64_t ld, int T,
                                                              const int* __restrict__ rm,
                                                              const int* __restrict__ shift,
                                                              const int* __restrict__ lim, int dk, int64_t B, int L,
                                                              float period, int I, const uint4* __restrict__ Wpack,
                                                              float* __restrict__ h_out, float* __restrict__ c_out,
                                                              float* __restrict__ mu_out, float* __restrict__ sd_out) {
  __shared__ __attribute__((aligned(16))) unsigned short hbuf[64 * (H + 8)];
  __shared__ float smu[64], sinv[64];
  __shared__ float2 stab[kLstmPhaseTab];
  const int lane = lane_id(), w = wave_id();
  constexpr int NW = H / 16;
  const int64_t b0 = (int64_t)blockIdx.x * 64;
  // prologue: the window statistics of this workgroup's sequences
  for (int q = w; q < 64; q += NW) {
    const int64_t bb = b0 + q;
    float mu = 0.f, sd = 1e-6f;
    if (bb < B) {
      const int64_t r = rm != nullptr ? rm[bb] : bb;
      const int off = shift != nullptr ? dk - shift[bb] : 0;
      const int lm = lim != nullptr ? lim[bb] + dk : T;
      const float* hr = hist + r * ld;
      float s = 0.f;
      int n = 0;
      for (int i = lane; i < L; i += 64) {
        const int bc = T - L + i + off;
        const float v = (bc >= 0 && bc < lm) ? hr[bc] : __builtin_nanf("");
        if (isfinite(v)) { s += v; ++n; }
      }
      s = wave_sum(s);
      n = wave_sum(n);
      mu = s / (float)(n > 0 ? n : 1);
      float qq = 0.f;
      for (int i = lane; i < L; i += 64) {
        const int bc = T - L + i + off;
        const float v = (bc >= 0 && bc < lm) ? hr[bc] : __builtin_nanf("");
        if (isfinite(v)) { const float d = v - mu; qq += d * d; }
      }
      qq = wave_sum(qq);
      sd = sqrtf(qq / (float)(n > 0 ? n : 1));
      sd = sd > 1e-6f ? sd : 1e-6f;
      if (lane == 0) { mu_out[bb] = mu; sd_out[bb] = sd; }
    }
    if (lane == 0) { smu[q] = mu; sinv[q] = 1.f / sd; }
  }
  __syncthreads();
  HistSource xs;
  const int col = lane & 31;
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    int64_t bb = b0 + 32 * ct + col;
    bb = bb < B ? bb : B - 1;
    const int64_t r = rm != nullptr ? rm[bb] : bb;
    xs.row[ct] = hist + r * ld;
    xs.off[ct] = shift != nullptr ? dk - shift[bb] : 0;
    xs.lim[ct] = lim != nullptr ? lim[bb] + dk : T;
    xs.mu[ct] = smu[32 * ct + col];
    xs.inv[ct] = sinv[32 * ct + col];
  }
  xs.c0 = T - L;
  xs.p = period;
  xs.ip = 1.f / period;
  xs.I = I;
  xs.lo_half = (lane >> 5) == 0;
  xs.tab = nullptr;
  if (L <= kLstmPhaseTab) {
    for (int t = threadIdx.x; t < L; t += H * 4) stab[t] = xs.phase_entry(t);
    __syncthreads();
    xs.tab = stab;
  }
  lstm_pipe_body<H, false>(xs, B, L, Wpack, nullptr, nullptr, h_out, c_out, nullptr, hbuf);
}

FM_API int fm_lstm_forward_hist(const float* hist, int64_t ld, int T, const int* rm, const int* shift, const int* lim,
                                int dk, int64_t B, int L, int H, float period, int I, const void* Wpack, float* h_out,
                                float* c_out, float* mu, float* sd, hipStream_t stream) {
  if (B <= 0) return 0;
  if (L <= 0 || L > T || I < 0 || I > 3 || !(period > 0.f) || (shift == nullptr) != (lim == nullptr))
    return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((B + 63) / 64));
#define FM_LSTMH(HH)                                                                                             \
  hipLaunchKernelGGL(lstm_fwd_hist_kernel<HH>, grid, dim3(HH * 4), 0, stream, hist, ld, T, rm, shift, lim, dk, B, L, \
                     period, I, (const uint4*)Wpack, h_out, c_out, mu, sd)
  if (H == 128) FM_LSTMH(128);
  else if (H == 64) FM_LSTMH(64);
  else if (H == 32) FM_LSTMH(32);
  else return (int)hipErrorInvalidValue;
#undef FM_LSTMH
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Forecaster features straight from the packed history: per row the last L
// samples are z-scored (finite mean / population std, missing -> 0) and laid
// out as the kernel's augmented input [z, sin(2 pi t/P), cos(2 pi t/P)][:I],
// 1.0 at k = I, zeros above, in bf16.  One wave per row.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void lstm_features_kernel(const float* __restrict__ hist, int64_t ld, int T,
                                                            int64_t R, int L, float period, int I,
                                                            uint4* __restrict__ xa, float* __restrict__ mu_out,
                                                            float* __restrict__ sd_out) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R) return;
  const int lane = lane_id();
  const float* hr = hist + row * ld + (T - L);
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
  const float w0 = 6.283185307179586f / period;
  for (int i = lane; i < L; i += 64) {
    const float v = hr[i];
    const float z = isfinite(v) ? (v - mu) * inv : 0.f;
    const float ph = w0 * (float)(T - L + i);
    float f[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) f[k] = 0.f;
    if (I > 0) f[0] = z;
    if (I > 1) f[1] = sinf(ph);
    if (I > 2) f[2] = cosf(ph);
    f[I < 15 ? I : 15] = 1.f;
    uint4 lo, hi;
    lo.x = pack_bf2(f[0], f[1]); lo.y = pack_bf2(f[2], f[3]); lo.z = pack_bf2(f[4], f[5]); lo.w = pack_bf2(f[6], f[7]);
    hi.x = pack_bf2(f[8], f[9]); hi.y = pack_bf2(f[10], f[11]); hi.z = pack_bf2(f[12], f[13]);
    hi.w = pack_bf2(f[14], f[15]);
    xa[(row * L + i) * 2 + 0] = lo;
    xa[(row * L + i) * 2 + 1] = hi;
  }
  if (lane == 0) { mu_out[row] = mu; sd_out[row] = sd; }
}

FM_API int fm_lstm_features(const float* hist, int64_t ld, int T, int64_t R, int L, float period, int I, void* xa,
                            float* mu, float* sd, hipStream_t stream) {
  if (R <= 0) return 0;
  if (L <= 0 || L > T || I < 0 || I > 3) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(lstm_features_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, hist, ld, T, R, L,
                     period, I, (uint4*)xa, mu, sd);
  FM_LAUNCH_CHECK();
  return 0;
}

// nct: batch column tiles per workgroup (1 or 2); 0 = tuned default.
// cell: 0 = separate sigm/tanh (10 transcendentals per unit-step), 1 = the
// fm_lstm_cell.h cell, 2 = that cell in the column-tile pipelined kernel
// (nct ignored); -1 = default.
FM_API int fm_lstm_forward_v(const void* xa, int64_t B, int L, int H, const void* Wpack, const float* h0,
                             const float* c0, float* h_out, float* c_out, unsigned short* hseq, int nct, int cell,
                             hipStream_t stream) {
  if (B <= 0 || L <= 0) return 0;
  const uint4* x = (const uint4*)xa;
  // Default 64 columns (2 tiles).  For H=128 one tile gives 162 VGPRs and 3
  // waves/SIMD instead of 2 but measured 1.5 % slower (tools/lstm_ab.py:
  // 3.66 vs 3.61 ms at 80k x 240).
  if (nct == 0) nct = 2;
  if (cell < 0) cell = 2;   // tools/lstm_ab.py: 3.21-3.29 ms vs 3.34-3.36 (cell 1) at 80k x 240 x H128
  if (cell == 2) {   // column-tile pipelined kernel (2 tiles, fused cell)
    const dim3 grid((unsigned)((B + 63) / 64));
#define FM_LSTMP(HH)                                                                                              \
    do {                                                                                                         \
      if (hseq != nullptr)                                                                                       \
        hipLaunchKernelGGL((lstm_fwd_pipe_kernel<HH, true>), grid, dim3(HH * 4), 0, stream, x, B, L,            \
                           (const uint4*)Wpack, h0, c0, h_out, c_out, hseq);                                     \
      else                                                                                                       \
        hipLaunchKernelGGL((lstm_fwd_pipe_kernel<HH, false>), grid, dim3(HH * 4), 0, stream, x, B, L,           \
                           (const uint4*)Wpack, h0, c0, h_out, c_out, hseq);                                     \
    } while (0)
    if (H == 128) FM_LSTMP(128);
    else if (H == 64) FM_LSTMP(64);
    else if (H == 32) FM_LSTMP(32);
    else return (int)hipErrorInvalidValue;
#undef FM_LSTMP
    FM_LAUNCH_CHECK();
    return 0;
  }
#define FM_LSTM(HH, NC, CC)                                                                                     \
  hipLaunchKernelGGL((lstm_fwd_kernel<HH, NC, CC>), dim3((unsigned)((B + 32 * NC - 1) / (32 * NC))),           \
                     dim3(HH * 4), 0, stream, x, B, L, (const uint4*)Wpack, h0, c0, h_out, c_out, hseq)
#define FM_LSTM_C(HH, NC) do { if (cell == 1) FM_LSTM(HH, NC, 1); else FM_LSTM(HH, NC, 0); } while (0)
  if (H == 128) { if (nct == 1) FM_LSTM_C(128, 1); else FM_LSTM_C(128, 2); }
  else if (H == 64) { if (nct == 1) FM_LSTM_C(64, 1); else FM_LSTM_C(64, 2); }
  else if (H == 32) { if (nct == 1) FM_LSTM_C(32, 1); else FM_LSTM_C(32, 2); }
  else return (int)hipErrorInvalidValue;
#undef FM_LSTM_C
#undef FM_LSTM
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_lstm_forward_nct(const void* xa, int64_t B, int L, int H, const void* Wpack, const float* h0,
                               const float* c0, float* h_out, float* c_out, unsigned short* hseq, int nct,
                               hipStream_t stream) {
  return fm_lstm_forward_v(xa, B, L, H, Wpack, h0, c0, h_out, c_out, hseq, nct, -1, stream);
}

FM_API int fm_lstm_forward(const void* xa, int64_t B, int L, int H, const void* Wpack, const float* h0,
                           const float* c0, float* h_out, float* c_out, unsigned short* hseq, hipStream_t stream) {
  return fm_lstm_forward_nct(xa, B, L, H, Wpack, h0, c0, h_out, c_out, hseq, 0, stream);
}

// ---------------------------------------------------------------------------
// The forecaster's linear head and de-normalisation in one pass:
//   fc[b, j] = mu[b] + sd[b] * (h[b, :] . W[min(j, Hz - 1), :] + bias[min(j, Hz - 1)])
// for j < Hout (a horizon past the head's Hz repeats its last step, as
// LSTMForecaster._head).  One thread per sequence, W and bias in LDS (Hz x H
// <= 64 x 256 floats); replaces mm + add + cat + mul + add.
// ---------------------------------------------------------------------------
template <int H, int NZ>
__global__ __launch_bounds__(256) void lstm_head_kernel(const float* __restrict__ h, int64_t B,
                                                        const float* __restrict__ W, const float* __restrict__ bias,
                                                        int Hz, const float* __restrict__ mu,
                                                        const float* __restrict__ sd, int Hout,
                                                        float* __restrict__ fc) {
  // one thread per sequence; W / bias in LDS (every lane reads the same
  // word: a broadcast); NZ >= Hz is the compile-time bound of the head's
  // outputs, so the accumulators stay in registers and the horizon padding
  // (Hout > Hz repeats the last output) needs no runtime register indexing
  extern __shared__ float sw[];            // [Hz][H] then bias [Hz]
  for (int i = threadIdx.x; i < Hz * H; i += blockDim.x) sw[i] = W[i];
  for (int i = threadIdx.x; i < Hz; i += blockDim.x) sw[Hz * H + i] = bias[i];
  __syncthreads();
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float4* hr = reinterpret_cast<const float4*>(h + b * H);
  float acc[NZ];
#pragma unroll
  for (int j = 0; j < NZ; ++j) acc[j] = 0.f;
#pragma unroll 4
  for (int k4 = 0; k4 < H / 4; ++k4) {
    const float4 x = hr[k4];
#pragma unroll
    for (int j = 0; j < NZ; ++j) {
      if (j < Hz) {
        const float4 w = *reinterpret_cast<const float4*>(sw + j * H + 4 * k4);
        acc[j] = __builtin_fmaf(x.x, w.x, __builtin_fmaf(x.y, w.y, __builtin_fmaf(x.z, w.z, __builtin_fmaf(x.w, w.w, acc[j]))));
      }
    }
  }
  const float m = mu[b], s = sd[b];
  float last = 0.f;
#pragma unroll
  for (int j = 0; j < NZ; ++j)
    if (j < Hz) acc[j] = __builtin_fmaf(s, acc[j] + sw[Hz * H + j], m), last = acc[j];
  float* out = fc + b * Hout;
#pragma unroll
  for (int j = 0; j < NZ; ++j)
    if (j < Hout) out[j] = j < Hz ? acc[j] : last;
  for (int j = NZ; j < Hout; ++j) out[j] = last;
}

FM_API int fm_lstm_head(const float* h, int64_t B, int H, const float* W, const float* bias, int Hz, const float* mu,
                        const float* sd, int Hout, float* fc, hipStream_t stream) {
  if (B <= 0) return 0;
  if (Hz < 1 || Hz > 64 || Hout < 1) return (int)hipErrorInvalidValue;
  const dim3 grid((unsigned)((B + 255) / 256));
  const size_t lds = (size_t)(Hz * H + Hz) * sizeof(float);
#define FM_HEAD(HH)                                                                                              \
  do {                                                                                                         \
    if (Hz <= 16)                                                                                              \
      hipLaunchKernelGGL((lstm_head_kernel<HH, 16>), grid, dim3(256), lds, stream, h, B, W, bias, Hz, mu, sd, Hout, fc); \
    else                                                                                                       \
      hipLaunchKernelGGL((lstm_head_kernel<HH, 64>), grid, dim3(256), lds, stream, h, B, W, bias, Hz, mu, sd, Hout, fc); \
  } while (0)
  if (H == 128) FM_HEAD(128);
  else if (H == 64) FM_HEAD(64);
  else if (H == 32) FM_HEAD(32);
  else if (H == 256) FM_HEAD(256);
  else return (int)hipErrorInvalidValue;
#undef FM_HEAD
  FM_LAUNCH_CHECK();
  return 0;
}
