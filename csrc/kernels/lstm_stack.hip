// fm-hipcc-flags: -fno-slp-vectorize
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
#include "fm_lstm_cell.h"

#include <type_traits>

using namespace fm;

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

namespace {

__device__ __forceinline__ unsigned pack_bf2(float lo, float hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(unsigned, v);
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  const __bf16 b = (__bf16)f;
  return __builtin_bit_cast(unsigned short, b);
}
// the cell update: fm_lstm_cell.h (pre-scaled gates, scaled c)
__device__ __forceinline__ void cell(float ai, float af, float ag, float ao, float& cs, float& h) {
  lstm_cell(ai, af, ag, ao, cs, h);
}

union Frag {
  bf16x8 v;
  uint4 u;
};
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

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
  uint4 onesv[NCT];                                   // layer-1 bias step: B = [1, 0, ..., 0]
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) onesv[ct] = make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);

  // gates[rt][ct] = sum_ks A[rt][ks] B[ks][ct].  B of k-step ks < KH is h
  // image ``lo``, ks >= KH image ``hi`` (at ks - KH), except the last step
  // whose B is the register ``breg`` (x_t / ones).  The LDS read is
  // unconditional (clamped address) and the register picked by VALUE: a
  // select between an LDS and a register address makes the compiler emit a
  // flat load, whose vmcnt(0) wait also drains the weight lookahead.
  auto gemm = [&](const uint4* Ww, int KS, const uint4 (&breg)[NCT], const unsigned short* lo,
                  const unsigned short* hi, f32x16 (&acc)[RT][NCT]) {
    Frag a[RT], an[RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[rt].u = Ww[(rt * KS + 0) * 64];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = (f32x16){};
    // not unrolled: unrolling lets the scheduler hoist every k-step's A
    // fragments (33 x RT x 16 B per lane at H = 256) and spill; one k-step of
    // lookahead is what the L2 latency needs with 2 waves per SIMD
#pragma unroll 1
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) an[rt].u = Ww[(rt * KS + ks + 1) * 64];
      }
      const int kc = ks < KH ? ks : ks - KH < KH ? ks - KH : KH - 1;
      const unsigned short* src = (ks < KH ? lo : hi) + 16 * kc + 8 * hf;
      Frag bf[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        const uint4 v = *reinterpret_cast<const uint4*>(&src[(32 * ct + col) * HP]);
        bf[ct].u = ks == KS - 1 ? breg[ct] : v;
      }
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
              make_float4(c[rt][ct][0] * kLstmInvK, c[rt][ct][1] * kLstmInvK, c[rt][ct][2] * kLstmInvK,
                          c[rt][ct][3] * kLstmInvK);
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
    gemm(W0w, KS0, xt, h0p, h0p, acc);
    update(acc, c0, h0b + cur * BT * HP, last && LAYERS == 1);
    __syncthreads();
    if (LAYERS == 2) {
      const unsigned short* h1p = h1b + prv * BT * HP;
      const unsigned short* h0c = h0b + cur * BT * HP;
      gemm(W1w, KS1, onesv, h1p, h0c, acc);
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

// ---------------------------------------------------------------------------
// Two layers, software-pipelined across the layer boundary so that the cell
// updates (VALU: the fm_lstm_cell.h update) issue beside MFMAs instead of
// between barriers.  Layer 0 at step t+1 needs only h0_t, and layer 1's
// k-steps over h1_t do not need h0_{t+1}, so one step is two barrier-separated
// phases:
//
//   A: L1(t)   k-steps over [h0_t; 1]      -> accB  (MFMA only)
//      L0(t+1) k-steps over [x_{t+1}; h0_t] -> accA  ||  cell L1(t)   -> h1_t
//   B: L1(t+1) k-steps over h1_t           -> accB  ||  cell L0(t+1) -> h0_{t+1}
//
// Two barriers per step instead of four, single-buffered h images, one cell
// (4 gate values of one unit per lane) per k-step, interleaved with that
// k-step's MFMAs -- the k-loops are unrolled so every cell's accumulator
// registers are static.  BT = 32 sequences (one column tile); the A fragments
// stay one k-step ahead across phase boundaries, and the barriers wait only
// for LDS (workgroup fence on the local address space), so those loads stay
// in flight across them.
namespace {
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
template <int N>
using ic = std::integral_constant<int, N>;
// f(ic<0>{}), ..., f(ic<N-1>{}): a compile-time unrolled loop of any length
// (#pragma unroll gives up on long bodies and falls back to a rolled loop
// with dynamically indexed -- scratch -- register arrays)
template <class F, int... I>
__device__ __forceinline__ void static_for_(F&& f, std::integer_sequence<int, I...>) {
  (f(ic<I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_(f, std::make_integer_sequence<int, N>{});
}
}  // namespace

// ABL (measurement only, 0 in production): bit 0 replaces the cell math by a
// copy, bit 1 reads every A fragment from one k-step's address (L2-hot), bit
// 2 keeps the A fragments one k-step ahead instead of two
template <int H, int RT, int ABL = 0>
__global__ __launch_bounds__(64 * H / (8 * RT)) void lstm_stack2_pipe_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out, float* __restrict__ c_out) {
  constexpr int NW = H / (8 * RT);
  constexpr int KH = H / 16;
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 32;
  constexpr int NC = 4 * RT;                           // cells per lane per layer-step
  static_assert(NC <= KH, "one cell per k-step of the h1 phase");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                           // [BT][HP] h0 (single-buffered)
  unsigned short* h1b = lds + BT * HP;                 // [BT][HP] h1
  const int lane = lane_id(), w = wave_id();
  const int hf = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  for (int i = threadIdx.x; i < 2 * BT * HP; i += 64 * NW) lds[i] = 0;   // h_{-1} = 0
  float c0[RT][4], c1[RT][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int j = 0; j < 4; ++j) c0[rt][j] = c1[rt][j] = 0.f;
  __syncthreads();

  int64_t bb = b0 + col;
  const bool inb = bb < B;
  bb = inb ? bb : B - 1;
  const uint4* xp = xa + (bb * L) * 2 + hf;
  // weights through buffer loads: a wave-uniform resource (SGPRs), the lane's
  // 16 B as the VGPR offset and the k-step as a scalar offset -- no per-load
  // 64-bit VGPR address (with 268 loads in the unrolled step those addresses
  // are what the compiler hoists and spills)
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t W0w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W0 + (int64_t)wu * RT * KS0 * 64), (short)0, RT * KS0 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t W1w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W1 + (int64_t)wu * RT * KS1 * 64), (short)0, RT * KS1 * 1024, 0x00020000);
  const int voff = 16 * lane;
  const uint4 onesv = make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);
  const unsigned short* h0r = h0b + col * HP + 8 * hf;     // this lane's B-fragment row
  const unsigned short* h1r = h1b + col * HP + 8 * hf;
  unsigned short* h0w = h0b + col * HP;
  unsigned short* h1w = h1b + col * HP;
  auto lds16 = [](const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); };

  Frag a[RT], an[RT];                                  // A fragments of the current / next k-step
  auto loadA = [&](Frag (&f)[RT], __amdgpu_buffer_rsrc_t Ww, int KS, int ks) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(Ww, voff, (ABL & 2) ? rt * 1024 : (rt * KS + ks) * 1024,
                                                            0);
      f[rt].u = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // NK unrolled k-steps: A of step i from (Ww, KS, ks_of(i)), B = b_of(i),
  // then cell_at(i); the A fragments of (Wn, KSn, ksn) are prefetched during
  // the last step (the first k-step of whatever follows)
  auto segment = [&](auto NK, f32x16 (&acc)[RT], __amdgpu_buffer_rsrc_t Ww, int KS, auto ks_of, auto b_of,
                     __amdgpu_buffer_rsrc_t Wn, int KSn, int kn0, int kn1, auto cell_at) {
    // A fragments run two k-steps ahead (a: this step, an: the next; on
    // entry both were issued by whatever ran before), across segments: the
    // last two steps prefetch the next segment's (Wn, KSn) k-steps kn0, kn1.
    // The B fragment (h image in LDS, stable for the whole segment) is read
    // one k-step ahead.
    constexpr int N = decltype(NK)::value;
    uint4 bcur = b_of(0);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      __builtin_amdgcn_sched_barrier(0);             // k-steps stay in order: no hoisted loads
      Frag ann[RT];
      if (ABL & 4) {                                 // one k-step ahead only
        if (i + 1 < N) loadA(an, Ww, KS, ks_of(i + 1));
        else loadA(an, Wn, KSn, kn0);
      } else if (i + 2 < N) {
        loadA(ann, Ww, KS, ks_of(i + 2));
      } else {
        loadA(ann, Wn, KSn, i + 2 == N ? kn0 : kn1);
      }
      const uint4 bnext = i + 1 < N ? b_of(i + 1) : bcur;
      Frag bf;
      bf.u = bcur;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt].v, bf.v, acc[rt], 0, 0, 0);
      cell_at(i);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        a[rt] = an[rt];
        if (!(ABL & 4)) an[rt] = ann[rt];
      }
      bcur = bnext;
    }
  };
  auto zero = [](f32x16 (&acc)[RT]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = (f32x16){};
  };
  // cell q (row tile q / 4, unit q % 4 of the lane's 4) of a finished layer
  // accumulator; the tile's 4 h values go to LDS with its last cell
  float hv[4];
  auto cell_q = [&](int q, const f32x16 (&acc)[RT], float (&c)[RT][4], unsigned short* hw, bool out) {
    const int rt = q >> 2, j = q & 3;
    if (ABL & 1) {
      hv[j] = acc[rt][j] * 1e-3f;
      c[rt][j] = acc[rt][4 + j];
    } else {
      cell(acc[rt][j], acc[rt][4 + j], acc[rt][8 + j], acc[rt][12 + j], c[rt][j], hv[j]);
    }
    if (j == 3) {
      const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
      uint2 pk;
      pk.x = pack_bf2(hv[0], hv[1]);
      pk.y = pack_bf2(hv[2], hv[3]);
      *reinterpret_cast<uint2*>(&hw[u0]) = pk;
      if (out && inb) {
        *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        *reinterpret_cast<float4*>(&c_out[bb * H + u0]) =
            make_float4(c[rt][0] * kLstmInvK, c[rt][1] * kLstmInvK, c[rt][2] * kLstmInvK, c[rt][3] * kLstmInvK);
      }
    }
  };
  const auto ks_l0 = [](int i) { return i == 0 ? KH : i - 1; };        // layer 0: x/bias step first
  const auto ks_l1b = [](int i) { return KH + i; };                    // layer 1 over [h0; 1]
  const auto ks_l1a = [](int i) { return i; };                         // layer 1 over h1
  const auto no_cell = [](int) {};

  f32x16 accA[RT], accB[RT];
  uint4 xt = xp[0];
  // prologue: L0(0) (h0_{-1} = 0), its cells, barrier; L1(0)'s k-steps over
  // h1_{-1} = 0 contribute nothing: accB starts at zero
  loadA(a, W0w, KS0, KH);
  if (!(ABL & 4)) loadA(an, W0w, KS0, 0);
  zero(accA);
  segment(ic<KS0>{}, accA, W0w, KS0, ks_l0,
          [&](int i) { const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1)); return i == 0 ? xt : v; },
          W1w, KS1, KH, KH + 1, no_cell);
#pragma unroll
  for (int q = 0; q < NC; ++q) cell_q(q, accA, c0, h0w, false);
  lds_barrier();
  zero(accB);
  const auto b_l1b = [&](int i) { const uint4 v = lds16(h0r + 16 * (i < KH ? i : KH - 1)); return i == KH ? onesv : v; };
  for (int t = 0; t < L - 1; ++t) {
    xt = xp[(t + 1) * 2];
    // phase A: L1(t) over [h0_t; 1]
    segment(ic<KH + 1>{}, accB, W1w, KS1, ks_l1b, b_l1b, W0w, KS0, KH, 0, no_cell);
    //          L0(t+1) over [x_{t+1}; h0_t]  ||  cells of L1(t)
    zero(accA);
    segment(ic<KS0>{}, accA, W0w, KS0, ks_l0,
            [&](int i) { const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1)); return i == 0 ? xt : v; },
            W1w, KS1, 0, 1, [&](int i) { if (i < NC) cell_q(i, accB, c1, h1w, false); });
    lds_barrier();                                   // h1_t complete; every read of h0_t done
    // phase B: L1(t+1) over h1_t  ||  cells of L0(t+1)
    zero(accB);
    segment(ic<KH>{}, accB, W1w, KS1, ks_l1a, [&](int i) { return lds16(h1r + 16 * i); },
            W1w, KS1, KH, KH + 1, [&](int i) { if (i < NC) cell_q(i, accA, c0, h0w, false); });
    lds_barrier();                                   // h0_{t+1} complete; every read of h1_t done
  }
  // the last step's layer 1 (out of the loop: its output addresses are not
  // live across the time loop)
  segment(ic<KH + 1>{}, accB, W1w, KS1, ks_l1b, b_l1b, W1w, KS1, 0, 1, no_cell);
#pragma unroll
  for (int q = 0; q < NC; ++q) cell_q(q, accB, c1, h1w, true);
}

template <int H, int RT, int ABL = 0>
static int launch_stack2_pipe(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                              float* c_out, hipStream_t stream) {
  constexpr int NW = H / (8 * RT);
  const size_t lds = (size_t)2 * 32 * (H + 8) * sizeof(unsigned short);
  auto k = lstm_stack2_pipe_kernel<H, RT, ABL>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + 31) / 32)), dim3(64 * NW), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Two layers, row-tile streamed, BT = 64 sequences per workgroup.  The
// pipelined kernel above is bound by the weight stream: every workgroup
// pulls all 1.6 MB of [W0 | W1] through its CU's vector-memory path each step
// for only 32 sequences (profiles/lstm_pipe_ablation_r3.jsonl: L1-resident
// weights 4.7 ms vs 6.7), and 64 sequences x both layers' accumulators do not
// fit in registers.  Here a wave works through its row tiles one at a time
// ("tasks": one row tile of one layer, both column tiles), so only two tiles'
// accumulators are live -- the one accumulating and the one whose cells are
// being updated beside its MFMAs -- and each weight fragment feeds 64
// sequences, halving weight bytes per sequence.
//
// Iteration s runs layer 0 at step s and layer 1 at step s - 1 (both read
// only outputs of iteration s - 1), as 8 tasks: L0 rt0..3, L1 rt0..3.  The
// cells of task T run during task T + 1 (those of L1 rt3 in the next
// iteration's L0 rt0).  h images are double-buffered per layer; two barriers
// per iteration: before L0 rt0 (h0_{s-1} complete) and before L1 rt0
// (h1_{s-2} complete: its last cells ran in L0 rt0).  Iteration 0 has no
// layer-1 cells, iteration L no layer-0 input (x clamped, outputs unused);
// the final L1 rt3 cells (h_out / c_out) run after the loop.
template <int H>
__global__ __launch_bounds__(512) void lstm_stack2_rs_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out, float* __restrict__ c_out) {
  constexpr int RT = 4;
  constexpr int NW = H / (8 * RT);
  static_assert(NW == 8, "8 waves");
  constexpr int KH = H / 16;
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 64;
  constexpr int IMG = BT * HP;
  constexpr int G0 = RT * KS0;                          // k-steps of the layer-0 tasks
  constexpr int G = G0 + RT * KS1;                      // k-steps per iteration
  constexpr int DA = 3;                                 // A fragments DA k-steps ahead
  static_assert(G % (DA + 1) == 0, "A ring wraps at the iteration boundary");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                            // [2][BT][HP]
  unsigned short* h1b = lds + 2 * IMG;                  // [2][BT][HP]
  const int lane = lane_id(), w = wave_id();
  const int hf = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  for (int i = threadIdx.x; i < 4 * IMG; i += 64 * NW) lds[i] = 0;   // h_{-1} = 0
  float c0[RT][2][4], c1[RT][2][4];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
      for (int j = 0; j < 4; ++j) c0[rt][ct][j] = c1[rt][ct][j] = 0.f;
  __syncthreads();

  const uint4* xp[2];
  bool inb[2];
  int64_t bbo[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) {
    int64_t bb = b0 + 32 * ct + col;
    inb[ct] = bb < B;
    bb = bb < B ? bb : B - 1;
    bbo[ct] = bb;
    xp[ct] = xa + (bb * L) * 2 + hf;
  }
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t W0w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W0 + (int64_t)wu * RT * KS0 * 64), (short)0, RT * KS0 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t W1w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W1 + (int64_t)wu * RT * KS1 * 64), (short)0, RT * KS1 * 1024, 0x00020000);
  const int voff = 16 * lane;
  const uint4 onesv = make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);
  const int lro = col * HP + 8 * hf;                    // this lane's B-fragment row (column tile 0)
  auto lds16 = [](const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); };

  // k-step g of an iteration -> (layer, row tile, k index within the task)
  auto lay = [](int g) { return g >= G0 ? 1 : 0; };
  auto tsk = [](int g) { return g < G0 ? g / KS0 : RT + (g - G0) / KS1; };
  auto kin = [](int g) { return g < G0 ? g % KS0 : (g - G0) % KS1; };
  auto loadA = [&](Frag& f, int g) {
    const int rt = tsk(g) & (RT - 1), i = kin(g);
    const u32x4 v = lay(g) ? __builtin_amdgcn_raw_buffer_load_b128(W1w, voff, (rt * KS1 + i) * 1024, 0)
                           : __builtin_amdgcn_raw_buffer_load_b128(W0w, voff, (rt * KS0 + (i == 0 ? KH : i - 1)) * 1024, 0);
    f.u = make_uint4(v.x, v.y, v.z, v.w);
  };

  f32x16 acc[2][2];                                     // [task parity][column tile]
  Frag ar[DA + 1];
  float hv[4];
  // cell q (column tile q / 4, unit q % 4) of the finished task T's
  // accumulator; the tile's 4 h values go to image ``img`` with its last cell
  auto cell_q = [&](int T, int q, unsigned short* img, bool out) {
    const int rt = T & (RT - 1), ct = q >> 2, j = q & 3;
    const f32x16& a = acc[T & 1][ct];
    if (T >= RT) cell(a[j], a[4 + j], a[8 + j], a[12 + j], c1[rt][ct][j], hv[j]);
    else cell(a[j], a[4 + j], a[8 + j], a[12 + j], c0[rt][ct][j], hv[j]);
    if (j == 3) {
      const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
      uint2 pk;
      pk.x = pack_bf2(hv[0], hv[1]);
      pk.y = pack_bf2(hv[2], hv[3]);
      *reinterpret_cast<uint2*>(&img[(32 * ct + col) * HP + u0]) = pk;
      if (out && inb[ct]) {
        const float(&c)[RT][2][4] = c1;
        *reinterpret_cast<float4*>(&h_out[bbo[ct] * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        *reinterpret_cast<float4*>(&c_out[bbo[ct] * H + u0]) =
            make_float4(c[rt][ct][0] * kLstmInvK, c[rt][ct][1] * kLstmInvK, c[rt][ct][2] * kLstmInvK,
                        c[rt][ct][3] * kLstmInvK);
      }
    }
  };

#pragma unroll
  for (int g = 0; g < DA; ++g) loadA(ar[g], g);
  uint4 xn[2];
#pragma unroll
  for (int ct = 0; ct < 2; ++ct) xn[ct] = xp[ct][0];

  for (int s = 0; s <= L; ++s) {
    const int p = s & 1;
    const unsigned short* h0r = h0b + (p ^ 1) * IMG + lro;   // h0_{s-1}
    const unsigned short* h1r = h1b + p * IMG + lro;         // h1_{s-2}
    unsigned short* h0w = h0b + p * IMG;                     // h0_s
    unsigned short* h1w_old = h1b + p * IMG;                 // h1_{s-2} (L1 rt3 cells of iteration s - 1)
    unsigned short* h1w = h1b + (p ^ 1) * IMG;               // h1_{s-1}
    const bool l1prev = s >= 2, l1cur = s >= 1, fin = s == L;
    uint4 xt[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      xt[ct] = xn[ct];
      xn[ct] = xp[ct][(s + 1 < L ? s + 1 : L - 1) * 2];
    }
    // B of k-step g, column tile ct (by value: see gemm above)
    auto bread = [&](int g, int ct) {
      const int i = kin(g);
      if (lay(g) == 0) {
        const uint4 v = lds16(h0r + 32 * ct * HP + 16 * (i == 0 ? 0 : i - 1));
        return i == 0 ? xt[ct] : v;
      }
      if (i < KH) return lds16(h1r + 32 * ct * HP + 16 * i);
      const uint4 v = lds16(h0r + 32 * ct * HP + 16 * (i < 2 * KH ? i - KH : KH - 1));
      return i == 2 * KH ? onesv : v;
    };
    uint4 bcur[2] = {xt[0], xt[1]};
    static_for<G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (g == 0 || g == G0) lds_barrier();
      loadA(ar[(g + DA) % (DA + 1)], (g + DA) % G);
      if constexpr (g == G0) {                                 // not prefetched across the barrier
        bcur[0] = bread(g, 0);
        bcur[1] = bread(g, 1);
      }
      uint4 bnext[2] = {bcur[0], bcur[1]};
      if constexpr (g + 1 < G && g + 1 != G0) {
        bnext[0] = bread(g + 1, 0);
        bnext[1] = bread(g + 1, 1);
      }
      constexpr int T = g < G0 ? g / KS0 : RT + (g - G0) / KS1;
      constexpr int i = g < G0 ? g % KS0 : (g - G0) % KS1;
      const Frag& a = ar[g % (DA + 1)];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        Frag bf;
        bf.u = bcur[ct];
        acc[T & 1][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.v, bf.v, i == 0 ? (f32x16){} : acc[T & 1][ct],
                                                                 0, 0, 0);
      }
      // one cell of the previous task every 2 (layer-0 task) or 4 (layer-1
      // task) k-steps from the second k-step on
      constexpr int stride = g >= G0 ? 4 : 2;
      if constexpr (i >= 1 && (i - 1) % stride == 0 && (i - 1) / stride < 8) {
        constexpr int q = (i - 1) / stride, Tp = (T + 2 * RT - 1) % (2 * RT);
        if constexpr (T == 0) {
          if (l1prev) cell_q(Tp, q, h1w_old, false);
        } else if constexpr (Tp < RT) {
          cell_q(Tp, q, h0w, false);
        } else if (l1cur) {
          cell_q(Tp, q, h1w, fin);
        }
      }
      bcur[0] = bnext[0];
      bcur[1] = bnext[1];
    });
  }
  // L1(L-1) rt3: its cells would run in iteration L + 1
#pragma unroll
  for (int q = 0; q < 8; ++q) cell_q(2 * RT - 1, q, h1b + ((L + 1) & 1) * IMG, true);
}

template <int H>
static int launch_stack2_rs(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                            float* c_out, hipStream_t stream) {
  const size_t lds = (size_t)4 * 64 * (H + 8) * sizeof(unsigned short);
  auto k = lstm_stack2_rs_kernel<H>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + 63) / 64)), dim3(512), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
}

// Two layers at H = 256 on 16x16 tiles: v_mfma_f32_16x16x32_bf16, BT = 48
// sequences (three 16-column tiles) per workgroup.  The 32-column kernel
// above needs 64 sequences per workgroup to halve the weight stream, which
// leaves a 10k-service fleet at ceil(10000 / 64) = 157 workgroups: 99 of the
// 256 CUs idle for the whole recurrence.  With 16-column tiles the workgroup
// takes 48 sequences -> 209 workgroups (82 % of the CUs), 25 % less MFMA work
// per workgroup for the same weight bytes per step.
//
// Layout (cdna_hip_programming.md §3, 16x16x32): lane l holds A[row l & 15][k
// 8 (l >> 4) + j], B[k 8 (l >> 4) + j][col l & 15] and C rows 4 (l >> 4) .. +3
// of column l & 15.  A 16-row tile is 4 hidden units x [i f g o] (row 4u + gate),
// so a lane's four accumulators are one unit's gates of one sequence: the
// cell stays lane-local.  Wave w owns units 32 w .. 32 w + 31 as 8 row tiles per
// layer.  K order of the packed weights (ops/lstm.py pack_stack_t16) is the
// order the k-steps run: layer 0 [x_t, 1 | pad] then h0_{t-1} (9 k-steps of
// 32); layer 1 h1_{t-1}, h0_t, then [1 | pad] (17 k-steps).
//
// Schedule: lstm_stack2_rs_kernel's, with 16 tasks per iteration (L0 rt0..7 at
// step s, L1 rt0..7 at step s - 1), the three cells of task T beside the
// first k-steps of task T + 1, A fragments DA k-steps ahead, two barriers per
// iteration (before L0 rt0 and L1 rt0).
template <int H>
__global__ __launch_bounds__(512) void lstm_stack2_t16_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out, float* __restrict__ c_out) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  constexpr int NW = 8;
  constexpr int RT = H / (4 * NW);                      // 16-row tiles per wave per layer (8)
  constexpr int NCT = 3;
  constexpr int KH = H / 32;                            // 32-k steps over one hidden vector
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 16 * NCT;
  constexpr int IMG = BT * HP;
  constexpr int G0 = RT * KS0;                          // k-steps of the layer-0 tasks
  constexpr int G = G0 + RT * KS1;                      // k-steps per iteration
  constexpr int DA = 3;                                 // A fragments DA k-steps ahead
  static_assert(G % (DA + 1) == 0, "A ring wraps at the iteration boundary");
  static_assert(KS0 >= 2 * NCT && KS1 >= 4 * NCT - 3, "a task's cells fit beside the next task's k-steps");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                            // [2][BT][HP]
  unsigned short* h1b = lds + 2 * IMG;                  // [2][BT][HP]
  const int lane = lane_id(), w = wave_id();
  const int q4 = lane >> 4, col = lane & 15;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  for (int i = threadIdx.x; i < 4 * IMG; i += 64 * NW) lds[i] = 0;   // h_{-1} = 0
  float c0[RT][NCT], c1[RT][NCT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) c0[rt][ct] = c1[rt][ct] = 0.f;
  __syncthreads();

  const uint4* xp[NCT];
  bool inb[NCT];
  int64_t bbo[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) {
    int64_t bb = b0 + 16 * ct + col;
    inb[ct] = bb < B;
    bb = bb < B ? bb : B - 1;
    bbo[ct] = bb;
    xp[ct] = xa + (bb * L) * 2 + (q4 & 1);              // lanes q4 >= 2 hold the zero pad
  }
  const bool xlane = q4 < 2;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t W0w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W0 + (int64_t)wu * RT * KS0 * 64), (short)0, RT * KS0 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t W1w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W1 + (int64_t)wu * RT * KS1 * 64), (short)0, RT * KS1 * 1024, 0x00020000);
  const int voff = 16 * lane;
  const uint4 zero4 = make_uint4(0u, 0u, 0u, 0u);
  const uint4 onesv = make_uint4(q4 == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);
  const int lro = col * HP + 8 * q4;                    // this lane's B-fragment row (column tile 0)
  auto lds16 = [](const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); };

  auto lay = [](int g) { return g >= G0 ? 1 : 0; };
  auto tsk = [](int g) { return g < G0 ? g / KS0 : RT + (g - G0) / KS1; };
  auto kin = [](int g) { return g < G0 ? g % KS0 : (g - G0) % KS1; };
  auto loadA = [&](Frag& f, int g) {
    const int rt = tsk(g) & (RT - 1), i = kin(g);
    const u32x4 v = lay(g) ? __builtin_amdgcn_raw_buffer_load_b128(W1w, voff, (rt * KS1 + i) * 1024, 0)
                           : __builtin_amdgcn_raw_buffer_load_b128(W0w, voff, (rt * KS0 + i) * 1024, 0);
    f.u = make_uint4(v.x, v.y, v.z, v.w);
  };

  f32x4 acc[2][NCT];                                    // [task parity][column tile]
  Frag ar[DA + 1];
  // the cell of column tile ct of the finished task T: unit 32 w + 4 rt + q4 of
  // sequence 16 ct + col; its h goes to image ``img`` (bf16), and with ``out``
  // to h_out / c_out
  auto cell_q = [&](int T, int ct, unsigned short* img, bool out) {
    const int rt = T & (RT - 1);
    const f32x4& a = acc[T & 1][ct];
    float hv;
    if (T >= RT) cell(a[0], a[1], a[2], a[3], c1[rt][ct], hv);
    else cell(a[0], a[1], a[2], a[3], c0[rt][ct], hv);
    const int u = 4 * RT * w + 4 * rt + q4;
    img[(16 * ct + col) * HP + u] = f2bf(hv);
    if (out && inb[ct]) {
      h_out[bbo[ct] * H + u] = hv;
      c_out[bbo[ct] * H + u] = c1[rt][ct] * kLstmInvK;
    }
  };

#pragma unroll
  for (int g = 0; g < DA; ++g) loadA(ar[g], g);
  uint4 xn[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) xn[ct] = xlane ? xp[ct][0] : zero4;

  for (int s = 0; s <= L; ++s) {
    const int p = s & 1;
    const unsigned short* h0r = h0b + (p ^ 1) * IMG + lro;   // h0_{s-1}
    const unsigned short* h1r = h1b + p * IMG + lro;         // h1_{s-2}
    unsigned short* h0w = h0b + p * IMG;                     // h0_s
    unsigned short* h1w_old = h1b + p * IMG;                 // h1_{s-2} (L1 rt7 cells of iteration s - 1)
    unsigned short* h1w = h1b + (p ^ 1) * IMG;               // h1_{s-1}
    const bool l1prev = s >= 2, l1cur = s >= 1, fin = s == L;
    uint4 xt[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      xt[ct] = xn[ct];
      xn[ct] = xlane ? xp[ct][(s + 1 < L ? s + 1 : L - 1) * 2] : zero4;
    }
    // B of k-step g, column tile ct (by value: see gemm above)
    auto bread = [&](int g, int ct) {
      const int i = kin(g);
      if (lay(g) == 0) {
        const uint4 v = lds16(h0r + 16 * ct * HP + 32 * (i == 0 ? 0 : i - 1));
        return i == 0 ? xt[ct] : v;
      }
      if (i < KH) return lds16(h1r + 16 * ct * HP + 32 * i);
      const uint4 v = lds16(h0r + 16 * ct * HP + 32 * (i < 2 * KH ? i - KH : KH - 1));
      return i == 2 * KH ? onesv : v;
    };
    uint4 bcur[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) bcur[ct] = xt[ct];
    static_for<G>([&](auto gc) {
      constexpr int g = decltype(gc)::value;
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (g == 0 || g == G0) lds_barrier();
      loadA(ar[(g + DA) % (DA + 1)], (g + DA) % G);
      if constexpr (g == G0) {                                 // not prefetched across the barrier
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) bcur[ct] = bread(g, ct);
      }
      uint4 bnext[NCT];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) bnext[ct] = bcur[ct];
      if constexpr (g + 1 < G && g + 1 != G0) {
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) bnext[ct] = bread(g + 1, ct);
      }
      constexpr int T = g < G0 ? g / KS0 : RT + (g - G0) / KS1;
      constexpr int i = g < G0 ? g % KS0 : (g - G0) % KS1;
      const Frag& a = ar[g % (DA + 1)];
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        Frag bf;
        bf.u = bcur[ct];
        acc[T & 1][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, bf.v, i == 0 ? (f32x4){} : acc[T & 1][ct],
                                                                 0, 0, 0);
      }
      // one cell of the previous task every 2 (layer-0 task) or 4 (layer-1
      // task) k-steps from the second k-step on
      constexpr int stride = g >= G0 ? 4 : 2;
      if constexpr (i >= 1 && (i - 1) % stride == 0 && (i - 1) / stride < NCT) {
        constexpr int q = (i - 1) / stride, Tp = (T + 2 * RT - 1) % (2 * RT);
        if constexpr (T == 0) {
          if (l1prev) cell_q(Tp, q, h1w_old, false);
        } else if constexpr (Tp < RT) {
          cell_q(Tp, q, h0w, false);
        } else if (l1cur) {
          cell_q(Tp, q, h1w, fin);
        }
      }
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) bcur[ct] = bnext[ct];
    });
  }
  // L1(L-1) rt7: its cells would run in iteration L + 1
#pragma unroll
  for (int q = 0; q < NCT; ++q) cell_q(2 * RT - 1, q, h1b + ((L + 1) & 1) * IMG, true);
}

template <int H>
static int launch_stack2_t16(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                             float* c_out, hipStream_t stream) {
  const size_t lds = (size_t)4 * 48 * (H + 8) * sizeof(unsigned short);
  auto k = lstm_stack2_t16_kernel<H>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + 47) / 48)), dim3(512), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
}

// Row tiles per wave / column tiles per workgroup (see ops/lstm.py
// STACK_TILING / STACK_TILING_2L): two layers at H=256 run the row-streamed
// BT = 64 kernel (nct = 202, RT = 4: 10k x 240 in 4.6 ms, 80k in 29.6; the
// layer-pipelined nct = 201 kernel 6.8 / 35.9, the 4 x 2 register kernel 8.2 /
// 42.0, profiles/lstm_stack_rs_r3.jsonl); one layer at H=256: 4 x 2 (8 waves, 64
// sequences share every streamed weight fragment); H<=128: 2 x 2 (H/16
// waves, 64 sequences).  rt / nct = 0 pick 4 x 2 / 2 x 2; the other H = 256
// tilings (4 x 1, 2 x 2, 2 x 1, 2 x 1 pipelined) stay instantiated for the
// A/B (ops/lstm.py FM_LSTM_STACK_TILING) and need weights packed with the
// same RT.  Measured and removed: an LDS-DMA weight ring (LDS-bandwidth
// bound, 9.8 ms) and a flat-step pipelined kernel with a 4-deep register
// ring (7.1 ms), profiles/lstm_stack_ab_r3*.jsonl.
FM_API int fm_lstm_stack(const void* xa, int64_t B, int L, int H, int layers, const void* W0, const void* W1,
                         float* h_out, float* c_out, int rt, int nct, hipStream_t stream) {
  if (B <= 0 || L <= 0) return 0;
  if (layers != 1 && layers != 2) return (int)hipErrorInvalidValue;
  if (layers == 2 && W1 == nullptr) return (int)hipErrorInvalidValue;
#define FM_STK(HH, RTT, NCC)                                                                              \
  return layers == 2 ? launch_stack<HH, RTT, NCC, 2>(xa, B, L, W0, W1, h_out, c_out, stream)            \
                     : launch_stack<HH, RTT, NCC, 1>(xa, B, L, W0, W1, h_out, c_out, stream)
  if (nct == 201 && layers == 2) {     // layer-pipelined 2-layer kernel (lstm_stack2_pipe_kernel), 1 column tile
    if (H == 256 && rt == 4) return launch_stack2_pipe<256, 4>(xa, B, L, W0, W1, h_out, c_out, stream);
    if (H == 256 && rt == 2) return launch_stack2_pipe<256, 2>(xa, B, L, W0, W1, h_out, c_out, stream);
    return (int)hipErrorInvalidValue;
  }
  if (nct == 216 && layers == 2) {     // 16x16-tile 2-layer kernel (lstm_stack2_t16_kernel), 48 sequences
    if (H == 256 && rt == 8) return launch_stack2_t16<256>(xa, B, L, W0, W1, h_out, c_out, stream);
    return (int)hipErrorInvalidValue;
  }
  if (nct == 202 && layers == 2) {     // row-tile streamed 2-layer kernel (lstm_stack2_rs_kernel), 2 column tiles
    if (H == 256 && rt == 4) return launch_stack2_rs<256>(xa, B, L, W0, W1, h_out, c_out, stream);
    return (int)hipErrorInvalidValue;
  }
  if (nct >= 211 && nct <= 214 && layers == 2 && H == 256 && rt == 4) {   // ablations (measurement only)
    if (nct == 211) return launch_stack2_pipe<256, 4, 1>(xa, B, L, W0, W1, h_out, c_out, stream);
    if (nct == 212) return launch_stack2_pipe<256, 4, 2>(xa, B, L, W0, W1, h_out, c_out, stream);
    if (nct == 213) return launch_stack2_pipe<256, 4, 3>(xa, B, L, W0, W1, h_out, c_out, stream);
    return launch_stack2_pipe<256, 4, 4>(xa, B, L, W0, W1, h_out, c_out, stream);
  }
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
