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

#include <type_traits>

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

// ---------------------------------------------------------------------------
// Same recurrence, weights staged through LDS by LDS-DMA (global_load_lds
// dwordx4) in a DEPTH-deep per-wave ring instead of register lookahead.
// The streamed A fragments then cost no VGPRs (the register variant spills 65
// at 4 x 2), and DEPTH k-steps of weight loads stay in flight behind the MFMAs
// of the current one (counted s_waitcnt vmcnt, raw s_barrier so a stage in
// flight survives the barriers).  The packed fragment of one (rt, k-step) is
// 64 lanes x 16 B contiguous, exactly the lane-linear image one LDS-DMA
// wave-instruction writes, so each wave reads back its own fragments with
// ds_read_b128 and no wave touches another's ring.  To make room in LDS the
// h images are single-buffered, with one extra barrier per layer between the
// last read of h_{t-1} and the first write of h_t.
namespace {
__device__ __forceinline__ void glds16(const uint4* g, uint4* l) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)l, 16, 0, 0);
}
// s_waitcnt vmcnt(N), the other counters left alone (gfx9 encoding)
#define FM_VMCNT(N) __builtin_amdgcn_s_waitcnt((((N) & 15) | ((((N) >> 4) & 3) << 14) | 0x0F70))
#define FM_LGKM0() __builtin_amdgcn_s_waitcnt(0xC07F)
// The kernel's own LDS traffic while LDS-DMA stages are in flight goes through
// these: the compiler cannot tell a ring slot or an h image from the slots a
// pending LDS-DMA writes, and would put an s_waitcnt vmcnt(0) in front of
// every compiler-visible ds_read / ds_write (draining the ring each k-step).
// The reads carry no wait of their own: ``lds_fence`` (lgkmcnt(0)) ties every
// fragment read before it to the wait, so no use can be scheduled earlier.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned lds_off(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ u32x4 ds_read16(unsigned a) {
  u32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
__device__ __forceinline__ void ds_write8(unsigned a, u32x2 v) {
  asm volatile("ds_write_b64 %0, %1" : : "v"(a), "v"(v) : "memory");
}
template <int N>
__device__ __forceinline__ void lds_fence(u32x4 (&f)[N]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}
__device__ __forceinline__ uint4 as_uint4(u32x4 v) { return make_uint4(v.x, v.y, v.z, v.w); }
}  // namespace

template <int H, int RT, int NCT, int LAYERS, int DEPTH>
__global__ __launch_bounds__(64 * H / (8 * RT)) void lstm_stack_glds_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out, float* __restrict__ c_out) {
  constexpr int NW = H / (8 * RT);
  constexpr int KH = H / 16;
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 32 * NCT;
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                                   // [BT][HP]
  unsigned short* h1b = lds + BT * HP;                         // [BT][HP] (LAYERS == 2)
  const int lane = lane_id(), w = wave_id();
  uint4* ring = reinterpret_cast<uint4*>(lds + LAYERS * BT * HP) + (int64_t)w * DEPTH * RT * 64;
  const unsigned ring_off = lds_off(ring) + 16 * lane_id();
  const unsigned h0o = lds_off(h0b), h1o = lds_off(h1b);
  const int hf = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;

  for (int i = threadIdx.x; i < LAYERS * BT * HP; i += 64 * NW) lds[i] = 0;   // h_{-1} = 0
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
  uint4 onesv[NCT];
#pragma unroll
  for (int ct = 0; ct < NCT; ++ct) onesv[ct] = make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u);

  // k-step order of layer 0: the x/bias step first (its B fragment is the
  // register x_t, whose load the compiler waits for with vmcnt(0): taking it
  // first keeps that drain at the start of the layer, before the ring fills)
  auto ks_of0 = [](int i) { return i == 0 ? KH : i - 1; };
  auto stage = [&](const uint4* Ww, int KS, int ks, int slot) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) glds16(Ww + (rt * KS + ks) * 64, ring + (slot * RT + rt) * 64);
  };
  // gates[rt][ct] = sum_i A[rt][ks(i)] B[ks(i)][ct]; stages 0 .. DEPTH-1 were
  // issued by the caller; the stage of step i + DEPTH is issued after step i.
  // B of k-step ks < KH is h image ``lo``, ks >= KH image ``hi`` (at ks - KH),
  // except step ``sp`` whose B is the register ``breg`` (x_t / ones): the LDS
  // read is unconditional (clamped address) and the register picked by VALUE,
  // so no pointer select turns the ds_read into a flat load.
  auto gemm = [&](const uint4* Ww, int KS, auto ks_of, int sp, const uint4 (&breg)[NCT], unsigned lo, unsigned hi,
                  f32x16 (&acc)[RT][NCT]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = (f32x16){};
#pragma unroll 1
    for (int i = 0; i < KS; ++i) {
      const int slot = i % DEPTH;
      // stages still allowed in flight: the ones issued after step i's
      const int ahead = KS - 1 - i < DEPTH - 1 ? KS - 1 - i : DEPTH - 1;
      if (ahead >= 2) FM_VMCNT(2 * RT);
      else if (ahead == 1) FM_VMCNT(RT);
      else FM_VMCNT(0);
      const int ks = ks_of(i);
      const int kc = ks < KH ? ks : ks - KH < KH ? ks - KH : KH - 1;
      const unsigned src = (ks < KH ? lo : hi) + 2 * (16 * kc + 8 * hf + col * HP);
      u32x4 f[RT + NCT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) f[rt] = ds_read16(ring_off + 16 * ((slot * RT + rt) * 64));
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) f[RT + ct] = ds_read16(src + 2 * (32 * ct * HP));
      lds_fence(f);                              // fragments in VGPRs: the slot may be refilled
      Frag a[RT], bf[NCT];
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) a[rt].u = as_uint4(f[rt]);
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) bf[ct].u = i == sp ? breg[ct] : as_uint4(f[RT + ct]);
      if (i + DEPTH < KS) stage(Ww, KS, ks_of(i + DEPTH), slot);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct)
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt].v, bf[ct].v, acc[rt][ct], 0, 0, 0);
    }
  };
  auto update = [&](f32x16 (&acc)[RT][NCT], float (&c)[RT][NCT][4], unsigned hdst, bool last) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < NCT; ++ct) {
        float hv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          cell(acc[rt][ct][j], acc[rt][ct][4 + j], acc[rt][ct][8 + j], acc[rt][ct][12 + j], c[rt][ct][j], hv[j]);
        const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
        u32x2 pk;
        pk.x = pack_bf2(hv[0], hv[1]);
        pk.y = pack_bf2(hv[2], hv[3]);
        ds_write8(hdst + 2 * ((32 * ct + col) * HP + u0), pk);
        if (last && inb[ct]) {
          const int64_t bb = b0 + 32 * ct + col;
          *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          *reinterpret_cast<float4*>(&c_out[bb * H + u0]) =
              make_float4(c[rt][ct][0], c[rt][ct][1], c[rt][ct][2], c[rt][ct][3]);
        }
      }
  };
  auto barrier = [&]() {
    FM_LGKM0();                                  // this wave's LDS writes landed
    __builtin_amdgcn_s_barrier();               // raw: stages in flight survive it
  };

  // x_t is laundered through an empty asm once a drained k-step proves it
  // landed: a register loaded outside a loop that has VMEM of its own makes the
  // compiler flush vmcnt in the loop preheader, i.e. drain the ring stages
  uint4 xt[NCT];
  {
    u32x4 x0[NCT];
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const uint4 v = xp[ct][0];
      x0[ct] = (u32x4){v.x, v.y, v.z, v.w};
    }
    FM_VMCNT(0);
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      asm volatile("" : "+v"(x0[ct]));
      xt[ct] = as_uint4(x0[ct]);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) stage(W0w, KS0, ks_of0(d), d);
  for (int t = 0; t < L; ++t) {
    const bool last = t == L - 1;
    u32x4 xn[NCT];                               // x_{t+1}, in flight behind layer 0's k-steps
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      const uint4 v = xp[ct][(last ? t : t + 1) * 2];
      xn[ct] = (u32x4){v.x, v.y, v.z, v.w};
    }
    f32x16 acc[RT][NCT];
    gemm(W0w, KS0, ks_of0, 0, xt, h0o, h0o, acc);
    FM_VMCNT(0);                                 // free: the last k-step drained
#pragma unroll
    for (int ct = 0; ct < NCT; ++ct) {
      asm volatile("" : "+v"(xn[ct]));
      xt[ct] = as_uint4(xn[ct]);
    }
    if (LAYERS == 2) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) stage(W1w, KS1, d, d);
    }
    barrier();                                   // every wave done reading h0_{t-1}
    update(acc, c0, h0o, last && LAYERS == 1);
    if (LAYERS == 1 && !last) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) stage(W0w, KS0, ks_of0(d), d);
    }
    barrier();                                   // h0_t complete
    if (LAYERS == 2) {
      gemm(W1w, KS1, [](int i) { return i; }, KS1 - 1, onesv, h1o, h0o, acc);
      if (!last) {
#pragma unroll
        for (int d = 0; d < DEPTH; ++d) stage(W0w, KS0, ks_of0(d), d);
      }
      barrier();                                 // every wave done reading h1_{t-1} (and h0_t)
      update(acc, c1, h1o, last);
      barrier();                                 // h1_t complete
    }
  }
  FM_VMCNT(0);
}

template <int H, int RT, int NCT, int LAYERS, int DEPTH>
static int launch_stack_glds(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                             float* c_out, hipStream_t stream) {
  constexpr int NW = H / (8 * RT);
  constexpr int BT = 32 * NCT;
  const size_t lds = (size_t)LAYERS * BT * (H + 8) * sizeof(unsigned short) + (size_t)NW * DEPTH * RT * 64 * 16;
  auto k = lstm_stack_glds_kernel<H, RT, NCT, LAYERS, DEPTH>;
  if (lds > 160 * 1024) return (int)hipErrorInvalidValue;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + BT - 1) / BT)), dim3(64 * NW), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
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
// updates (VALU: 5 exp + 2 rcp per unit) issue beside MFMAs instead of
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
// f(ic<0>{}), ..., f(ic<N-1>{}): a compile-time-indexed unrolled sequence
template <class F, int... Gs>
__device__ __forceinline__ void for_each_ic(F&& f, std::integer_sequence<int, Gs...>) {
  (f(ic<Gs>{}), ...);
}
}  // namespace

template <int H, int RT>
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

  Frag a[RT];                                          // A fragments of the current k-step
  auto loadA = [&](Frag (&f)[RT], __amdgpu_buffer_rsrc_t Ww, int KS, int ks) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(Ww, voff, (rt * KS + ks) * 1024, 0);
      f[rt].u = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // NK unrolled k-steps: A of step i from (Ww, KS, ks_of(i)), B = b_of(i),
  // then cell_at(i); the A fragments of (Wn, KSn, ksn) are prefetched during
  // the last step (the first k-step of whatever follows)
  auto segment = [&](auto NK, f32x16 (&acc)[RT], __amdgpu_buffer_rsrc_t Ww, int KS, auto ks_of, auto b_of,
                     __amdgpu_buffer_rsrc_t Wn, int KSn, int ksn, auto cell_at) {
    // the B fragment (h image in LDS, stable for the whole segment) is read
    // one k-step ahead too, so its LDS latency hides behind the MFMAs
    uint4 bcur = b_of(0);
#pragma unroll
    for (int i = 0; i < decltype(NK)::value; ++i) {
      __builtin_amdgcn_sched_barrier(0);             // k-steps stay in order: no hoisted loads
      Frag an[RT];
      if (i + 1 < decltype(NK)::value) loadA(an, Ww, KS, ks_of(i + 1));
      else loadA(an, Wn, KSn, ksn);
      const uint4 bnext = i + 1 < decltype(NK)::value ? b_of(i + 1) : bcur;
      Frag bf;
      bf.u = bcur;
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
        acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[rt].v, bf.v, acc[rt], 0, 0, 0);
      cell_at(i);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) a[rt] = an[rt];
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
    cell(acc[rt][j], acc[rt][4 + j], acc[rt][8 + j], acc[rt][12 + j], c[rt][j], hv[j]);
    if (j == 3) {
      const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
      uint2 pk;
      pk.x = pack_bf2(hv[0], hv[1]);
      pk.y = pack_bf2(hv[2], hv[3]);
      *reinterpret_cast<uint2*>(&hw[u0]) = pk;
      if (out && inb) {
        *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        *reinterpret_cast<float4*>(&c_out[bb * H + u0]) = make_float4(c[rt][0], c[rt][1], c[rt][2], c[rt][3]);
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
  zero(accA);
  segment(ic<KS0>{}, accA, W0w, KS0, ks_l0,
          [&](int i) { const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1)); return i == 0 ? xt : v; },
          W1w, KS1, KH, no_cell);
#pragma unroll
  for (int q = 0; q < NC; ++q) cell_q(q, accA, c0, h0w, false);
  lds_barrier();
  zero(accB);
  const auto b_l1b = [&](int i) { const uint4 v = lds16(h0r + 16 * (i < KH ? i : KH - 1)); return i == KH ? onesv : v; };
  for (int t = 0; t < L - 1; ++t) {
    xt = xp[(t + 1) * 2];
    // phase A: L1(t) over [h0_t; 1]
    segment(ic<KH + 1>{}, accB, W1w, KS1, ks_l1b, b_l1b, W0w, KS0, KH, no_cell);
    //          L0(t+1) over [x_{t+1}; h0_t]  ||  cells of L1(t)
    zero(accA);
    segment(ic<KS0>{}, accA, W0w, KS0, ks_l0,
            [&](int i) { const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1)); return i == 0 ? xt : v; },
            W1w, KS1, 0, [&](int i) { if (i < NC) cell_q(i, accB, c1, h1w, false); });
    lds_barrier();                                   // h1_t complete; every read of h0_t done
    // phase B: L1(t+1) over h1_t  ||  cells of L0(t+1)
    zero(accB);
    segment(ic<KH>{}, accB, W1w, KS1, ks_l1a, [&](int i) { return lds16(h1r + 16 * i); },
            W1w, KS1, KH, [&](int i) { if (i < NC) cell_q(i, accA, c0, h0w, false); });
    lds_barrier();                                   // h0_{t+1} complete; every read of h1_t done
  }
  // the last step's layer 1 (out of the loop: its output addresses are not
  // live across the time loop)
  segment(ic<KH + 1>{}, accB, W1w, KS1, ks_l1b, b_l1b, W1w, KS1, 0, no_cell);
#pragma unroll
  for (int q = 0; q < NC; ++q) cell_q(q, accB, c1, h1w, true);
}

// The same two-phase schedule as one flat, unrolled sequence of the step's
// NG = 3 H/16 + 2 k-steps (L1 over [h0; 1], L0 over [x; h0], L1 over h1), so
// the A fragments run D k-steps ahead through a ring of D + 1 register sets
// -- across phase boundaries, barriers and time steps (NG % (D + 1) == 0
// keeps the ring aligned from one step to the next).  c of both layers lives
// in LDS (lane-linear float4 per row tile) to leave the registers to the ring.
template <int H, int RT, int D>
__global__ __launch_bounds__(64 * H / (8 * RT)) void lstm_stack2_flow_kernel(
    const uint4* __restrict__ xa, int64_t B, int L, const uint4* __restrict__ W0, const uint4* __restrict__ W1,
    float* __restrict__ h_out, float* __restrict__ c_out) {
  constexpr int NW = H / (8 * RT);
  constexpr int KH = H / 16;
  constexpr int KS0 = KH + 1;
  constexpr int KS1 = 2 * KH + 1;
  constexpr int HP = H + 8;
  constexpr int BT = 32;
  constexpr int NC = 4 * RT;
  constexpr int NG = 3 * KH + 2;
  constexpr int G2 = KH + 1, G3 = 2 * KH + 2;          // first k-step of the L0 / L1-over-h1 phases
  constexpr int R = D + 1;
  static_assert(NC <= KH && NG % R == 0, "ring must stay aligned across steps");
  extern __shared__ __attribute__((aligned(16))) unsigned short lds[];
  unsigned short* h0b = lds;                           // [BT][HP]
  unsigned short* h1b = lds + BT * HP;                 // [BT][HP]
  float4* cst = reinterpret_cast<float4*>(lds + 2 * BT * HP);   // [2][NW][RT][64] c of both layers
  const int lane = lane_id(), w = wave_id();
  const int hf = lane >> 5, col = lane & 31;
  const int64_t b0 = (int64_t)blockIdx.x * BT;
  {
    unsigned* z = reinterpret_cast<unsigned*>(lds);
    constexpr int NZ = BT * HP + 2 * NW * RT * 64 * 4;           // dwords: h images + c
    for (int i = threadIdx.x; i < NZ; i += 64 * NW) z[i] = 0u;
  }
  __syncthreads();

  int64_t bb = b0 + col;
  const bool inb = bb < B;
  bb = inb ? bb : B - 1;
  const uint4* xp = xa + (bb * L) * 2 + hf;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const __amdgpu_buffer_rsrc_t W0w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W0 + (int64_t)wu * RT * KS0 * 64), (short)0, RT * KS0 * 1024, 0x00020000);
  const __amdgpu_buffer_rsrc_t W1w = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(W1 + (int64_t)wu * RT * KS1 * 64), (short)0, RT * KS1 * 1024, 0x00020000);
  const int voff = 16 * lane;
  const unsigned short* h0r = h0b + col * HP + 8 * hf;
  const unsigned short* h1r = h1b + col * HP + 8 * hf;
  unsigned short* h0w = h0b + col * HP;
  unsigned short* h1w = h1b + col * HP;
  auto lds16 = [](const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); };
  auto ones = [&]() { return make_uint4(hf == 0 ? 0x3F80u : 0u, 0u, 0u, 0u); };

  auto loadA = [&](Frag (&f)[RT], __amdgpu_buffer_rsrc_t Ww, int KS, int ks) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(Ww, voff, (rt * KS + ks) * 1024, 0);
      f[rt].u = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  // k-step g of a time step -> A fragments
  auto load_g = [&](Frag (&f)[RT], int g) {
    if (g < G2) loadA(f, W1w, KS1, KH + g);                          // L1 over [h0; 1]
    else if (g < G3) loadA(f, W0w, KS0, g == G2 ? KH : g - G2 - 1);  // L0: x/bias step first
    else loadA(f, W1w, KS1, g - G3);                                 // L1 over h1
  };
  auto mfma = [&](f32x16 (&acc)[RT], const Frag (&f)[RT], uint4 b) {
    Frag bf;
    bf.u = b;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
      acc[rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f[rt].v, bf.v, acc[rt], 0, 0, 0);
  };
  auto zero = [](f32x16 (&acc)[RT]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt] = (f32x16){};
  };
  float hv[4], cq[4];
  auto cell_q = [&](int q, const f32x16 (&acc)[RT], int layer, unsigned short* hw, bool out) {
    const int rt = q >> 2, j = q & 3;
    float4* cp = cst + ((layer * NW + w) * RT + rt) * 64 + lane;
    if (j == 0) {
      const float4 c4 = *cp;
      cq[0] = c4.x; cq[1] = c4.y; cq[2] = c4.z; cq[3] = c4.w;
    }
    cell(acc[rt][j], acc[rt][4 + j], acc[rt][8 + j], acc[rt][12 + j], cq[j], hv[j]);
    if (j == 3) {
      const int u0 = 8 * RT * w + 8 * rt + 4 * hf;
      uint2 pk;
      pk.x = pack_bf2(hv[0], hv[1]);
      pk.y = pack_bf2(hv[2], hv[3]);
      *reinterpret_cast<uint2*>(&hw[u0]) = pk;
      *cp = make_float4(cq[0], cq[1], cq[2], cq[3]);
      if (out && inb) {
        *reinterpret_cast<float4*>(&h_out[bb * H + u0]) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        *reinterpret_cast<float4*>(&c_out[bb * H + u0]) = make_float4(cq[0], cq[1], cq[2], cq[3]);
      }
    }
  };

  f32x16 accA[RT], accB[RT];
  Frag fr[R][RT];
  // prologue: L0(0) with h0_{-1} = 0 (one k-step lookahead), its cells, barrier
  {
    uint4 x0 = xp[0];
    Frag a[RT], an[RT];
    loadA(a, W0w, KS0, KH);
    zero(accA);
#pragma unroll
    for (int i = 0; i < KS0; ++i) {
      __builtin_amdgcn_sched_barrier(0);
      if (i + 1 < KS0) loadA(an, W0w, KS0, i);
      const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1));
      mfma(accA, a, i == 0 ? x0 : v);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) a[rt] = an[rt];
    }
#pragma unroll
    for (int d = 0; d < D; ++d) load_g(fr[d], d);      // the ring: first k-steps of step 0
#pragma unroll
    for (int q = 0; q < NC; ++q) cell_q(q, accA, 0, h0w, false);
    lds_barrier();
  }
  zero(accB);                                          // L1(0) over h1_{-1} = 0
  uint4 xt = make_uint4(0u, 0u, 0u, 0u);
  for (int t = 0; t < L - 1; ++t) {
    for_each_ic([&](auto G) {
      constexpr int g = decltype(G)::value;
      __builtin_amdgcn_sched_barrier(0);               // k-steps stay in order
      load_g(fr[(g + D) % R], (g + D) % NG);           // D ahead (wrapping into step t + 1)
      if constexpr (g == 0) xt = xp[(t + 1) * 2];
      if constexpr (g < G2) {                          // phase A: L1(t) over [h0_t; 1]
        const uint4 v = lds16(h0r + 16 * (g < KH ? g : KH - 1));
        mfma(accB, fr[g % R], g == KH ? ones() : v);
      } else if constexpr (g < G3) {                   //   L0(t+1) over [x_{t+1}; h0_t] || cells L1(t)
        constexpr int i = g - G2;
        if constexpr (i == 0) zero(accA);
        const uint4 v = lds16(h0r + 16 * (i == 0 ? 0 : i - 1));
        mfma(accA, fr[g % R], i == 0 ? xt : v);
        if constexpr (i < NC) cell_q(i, accB, 1, h1w, false);
        if constexpr (g == G3 - 1) lds_barrier();      // h1_t complete; every read of h0_t done
      } else {                                         // phase B: L1(t+1) over h1_t || cells L0(t+1)
        constexpr int i = g - G3;
        if constexpr (i == 0) zero(accB);
        mfma(accB, fr[g % R], lds16(h1r + 16 * i));
        if constexpr (i < NC) cell_q(i, accA, 0, h0w, false);
        if constexpr (g == NG - 1) lds_barrier();      // h0_{t+1} complete; every read of h1_t done
      }
    }, std::make_integer_sequence<int, NG>{});
  }
  // the last step's layer 1 over [h0; 1] (its ring sets were loaded ahead)
#pragma unroll
  for (int g = 0; g < G2; ++g) {
    __builtin_amdgcn_sched_barrier(0);
    if (g + D < G2) load_g(fr[(g + D) % R], g + D);
    const uint4 v = lds16(h0r + 16 * (g < KH ? g : KH - 1));
    mfma(accB, fr[g % R], g == KH ? ones() : v);
  }
#pragma unroll
  for (int q = 0; q < NC; ++q) cell_q(q, accB, 1, h1w, true);
}

template <int H, int RT, int D>
static int launch_stack2_flow(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                              float* c_out, hipStream_t stream) {
  constexpr int NW = H / (8 * RT);
  const size_t lds = (size_t)2 * 32 * (H + 8) * sizeof(unsigned short) + (size_t)2 * NW * RT * 64 * 16;
  auto k = lstm_stack2_flow_kernel<H, RT, D>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + 31) / 32)), dim3(64 * NW), lds, stream, (const uint4*)xa, B, L,
                     (const uint4*)W0, (const uint4*)W1, h_out, c_out);
  FM_LAUNCH_CHECK();
  return 0;
}

template <int H, int RT>
static int launch_stack2_pipe(const void* xa, int64_t B, int L, const void* W0, const void* W1, float* h_out,
                              float* c_out, hipStream_t stream) {
  constexpr int NW = H / (8 * RT);
  const size_t lds = (size_t)2 * 32 * (H + 8) * sizeof(unsigned short);
  auto k = lstm_stack2_pipe_kernel<H, RT>;
  if (lds > 64 * 1024) {
    const hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return (int)e;
  }
  hipLaunchKernelGGL(k, dim3((unsigned)((B + 31) / 32)), dim3(64 * NW), lds, stream, (const uint4*)xa, B, L,
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
  if (nct == 202 && layers == 2) {     // flat-sequence pipelined kernel (lstm_stack2_flow_kernel), ring depth 4
    if (H == 256 && rt == 4) return launch_stack2_flow<256, 4, 4>(xa, B, L, W0, W1, h_out, c_out, stream);
    if (H == 256 && rt == 2) return launch_stack2_flow<256, 2, 4>(xa, B, L, W0, W1, h_out, c_out, stream);
    return (int)hipErrorInvalidValue;
  }
  if (nct == 201 && layers == 2) {     // layer-pipelined 2-layer kernel (lstm_stack2_pipe_kernel), 1 column tile
    if (H == 256 && rt == 4) return launch_stack2_pipe<256, 4>(xa, B, L, W0, W1, h_out, c_out, stream);
    if (H == 256 && rt == 2) return launch_stack2_pipe<256, 2>(xa, B, L, W0, W1, h_out, c_out, stream);
    return (int)hipErrorInvalidValue;
  }
  if (nct >= 100) {                    // LDS-DMA weight ring (lstm_stack_glds_kernel), nct - 100 column tiles
#define FM_GLDS(HH, RTT, NCC, DD)                                                                              \
  return layers == 2 ? launch_stack_glds<HH, RTT, NCC, 2, DD>(xa, B, L, W0, W1, h_out, c_out, stream)         \
                     : launch_stack_glds<HH, RTT, NCC, 1, DD>(xa, B, L, W0, W1, h_out, c_out, stream)
    if (H == 256 && rt == 4 && nct == 102) FM_GLDS(256, 4, 2, 2);
    if (H == 256 && rt == 4 && nct == 101) FM_GLDS(256, 4, 1, 3);
    if (H == 256 && rt == 2 && nct == 102) FM_GLDS(256, 2, 2, 2);
    return (int)hipErrorInvalidValue;
#undef FM_GLDS
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
