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
