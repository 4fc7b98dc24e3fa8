// The LSTM cell update shared by lstm.hip and lstm_stack.hip (K6).
//
// Issue-cost budget (MI355X_MICROARCH.md, "vector-instruction ISSUE cost"):
// a v_exp_f32 / v_rcp_f32 issues in 8 cycles, a v_add / v_fma / v_med3 in 4.
// A transcendental is therefore worth two plain VALU ops, and any FMA-only
// sigmoid / tanh (a clamp, a square, a Horner chain of 5+ FMAs, a final
// scale) costs MORE than the 2-3 ops it replaces.  What pays is taking the
// plain ops out around the transcendentals:
//
//   * the gate pre-activations arrive pre-scaled by the packed weights
//     (ops/lstm.py gate_scales): i, f, o rows by -log2(e), g rows by
//     -2 log2(e), so exp2 of the MFMA output IS e^{-x} / e^{-2x}: no v_mul;
//   * the cell state is kept scaled, cs = -2 log2(e) c, so tanh(c) needs no
//     v_mul either; the scale is folded into the i*g term for free
//     (K (1 - E_g) = fma(E_g, -K, K));
//   * only the exponents that could turn a product into inf * 0 are clamped
//     (g and c; an overflowing E_i / E_f / E_o drives its rcp to 0, the
//     correct saturated gate):
//
//     sf = 1 / (1 + E_f)                           v_exp v_add v_rcp
//     K i g = K (1 - E_g) / (E_i (1 + E_g) + (1 + E_g))
//                                                  2 v_exp, v_med3, v_add, 2 v_fma, v_mul, v_rcp
//     cs' = fma(cs, sf, K i g)                      v_fma
//     h = (1 - E_c) / (E_o (1 + E_c) + (1 + E_c))   2 v_exp, v_med3, v_add, 2 v_fma, v_rcp
//       (the numerator folded: (1 - E_c) r = fma(-E_c, r, r))
//
// = 11 VALU + 8 transcendental = 108 issue cycles per unit-step, against
// 20 + 7 = 136 for the fused-fraction form with in-kernel scaling and clamps
// on every exponent (152 before the weights carried the scale).
#pragma once

namespace fm {

constexpr float kLstmLog2e = 1.4426950408889634f;
constexpr float kLstmK = -2.f * kLstmLog2e;       // cs = kLstmK * c
constexpr float kLstmInvK = 1.f / kLstmK;
constexpr float kLstmExpClamp = 60.f;             // E <= 2^60: (1 + E_i)(1 + E_g) and (1 + E_o)(1 + E_c) stay finite

__device__ __forceinline__ float lstm_exp2(float x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ float lstm_exp2_clamped(float x) {
  return __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(x, -kLstmExpClamp, kLstmExpClamp));
}

// ai, af, ao: -log2(e) x;  ag: -2 log2(e) x (pre-scaled gate pre-activations)
// cs: the scaled cell state (in / out);  h: the hidden output (unscaled)
__device__ __forceinline__ void lstm_cell(float ai, float af, float ag, float ao, float& cs, float& h) {
#if defined(FM_LSTM_CELL_AB) && FM_LSTM_CELL_AB == 12
  // A/B build only (tools/build_native.py --variant): the 12-VALU form
  {
    const float sf1 = __builtin_amdgcn_rcpf(1.f + lstm_exp2(af));
    const float eg1 = lstm_exp2_clamped(ag);
    const float pg1 = 1.f + eg1;
    const float kig1 = __builtin_fmaf(eg1, -kLstmK, kLstmK) * __builtin_amdgcn_rcpf(__builtin_fmaf(lstm_exp2(ai), pg1, pg1));
    cs = __builtin_fmaf(cs, sf1, kig1);
    const float ec1 = lstm_exp2_clamped(cs);
    const float pc1 = 1.f + ec1;
    h = (1.f - ec1) * __builtin_amdgcn_rcpf(__builtin_fmaf(lstm_exp2(ao), pc1, pc1));
    return;
  }
#endif
#if defined(FM_LSTM_CELL_AB) && FM_LSTM_CELL_AB == 14
  // A/B build only (tools/build_native.py --variant): the 14-VALU form
  const float sf0 = __builtin_amdgcn_rcpf(1.f + lstm_exp2(af));
  const float eg0 = lstm_exp2_clamped(ag);
  const float kig0 = __builtin_fmaf(eg0, -kLstmK, kLstmK) * __builtin_amdgcn_rcpf((1.f + lstm_exp2(ai)) * (1.f + eg0));
  cs = __builtin_fmaf(cs, sf0, kig0);
  const float ec0 = lstm_exp2_clamped(cs);
  h = (1.f - ec0) * __builtin_amdgcn_rcpf((1.f + lstm_exp2(ao)) * (1.f + ec0));
  return;
#endif
  const float sf = __builtin_amdgcn_rcpf(1.f + lstm_exp2(af));
  const float eg = lstm_exp2_clamped(ag);
  const float pg = 1.f + eg;
  const float pig = __builtin_fmaf(lstm_exp2(ai), pg, pg);            // (1 + E_i)(1 + E_g)
  const float kig = __builtin_fmaf(eg, -kLstmK, kLstmK) * __builtin_amdgcn_rcpf(pig);
  cs = __builtin_fmaf(cs, sf, kig);
  const float ec = lstm_exp2_clamped(cs);
  const float pc = 1.f + ec;
  const float r = __builtin_amdgcn_rcpf(__builtin_fmaf(lstm_exp2(ao), pc, pc));   // 1 / ((1 + E_o)(1 + E_c))
  h = __builtin_fmaf(-ec, r, r);                                                  // (1 - E_c) r
}

// Separate-gate form of the same pre-scaled recurrence (10 transcendentals;
// A/B timing only): sigm(x) = 1 / (1 + E), tanh(x) = 2 / (1 + E_2x) - 1.
__device__ __forceinline__ float lstm_sigm_s(float xs) { return __builtin_amdgcn_rcpf(1.f + lstm_exp2(xs)); }
__device__ __forceinline__ float lstm_tanh_s(float xs) {
  return 2.f * __builtin_amdgcn_rcpf(1.f + lstm_exp2(xs)) - 1.f;
}
__device__ __forceinline__ void lstm_cell_separate(float ai, float af, float ag, float ao, float& cs, float& h) {
  const float c = cs * kLstmInvK;
  const float cn = lstm_sigm_s(af) * c + lstm_sigm_s(ai) * lstm_tanh_s(ag);
  cs = cn * kLstmK;
  h = lstm_sigm_s(ao) * lstm_tanh_s(cs);
}

}  // namespace fm
