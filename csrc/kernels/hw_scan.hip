// K2: additive Holt-Winters grid fit as a TIME-PARALLEL scan, seasons in
// registers (no seasonal scratch in HBM at all).
//
// Why: the serial grid fit (smoothing.hip hw2_fit_kernel, one thread per
// (row, candidate pair) running all T steps) has to park m seasonal indices
// per candidate somewhere between laps; at the config-2 shape (40k rows x 27
// candidates x m = 1440) that is 37 GB of fp16 scratch traffic per fit, and
// the fit sat at 76 % of the read+write HBM floor (profiles/pmc_c2_requests_r3.txt).
//
// The additive recursion is LINEAR in its (level, trend) state.  In the
// one-step error e = x - (l + t + s):
//     l' = l + t + a e,   t' = t + a b e,   s' = s + g (1 - a) e
// i.e. v' = A v + k u with v = (l, t), u = x - s, k = (a, a b) and
// A = J - k 1^T (J = [[1, 1], [0, 1]]); a missing sample gives e = 0, v' = J v.
// Inside one season lap every seasonal index s(p) is read once, so the lap's
// inputs u are all known at the lap's start.  One WAVE owns one (row,
// candidate pair) and splits the lap's m steps into 64 contiguous chunks of C
// (lane i: lap offsets [iC, iC + C)), keeping its C seasonal indices of both
// candidates in VGPRs for the whole fit:
//   pass 1  each lane folds its chunk into an affine map v -> A^C v + b
//           (zero-state response; lane 0 starts from the lap's entering state
//           instead of zero; 5 packed ops / step);
//   scan    Hillis-Steele over the 64 lanes: b_i += A^{C d} b_{i-d}, d = 1..32
//           (the lane-uniform powers A^{C 2^j} sit in LDS); the prefix of
//           lanes 0..i-1 is then the (level, trend) entering lane i;
//   pass 2  the textbook recursion over the chunk from that state, updating
//           the lane's seasonal indices and the SSE (exactly the serial
//           kernel's arithmetic).
// A lap that contains a missing sample (rare: rows are right-aligned, the
// left NaN padding is skipped via the row's first finite sample) runs pass 1
// and the scan with explicit 2x2 chunk matrices (J for missing steps).
//
// Work per step is ~12 packed VALU ops instead of ~7, but there is no
// seasonal traffic left: the row's history is staged once in LDS (the 14
// waves of a row read it from there) and the fit becomes VALU-bound.  One
// workgroup per row (ceil(G/2) waves): after the fit the workgroup picks the
// best candidate (hw2_forecast_kernel's rule), and only the winning wave
// writes its seasons (the model cache's fp32 [R, m] state, by absolute phase)
// and the H-step forecast.  Seasons stay fp32 end to end (the serial kernel's
// fp16 scratch rounded them by 2^-11 per lap).
//
// Reference: foremast-brain's Holt-Winters model (docs/guides/design.md:62-72,
// deploy/foremast/3_brain/foremast-brain.yaml ML_ALGORITHM); the recursion and
// its initialisation follow docs/BRAIN_SPEC.md §3.2 and ops/smoothing.py's
// fp64 reference (ref_es_fit).
#include <cstdlib>

#include "fm_common.h"

using namespace fm;

namespace {

typedef float f2 __attribute__((ext_vector_type(2)));

struct M2 {      // [[a, b], [c, d]] for two candidates at once
  f2 a, b, c, d;
};

__device__ __forceinline__ M2 mmul(const M2& p, const M2& q) {
  return {p.a * q.a + p.b * q.c, p.a * q.b + p.b * q.d, p.c * q.a + p.d * q.c, p.c * q.b + p.d * q.d};
}

// value of lane (lane - d) & 63 (callers ignore lanes < d); d = 1 rides DPP wave_shr:1
// (bound_ctrl: lane 0 reads 0, no old value to materialise)
__device__ __forceinline__ float up1(float v, int d) {
  if (d == 1) return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(((lane_id() - d) & 63) << 2, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ f2 up(f2 v, int d) { return (f2){up1(v.x, d), up1(v.y, d)}; }
// lane - 1's pair, zeros into lane 0 (row_shr-style DPP with bound_ctrl: no
// old value to materialise first)
__device__ __forceinline__ float up0_1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x138, 0xF, 0xF, true));
}
__device__ __forceinline__ f2 up0(f2 v) {
  const float vx = v.x, vy = v.y;
  return (f2){up0_1(vx), up0_1(vy)};
}

// lane l's pair, for every lane.  The halves go through named floats:
// __builtin_bit_cast of a vector element (bit_cast(int, v.y)) reads the
// vector's FIRST element with this clang, which silently turned every .y
// broadcast into a copy of .x.
__device__ __forceinline__ f2 rdl(f2 v, int l) {
  const float vx = v.x, vy = v.y;
  return (f2){__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vx), l)),
              __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vy), l))};
}

constexpr int kLevels = 6;          // log2(64) scan levels

// lane l's pair (per-lane l)
__device__ __forceinline__ f2 bperm2(f2 v, int l) {
  const float vx = v.x, vy = v.y;
  return (f2){__builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(l << 2, __builtin_bit_cast(int, vx))),
              __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(l << 2, __builtin_bit_cast(int, vy)))};
}

// sum over each group of N lanes (N = 64: the whole wave, 32: each half)
template <int N, typename T>
__device__ __forceinline__ T group_sum(T v) {
  v += xor_lane<1>(v); v += xor_lane<2>(v); v += xor_lane<4>(v);
  v += xor_lane<8>(v); v += xor_lane<16>(v);
  if constexpr (N == 64) v += xor_lane<32>(v);
  return v;
}
constexpr int kMaxG = 32;           // candidates per row (<= 16 waves of two)
constexpr int kMaxLaps = 128;       // season laps per row (T / m)

}  // namespace

// Row layout in LDS: sample t >= base (the row's first finite sample) sits at
// xs[pad(t - base)], pad(r) = r + (r >> S) with S = ctz(C) (C = 2^S * odd,
// S >= 2, m a multiple of C; S = 31 -- no padding -- otherwise).  A lane's chunk then starts
// o (2^S + 1) words after its left neighbour's (o = C / 2^S): an odd stride,
// so the 32 lanes of a ds_read_b32 group hit 32 different banks (a stride of
// C = 24 words put them on 4 banks: 8-way conflicts, half the fit's time).
// Lap starts are multiples of m = (lanes) * C past base in the exact case, so
// the within-chunk offsets j + (j >> S) are compile-time immediates.
template <int C, bool EXACT>
struct RowPad {
  static constexpr int S = (EXACT && C % 4 == 0) ? __builtin_ctz(C) : 31;
  static __device__ __forceinline__ int at(int r) { return r + (r >> S); }
  static __host__ __device__ constexpr int words(int r) { return r + (S < 31 ? (r >> S) : 0) + 1; }
};

// LDS: xs[pad(T - base + 64 C)] (the row from base on, NaN-padded) |
// pw[GP][kLevels][4] f2 (A^{C 2^j} per wave) | sse[32] | base, lap flags | wave sums,
// the L2 warm-up DMA landing zone, wave minima and the winner's state
template <int C, bool EXACT, bool FS, int LPP>
__global__ __launch_bounds__(1024) void hw_scan_fit_kernel(const float* __restrict__ x, int64_t ld, int T,
                                                           const float* __restrict__ cand, int G, int m, int H,
                                                           float* __restrict__ sse, float* __restrict__ state,
                                                           int* __restrict__ nobs, float* __restrict__ fc,
                                                           float* __restrict__ sigma, int* __restrict__ best,
                                                           int* __restrict__ nfin, float* __restrict__ sscale,
                                                           float* __restrict__ season_out, int xal, int64_t nrows,
                                                           int ahead, int npass, long long* __restrict__ probe,
                                                           float prune, int plap) {
  using RP = RowPad<C, EXACT>;
  // FOREMAST_HW_SCAN_DEBUG (instruction accounting with PMC, results are
  // garbage): 1 = stop after the row setup, 2 = skip the season laps
  const int dbg = (npass >> 8) & 255;
  const bool use_s0 = FS && (npass >> 16) != 0;   // LDS room for the first-season pairs
  npass &= 255;
  const long long pc0 = probe != nullptr ? clock64() : 0, pw0 = probe != nullptr ? wall_clock64() : 0;
  extern __shared__ float lds[];
  const int64_t row = blockIdx.x;
  const int GP = (G + 1) >> 1;
  const int Tx = (RP::words(T + 64 * C) + 3) & ~3;   // padded row + NaN tail for the last lap
  float* xs = lds;
  f2* pw = reinterpret_cast<f2*>(lds + Tx);
  float* sse_s = lds + Tx + (kMaxG / 2) * kLevels * 8;      // pw: one entry per pair slot
  int* ibase = reinterpret_cast<int*>(sse_s + kMaxG);
  int* lapnan = ibase + 4;                                     // FS: a missing sample in lap k
  float* wsum = reinterpret_cast<float*>(lapnan + kMaxLaps);  // FS: per-wave season sums
  const int tid = threadIdx.x, nth = blockDim.x;
  const int lane = lane_id(), w = wave_id();
  // LPP lanes per candidate pair: 64 (one pair per wave) or 32 (two pairs per
  // wave, half-waves scanning 32 chunks: short seasons, fewer scan levels)
  static_assert(LPP == 64 || (LPP == 32 && FS), "half-wave pairs need the cooperative setup");
  constexpr int PPW = 64 / LPP, NLV = LPP == 64 ? 6 : 5;
  const int half = lane / LPP, li = lane % LPP;
  // pair slots: slot `slot` fits pairs slot, slot + SL, ... in npass passes
  // (fewer waves per row, so two rows share a CU: one's setup and selection
  // run beside the other's laps); an idle slot shadows the last pair
  const int slot = w * PPW + half, SL = (nth / FM_WAVE) * PPW;
  const f2 one = {1.f, 1.f}, zero = {0.f, 0.f};
  const f2 m0 = li == 0 ? one : zero;                 // the lane that starts a lap's scan
  const float* xr = x + row * ld;

  // ---- stage the row.  FS with an aligned row of <= 16 floats per thread
  // (config 2: 10,080 over 448 threads, KREG = 6): ONE read of the row, held in
  // registers while the first finite sample is found, then written to LDS
  // from base on -- with the lap flags and the first two seasons' sums on the
  // way.  Otherwise: find base, then re-read the row (L2) into LDS.  The
  // candidate powers are computed while the row's loads are in flight.
  constexpr int KREG = 6;
  const bool rs = FS && xal && T <= KREG * 4 * nth;
  // wsum[64..128) is the L2 warm-up DMA's landing zone (one dword per lane of
  // a wave): the per-wave minima and the winner's state live past it
  int* wmin = reinterpret_cast<int*>(wsum + 128);             // per-wave first finite sample
  if constexpr (FS)
    for (int i = tid; i < kMaxLaps; i += nth) lapnan[i] = 0;
  float4 rv[KREG];
  if (rs) {
#pragma unroll
    for (int k = 0; k < KREG; ++k) {
      const int i = (k * nth + tid) * 4;
      if (i + 4 <= T) {
        rv[k] = *reinterpret_cast<const float4*>(xr + i);
      } else {
        const float nan = __builtin_nanf("");
        rv[k] = make_float4(nan, nan, nan, nan);
        if (i < T) rv[k].x = xr[i];
        if (i + 1 < T) rv[k].y = xr[i + 1];
        if (i + 2 < T) rv[k].z = xr[i + 2];
      }
    }
  }
  // ---- per slot: two candidates, A = J - k 1^T and its lane-uniform powers
  // A^{C 2^lv} into the slot's LDS entry
  f2 al, ab, gs;
  auto powers = [&](int pair) {
    const int ga = 2 * pair, gb = 2 * pair + 1 < G ? 2 * pair + 1 : 2 * pair;
    al = (f2){cand[3 * ga], cand[3 * gb]};
    const f2 be = {cand[3 * ga + 1], cand[3 * gb + 1]}, gm = {cand[3 * ga + 2], cand[3 * gb + 2]};
    ab = al * be;
    gs = gm * (one - al);
    // FS laps run in (P, T) coordinates (see the lap loop), the others in (L, T)
    const M2 A = FS ? M2{one - al - ab, one, -ab, one} : M2{one - al, one - al, -ab, one - ab};
    M2 Q = A;
    if constexpr (FS) {
      M2 Pw = A;
      Q = {one, zero, zero, one};
#pragma unroll
      for (int k = C; k > 0; k >>= 1) {                  // A^C by squaring
        if (k & 1) Q = mmul(Q, Pw);
        Pw = mmul(Pw, Pw);
      }
    } else {
#pragma unroll 1
      for (int k = 1; k < C; ++k) Q = mmul(Q, A);        // A^C
    }
    if (li == 0) {
#pragma unroll 1
      for (int lv = 0; lv < kLevels; ++lv) {
        f2* p = pw + (slot * kLevels + lv) * 4;
        p[0] = Q.a; p[1] = Q.b; p[2] = Q.c; p[3] = Q.d;
        Q = mmul(Q, Q);
      }
    }
  };
  powers(min(slot, GP - 1));                   // pass 0, while the row's loads are in flight

  int fmin = T;
  if (rs) {
#pragma unroll
    for (int k = 0; k < KREG; ++k) {
      const float4 v = rv[k];
      const int f = isfinite(v.x) ? 0 : isfinite(v.y) ? 1 : isfinite(v.z) ? 2 : isfinite(v.w) ? 3 : 4;
      if (f < 4) fmin = min(fmin, (k * nth + tid) * 4 + f);
    }
  } else if (xal) {
    for (int i = tid * 4; i < T; i += nth * 4) {
      if (i + 4 <= T) {
        const float4 v = *reinterpret_cast<const float4*>(xr + i);
        const int f = isfinite(v.x) ? 0 : isfinite(v.y) ? 1 : isfinite(v.z) ? 2 : isfinite(v.w) ? 3 : 4;
        if (f < 4) fmin = min(fmin, i + f);
      } else {
        for (int k = i; k < T; ++k)
          if (isfinite(xr[k])) fmin = min(fmin, k);
      }
    }
  } else {
    for (int i = tid; i < T; i += nth)
      if (isfinite(xr[i])) fmin = min(fmin, i);
  }
  fmin = wave_min(fmin);
  if (lane == 0) wmin[w] = fmin;
  __syncthreads();                          // wmin, pw, lapnan zeroed
  const long long pcb = probe != nullptr ? clock64() : 0;
  int base = T;
  for (int v = 0; v < nth / FM_WAVE; ++v) base = min(base, wmin[v]);
  base = __builtin_amdgcn_readfirstlane(base);    // uniform (SGPR): it outlives the passes
  float sa1 = 0.f, sb1 = 0.f, fa1 = 0.f, fb1 = 0.f;   // FS: this thread's first / second season sums
  {
    const int e1 = min(base + m, T), e2 = min(base + 2 * m, T);
    if (rs) {
      const bool b4 = (base & 3) == 0;        // float4s stay whole in the padded row (S >= 2)
#pragma unroll
      for (int k = 0; k < KREG; ++k) {
        const float vv[4] = {rv[k].x, rv[k].y, rv[k].z, rv[k].w};
        const int i0 = (k * nth + tid) * 4;
        if (b4 && i0 >= base && i0 + 4 <= T) {
          // whole float4 inside the row: 4 stores at consecutive padded slots;
          // all finite and inside one season -> the sums without selects
          const int r0 = i0 - base;
          float* dst = xs + RP::at(r0);
          dst[0] = vv[0]; dst[1] = vv[1]; dst[2] = vv[2]; dst[3] = vv[3];
          const bool fin = isfinite(vv[0]) && isfinite(vv[1]) && isfinite(vv[2]) && isfinite(vv[3]);
          const float s4 = (vv[0] + vv[1]) + (vv[2] + vv[3]);
          if (fin && i0 + 4 <= e1) { sa1 += s4; fa1 += 4.f; continue; }
          if (fin && i0 >= e1 && i0 + 4 <= e2) { sb1 += s4; fb1 += 4.f; continue; }
          if (fin && i0 >= e2) continue;
        }
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int i = i0 + c;
          if (i >= base && i < T) {
            const float v = vv[c];
            const bool f = isfinite(v);
            xs[RP::at(i - base)] = v;
            if (!f && i >= base + m) lapnan[(i - base - m) / m] = 1;   // that lap takes the general scan
            if (i < e1) { sa1 += f ? v : 0.f; fa1 += f ? 1.f : 0.f; }
            else if (i < e2) { sb1 += f ? v : 0.f; fb1 += f ? 1.f : 0.f; }
          }
        }
      }
    } else {
      for (int i = base + tid; i < T; i += nth) {
        const float v = xr[i];
        xs[RP::at(i - base)] = v;
        if constexpr (FS)
          if (!isfinite(v) && i >= base + m) lapnan[(i - base - m) / m] = 1;   // that lap takes the general scan
      }
    }
    for (int r = T - base + tid; r < T - base + 64 * C; r += nth) xs[RP::at(r)] = __builtin_nanf("");
    if constexpr (FS) {
      // first- and second-season sums split over the workgroup's waves, then
      // added in a fixed order (deterministic, the same in every wave)
      if (!rs) {
        __syncthreads();                    // the staged row
        for (int i = base + tid; i < e2; i += nth) {
          const float v = xs[RP::at(i - base)];
          const bool f = isfinite(v);
          if (i < e1) { sa1 += f ? v : 0.f; fa1 += f ? 1.f : 0.f; }
          else { sb1 += f ? v : 0.f; fb1 += f ? 1.f : 0.f; }
        }
      }
      sa1 = wave_sum(sa1); sb1 = wave_sum(sb1); fa1 = wave_sum(fa1); fb1 = wave_sum(fb1);
      if (lane == 0) { wsum[4 * w] = sa1; wsum[4 * w + 1] = sb1; wsum[4 * w + 2] = fa1; wsum[4 * w + 3] = fb1; }
    }
  }
  __syncthreads();                          // the row, lap flags and season sums
  if (dbg == 1) return;
  if constexpr (FS) {
    // warm L2 (and the Infinity Cache) with the row the workgroup `ahead`
    // dispatches later will read -- the same XCD when ahead % 8 == 0: one dword
    // per 128-B line, DMA'd into a scratch LDS zone (no VGPR).  Issued after
    // the setup's last barrier: a barrier waits for every outstanding memory
    // operation, so the next one (after the laps) finds it long landed
    const int64_t nxt = row + ahead;
    if (ahead > 0 && nxt < nrows) {
      const float* src = x + nxt * ld;
      const int lines = (T + 31) / 32;
      for (int c = tid; c < lines; c += nth)
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + c * 32),
                                         (__attribute__((address_space(3))) void*)(wsum + 16 * 4), 4, 0, 0);
    }
  }


  // ---- initial level / trend (the same for every candidate): level = mean of
  // the first season, trend = (mean of the second - mean of the first) / m
  float m1 = __builtin_nanf(""), trd = 0.f;
  int c1 = 0;
  if (base < T) {
    const int e1 = min(base + m, T), e2 = min(base + 2 * m, T);
    float sa = 0.f, sb = 0.f;
    int ca = 0, cb = 0;
    if constexpr (FS) {
      float fa = 0.f, fb = 0.f;
      for (int v = 0; v < nth / FM_WAVE; ++v) {
        sa += wsum[4 * v]; sb += wsum[4 * v + 1]; fa += wsum[4 * v + 2]; fb += wsum[4 * v + 3];
      }
      ca = (int)fa;
      cb = (int)fb;
    } else {
      for (int i = base + lane; i < e1; i += FM_WAVE) {
        const float v = xs[RP::at(i - base)];
        const bool f = isfinite(v);
        sa += f ? v : 0.f;
        ca += f;
      }
      for (int i = e1 + lane; i < e2; i += FM_WAVE) {
        const float v = xs[RP::at(i - base)];
        const bool f = isfinite(v);
        sb += f ? v : 0.f;
        cb += f;
      }
      sa = wave_sum(sa); sb = wave_sum(sb); ca = wave_sum(ca); cb = wave_sum(cb);
    }
    m1 = ca > 0 ? sa / ca : 0.f;
    const float m2 = cb > 0 ? sb / cb : 0.f;
    trd = cb > 0 ? (m2 - m1) / m : 0.f;
    c1 = ca;
  }
  // uniform across the workgroup: SGPRs, not VGPRs held through the passes
  m1 = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, m1)));
  trd = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, trd)));
  c1 = __builtin_amdgcn_readfirstlane(c1);
  const int q0 = li * C;
  f2 s[C];
  int n = 0;                                // finite steps after the first season (every candidate)
  int bg = 0;                               // the best candidate so far and its SSE (uniform)
  float bs = 0.f;
  float* lbt = wsum + 144;                  // the winner's level, trend
  float* sbst = wsum + 160;                 // the winner's seasons by absolute phase [m]
  // FS: the first season's indices (the same for every candidate) in the
  // lanes' register order, [C][LPP] pairs: a pass loads its C seasons with C
  // conflict-free ds_read_b64 instead of recomputing them
  f2* s0T = reinterpret_cast<f2*>(sbst + ((m + 3) & ~3));
  if (use_s0) {
    for (int i = tid; i < C * LPP; i += nth) {
      const int j = i / LPP, q = (i % LPP) * C + j;
      const float v = (q < m && base + q < T) ? xs[RP::at(q)] : __builtin_nanf("");
      const float si = isfinite(v) ? v - m1 : 0.f;
      s0T[i] = (f2){si, si};
    }
    __syncthreads();
  }
  long long pc1 = 0, pc2 = 0, pcs = 0;
  // early candidate pruning (FS, one pair per wave): after lap `plap` every
  // candidate's partial SSE is published (psse: the setup's per-wave season
  // sums, dead by then); a pair whose two partials both exceed `prune` x the
  // smallest partial of the candidates fitted so far stops its laps and
  // reports SSE = inf (never selected).  The leader is never pruned, so each
  // pass keeps at least the pass-0 winner's full fit; nfull = the finite-step
  // count of a completed fit (sigma / nfin of the row)
  float* psse = wsum;
  int* nfull = reinterpret_cast<int*>(wsum + 146);
  const bool pr_on = FS && LPP == 64 && prune > 0.f && plap > 0;
#pragma unroll 1
  for (int pass = 0; pass < npass; ++pass) {
  const int pidx = slot + pass * SL;
  const bool pvalid = pidx < GP;
  const int pair = pvalid ? pidx : GP - 1;
  if (pass > 0) {
    powers(pair);
    __syncthreads();                        // the slot's powers (every wave runs every pass)
  }
  const int ga = 2 * pair, gb = 2 * pair + 1 < G ? 2 * pair + 1 : 2 * pair;
  // ---- initial state, seasonal indices from the first season (an opaque
  // lane offset: hoisted out of the pass loop, the C per-step conditions and
  // addresses took 70 registers for the whole loop)
  f2 l = (f2){m1, m1}, tr = (f2){trd, trd};
  if constexpr (FS) l = l + tr;             // the FS laps carry P = level + trend
  int q0p = q0;
  asm volatile("" : "+v"(q0p));
  if (use_s0) {
#pragma unroll
    for (int j = 0; j < C; ++j) s[j] = s0T[j * LPP + li];
  } else if (base < T) {
#pragma unroll
    for (int j = 0; j < C; ++j) {
      const int q = q0p + j;
      const float v = (q < m && base + q < T) ? xs[RP::at(q)] : __builtin_nanf("");
      const float si = isfinite(v) ? v - m1 : 0.f;
      s[j] = (f2){si, si};
    }
  } else {
#pragma unroll
    for (int j = 0; j < C; ++j) s[j] = zero;
  }

  if (probe != nullptr && pass == 0) pc1 = clock64();
  // ---- season laps.  Steps past the lap's end (the last active lane's tail,
  // later lanes) act as missing samples (e = 0: seasons, SSE and count stay
  // unchanged), so the step loops carry no per-step branches; xs is padded
  // with NaN past T so their reads stay inside the allocation.
  double ea = 0.0, eb = 0.0;
  n = 0;
  bool pruned = false;
  if constexpr (FS) {
  // One code path for every lap: the general arithmetic (missing samples,
  // inactive steps) sits behind lap-uniform scalar branches inside the step
  // loops.  Separate lap variants each produced their own updated seasons and
  // the register allocator copied all C of them back at the join (+48 VGPRs
  // and 24 v_mov_b64 per lap at C = 24).
  //
  // The state is carried as (P, T), P = level + trend (the prediction before
  // the season): e = x - s - P;  P' = P + T + c e  (c = a + a b);  T' = T + a b e;
  // s' = s + g (1 - a) e.  The same recursion as (level, trend), but each step
  // has two dependent ops on its critical path (e, then P') instead of four,
  // so the scheduler has independent work for the hazard slots.  The powers
  // in pw are of A = [[1 - c, 1], [-a b, 1]] (powers() for FS).
  const f2 cc = al + ab;
  f2 accp = zero;                             // this lane's SSE over the laps (fp32: <= C * laps terms)
  int lap = 0;
#pragma unroll 1
  for (int tl = dbg == 2 ? T : base + m; tl < T; tl += m, ++lap) {
    int pwo = slot * kLevels * 4;
    if constexpr (LPP == 64) asm volatile("" : "+s"(pwo));
    else asm volatile("" : "+v"(pwo));
    const f2* pwv = pw + pwo;
    const int nact = min(m, T - tl);
    const int last = (nact - 1) / C;          // lane holding the lap's last step
    const int cnt = nact - q0;                // active steps of this lane (may be <= 0 or > C)
    const bool gaps = lapnan[lap] != 0;       // a missing sample (the staging's flags)
    // pass 2 needs the masked arithmetic for gaps and for inactive steps
    // (a partial last lap; every lap when the chunks do not tile the season)
    const bool gen2 = gaps || !EXACT || nact != m;
    const int xo0 = RP::at(tl - base + q0);
    const float* xl = xs + xo0;
    // pass 1 (lanes before `last` feed the scan; their chunks are full):
    // lane 0 starts from the lap's entering state, the others from zero
    f2 bP = l * m0, bT = tr * m0;
    M2 Mm = {one, zero, zero, one};
    // the step loops read their samples in groups of 8 issued together: the
    // lap-uniform branches split every step into its own basic block, so the
    // compiler would otherwise wait on each step's LDS read in turn
    float xg[8];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (j % 8 == 0) {
        if (j > 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 8 && j + k < C; ++k) xg[k] = xl[(j + k) + ((j + k) >> RP::S)];
      }
      const float xq = xg[j % 8];
      const f2 u = xq - s[j];
      f2 e = u - bP;
      const f2 w = bP + bT;
      if (gaps) {                             // uniform branch: missing sample -> J, no input
        asm volatile("");
        const bool fin = isfinite(xq);
        e = fin ? e : zero;
        // Mm <- (J - k e1^T) Mm with k = (c, a b) on a sample, 0 when missing
        const f2 kP = fin ? cc : zero, kT = fin ? ab : zero;
        const f2 w0 = Mm.a + Mm.c, w1 = Mm.b + Mm.d;
        const f2 na = w0 - kP * Mm.a, nb = w1 - kP * Mm.b;
        Mm.c = Mm.c - kT * Mm.a;
        Mm.d = Mm.d - kT * Mm.b;
        Mm.a = na;
        Mm.b = nb;
      }
      bP = __builtin_elementwise_fma(cc, e, w);
      bT = __builtin_elementwise_fma(ab, e, bT);
    }
    if (!gaps) {
      // full, finite chunks: lane i's window at level d is A^{C d}
#pragma unroll
      for (int lv = 0; lv < NLV; ++lv) {
        const int d = 1 << lv;
        const f2 n0 = up(bP, d), n1 = up(bT, d);
        const f2 p0 = pwv[lv * 4 + 0], p1 = pwv[lv * 4 + 1], p2 = pwv[lv * 4 + 2], p3 = pwv[lv * 4 + 3];
        if (li >= d) {
          bP = bP + p0 * n0 + p1 * n1;
          bT = bT + p2 * n0 + p3 * n1;
        }
      }
    } else {
#pragma unroll
      for (int lv = 0; lv < NLV; ++lv) {
        const int d = 1 << lv;
        const M2 nm = {up(Mm.a, d), up(Mm.b, d), up(Mm.c, d), up(Mm.d, d)};
        const f2 n0 = up(bP, d), n1 = up(bT, d);
        if (li >= d) {
          bP = bP + Mm.a * n0 + Mm.b * n1;
          bT = bT + Mm.c * n0 + Mm.d * n1;
          Mm = mmul(Mm, nm);
        }
      }
    }
    // exclusive prefix: the state entering this lane's chunk (lane 0: the
    // lap's entering state; the shift brings lane 0 zeros)
    f2 P, Tt;
    if constexpr (LPP == 64) {
      P = __builtin_elementwise_fma(l, m0, up0(bP));
      Tt = __builtin_elementwise_fma(tr, m0, up0(bT));
    } else {
      // lane 32 reads lane 31 (the other half, possibly an idle lane's NaN):
      // selected, with the shifts taken first in uniform control flow (inside
      // a ?: arm the DPP would run under a divergent exec mask, and a DPP read
      // from an inactive lane returns 0)
      const f2 shP = up0(bP), shT = up0(bT);
      P = li == 0 ? l : shP;
      Tt = li == 0 ? tr : shT;
    }
    int xo = xo0;
    asm volatile("" : "+v"(xo));
    xl = xs + xo;
    f2 acc = accp;
    int nn = 0;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (j % 8 == 0) {
        if (j > 0) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 8 && j + k < C; ++k) xg[k] = xl[(j + k) + ((j + k) >> RP::S)];
      }
      const float xq = xg[j % 8];
      const f2 d = xq - s[j];                 // off the critical path
      f2 e = d - P;
      f2 w = P + Tt;
      if (gen2) {                             // uniform branch: inactive steps are exact no-ops,
        asm volatile("");                     // missing samples leave e = 0
        const bool act = j < cnt;
        const bool fin = act && isfinite(xq);
        w = act ? w : P;
        e = fin ? e : zero;
        nn += fin ? 1 : 0;
      }
      P = __builtin_elementwise_fma(cc, e, w);
      Tt = __builtin_elementwise_fma(ab, e, Tt);
      s[j] = __builtin_elementwise_fma(gs, e, s[j]);
      acc = __builtin_elementwise_fma(e, e, acc);
    }
    accp = acc;
    n += gen2 ? nn : C;
    if constexpr (LPP == 64) {
      l = rdl(P, last);
      tr = rdl(Tt, last);
    } else {                                  // each half reads its own last lane
      l = bperm2(P, (lane & ~(LPP - 1)) + last);
      tr = bperm2(Tt, (lane & ~(LPP - 1)) + last);
    }
    if (pr_on && lap + 1 == plap) {           // workgroup-uniform: every wave runs the same laps
      const f2 a = q0 < m ? accp : zero;
      const float pa = group_sum<LPP>(a.x), pb = group_sum<LPP>(a.y);
      __syncthreads();                        // (psse reuses the setup's season sums)
      if (li == 0 && pvalid) {
        psse[ga] = pa;
        psse[gb] = pb;
      }
      __syncthreads();
      const int gk = min(G, 2 * (pass + 1) * SL);     // candidates with a partial so far
      const float inf = __builtin_inff();
      float mn = lane < gk && isfinite(psse[lane]) ? psse[lane] : inf;
      mn = fminf(mn, xor_lane<1>(mn)); mn = fminf(mn, xor_lane<2>(mn)); mn = fminf(mn, xor_lane<4>(mn));
      mn = fminf(mn, xor_lane<8>(mn)); mn = fminf(mn, xor_lane<16>(mn)); mn = fminf(mn, xor_lane<32>(mn));
      const float lim = prune * mn;
      if (pvalid && mn > 0.f && mn < inf && pa > lim && pb > lim) {
        pruned = true;
        break;
      }
    }
  }
  l = l - tr;                                 // (P, T) -> (level, trend)
  if (q0 >= m) { accp = zero; n = 0; }        // idle lanes ran past the season
  ea = accp.x;
  eb = accp.y;
  } else {
#pragma unroll 1
  for (int tl = base + m; tl < T; tl += m) {
    // re-read the powers every lap (an opaque offset keeps the compiler from
    // hoisting 24 loop-invariant LDS loads into 48 live VGPRs)
    int pwo = slot * kLevels * 4;
    if constexpr (LPP == 64) asm volatile("" : "+s"(pwo));
    else asm volatile("" : "+v"(pwo));
    const f2* pwv = pw + pwo;
    const int nact = min(m, T - tl);
    const int last = (nact - 1) / C;          // lane holding the lap's last step
    const int cnt = nact - q0;                // active steps of this lane (may be <= 0 or > C)
    const float* xl = xs + RP::at(tl - base + q0);   // reassigned for pass 2
    // lane 0 folds the lap's entering state into its chunk, so the scanned
    // prefix of lanes 0..i-1 IS the state entering lane i (no carry matrix)
    const f2 l0 = li == 0 ? l : zero, t0v = li == 0 ? tr : zero;
    bool bad = false;
    bool gaps = false;                      // FS: the staging flagged a missing sample in this lap
    if constexpr (FS) gaps = lapnan[(tl - base - m) / m] != 0;
    f2 b0 = l0, b1 = t0v;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (j % 8 == 0 && j > 0) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight (VGPRs)
      const float xq = xl[j + (j >> RP::S)];
      if constexpr (!FS) bad |= !isfinite(xq);
      const f2 u = xq - s[j];
      const f2 wb = b0 + b1;
      const f2 e = u - wb;
      b0 = __builtin_elementwise_fma(al, e, wb);
      b1 = __builtin_elementwise_fma(ab, e, b1);
    }
    // only the lanes before the last active one feed the scan
    if (FS ? !gaps : !__any(bad && lane < last)) {
      // those chunks are full and finite: lane i's window at level d is
      // A^{C d}, the same for every lane >= d
#pragma unroll
      for (int lv = 0; lv < NLV; ++lv) {
        const int d = 1 << lv;
        const f2 n0 = up(b0, d), n1 = up(b1, d);
        const f2 p0 = pwv[lv * 4 + 0], p1 = pwv[lv * 4 + 1], p2 = pwv[lv * 4 + 2], p3 = pwv[lv * 4 + 3];
        if (li >= d) {
          b0 = b0 + p0 * n0 + p1 * n1;
          b1 = b1 + p2 * n0 + p3 * n1;
        }
      }
    } else {
      // general chunks: explicit 2x2 maps (missing or inactive step: J, no input)
      M2 Mm = {one, zero, zero, one};
      b0 = l0;
      b1 = t0v;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (j % 8 == 0 && j > 0) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight (VGPRs)
        const float xq = xl[j + (j >> RP::S)];
        const bool fin = j < cnt && isfinite(xq);
        const f2 u = xq - s[j];
        const f2 wb = b0 + b1;
        const f2 e = fin ? u - wb : zero;
        b0 = __builtin_elementwise_fma(al, e, wb);
        b1 = __builtin_elementwise_fma(ab, e, b1);
        const f2 ka = fin ? al : zero, kb = fin ? ab : zero;
        const f2 w0 = Mm.a + Mm.c, w1 = Mm.b + Mm.d;
        Mm.a = w0 - ka * w0;
        Mm.b = w1 - ka * w1;
        Mm.c = Mm.c - kb * w0;
        Mm.d = Mm.d - kb * w1;
      }
#pragma unroll
      for (int lv = 0; lv < NLV; ++lv) {
        const int d = 1 << lv;
        const M2 nm = {up(Mm.a, d), up(Mm.b, d), up(Mm.c, d), up(Mm.d, d)};
        const f2 n0 = up(b0, d), n1 = up(b1, d);
        if (li >= d) {
          b0 = b0 + Mm.a * n0 + Mm.b * n1;
          b1 = b1 + Mm.c * n0 + Mm.d * n1;
          Mm = mmul(Mm, nm);
        }
      }
    }
    // exclusive prefix: the (level, trend) entering this lane's chunk
    f2 L = up(b0, 1), Tt = up(b1, 1);
    if (li == 0) { L = l; Tt = tr; }
    // re-read the lap's samples (an opaque offset: otherwise the compiler keeps
    // pass 1's C loads live across the scan)
    int xo = RP::at(tl - base + q0);
    asm volatile("" : "+v"(xo));
    xl = xs + xo;
    f2 acc = zero;
    int nn = 0;
    if (EXACT && nact == m && (FS ? !gaps : !__any(bad && q0 < m))) {
      // full lap without a missing sample, m = C * (lanes in use): no
      // inactive or missing step in a used lane, so no per-step select
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (j % 8 == 0 && j > 0) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight (VGPRs)
        const float xq = xl[j + (j >> RP::S)];
        const f2 lt = L + Tt;
        const f2 e = xq - (lt + s[j]);
        L = __builtin_elementwise_fma(al, e, lt);
        Tt = __builtin_elementwise_fma(ab, e, Tt);
        s[j] = __builtin_elementwise_fma(gs, e, s[j]);
        acc = __builtin_elementwise_fma(e, e, acc);
      }
      nn = C;
      if (q0 >= m) { acc = zero; nn = 0; }   // idle lanes ran the next lap's samples
    } else if (EXACT && nact == m) {
      // full lap, m = C * (lanes in use): no inactive step in a used lane
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (j % 8 == 0 && j > 0) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight (VGPRs)
        const float xq = xl[j + (j >> RP::S)];
        const bool fin = isfinite(xq);
        const f2 lt = L + Tt;
        const f2 pred = lt + s[j];
        const f2 e = fin ? xq - pred : zero;
        L = __builtin_elementwise_fma(al, e, lt);
        Tt = __builtin_elementwise_fma(ab, e, Tt);
        s[j] = __builtin_elementwise_fma(gs, e, s[j]);
        acc = __builtin_elementwise_fma(e, e, acc);
        nn += fin ? 1 : 0;
      }
      if (q0 >= m) { acc = zero; nn = 0; }   // idle lanes ran the next lap's samples
    } else {
      // inactive steps are exact no-ops (lt = L, e = 0), so the last active
      // lane ends on the lap's end state
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (j % 8 == 0 && j > 0) __builtin_amdgcn_sched_barrier(0);   // bound the loads in flight (VGPRs)
        const float xq = xl[j + (j >> RP::S)];
        const bool act = j < cnt;
        const bool fin = act && isfinite(xq);
        const f2 lt = __builtin_elementwise_fma(Tt, (f2){act ? 1.f : 0.f, act ? 1.f : 0.f}, L);
        const f2 pred = lt + s[j];
        const f2 e = fin ? xq - pred : zero;
        L = __builtin_elementwise_fma(al, e, lt);
        Tt = __builtin_elementwise_fma(ab, e, Tt);
        s[j] = __builtin_elementwise_fma(gs, e, s[j]);
        acc = __builtin_elementwise_fma(e, e, acc);
        nn += fin ? 1 : 0;
      }
    }
    ea += acc.x;
    eb += acc.y;
    n += nn;
    if constexpr (LPP == 64) {
      l = rdl(L, last);
      tr = rdl(Tt, last);
    } else {                                 // each half reads its own last lane
      l = bperm2(L, (lane & ~(LPP - 1)) + last);
      tr = bperm2(Tt, (lane & ~(LPP - 1)) + last);
    }
  }
  }  // !FS
  if (probe != nullptr) pc2 = clock64();
  // lanes' fp64 lap sums, reduced across the lanes in fp32 (the SSE is fp32)
  float fa = group_sum<LPP>((float)ea), fb = group_sum<LPP>((float)eb);
  n = __builtin_amdgcn_readfirstlane(group_sum<LPP>(n));   // the same for every candidate
  if (pruned) {
    fa = fb = __builtin_inff();
  } else if (pr_on && lane == 0) {
    *nfull = n;
  }

  // ---- per-candidate results
  const float tph = (float)(T % m);
  if (li == 0 && pvalid) {
    const int64_t pa = row * G + ga;
    sse[pa] = fa;
    state[pa * 3 + 0] = l.x;
    state[pa * 3 + 1] = tr.x;
    state[pa * 3 + 2] = tph;
    nobs[pa] = n;
    sse_s[ga] = fa;
    if (2 * pair + 1 < G) {
      const int64_t pb = pa + 1;
      sse[pb] = fb;
      state[pb * 3 + 0] = l.y;
      state[pb * 3 + 1] = tr.y;
      state[pb * 3 + 2] = tph;
      nobs[pb] = n;
      sse_s[gb] = fb;
    }
  }
  __syncthreads();
  if (probe != nullptr) pcs = clock64();
  // ---- the best candidate so far: this pass covers candidates [g0, g1), so
  // continuing the ascending scan picks as one scan over all G would
  // (hw2_forecast_kernel's rule); a new winner parks its state in LDS
  // The rule's outcome over [0, g1): the first smallest finite SSE, else the
  // last candidate -- one lane per candidate (G <= 32), a wave min and two ballots
  const int g0 = 2 * pass * SL, g1 = min(G, 2 * (pass + 1) * SL);
  {
    const float inf = __builtin_inff();
    const float v = lane < g1 ? sse_s[lane] : inf;
    const bool fv = lane < g1 && isfinite(v);
    float mn = fv ? v : inf;
    mn = fminf(mn, xor_lane<1>(mn)); mn = fminf(mn, xor_lane<2>(mn)); mn = fminf(mn, xor_lane<4>(mn));
    mn = fminf(mn, xor_lane<8>(mn)); mn = fminf(mn, xor_lane<16>(mn)); mn = fminf(mn, xor_lane<32>(mn));
    const uint64_t at_min = __ballot(fv && v == mn);
    if (at_min != 0) {
      bg = (int)__builtin_ctzll(at_min);
      bs = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, mn)));
    } else {
      bg = g1 - 1;
      bs = sse_s[g1 - 1];
    }
    bs = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, bs)));
    bg = __builtin_amdgcn_readfirstlane(bg);
  }
  if (bg >= g0 && (bg >> 1) == pair && pvalid) {
    const bool hi = (bg & 1) != 0;
    int p = (base + q0p) % m;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (q0p + j < m) sbst[p] = hi ? s[j].y : s[j].x;     // seasons by absolute phase
      p = p + 1 == m ? 0 : p + 1;
    }
    if (li == 0) {
      lbt[0] = hi ? l.y : l.x;
      lbt[1] = hi ? tr.y : tr.x;
    }
  }
  }  // passes
  __syncthreads();
  // the winner's forecast and seasons, spread over the whole workgroup
  if (pr_on) n = *nfull;                       // (this wave's own count may be a pruned fit's)
  {
    const float lb = lbt[0], tb = lbt[1];
    const int t0 = T % m;
    float* fcr = fc + row * H;
    for (int h = 1 + tid; h <= H; h += nth) {
      int p = t0 + h - 1;
      while (p >= m) p -= m;
      fcr[h - 1] = lb + h * tb + sbst[p];
    }
    if (season_out != nullptr) {
      float* so = season_out + row * m;
      for (int p = tid; p < m; p += nth) so[p] = sbst[p];
    }
    if (tid == 0) {
      sigma[row] = n > 1 ? sqrtf(bs / (float)(n - 1)) : 0.f;
      best[row] = bg;
      sscale[row] = 1.f;
      if (nfin != nullptr) nfin[row] = c1 + n;
    }
  }
  if constexpr (FS) __builtin_amdgcn_s_waitcnt(0);   // no L2 warm-up DMA outlives the workgroup's LDS
  if (probe != nullptr && lane == 0) {
    // phase timing (fm_hw_scan_set_probe), per wave: clocks at start, after
    // the first barrier, at the laps, after the laps, after the selection
    // barrier and at exit; the wall clock at start; HW_ID (SIMD, CU, SE)
    long long* pr = probe + (row * 16 + w) * 8;
    pr[0] = pc0; pr[1] = pcb; pr[2] = pc1; pr[3] = pc2; pr[4] = pcs; pr[5] = clock64();
    const unsigned hwid = __builtin_amdgcn_s_getreg((31 << 11) | 4);     // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);      // HW_REG_XCC_ID [3:0]
    pr[6] = pw0; pr[7] = ((long long)xcc << 32) | hwid;
  }
}

namespace {
constexpr int kChunks[] = {4, 5, 6, 8, 9, 12, 16, 18, 20, 23, 24};
constexpr int kHalfMaxM = 32 * 24;       // seasons up to this length scan in 32-lane half-waves

constexpr size_t kMaxLds = 160 * 1024;   // a single gfx950 workgroup may take the whole LDS
constexpr int kPassWaves = 8;            // waves per row when candidates run in passes (2 rows / CU)

template <int C, bool EXACT, bool FS, int LPP>
void allow_big_lds() {
  static bool done = false;            // once per instantiation (idempotent if raced)
  if (!done) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(hw_scan_fit_kernel<C, EXACT, FS, LPP>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)kMaxLds);
    done = true;
  }
}

// FOREMAST_HW_SCAN_SETUP=0: the original setup (per-wave season means, A^C by
// C - 1 products, per-step NaN ballots; one pair per wave) for A/B runs
bool scan_fast_setup() {
  static const bool fs = [] {
    const char* e = getenv("FOREMAST_HW_SCAN_SETUP");
    return e == nullptr || e[0] != '0';
  }();
  return fs;
}

// FOREMAST_HW_SCAN_PASSES=1: one pass over the candidate pairs (one wave per
// pair, one row per CU at config 2) for A/B runs
bool scan_passes_allowed() {
  static const bool ok = [] {
    const char* e = getenv("FOREMAST_HW_SCAN_PASSES");
    return e == nullptr || e[0] != '1';
  }();
  return ok;
}

// lanes per candidate pair for a season of m steps
int scan_lpp(int m) {
  static const int force = [] {
    const char* e = getenv("FOREMAST_HW_SCAN_LPP");
    return e == nullptr ? 0 : atoi(e);
  }();
  // half-wave pairs for short seasons (FOREMAST_HW_SCAN_LPP=64 for A/B runs):
  // 40k rows x 10,080, m = 288: 5.36 vs 11.3 ms; m = 720: 4.36 vs 6.37 ms
  // (profiles/hw_scan_halfwave_ab_r3.jsonl)
  if (!scan_fast_setup() || force == 64) return 64;
  return m <= kHalfMaxM ? 32 : 64;
}

int scan_debug() {
  static const int d = [] {
    const char* e = getenv("FOREMAST_HW_SCAN_DEBUG");
    return e == nullptr ? 0 : atoi(e);
  }();
  return d;
}

long long* g_probe = nullptr;            // fm_hw_scan_set_probe: [R, 16, 8] int64 phase timings, or null

template <int C>
int launch_one(const float* x, int64_t ld, int T, int64_t R, const float* cand, int G, int m, int H, float* sse,
               float* state, int* nobs, float* fc, float* sigma, int* best, int* nfin, float* sscale,
               float* season_out, size_t lds, int xal, int lpp, int npass, int s0, float prune, int plap,
               hipStream_t stream) {
  const int GP = (G + 1) / 2;
  const int slots = lpp == 64 ? GP : (GP + 1) / 2;          // waves for one pass over the pairs
  const int waves = (slots + npass - 1) / npass;
  const bool fs = scan_fast_setup();
  // L2 warm-up distance: the workgroups resident at once (one per CU at 14
  // waves), a multiple of the 8 XCDs so the warmed row is read on the same XCD
  static const int ahead = [] {
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const char* e = getenv("FOREMAST_HW_SCAN_AHEAD");
    return e != nullptr ? atoi(e) : (cus / 8) * 8;
  }();
#define FM_HWS_LAUNCH(EX, FSV, LP)                                                                          \
  do {                                                                                                     \
    if (lds > 65536) allow_big_lds<C, EX, FSV, LP>();                                                       \
    hipLaunchKernelGGL((hw_scan_fit_kernel<C, EX, FSV, LP>), dim3((unsigned)R), dim3(64 * waves), lds, stream, x, \
                       ld, T, cand, G, m, H, sse, state, nobs, fc, sigma, best, nfin, sscale, season_out, xal,  \
                       R, ahead * (npass > 1 ? 2 : 1), npass | (scan_debug() << 8) | (s0 << 16), g_probe,   \
                       prune, plap);                                                                        \
  } while (0)
  const bool ex = m % C == 0;
  if (lpp == 32) {
    if (ex) FM_HWS_LAUNCH(true, true, 32);
    else FM_HWS_LAUNCH(false, true, 32);
  } else if (ex && fs) FM_HWS_LAUNCH(true, true, 64);
  else if (ex) FM_HWS_LAUNCH(true, false, 64);
  else if (fs) FM_HWS_LAUNCH(false, true, 64);
  else FM_HWS_LAUNCH(false, false, 64);
#undef FM_HWS_LAUNCH
  FM_LAUNCH_CHECK();
  return 0;
}

// Additive Holt-Winters grid fit + best-candidate forecast in one launch
// (one workgroup per row).  Same outputs as fm_es_fit(kind = 2) --
// sse [R, G], state [R*G, 3], nobs [R*G], fc [R, H], sigma / best / nfin [R],
// sscale [R] (= 1: data units) -- plus, when season_out is not null, the best
// candidate's seasonal indices [R, m] by absolute phase.  Returns
// hipErrorInvalidValue for shapes it does not cover (the caller then uses the
// serial kernel): m > 64 * 24 or m < 192 (chunks of 4..24 steps per lane; seasons
// up to 768 steps run two candidate pairs per wave, 32 lanes each),
// G > 32, 2 m > T, or a row beyond the 160 KB of LDS a workgroup may take.
// The plan of a scan fit for (T, G, m): chunk length C, lanes per pair and
// the dynamic LDS bytes, or C = 0 when the shape is not covered.  One place
// decides, for the launcher and for the Python-side shape query
// (fm_hw_scan_supported), so the two can never disagree.
struct ScanPlan {
  int C = 0, lpp = 64, npass = 1, s0 = 0;
  size_t lds = 0;
};

ScanPlan scan_plan(int T, int G, int m) {
  ScanPlan p;
  if (G < 1 || G > kMaxG || m < 2 || 2 * m > T) return p;
  const int lpp = scan_lpp(m);
  const int need = (m + lpp - 1) / lpp;
  int C = 0;
  // 9 and 18 (the 32-lane chunks of 288 / 576-step seasons) only for half-waves:
  // the one-pair-per-wave kernel keeps its measured chunk choice
  auto usable = [lpp](int c) { return lpp == 32 || (c != 9 && c != 18); };
  for (int c : kChunks)                      // an exact chunk (no masked steps in full laps) ...
    if (usable(c) && c >= need && m % c == 0) { C = c; break; }
  if (C == 0)
    for (int c : kChunks)                    // ... else the shortest that covers the lap
      if (usable(c) && c >= need) { C = c; break; }
  if (C == 0 || m < 3 * 64) return p;
  const int GP = (G + 1) / 2;
  const int S = (m % C == 0 && C % 4 == 0) ? __builtin_ctz(C) : 31;   // RowPad<C, EXACT>::S
  const size_t words = ((size_t)(T + 64 * C) + (S < 31 ? (size_t)(T + 64 * C) >> S : 0) + 1 + 3) & ~(size_t)3;
  const size_t lds = words * 4 + (size_t)(kMaxG / 2) * kLevels * 8 * 4 + kMaxG * 4 + 16 + kMaxLaps * 4 + 16 * 4 * 4 + 64 * 4 +
                     32 * 4 + (size_t)((m + 3) & ~3) * 4;   // wsum | DMA landing zone | wmin, lbt | seasons
  if (lds > kMaxLds || (T - m) / m >= kMaxLaps) return p;
  p.C = C;
  p.lpp = lpp;
  p.lds = lds;
  // candidate passes: a row's waves beyond kPassWaves leave room for one
  // workgroup per CU (4 waves / SIMD at 128 VGPRs); in passes of at most
  // kPassWaves waves two rows share a CU when their LDS fits twice
  const int slots = lpp == 64 ? GP : (GP + 1) / 2;
  if (scan_fast_setup() && slots > kPassWaves && 2 * lds <= kMaxLds && scan_passes_allowed())
    p.npass = (slots + kPassWaves - 1) / kPassWaves;
  // the first-season pairs (C x lpp, FS) when they fit beside the row (and
  // keep two rows per CU when the candidates run in passes)
  const size_t s0b = (size_t)C * lpp * 8;
  if (scan_fast_setup() && (p.npass > 1 ? 2 : 1) * (lds + s0b) <= kMaxLds) {
    p.lds = lds + s0b;
    p.s0 = 1;
  }
  return p;
}
}  // namespace

// Phase-timing buffer for the next fits (tools/hw_scan_probe.py): [R, 16
// waves, 8] int64, null to switch it off.
FM_API int fm_hw_scan_set_probe(void* p) {
  g_probe = static_cast<long long*>(p);
  return 0;
}

// 1 when fm_hw_scan_fit covers (T, G, m) in this process (environment
// overrides included, read once), else 0.
FM_API int fm_hw_scan_supported(int T, int G, int m) { return scan_plan(T, G, m).C != 0; }

//
// ``prune`` > 0 (FS plans with one candidate pair per wave): after ``plap``
// season laps (0: a third of the row's laps, at least 3 laps needed) a pair
// whose two partial SSEs both exceed prune x the smallest partial so far stops
// fitting; its candidates report SSE = inf (never selected), their state /
// nobs are partial.  prune <= 0: the exact full grid.
FM_API int fm_hw_scan_fit(const float* x, int64_t ld, int T, int64_t R, const float* cand, int G, int m, int H,
                          float* sse, float* state, int* nobs, float* fc, float* sigma, int* best, int* nfin,
                          float* sscale, float* season_out, float prune, int plap, hipStream_t stream) {
  if (R <= 0) return 0;
  if (H < 0) return (int)hipErrorInvalidValue;
  const ScanPlan pl = scan_plan(T, G, m);
  if (pl.C == 0) return (int)hipErrorInvalidValue;
  const int C = pl.C, lpp = pl.lpp, npass = pl.npass, s0 = pl.s0;
  const size_t lds = pl.lds;
  const int xal = ((uintptr_t)x % 16 == 0) && (ld % 4 == 0);
  if (plap <= 0) plap = (T - m) / m >= 3 ? (T - m) / m / 3 : 0;
  if (prune <= 0.f || plap <= 0) {
    prune = 0.f;
    plap = 0;
  }
#define FM_HWS(CC)                                                                                         \
  case CC:                                                                                                 \
    return launch_one<CC>(x, ld, T, R, cand, G, m, H, sse, state, nobs, fc, sigma, best, nfin, sscale,    \
                          season_out, lds, xal, lpp, npass, s0, prune, plap, stream);
  switch (C) {
    FM_HWS(4) FM_HWS(5) FM_HWS(6) FM_HWS(8) FM_HWS(9) FM_HWS(12) FM_HWS(16) FM_HWS(18) FM_HWS(20) FM_HWS(23)
    FM_HWS(24)
    default: return (int)hipErrorInvalidValue;
  }
#undef FM_HWS
}
