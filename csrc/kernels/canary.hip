// fm-hipcc-flags: -mllvm -pragma-unroll-threshold=1000000
// (the 1024-sample pairwise sort, K = 16: past LLVM's default pragma-unroll
// size limit the stage loops stayed rolled -- runtime register indexing
// through scratch (132 B/lane) and s_set_gpr_idx; fully unrolled: 0 scratch)
// Canary-scoring kernels (K4 pairwise rank tests, K1+K7 fused history-stats +
// anomaly decision, service reduce, anomaly compaction, K11 synthetic fleet).
//
// Reference behaviour being rebuilt (foremast-brain is external; see
// docs/BRAIN_SPEC.md): per (service, metric) the brain fits a historical model
// (ML_ALGORITHM=moving_average_all, deploy/foremast/3_brain/foremast-brain.yaml:24-25),
// compares canary vs baseline with pairwise tests (foremast-brain/README.md:32-38,
// docs/guides/design.md:35) and flags current points outside the bounds
// (design.md:43, fail fast).
//
// Layout: rows = services x metrics, row r -> metric r % M.  history [R, ld_h]
// fp32 (NaN = missing sample), current [R, ld_c], baseline [R, ld_b].
#include "fm_common.h"

using namespace fm;

// ---------------------------------------------------------------------------
// K4: pairwise tests. One wave per (service, metric) row, 4 rows per 256-thread
// workgroup.  The pooled sample (n1 + n2 <= 64*K) is sorted in registers with a
// bitonic network (in-register swaps for strides >= 64, __shfl_xor below),
// average ranks with ties come from a max-scan / suffix-min-scan over tie runs.
// ---------------------------------------------------------------------------
namespace {

constexpr float kPad = INFINITY;

// SPLIT (K == 2 only): register 0 holds sample 1 and register 1 sample 2
// (each <= 64 values).  Every stage up to size 64 then stays inside one
// register, so a value's sample is its register index and the tags need no
// exchange; they are rebuilt (k, or -1 for pads) before the final 128-merge.
// That drops the tag exchange and select from 21 of the 27 lane-exchange
// steps.
template <int K, bool SPLIT = false>
__device__ __forceinline__ void bitonic_sort(float (&v)[K], int (&tag)[K]) {
  // Branch-free compare-exchange (selects, no exec-mask branches): strides
  // >= 64 swap registers inside the lane, smaller strides exchange with the
  // partner lane through DPP / permlane (xor_lane_any).
  static_assert(!SPLIT || K == 2, "split layout is two 64-lane registers");
  const int lane = lane_id();
#pragma unroll
  for (int size = 2; size <= 64 * K; size <<= 1) {
    const bool tags = !SPLIT || size > 64;
    if (SPLIT && size == 128) {
#pragma unroll
      for (int k = 0; k < K; ++k) tag[k] = v[k] == kPad ? -1 : k;
    }
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      if (stride >= 64) {
        const int ks = stride / 64;
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int p = k ^ ks;
          if (p > k) {
            const int i = k * 64 + lane;
            const bool asc = (i & size) == 0;
            const float a = v[k], b = v[p];
            const int ta = tag[k], tb = tag[p];
            const bool alt = a < b;
            const float mn = alt ? a : b, mx = alt ? b : a;
            const int tmn = alt ? ta : tb, tmx = alt ? tb : ta;
            v[k] = asc ? mn : mx; v[p] = asc ? mx : mn;
            tag[k] = asc ? tmn : tmx; tag[p] = asc ? tmx : tmn;
          }
        }
      } else {
        float ov[K];
        int ot[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
          ov[k] = xor_lane_any(v[k], stride);
          ot[k] = tags ? xor_lane_any(tag[k], stride) : 0;
        }
#pragma unroll
        for (int k = 0; k < K; ++k) {
          const int i = k * 64 + lane;
          const bool asc = (i & size) == 0;
          const bool lower = (lane & stride) == 0;
          // keep the smaller value in the lower lane of an ascending pair
          const bool keep_min = lower == asc;
          // select min or max of the pair; the tag follows only when the value
          // actually moved (equal values keep their own tags on both lanes)
          const bool vlt = v[k] < ov[k];
          const float mn = vlt ? v[k] : ov[k], mx = vlt ? ov[k] : v[k];
          const float nv = keep_min ? mn : mx;
          if (tags) tag[k] = nv != v[k] ? ot[k] : tag[k];
          v[k] = nv;
        }
      }
    }
  }
}

// Average (1-based) ranks for a sorted register array whose first n entries are
// real.  tie_term accumulates sum(t^3 - t) over tie runs; is_end marks the last
// element of each run (where empirical CDFs are evaluated).
template <int K>
__device__ __forceinline__ void avg_ranks(const float (&v)[K], int n, int (&rank2)[K], bool (&is_end)[K],
                                          int& tie_term) {
  // rank2 = 2 x (1-based average rank) = start + end + 2: exact integers, so
  // rank sums and the tie term sum(t^3 - t) (<= 1024^3 < 2^31) need no doubles.
  const int lane = lane_id();
  int start_idx[K];
  int carry = 0;
  float last_prev = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * 64 + lane;
    const float prev = lane_prev(v[k], last_prev);
    const bool st = (i == 0) || (v[k] != prev);
    int s = st ? i : 0;
    s = wave_incl_max(s, 0);
    s = s > carry ? s : carry;
    start_idx[k] = s;
    carry = lane_bcast(s, 63);
    last_prev = lane_bcast(v[k], 63);
  }
  int carry_e = 0x7fffffff;
  float next_first = 0.f;
  int tl = 0;
#pragma unroll
  for (int k = K - 1; k >= 0; --k) {
    const int i = k * 64 + lane;
    const float next = lane_next(v[k], next_first);
    const bool en = (i < n) && ((i == n - 1) || (v[k] != next));
    int e = en ? i : 0x7fffffff;
    e = wave_incl_suffix_min(e, 0x7fffffff);
    e = e < carry_e ? e : carry_e;
    carry_e = lane_bcast(e, 0);
    next_first = lane_bcast(v[k], 0);
    is_end[k] = en;
    rank2[k] = start_idx[k] + e + 2;
    if (i < n && i == start_idx[k]) {
      const int t = e - start_idx[k] + 1;
      tl += t * t * t - t;
    }
  }
  tie_term = wave_sum(tl);
}

}  // namespace

enum { T_MW = 0, T_WIL = 1, T_KRU = 2, T_KS = 3, T_T = 4, T_FRI = 5, N_TESTS = 6 };
constexpr int kSuff = 14;

// Per-row pairwise inputs, split into a LOAD half (raw samples into
// registers, no arithmetic that would wait on them) and a COMPUTE half, so a
// fused kernel can put other loads in flight between the two.
template <int K>
struct PwIn {
  static constexpr int KW = (K + 1) / 2;
  float v[K];     // pooled sample slot i = k*64 + lane: cur[i] (i < n_cur) or base[i - n_cur]
  float pc[KW];   // position-paired cur[j], base[j] (Wilcoxon / Friedman)
  float pb[KW];
};

// SPLIT (K == 2, n_cur <= 64, n_base <= 64): v[0] = current, v[1] = baseline
// instead of the pooled order (see bitonic_sort).
template <int K, bool SPLIT = false>
__device__ __forceinline__ void pw_load(const float* __restrict__ c, const float* __restrict__ b, int n_cur,
                                        int n_base, PwIn<K>& in) {
  const int lane = lane_id();
  if constexpr (SPLIT) {
    in.v[0] = lane < n_cur ? c[lane] : kPad;
    in.v[1] = lane < n_base ? b[lane] : kPad;
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int i = k * 64 + lane;
      in.v[k] = i < n_cur ? c[i] : (i < n_cur + n_base ? b[i - n_cur] : kPad);
    }
  }
  const int npair = n_cur < n_base ? n_cur : n_base;
#pragma unroll
  for (int k = 0; k < PwIn<K>::KW; ++k) {
    const int j = k * 64 + lane;
    in.pc[k] = j < npair ? c[j] : 0.f;
    in.pb[k] = j < npair ? b[j] : 0.f;
  }
}

template <int K, bool SPLIT = false>
__device__ __forceinline__ void pw_compute(PwIn<K>& in, int n_cur, int n_base, double* __restrict__ o) {
  // Everything exact is carried in integers (counts, doubled rank sums, tie
  // terms, the KS numerator); only the Welch moments are floating point.
  const int lane = lane_id();
  float (&v)[K] = in.v;
  int tag[K];
  float s1 = 0.f, s2 = 0.f;
  int c12 = 0;  // n1 | n2 << 16
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * 64 + lane;
    int t = SPLIT ? (lane < (k == 0 ? n_cur : n_base) ? k : -1) : (i < n_cur ? 0 : (i < n_cur + n_base ? 1 : -1));
    float x = v[k];
    if (!isfinite(x)) { x = kPad; t = -1; }
    v[k] = x; tag[k] = t;
    if (t == 0) { s1 += x; c12 += 1; }
    if (t == 1) { s2 += x; c12 += 1 << 16; }
  }
  c12 = wave_sum(c12);
  const int n1 = c12 & 0xFFFF, n2 = c12 >> 16;
  const int n = n1 + n2;
  const float m1 = wave_sum(s1) / (float)(n1 > 0 ? n1 : 1), m2 = wave_sum(s2) / (float)(n2 > 0 ? n2 : 1);
  float q1 = 0.f, q2 = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (tag[k] == 0) { const float d = v[k] - m1; q1 += d * d; }
    if (tag[k] == 1) { const float d = v[k] - m2; q2 += d * d; }
  }
  q1 = wave_sum(q1); q2 = wave_sum(q2);

  // ---- Wilcoxon signed-rank on position-paired differences (zero_method='wilcox')
  constexpr int KW = PwIn<K>::KW;
  float dv[KW];
  int dt[KW];
  const int npair = n_cur < n_base ? n_cur : n_base;
  int cwz = 0;  // nonzero | positive << 10 | zero << 20 (each <= 512)
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int j = k * 64 + lane;
    float d = kPad;
    int t = -1;
    if (j < npair) {
      const float xc = in.pc[k], xb = in.pb[k];
      if (isfinite(xc) && isfinite(xb)) {
        const float dd = xc - xb;
        if (dd != 0.f) { d = fabsf(dd); t = dd > 0.f ? 1 : 0; cwz += 1 + (t << 10); }
        else cwz += 1 << 20;
      }
    }
    dv[k] = d; dt[k] = t;
  }
  cwz = wave_sum(cwz);
  const int nw = cwz & 0x3FF, npos = (cwz >> 10) & 0x3FF, nzero = cwz >> 20;

  bitonic_sort<K, SPLIT>(v, tag);
  int rk2[K];
  bool en[K];
  int tie = 0;
  avg_ranks<K>(v, n, rk2, en, tie);

  int r1x2 = 0;
  int dnum = 0;   // max |a1 n2 - a2 n1| over tie-run ends = D n1 n2
  int base12 = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (tag[k] == 0) r1x2 += rk2[k];
    // KS: inclusive prefix counts of both samples along the sorted order, one packed scan
    const int a12 = wave_incl_sum(tag[k] == 0 ? 1 : (tag[k] == 1 ? (1 << 16) : 0)) + base12;
    base12 = lane_bcast(a12, 63);
    if (en[k] && n1 > 0 && n2 > 0) {
      const int a1 = a12 & 0xFFFF, a2 = a12 >> 16;
      const int dd = abs(a1 * n2 - a2 * n1);
      dnum = dd > dnum ? dd : dnum;
    }
  }
  r1x2 = wave_sum(r1x2);
  dnum = wave_max(dnum);

  bitonic_sort<KW>(dv, dt);
  int rw2[KW];
  bool ew[KW];
  int tiew = 0;
  avg_ranks<KW>(dv, nw, rw2, ew, tiew);
  int rplus2 = 0;
#pragma unroll
  for (int k = 0; k < KW; ++k)
    if (dt[k] == 1) rplus2 += rw2[k];
  rplus2 = wave_sum(rplus2);

  // Per-row sufficient statistics; p-values are evaluated one row per THREAD
  // by pvalue_kernel (the double-precision special functions would otherwise
  // run on lane 0 with 63 lanes idle).
  if (lane == 0) {
    o[0] = n1; o[1] = n2; o[2] = nw; o[3] = 0.5 * r1x2; o[4] = tie;
    o[5] = (n1 > 0 && n2 > 0) ? (double)dnum / ((double)n1 * n2) : 0.0;
    o[6] = 0.5 * rplus2; o[7] = tiew; o[8] = m1; o[9] = m2; o[10] = q1; o[11] = q2;
    o[12] = npos; o[13] = nzero;
  }
}

// ---------------------------------------------------------------------------
// Counting form of the same statistics (no sort).  Every average rank is
// 2*rank = 2*#(v < x) + #(v == x) + 1, the KS empirical CDFs at x are the
// "<=" counts per sample, the tie term is sum over samples of (t_i^2 - 1)
// (t_i = size of x's tie run), and the Wilcoxon ranks are the same counts over
// the non-zero |d|.  The row's values go to LDS once; each lane then sweeps
// them with broadcast ds_read_b128 (4 values per instruction, one address for
// the whole wave: conflict-free), so the work is ~n independent compare/adds
// per owned value instead of the bitonic network's dependent exchange chain.
// ---------------------------------------------------------------------------
template <int K>
__device__ __forceinline__ void pw_compute_count(PwIn<K>& in, int n_cur, int n_base, double* __restrict__ o,
                                                 float* __restrict__ lds /* >= 3*64*K + 12 floats */) {
  constexpr int KW = PwIn<K>::KW;
  const int lane = lane_id();
  const int n = n_cur + n_base;
  const int nc4 = (n_cur + 3) & ~3, nb4 = (n_base + 3) & ~3;
  float* pc = lds;                      // current sample, +inf for missing / padding
  float* pb = lds + 64 * K + 4;         // baseline sample
  float* pd = lds + 128 * K + 8;        // |d| of non-zero pairs, +inf otherwise
  float x[K];
  int tag[K];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int i = k * 64 + lane;
    int t = i < n_cur ? 0 : (i < n ? 1 : -1);
    float v = in.v[k];
    if (!isfinite(v)) { v = kPad; t = -1; }
    x[k] = v; tag[k] = t;
    if (t == 0) s1 += v;
    if (t == 1) s2 += v;
    if (i < n_cur) pc[i] = v;
    else if (i < n) pb[i - n_cur] = v;
  }
  if (lane < 4) {
    if (n_cur + lane < nc4) pc[n_cur + lane] = kPad;
    if (n_base + lane < nb4) pb[n_base + lane] = kPad;
  }
  int n1 = 0, n2 = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    n1 += __popcll(__ballot(tag[k] == 0));
    n2 += __popcll(__ballot(tag[k] == 1));
  }
  const float m1 = wave_sum(s1) / (float)(n1 > 0 ? n1 : 1), m2 = wave_sum(s2) / (float)(n2 > 0 ? n2 : 1);
  float q1 = 0.f, q2 = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (tag[k] == 0) { const float d = x[k] - m1; q1 += d * d; }
    if (tag[k] == 1) { const float d = x[k] - m2; q2 += d * d; }
  }
  q1 = wave_sum(q1); q2 = wave_sum(q2);

  const int npair = n_cur < n_base ? n_cur : n_base;
  const int npp4 = (npair + 3) & ~3;
  float dabs[KW];
  int dsgn[KW];   // 1 positive, 0 negative, -1 excluded
  int npos = 0, nneg = 0, nzero = 0;
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int j = k * 64 + lane;
    float d = kPad;
    int t = -1;
    bool zero = false;
    if (j < npair) {
      const float xc = in.pc[k], xb = in.pb[k];
      if (isfinite(xc) && isfinite(xb)) {
        const float dd = xc - xb;
        if (dd != 0.f) { d = fabsf(dd); t = dd > 0.f ? 1 : 0; }
        else zero = true;
      }
    }
    dabs[k] = d; dsgn[k] = t;
    npos += __popcll(__ballot(t == 1));
    nneg += __popcll(__ballot(t == 0));
    nzero += __popcll(__ballot(zero));
    if (j < npp4) pd[j] = d;
  }
  const int nw = npos + nneg;
  __builtin_amdgcn_wave_barrier();   // LDS stores of this wave visible to its own reads
  __builtin_amdgcn_s_waitcnt(0xc07f);

  // pooled sample: per owned value, "<" and "==" counts against cur and base
  int lt_c[K], eq_c[K], lt_b[K], eq_b[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { lt_c[k] = 0; eq_c[k] = 0; lt_b[k] = 0; eq_b[k] = 0; }
  for (int j = 0; j < nc4; j += 4) {
    const float4 w = *reinterpret_cast<const float4*>(pc + j);
#pragma unroll
    for (int k = 0; k < K; ++k)
      lt_c[k] += (w.x < x[k]) + (w.y < x[k]) + (w.z < x[k]) + (w.w < x[k]),
      eq_c[k] += (w.x == x[k]) + (w.y == x[k]) + (w.z == x[k]) + (w.w == x[k]);
  }
  for (int j = 0; j < nb4; j += 4) {
    const float4 w = *reinterpret_cast<const float4*>(pb + j);
#pragma unroll
    for (int k = 0; k < K; ++k)
      lt_b[k] += (w.x < x[k]) + (w.y < x[k]) + (w.z < x[k]) + (w.w < x[k]),
      eq_b[k] += (w.x == x[k]) + (w.y == x[k]) + (w.z == x[k]) + (w.w == x[k]);
  }
  int r1x2 = 0, tie = 0, dnum = 0;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (tag[k] >= 0) {
      const int lt = lt_c[k] + lt_b[k], t = eq_c[k] + eq_b[k];
      if (tag[k] == 0) r1x2 += 2 * lt + t + 1;
      tie += t * t - 1;
      if (n1 > 0 && n2 > 0) {
        const int a1 = lt_c[k] + eq_c[k], a2 = lt_b[k] + eq_b[k];
        const int dd = abs(a1 * n2 - a2 * n1);
        dnum = dd > dnum ? dd : dnum;
      }
    }
  }
  r1x2 = wave_sum(r1x2);
  tie = wave_sum(tie);
  dnum = wave_max(dnum);

  // Wilcoxon ranks among the non-zero |d|
  int rp2 = 0, tiew = 0;
  {
    int ltw[KW], eqw[KW];
#pragma unroll
    for (int k = 0; k < KW; ++k) { ltw[k] = 0; eqw[k] = 0; }
    for (int j = 0; j < npp4; j += 4) {
      const float4 w = *reinterpret_cast<const float4*>(pd + j);
      const float wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < KW; ++k) ltw[k] += wv[u] < dabs[k], eqw[k] += wv[u] == dabs[k];
    }
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      if (dsgn[k] >= 0) {
        tiew += eqw[k] * eqw[k] - 1;
        if (dsgn[k] == 1) rp2 += 2 * ltw[k] + eqw[k] + 1;
      }
    }
  }
  rp2 = wave_sum(rp2);
  tiew = wave_sum(tiew);
  __builtin_amdgcn_wave_barrier();   // the LDS slot is reused by the next row

  if (lane == 0) {
    o[0] = n1; o[1] = n2; o[2] = nw; o[3] = 0.5 * r1x2; o[4] = tie;
    o[5] = (n1 > 0 && n2 > 0) ? (double)dnum / ((double)n1 * n2) : 0.0;
    o[6] = 0.5 * rp2; o[7] = tiew; o[8] = m1; o[9] = m2; o[10] = q1; o[11] = q2;
    o[12] = npos; o[13] = nzero;
  }
}

// One row's sufficient statistics (sort form): the split layout when both
// samples fit one register each (the usual 5 pods x 10 points per side).
template <int K>
__device__ __forceinline__ void pw_row(const float* __restrict__ c, const float* __restrict__ b, int n_cur,
                                       int n_base, double* __restrict__ o) {
  PwIn<K> in;
  if constexpr (K == 2) {
    if (n_cur <= 64 && n_base <= 64) {
      pw_load<K, true>(c, b, n_cur, n_base, in);
      pw_compute<K, true>(in, n_cur, n_base, o);
      return;
    }
  }
  pw_load<K>(c, b, n_cur, n_base, in);
  pw_compute<K>(in, n_cur, n_base, o);
}

template <int K>
__global__ __launch_bounds__(256) void pairwise_count_kernel(
    const float* __restrict__ cur, int64_t ld_c, int n_cur, const float* __restrict__ base, int64_t ld_b,
    int n_base, int64_t R, double* __restrict__ suff) {
  constexpr int KW = PwIn<K>::KW;
  constexpr int PER_WAVE = 3 * 64 * K + 12;
  __shared__ __attribute__((aligned(16))) float lds[4 * PER_WAVE];
  float* my = lds + wave_id() * PER_WAVE;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave_id(); row < R; row += (int64_t)gridDim.x * 4) {
    PwIn<K> in;
    pw_load<K>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, in);
    pw_compute_count<K>(in, n_cur, n_base, suff + row * kSuff, my);
  }
}

// Grid-stride over rows: launched with one wave per row, or capped to a few
// workgroups per CU so a concurrently running HBM-bound kernel keeps most of
// the wave slots (two-stream tick).
template <int K>
__global__ __launch_bounds__(256) void pairwise_kernel(
    const float* __restrict__ cur, int64_t ld_c, int n_cur, const float* __restrict__ base, int64_t ld_b,
    int n_base, int64_t R, double* __restrict__ suff) {
  for (int64_t row = (int64_t)blockIdx.x * 4 + wave_id(); row < R; row += (int64_t)gridDim.x * 4) {
    pw_row<K>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, suff + row * kSuff);
  }
}

// ---------------------------------------------------------------------------
// Fused canary row kernel: ONE wave per (service, metric) row does both the
// HBM-bound history statistics (mean / std / count over the 7-day row) and the
// compute-bound pairwise rank tests.  Order inside the wave: the small
// cur/base loads, then the whole history row (NQ float4 per lane, streamed,
// non-temporal), then the pairwise compute runs while the history is still in
// flight (vmcnt waits only for the first, small loads: in-order completion),
// then the history is reduced from registers.  The separate two-stream form
// (pairwise on a side stream || hist_stats) shares the CUs between two kernels
// whose waves compete for slots; here each wave carries both.
// ---------------------------------------------------------------------------
template <int NQ, int K>
__global__ __launch_bounds__(256) void canary_row_kernel(
    const float* __restrict__ hist, int64_t ld_h, int T, const float* __restrict__ cur, int64_t ld_c, int n_cur,
    const float* __restrict__ base, int64_t ld_b, int n_base, int64_t R, float* __restrict__ hs /*[R,3]*/,
    double* __restrict__ suff) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R) return;
  const int lane = lane_id();
  const bool do_pw = n_base > 0;
  PwIn<K> in;
  // same layout choice as pw_row, so every tick mode sums the Welch moments
  // in the same order (bit-identical p-values across modes)
  const bool split = K == 2 && n_cur <= 64 && n_base <= 64;
  if (do_pw) {
    if constexpr (K == 2) {
      if (split) pw_load<K, true>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, in);
      else pw_load<K>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, in);
    } else {
      pw_load<K>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, in);
    }
  }

  typedef float nt4 __attribute__((ext_vector_type(4)));
  const nt4* h = reinterpret_cast<const nt4*>(hist + row * ld_h);
  const int nq = (T + 3) >> 2;
  nt4 q[NQ];
  // Unpredicated loads (index clamped into the row, surplus masked by e0 < T
  // in the reduction): with exec-masked branches around them the waitcnt pass
  // could not prove how many loads are outstanding and waited for all of them
  // before the pairwise compute.
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int qi = lane + j * 64;
    q[j] = __builtin_nontemporal_load(h + (qi < nq ? qi : nq - 1));
  }

  if (do_pw) {
    if constexpr (K == 2) {
      if (split) pw_compute<K, true>(in, n_cur, n_base, suff + row * kSuff);
      else pw_compute<K>(in, n_cur, n_base, suff + row * kSuff);
    } else {
      pw_compute<K>(in, n_cur, n_base, suff + row * kSuff);
    }
  }

  float ls = 0.f;
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int e0 = (lane + j * 64) * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = q[j][c];
      if (e0 + c < T && isfinite(x)) { ls += x; ++cnt; }
    }
  }
  const double tot = wave_sum((double)ls);
  const int n = wave_sum(cnt);
  const float mf = n > 0 ? (float)(tot / n) : 0.f;
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < NQ; ++j) {
    const int e0 = (lane + j * 64) * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = q[j][c];
      if (e0 + c < T && isfinite(x)) { const float d = x - mf; ss += d * d; }
    }
  }
  const double sst = wave_sum((double)ss);
  if (lane == 0) {
    hs[row * 3 + 0] = mf;
    hs[row * 3 + 1] = n > 0 ? (float)sqrt(sst / n) : 0.f;
    hs[row * 3 + 2] = (float)n;
  }
}

FM_API int fm_canary_rows(const float* hist, int64_t ld_h, int T, const float* cur, int64_t ld_c, int n_cur,
                          const float* base, int64_t ld_b, int n_base, int64_t R, float* hs, double* suff,
                          hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_h & 3) != 0 || (((uintptr_t)hist) & 15) != 0) return (int)hipErrorInvalidValue;
  const int nq = (T + 3) / 4;
  const int n = n_cur + (n_base > 0 ? n_base : 0);
  const dim3 grid((unsigned)((R + 3) / 4)), block(256);
#define FM_CR(NQQ, KK) hipLaunchKernelGGL((canary_row_kernel<NQQ, KK>), grid, block, 0, stream, hist, ld_h, T, cur, \
                                          ld_c, n_cur, base, ld_b, n_base, R, hs, suff)
#define FM_CR_K(NQQ)              \
  if (n <= 64) FM_CR(NQQ, 1);     \
  else if (n <= 128) FM_CR(NQQ, 2); \
  else if (n <= 256) FM_CR(NQQ, 4); \
  else return (int)hipErrorInvalidValue;
  if (nq <= 64 * 8) { FM_CR_K(8) }
  else if (nq <= 64 * 16) { FM_CR_K(16) }
  else if (nq <= 64 * 24) { FM_CR_K(24) }
  else if (nq <= 64 * 32) { FM_CR_K(32) }
  else if (nq <= 64 * 40) { FM_CR_K(40) }
  else return (int)hipErrorInvalidValue;
#undef FM_CR_K
#undef FM_CR
  FM_LAUNCH_CHECK();
  return 0;
}

// p-value of ONE test for one row from its sufficient statistics (NaN when the
// test is gated out).  t is uniform per workgroup (grid y), so the fp64
// special-function code paths never diverge inside a wave.
__device__ __forceinline__ void eval_test(int t, const double* __restrict__ o, int min_mw, int min_wil, int min_kru,
                                          double& pv, double& sv) {
  const int n1 = (int)o[0], n2 = (int)o[1], nw = (int)o[2];
  const double r1 = o[3], tie = o[4], dmax = o[5], rplus = o[6], tiew = o[7];
  const double m1 = o[8], m2 = o[9], q1 = o[10], q2 = o[11];
  const int n = n1 + n2;
  const double NaN = __builtin_nan("");
  pv = NaN;
  sv = NaN;
  const double dn1 = n1, dn2 = n2, dn = n;
  switch (t) {
    case T_MW:
      if (n1 >= min_mw && n2 >= min_mw && n1 > 0 && n2 > 0) {
        const double u1 = r1 - dn1 * (dn1 + 1.0) / 2.0;
        const double u2 = dn1 * dn2 - u1;
        const double u = u1 > u2 ? u1 : u2;
        const double mu = dn1 * dn2 / 2.0;
        const double var = dn1 * dn2 / 12.0 * ((dn + 1.0) - tie / (dn * (dn - 1.0)));
        sv = u1;
        if (var > 0) {
          const double z = (u - mu - 0.5) / sqrt(var);
          double pp = 2.0 * norm_sf(z);
          pv = pp > 1.0 ? 1.0 : pp;
        } else {
          pv = 1.0;
        }
      }
      break;
    case T_KRU:
      if (n1 >= min_kru && n2 >= min_kru && n1 > 0 && n2 > 0) {
        const double r2 = dn * (dn + 1.0) / 2.0 - r1;
        double h = 12.0 / (dn * (dn + 1.0)) * (r1 * r1 / dn1 + r2 * r2 / dn2) - 3.0 * (dn + 1.0);
        const double corr = 1.0 - tie / (dn * dn * dn - dn);
        if (corr > 0) {
          sv = h / corr;
          pv = h / corr > 0 ? erfc(sqrt(0.5 * h / corr)) : 1.0;   // chi2(1) survival
        }
      }
      break;
    case T_KS:
      if (n1 >= min_mw && n2 >= min_mw && n1 > 0 && n2 > 0) {
        const double en_ = dn1 * dn2 / (dn1 + dn2);
        sv = dmax;
        pv = kolmogorov_sf(sqrt(en_) * dmax);
      }
      break;
    case T_T:
      if (n1 >= 2 && n2 >= 2 && n1 >= min_kru && n2 >= min_kru) {
        const double v1 = q1 / (dn1 - 1.0), v2 = q2 / (dn2 - 1.0);
        const double se2 = v1 / dn1 + v2 / dn2;
        if (se2 > 0) {
          const double tt = (m1 - m2) / sqrt(se2);
          const double a = v1 / dn1, bb = v2 / dn2;
          const double df = se2 * se2 / (a * a / (dn1 - 1.0) + bb * bb / (dn2 - 1.0));
          sv = tt;
          pv = student_t_2sided(tt, df);
        }
      }
      break;
    case T_WIL:
      if (nw >= min_wil && nw > 0) {
        const double dnw = nw;
        const double tot = dnw * (dnw + 1.0) / 2.0;
        const double rminus = tot - rplus;
        const double T = rplus < rminus ? rplus : rminus;
        const double mn = dnw * (dnw + 1.0) / 4.0;
        const double se = sqrt(dnw * (dnw + 1.0) * (2.0 * dnw + 1.0) / 24.0 - tiew / 48.0);
        sv = T;
        if (se > 0) {
          double pp = 2.0 * norm_sf(fabs((T - mn) / se));
          pv = pp > 1.0 ? 1.0 : pp;
        }
      }
      break;
    default: {  // T_FRI: k = 2 treatments over paired blocks, (n+ - n-)^2 / (n+ + n-), chi2(1)
      const int npos = (int)o[12], nzero = (int)o[13];
      const int nneg = nw - npos, b = nw + nzero;
      if (b >= min_wil && b > 0) {
        const double q = nw > 0 ? (double)(npos - nneg) * (npos - nneg) / nw : 0.0;
        sv = q;
        pv = q > 0 ? erfc(sqrt(0.5 * q)) : 1.0;
      }
    }
  }
}

__global__ __launch_bounds__(256) void pvalue_kernel(const double* __restrict__ suff, int64_t R, int min_mw,
                                                     int min_wil, int min_kru, float* __restrict__ pvals,
                                                     float* __restrict__ stats, int t0 = 0) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int t = blockIdx.y + t0;
  if (row >= R) return;
  double pv, sv;
  eval_test(t, suff + row * kSuff, min_mw, min_wil, min_kru, pv, sv);
  pvals[row * N_TESTS + t] = (float)pv;
  stats[row * N_TESTS + t] = (float)sv;
}

// ALL / ANY over the selected, applicable tests -> "distribution differs".
__global__ __launch_bounds__(256) void pcombine_kernel(const float* __restrict__ pvals, int64_t R, int test_mask,
                                                       int combine_any, float p_thr, int8_t* __restrict__ diff) {
  const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= R) return;
  int applicable = 0, significant = 0;
#pragma unroll
  for (int t = 0; t < N_TESTS; ++t) {
    const float p = pvals[row * N_TESTS + t];
    if (((test_mask >> t) & 1) && !isnan(p)) {
      ++applicable;
      if (p < p_thr) ++significant;
    }
  }
  diff[row] = applicable > 0 ? (int8_t)(combine_any ? (significant > 0) : (significant == applicable)) : (int8_t)0;
}

static int launch_pvalues(const double* suff, int64_t R, int test_mask, int combine_any, float p_thr, int min_mw,
                          int min_wil, int min_kru, float* pvals, float* stats, int8_t* diff, hipStream_t stream) {
  const unsigned nb = (unsigned)((R + 255) / 256);
  hipLaunchKernelGGL(pvalue_kernel, dim3(nb, N_TESTS), dim3(256), 0, stream, suff, R, min_mw, min_wil, min_kru, pvals,
                     stats, 0);
  FM_LAUNCH_CHECK();
  hipLaunchKernelGGL(pcombine_kernel, dim3(nb), dim3(256), 0, stream, pvals, R, test_mask, combine_any, p_thr, diff);
  FM_LAUNCH_CHECK();
  return 0;
}

// variant: 0 = bitonic-sort form (default), 1 = counting form.  Measured at
// 80k rows x (50 + 50): sort 140 us, counting 184 us (tools/tick_breakdown.py):
// the counting sweep issues ~n compares per owned value, more instructions
// than the log^2 network now that its exchanges are DPP / permlane.
FM_API int fm_pairwise_suff_v(const float* cur, int64_t ld_c, int n_cur, const float* base, int64_t ld_b,
                              int n_base, int64_t R, double* suff, int max_blocks, int variant, hipStream_t stream) {
  if (R <= 0) return 0;
  const int n = n_cur + n_base;
  int64_t blocks = (R + 3) / 4;
  if (max_blocks > 0 && blocks > max_blocks) blocks = max_blocks;
  const dim3 grid((unsigned)blocks), block(256);
#define FM_PW(KK)                                                                                                 \
  do {                                                                                                           \
    if (variant == 0)                                                                                            \
      hipLaunchKernelGGL(pairwise_kernel<KK>, grid, block, 0, stream, cur, ld_c, n_cur, base, ld_b, n_base, R,    \
                         suff);                                                                                  \
    else                                                                                                         \
      hipLaunchKernelGGL(pairwise_count_kernel<KK>, grid, block, 0, stream, cur, ld_c, n_cur, base, ld_b, n_base, \
                         R, suff);                                                                               \
  } while (0)
  if (n <= 64) FM_PW(1);
  else if (n <= 128) FM_PW(2);
  else if (n <= 256) FM_PW(4);
  else if (n <= 512) FM_PW(8);
  else if (n <= 1024) FM_PW(16);
  else return (int)hipErrorInvalidValue;
#undef FM_PW
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_pairwise_suff(const float* cur, int64_t ld_c, int n_cur, const float* base, int64_t ld_b, int n_base,
                            int64_t R, double* suff, int max_blocks, hipStream_t stream) {
  return fm_pairwise_suff_v(cur, ld_c, n_cur, base, ld_b, n_base, R, suff, max_blocks, 0, stream);
}

FM_API int fm_pvalues(const double* suff, int64_t R, int test_mask, int combine_any, float p_thr, int min_mw,
                      int min_wil, int min_kru, float* pvals, float* stats, int8_t* diff, hipStream_t stream) {
  if (R <= 0) return 0;
  return launch_pvalues(suff, R, test_mask, combine_any, p_thr, min_mw, min_wil, min_kru, pvals, stats, diff,
                        stream);
}

FM_API int fm_pairwise_tests(const float* cur, int64_t ld_c, int n_cur, const float* base, int64_t ld_b, int n_base,
                             int64_t R, int test_mask, int combine_any, float p_thr, int min_mw, int min_wil,
                             int min_kru, float* pvals, float* stats, int8_t* diff, double* suff,
                             hipStream_t stream) {
  if (R <= 0) return 0;
  const int n = n_cur + n_base;
  const dim3 grid((unsigned)((R + 3) / 4)), block(256);
#define FM_PW(KK) hipLaunchKernelGGL(pairwise_kernel<KK>, grid, block, 0, stream, cur, ld_c, n_cur, base, ld_b, \
                                     n_base, R, suff)
  if (n <= 64) FM_PW(1);
  else if (n <= 128) FM_PW(2);
  else if (n <= 256) FM_PW(4);
  else if (n <= 512) FM_PW(8);
  else if (n <= 1024) FM_PW(16);
  else return (int)hipErrorInvalidValue;
#undef FM_PW
  FM_LAUNCH_CHECK();
  return launch_pvalues(suff, R, test_mask, combine_any, p_thr, min_mw, min_wil, min_kru, pvals, stats, diff,
                        stream);
}

// Mean / population std / finite count of one history row, computed by a
// 256-thread block with the row held in registers (NV float4 per thread).
// Fast path for rows without missing samples (the common case): the plain
// sum is computed with packed f32 adds (v_pk_add_f32, 2 elements per
// instruction) and is finite iff every sample is; only a non-finite sum sends
// the block to the masked per-element path.  Per element that is ~0.75 VALU
// instructions instead of ~8, which leaves the CU's issue slots to the
// pairwise kernel running concurrently on the side stream.
// The row is read through a buffer resource (wave-uniform, in SGPRs) with the
// thread's 16 B as the VGPR offset and the 4-KB step as a scalar offset: no
// 64-bit VGPR address per load, and the range check returns zeros past the
// row (no clamp).  109 -> 72 VGPRs for the history kernel; the front kernel
// drops from 111 to 87 (the p-value call now bounds it): five waves per SIMD
// instead of four, i.e. one pairwise + four history workgroups per CU.
template <int NV>
__device__ __forceinline__ void block_row_stats(const float* __restrict__ hrow, int T, double* red, int* redi,
                                                float& mf, float& sd, int& n) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  typedef float nt4 __attribute__((ext_vector_type(4)));
  const int tid = threadIdx.x;
  const int nq = (T + 3) >> 2;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)hrow, (short)0, nq * 16, 0x00020000);
  nt4 q[NV];
  f2 acc = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int qi = tid + j * 256;
#ifdef FM_HIST_FLAT
    // (A/B build: the round-5 flat loads, one 64-bit VGPR address each)
    nt4 v = __builtin_nontemporal_load(reinterpret_cast<const nt4*>(hrow) + (qi < nq ? qi : nq - 1));
    if (qi >= nq) v = (nt4){0.f, 0.f, 0.f, 0.f};
#else
    nt4 v = __builtin_bit_cast(nt4, __builtin_amdgcn_raw_buffer_load_b128(rs, tid * 16, j * 4096, 2 /* nt */));
#endif
    if (qi == nq - 1) {
      const int e0 = qi * 4;
      if (e0 + 1 >= T) v.y = 0.f;
      if (e0 + 2 >= T) v.z = 0.f;
      if (e0 + 3 >= T) v.w = 0.f;
    }
    q[j] = v;
    acc += v.xy;
    acc += v.zw;
  }
  const double tot = block_sum<256>((double)acc.x + (double)acc.y, red);
  if (isfinite(tot)) {
    n = T;
    mf = (float)(tot / T);
    const f2 mm = {mf, mf};
    f2 a2 = {0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int qi = tid + j * 256;
      if (qi < nq - 1) {
        const f2 d0 = q[j].xy - mm, d1 = q[j].zw - mm;
        a2 += d0 * d0;
        a2 += d1 * d1;
      } else if (qi == nq - 1) {
        const int e0 = qi * 4;
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (e0 + c < T) { const float d = q[j][c] - mf; a2.x += d * d; }
      }
    }
    const double sst = block_sum<256>((double)a2.x + (double)a2.y, red);
    sd = (float)sqrt(sst / n);
    return;
  }
  f2 ms = {0.f, 0.f};
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int e0 = (tid + j * 256) * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = q[j][c];
      const bool ok = e0 + c < T && isfinite(x);
      cnt += ok ? 1 : 0;
      ms[c & 1] += ok ? x : 0.f;
    }
  }
  const double t2 = block_sum<256>((double)ms.x + (double)ms.y, red);
  n = block_sum<256>(cnt, redi);
  mf = n > 0 ? (float)(t2 / n) : 0.f;
  f2 a2 = {0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int e0 = (tid + j * 256) * 4;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float x = q[j][c];
      const float d = (e0 + c < T && isfinite(x)) ? x - mf : 0.f;
      a2[c & 1] += d * d;
    }
  }
  const double sst = block_sum<256>((double)a2.x + (double)a2.y, red);
  sd = n > 0 ? (float)sqrt(sst / n) : 0.f;
}

// ---------------------------------------------------------------------------
// K1 + K7 fused: moving_average_all bounds over the whole history row and the
// anomaly decision on the current window, one 256-thread workgroup per row.
// The row is read once from HBM with 16-B loads and kept in registers
// (NV float4 per thread) so the two-pass mean / variance costs no re-read.
// ---------------------------------------------------------------------------
template <int NV>
__global__ __launch_bounds__(256) void stats_decide_kernel(
    const float* __restrict__ hist, int64_t ld_h, int T, const float* __restrict__ cur, int64_t ld_c, int n_cur,
    int64_t R, int M, const float* __restrict__ thr, const int* __restrict__ bound, const float* __restrict__ minlb,
    float pair_factor, const int8_t* __restrict__ diff, int min_hist, float* __restrict__ out_stats,
    unsigned long long* __restrict__ out_flags, int NW, int* __restrict__ out_count, float* __restrict__ out_score,
    int* __restrict__ out_valid) {
  __shared__ double red[4];
  __shared__ int redi[4];
  const int tid = threadIdx.x;
  const int64_t row = blockIdx.x;
  float mf, sd;
  int n;
  block_row_stats<NV>(hist + row * ld_h, T, red, redi, mf, sd, n);
  const int m = (int)(row % M);
  float th = thr[m];
  if (diff != nullptr && diff[row]) th *= pair_factor;
  const int bd = bound[m];
  const float up = mf + th * sd;
  float lo = mf - th * sd;
  const float mlb = minlb[m];
  if (lo < mlb) lo = mlb;
  const bool has_hist = n >= min_hist && n > 0;

  const float* cr = cur + row * ld_c;
  int acnt = 0, ccnt = 0;
  float best = 0.f;
  const float inv = sd > 0.f ? __builtin_amdgcn_rcpf(sd) : 0.f;   // z-score scale, 1-ulp rcp
  for (int i0 = 0; i0 < n_cur; i0 += 256) {
    const int i = i0 + tid;
    bool f = false;
    if (i < n_cur) {
      const float x = cr[i];
      if (isfinite(x)) {
        ++ccnt;
        if (has_hist) {
          const bool hi = (bd & 1) && x > up;
          const bool lw = (bd & 2) && x < lo;
          f = hi || lw;
          if (f) {
            ++acnt;
            const float e = hi ? (x - up) : (lo - x);
            const float z = sd > 0.f ? e * inv : 1e30f;
            best = z > best ? z : best;
          }
        }
      }
    }
    const unsigned long long bal = __ballot(f);
    const int w = i0 / 64 + wave_id();
    if (lane_id() == 0 && w < NW) out_flags[row * NW + w] = bal;
  }
  acnt = block_sum<256>(acnt, redi);
  ccnt = block_sum<256>(ccnt, redi);
  best = block_max<256>(best, (float*)red);
  if (tid == 0) {
    out_stats[row * 4 + 0] = mf;
    out_stats[row * 4 + 1] = sd;
    out_stats[row * 4 + 2] = up;
    out_stats[row * 4 + 3] = lo;
    out_count[row] = acnt;
    out_score[row] = best;
    out_valid[row] = (has_hist ? 1 : 0) | (ccnt > 0 ? 2 : 0);
  }
}

FM_API int fm_stats_decide(const float* hist, int64_t ld_h, int T, const float* cur, int64_t ld_c, int n_cur, int64_t R,
                           int M, const float* thr, const int* bound, const float* minlb, float pair_factor,
                           const int8_t* diff, int min_hist, float* out_stats, unsigned long long* out_flags, int NW,
                           int* out_count, float* out_score, int* out_valid, hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_h & 3) != 0 || (((uintptr_t)hist) & 15) != 0) return (int)hipErrorInvalidValue;
  if (NW * 64 < n_cur) return (int)hipErrorInvalidValue;
  const int nq = (T + 3) / 4;
  const dim3 grid((unsigned)R), block(256);
#define FM_SD(NVV)                                                                                                    \
  hipLaunchKernelGGL(stats_decide_kernel<NVV>, grid, block, 0, stream, hist, ld_h, T, cur, ld_c, n_cur, R, M, thr,     \
                     bound, minlb, pair_factor, diff, min_hist, out_stats, out_flags, NW, out_count, out_score,        \
                     out_valid)
  if (nq <= 256 * 2) FM_SD(2);
  else if (nq <= 256 * 4) FM_SD(4);
  else if (nq <= 256 * 8) FM_SD(8);
  else if (nq <= 256 * 10) FM_SD(10);
  else if (nq <= 256 * 12) FM_SD(12);
  else if (nq <= 256 * 16) FM_SD(16);
  else return (int)hipErrorInvalidValue;
#undef FM_SD
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Split form of the same computation for the two-stream tick: hist_stats is
// the HBM-bound pass (mean, std, count per row) and runs concurrently with the
// compute-bound pairwise kernel on another stream; window_decide (one wave per
// row, reads only the small current window) applies the diff-dependent
// thresholds once both are done.
// ---------------------------------------------------------------------------
// History row of logical row `row`: identity, or a slot of the brain's
// device-resident history store (engine/resident.py) when a row map is given.
// The row index is wave-uniform, so the map read is one scalar load.
__device__ __forceinline__ int64_t hist_row(const int* __restrict__ rowmap, int64_t row) {
  return rowmap != nullptr ? (int64_t)rowmap[row] : row;
}

template <int NV>
__global__ __launch_bounds__(256) void hist_stats_kernel(const float* __restrict__ hist, int64_t ld_h, int T,
                                                         int64_t R, float* __restrict__ out /*[R,3]*/,
                                                         const int* __restrict__ rowmap) {
  __shared__ double red[4];
  __shared__ int redi[4];
  for (int64_t row = blockIdx.x; row < R; row += gridDim.x) {
    float mf, sd;
    int n;
    block_row_stats<NV>(hist + hist_row(rowmap, row) * ld_h, T, red, redi, mf, sd, n);
    if (threadIdx.x == 0) {
      out[row * 3 + 0] = mf;
      out[row * 3 + 1] = sd;
      out[row * 3 + 2] = (float)n;
    }
  }
}

FM_API int fm_hist_stats_rm(const float* hist, int64_t ld_h, int T, int64_t R, float* out, int max_blocks,
                            const int* rowmap, hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_h & 3) != 0 || (((uintptr_t)hist) & 15) != 0) return (int)hipErrorInvalidValue;
  const int nq = (T + 3) / 4;
  const dim3 grid((unsigned)(max_blocks > 0 && R > max_blocks ? max_blocks : R)), block(256);
#define FM_HS(NVV) hipLaunchKernelGGL(hist_stats_kernel<NVV>, grid, block, 0, stream, hist, ld_h, T, R, out, rowmap)
  if (nq <= 256 * 2) FM_HS(2);
  else if (nq <= 256 * 4) FM_HS(4);
  else if (nq <= 256 * 8) FM_HS(8);
  else if (nq <= 256 * 10) FM_HS(10);
  else if (nq <= 256 * 12) FM_HS(12);
  else if (nq <= 256 * 16) FM_HS(16);
  else return (int)hipErrorInvalidValue;
#undef FM_HS
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_hist_stats_capped(const float* hist, int64_t ld_h, int T, int64_t R, float* out, int max_blocks,
                                hipStream_t stream) {
  return fm_hist_stats_rm(hist, ld_h, T, R, out, max_blocks, nullptr, stream);
}

FM_API int fm_hist_stats(const float* hist, int64_t ld_h, int T, int64_t R, float* out, hipStream_t stream) {
  return fm_hist_stats_rm(hist, ld_h, T, R, out, 0, nullptr, stream);
}

// ---------------------------------------------------------------------------
// Horizontally fused front half of the canary tick: ONE launch whose
// workgroups take one of two roles by blockIdx.
//   * blockIdx <  nP: pairwise role — grid-stride over rows, one wave per row
//     (sorted-rank sufficient statistics), then the workgroup evaluates the
//     six p-values of its own rows, one (test, row) pair per thread,
//     test-major so a wave mostly runs one special function;
//   * blockIdx >= nP: history role — mean / std / count of a 7-day row per
//     workgroup (HBM-bound, grid-stride over rows).
// The compute-bound and the HBM-bound halves share every CU without a
// second stream: no fork/join in the graph (the side branch of a two-stream
// graph starts ~11-13 us late, and whether the branches land on different
// hardware queues varied run to run: profiles/tick_timeline_*.txt).  The
// pairwise workgroups have the lowest ids, so the dispatcher places them
// first and the history workgroups fill the remaining slots.
// ---------------------------------------------------------------------------
// Out-of-line p-value evaluation for the fused kernel: inlined into the
// role-split kernel the special functions pushed it to 256 VGPRs (one wave
// per SIMD); as a call the kernel keeps the history role's 96.
__device__ __attribute__((noinline)) void eval_test_call(int t, const double* __restrict__ o, int min_mw, int min_wil,
                                                         int min_kru, double& pv, double& sv) {
  eval_test(t, o, min_mw, min_wil, min_kru, pv, sv);
}

// FM_FRONT_TIMING builds (tools/front_timing.py): every workgroup of the
// front kernel records its start / end on the 100 MHz real-time counter, so
// the critical role (pairwise or history) of a shape can be read off.
#ifdef FM_FRONT_TIMING
__device__ unsigned long long g_front_t[2 * 8192];
#define FM_FT_MARK(k) \
  do { if (threadIdx.x == 0 && blockIdx.x < 8192) g_front_t[2 * blockIdx.x + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define FM_FT_MARK(k) do {} while (0)
#endif

#define FM_FRONT_PARAMS                                                                                        \
  const float *__restrict__ hist, int64_t ld_h, int T, int64_t R, float *__restrict__ hs /*[R,3]*/,            \
      const float *__restrict__ cur, int64_t ld_c, int n_cur, const float *__restrict__ base, int64_t ld_b,    \
      int n_base, double *__restrict__ suff, int nP, int min_mw, int min_wil, int min_kru,                     \
      float *__restrict__ pvals, float *__restrict__ pstats, unsigned *__restrict__ queue,                    \
      const int *__restrict__ rowmap
#define FM_FRONT_ARGS hist, ld_h, T, R, hs, cur, ld_c, n_cur, base, ld_b, n_base, suff, nP, min_mw, min_wil, \
      min_kru, pvals, pstats, queue, rowmap

// Control block of the front kernel's history queue (uint32 words from
// queue[kXcdCtl]; the queue is 8 x 32 counters + this block, zeroed by the
// host, kCtlOn set to 1 to enable the balancing): a split-is-set flag, the
// ranges done this tick, the 9 range bounds as fractions of the rows (2^-24
// fixed point, so a split survives the row count changing with fleet churn:
// range x is rows [R f[x] >> 24, R f[x+1] >> 24)), and per-XCD start / end
// times (u64, 100 MHz) of this tick.
constexpr int kXcdCtl = 256, kCtlR = 0, kCtlDone = 1, kCtlB = 2, kCtlOn = 31, kCtlT0 = 32, kCtlT1 = 48;
constexpr int64_t kXcdMinRows = 32768;
constexpr int kFracBits = 24;
__device__ inline int64_t xcd_bound(int64_t R, unsigned f) { return (R * (int64_t)f) >> kFracBits; }

// The last workgroup of XCD range ``xcd``: its end time; the last range of
// the tick to finish computes the next tick's bounds.
__device__ __attribute__((noinline)) void xcd_rebalance(unsigned* ctl, int xcd, int64_t R, int64_t lo, int64_t hi) {
  unsigned long long* t0 = reinterpret_cast<unsigned long long*>(ctl + kCtlT0);
  unsigned long long* t1 = reinterpret_cast<unsigned long long*>(ctl + kCtlT1);
  __hip_atomic_store(t1 + xcd, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned g = __hip_atomic_fetch_add(ctl + kCtlDone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  if (g != 7u) return;
  __hip_atomic_store(ctl + kCtlDone, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (R < 64 || R > 0x7fffffff) return;
  const bool had = __hip_atomic_load(ctl + kCtlR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
  constexpr double one = (double)(1u << kFracBits);
  double b[9], f[9], rate[8], tot = 0.0;
  for (int x = 0; x <= 8; ++x) {   // this tick's bounds, exactly as the history role derived them
    const unsigned fx = __hip_atomic_load(ctl + kCtlB + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    b[x] = had ? (double)xcd_bound(R, fx) : (double)(R * x / 8);
    f[x] = had ? (double)fx / one : (double)x / 8.0;
  }
  for (int x = 0; x < 8; ++x) {
    const unsigned long long a = __hip_atomic_load(t0 + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long e = __hip_atomic_load(t1 + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const double rows = b[x + 1] - b[x];
    if (!(e > a) || e - a > 100000000ull || rows < 1.0) return;   // (a range with no start this tick: keep the split)
    rate[x] = rows / (double)(e - a);
    tot += rate[x];
  }
  // a third of the way towards the split that would have ended every range
  // together, and only when the ranges ended more than 1.5 % apart (per-tick
  // noise is not steered by)
  double dmin = 1e300, dmax = 0.0;
  for (int x = 0; x < 8; ++x) {
    const double d = (b[x + 1] - b[x]) / rate[x];
    dmin = d < dmin ? d : dmin;
    dmax = d > dmax ? d : dmax;
  }
#ifndef FM_XCD_BAND
#define FM_XCD_BAND 1.015
#endif
#ifndef FM_XCD_STEP
#define FM_XCD_STEP 3.0
#endif
  if (had && dmax < FM_XCD_BAND * dmin) return;
  // in fraction space; every range keeps at least 1/64 of the rows (an XCD a
  // quarter of the mean speed), so no range empties and stops being timed
  constexpr double minf = 1.0 / 64.0;
  double acc = 0.0, prev = 0.0;
  unsigned nf[9];
  nf[0] = 0;
  for (int x = 0; x < 8; ++x) {
    acc += rate[x] / tot;
    double v = ((FM_XCD_STEP - 1.0) * f[x + 1] + acc) / FM_XCD_STEP;   // (1 / FM_XCD_STEP of the way)
    const double minv = prev + minf, maxv = 1.0 - (double)(7 - x) * minf;
    v = v < minv ? minv : (v > maxv ? maxv : v);
    nf[x + 1] = x == 7 ? (1u << kFracBits) : (unsigned)(v * one + 0.5);
    prev = (double)nf[x + 1] / one;
  }
  for (int x = 0; x <= 8; ++x) __hip_atomic_store(ctl + kCtlB + x, nf[x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(ctl + kCtlR, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NV, int K, bool PRIO>
__device__ __forceinline__ void tick_front_body(FM_FRONT_PARAMS) {
  __shared__ double red[4];
  __shared__ int redi[4];
  FM_FT_MARK(0);
  if ((int)blockIdx.x < nP) {
    if (PRIO) __builtin_amdgcn_s_setprio(2);
    const int64_t first = (int64_t)blockIdx.x * 4, stride = (int64_t)nP * 4;
    for (int64_t row = first + wave_id(); row < R; row += stride) {
      pw_row<K>(cur + row * ld_c, base + row * ld_b, n_cur, n_base, suff + row * kSuff);
    }
    __syncthreads();   // this workgroup's suff rows are visible to all its waves
    // local row j -> global row first + (j & 3) + (j >> 2) * stride
    const int64_t span = R > first ? R - first : 0;
    const int nr = (int)(((span + stride - 1) / stride) * 4);
    // wave-sized chunks of (test, 64 rows); the test is wave-uniform so the
    // special-function switch stays a scalar branch (a per-lane test index
    // made the compiler keep every path live: 256 VGPRs)
    const int cpt = (nr + 63) >> 6;
    for (int ci = wave_id(); ci < N_TESTS * cpt; ci += 4) {
      const int t = __builtin_amdgcn_readfirstlane(ci / cpt);
      const int j = (ci - t * cpt) * 64 + lane_id();
      const int64_t row = first + (j & 3) + (int64_t)(j >> 2) * stride;
      if (j < nr && row < R) {
        double pv, sv;
        eval_test_call(t, suff + row * kSuff, min_mw, min_wil, min_kru, pv, sv);
        pvals[row * N_TESTS + t] = (float)pv;
        pstats[row * N_TESTS + t] = (float)sv;
      }
    }
    FM_FT_MARK(1);
    return;
  }
  const int nH = (int)gridDim.x - nP;
  // PRIO: the co-resident pairwise waves issue ahead of the history waves
  // (history first measured 0.64-0.66 vs 0.53-0.56 ms per step: worse)
  if (PRIO) __builtin_amdgcn_s_setprio(0);
  if (queue == nullptr) {
    for (int64_t row = (int64_t)blockIdx.x - nP; row < R; row += nH) {
      float mf, sd;
      int n;
      block_row_stats<NV>(hist + hist_row(rowmap, row) * ld_h, T, red, redi, mf, sd, n);
      if (threadIdx.x == 0) {
        hs[row * 3 + 0] = mf;
        hs[row * 3 + 1] = sd;
        hs[row * 3 + 2] = (float)n;
      }
    }
    FM_FT_MARK(1);
    return;
  }
  // Dynamic history queue: the rows are split into 8 contiguous ranges, one
  // per XCD (workgroup ids are dealt round-robin over the XCDs), and the
  // history workgroups of a range grab chunks of kHistChunk rows from its
  // counter (one 128-B line per counter).  A slot freed by a finished
  // pairwise workgroup is then filled by a history workgroup that starts late
  // and simply takes what is left, instead of idling (static grid-stride).
  // The next chunk index is requested while the current chunk streams.  The
  // last workgroup of a range to find it empty resets the counters for the
  // next tick (every other workgroup of the range has already exited).
  // One row per grab: at the 1,250-service shard (~10 rows per workgroup) the
  // tail waits on at most one row instead of two (0.0951/0.0919 -> 0.0937/
  // 0.0904 ms per step, interleaved runs); neutral at 10k services.
#ifndef FM_HIST_CHUNK
#define FM_HIST_CHUNK 1
#endif
  constexpr int kHistChunk = FM_HIST_CHUNK;
  __shared__ unsigned s_next;
  const int hb = (int)blockIdx.x - nP;
  const int xcd = hb & 7;
  const int nwg = (nH >> 3) + ((nH & 7) > xcd ? 1 : 0);   // workgroups sharing this range
  // XCD-balanced ranges: the XCDs do not stream equally fast (per-XCD end
  // times of the history role, tools/front_timing.py: XCDs 3-5 end 30-40 us
  // after XCDs 0-2 at 80k rows, the same XCDs tick after tick), so the range
  // split adapts -- the last range to finish re-divides the rows in
  // proportion to each XCD's measured rows per microsecond for the next tick
  // (1/3 steps, as fractions of the rows, so the split carries over when the
  // fleet's row count changes).  queue[256..320): control block (kXcdCtl).
  unsigned* ctl = queue + kXcdCtl;
  int64_t lo = R * xcd / 8, hi = R * (xcd + 1) / 8;
  auto ld = [](const unsigned* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  // (agent-scope loads: written by another XCD last tick).  Small fleets keep
  // the even split: at the 1,250-service shard (10k rows) the per-tick
  // durations are too short and noisy to steer by (0.078 -> 0.081 ms measured)
  const bool bal = R >= kXcdMinRows && ld(ctl + kCtlOn) == 1u;
  if (bal && ld(ctl + kCtlR) != 0u) {
    lo = xcd_bound(R, ld(ctl + kCtlB + xcd));
    hi = xcd_bound(R, ld(ctl + kCtlB + xcd + 1));
  }
  unsigned* ctr = queue + xcd * 32;
  if (threadIdx.x == 0) {
    s_next = atomicAdd(ctr, (unsigned)kHistChunk);
    if (bal && s_next == 0u)       // the range's first grab: its start time
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(ctl + kCtlT0) + xcd, __builtin_amdgcn_s_memrealtime(),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  int64_t r0 = lo + (int64_t)s_next;
  while (r0 < hi) {
    unsigned nxt = 0;
    if (threadIdx.x == 0) nxt = atomicAdd(ctr, (unsigned)kHistChunk);
    const int64_t r1 = r0 + kHistChunk < hi ? r0 + kHistChunk : hi;
    for (int64_t row = r0; row < r1; ++row) {
      float mf, sd;
      int n;
      block_row_stats<NV>(hist + hist_row(rowmap, row) * ld_h, T, red, redi, mf, sd, n);
      if (threadIdx.x == 0) {
        hs[row * 3 + 0] = mf;
        hs[row * 3 + 1] = sd;
        hs[row * 3 + 2] = (float)n;
      }
    }
    __syncthreads();               // everyone is done reading s_next
    if (threadIdx.x == 0) s_next = nxt;
    __syncthreads();
    r0 = lo + (int64_t)s_next;
  }
  if (threadIdx.x == 0) {
    const unsigned d = atomicAdd(ctr + 1, 1u);
    if (d == (unsigned)nwg - 1) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (bal) xcd_rebalance(ctl, xcd, R, lo, hi);
    }
  }
  FM_FT_MARK(1);
}

template <int NV, int K, bool PRIO = false>
__global__ __launch_bounds__(256) void tick_front_kernel(FM_FRONT_PARAMS) {
  tick_front_body<NV, K, PRIO>(FM_FRONT_ARGS);
}

// The same kernel held to 5 waves per SIMD (96 VGPRs: the rest spills): one
// pairwise + four history workgroups per CU instead of one + three at the
// default 111 VGPRs.  FM_FRONT_OCC=5 selects it (A/B on one box).
template <int NV, int K, bool PRIO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5, 5))) void tick_front_kernel_o5(
    FM_FRONT_PARAMS) {
  tick_front_body<NV, K, PRIO>(FM_FRONT_ARGS);
}

// FM_FRONT_LDS=<bytes> (environment, read once): dynamic LDS requested per
// front-kernel workgroup, i.e. a cap on how many of them share a CU (160 KB
// of LDS: 33 KB -> at most four).  Default 33 KB: with the buffer-load history
// role the kernel fits five waves per SIMD, and a fifth concurrent workgroup
// per CU measured slower (more history streams during the pairwise phase).
static unsigned front_lds() {
  static const unsigned b = [] {
    const char* e = getenv("FM_FRONT_LDS");
    return e != nullptr ? (unsigned)atoi(e) : 33u * 1024u;
  }();
  return b;
}

static int front_occ() {
  static const int occ = [] {
    const char* e = getenv("FM_FRONT_OCC");
    return e != nullptr ? atoi(e) : 0;
  }();
  return occ;
}

// FM_FRONT_PRIO=1 (environment, read once): A/B of wave priorities in the
// front kernel (tools: bench.py with and without it on one box).
static bool front_prio() {
  static const bool on = [] {
    const char* e = getenv("FM_FRONT_PRIO");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

// nP / nH: workgroups of each role (0 = one pairwise workgroup per 4 rows /
// one history workgroup per row); queue: dynamic history rows (or nullptr):
// 8 x 32 + 64 zero-initialised uint32 -- the per-XCD counters and the
// XCD-balance control block (kXcdCtl; word kXcdCtl + kCtlOn = 1 enables it).
FM_API int fm_tick_front_rm(const float* hist, int64_t ld_h, int T, int64_t R, float* hs, const float* cur,
                            int64_t ld_c, int n_cur, const float* base, int64_t ld_b, int n_base, double* suff, int nP,
                            int nH, int min_mw, int min_wil, int min_kru, float* pvals, float* pstats,
                            unsigned* queue, const int* rowmap, hipStream_t stream) {
  if (R <= 0) return 0;
  if ((ld_h & 3) != 0 || (((uintptr_t)hist) & 15) != 0) return (int)hipErrorInvalidValue;
  const int n = n_cur + n_base;
  if (base == nullptr || n_base <= 0 || n > 256) return (int)hipErrorInvalidValue;
  const int64_t pmax = (R + 3) / 4;
  if (nP <= 0 || nP > pmax) nP = (int)pmax;
  if (nH <= 0 || nH > R) nH = (int)R;
  // queue: 8 x 32 + 64 zero-initialised uints (the counters are kept zero
  // between launches by the kernel itself); needs at least one history
  // workgroup per XCD range
  if (queue != nullptr && nH < 8) nH = 8;
  const int nq = (T + 3) / 4;
  const dim3 grid((unsigned)(nP + nH)), block(256);
  const unsigned lds = front_lds();
#define FM_TF(NVV, KK)                                                                                             \
  if (front_prio())                                                                                                 \
    hipLaunchKernelGGL((tick_front_kernel<NVV, KK, true>), grid, block, lds, stream, hist, ld_h, T, R, hs, cur, ld_c,  \
                       n_cur, base, ld_b, n_base, suff, nP, min_mw, min_wil, min_kru, pvals, pstats, queue, rowmap); \
  else if (front_occ() == 5)                                                                                         \
    hipLaunchKernelGGL((tick_front_kernel_o5<NVV, KK>), grid, block, lds, stream, hist, ld_h, T, R, hs, cur, ld_c,     \
                       n_cur, base, ld_b, n_base, suff, nP, min_mw, min_wil, min_kru, pvals, pstats, queue, rowmap); \
  else                                                                                                               \
  hipLaunchKernelGGL((tick_front_kernel<NVV, KK>), grid, block, lds, stream, hist, ld_h, T, R, hs, cur, ld_c, n_cur, \
                     base, ld_b, n_base, suff, nP, min_mw, min_wil, min_kru, pvals, pstats, queue, rowmap)
#define FM_TF_K(NVV)           \
  do {                         \
    if (n <= 64) FM_TF(NVV, 1);  \
    else if (n <= 128) FM_TF(NVV, 2); \
    else FM_TF(NVV, 4);        \
  } while (0)
  if (nq <= 256 * 2) FM_TF_K(2);
  else if (nq <= 256 * 4) FM_TF_K(4);
  else if (nq <= 256 * 8) FM_TF_K(8);
  else if (nq <= 256 * 10) FM_TF_K(10);
  else if (nq <= 256 * 12) FM_TF_K(12);
  else if (nq <= 256 * 16) FM_TF_K(16);
  else return (int)hipErrorInvalidValue;
#undef FM_TF_K
#undef FM_TF
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_tick_front(const float* hist, int64_t ld_h, int T, int64_t R, float* hs, const float* cur, int64_t ld_c,
                         int n_cur, const float* base, int64_t ld_b, int n_base, double* suff, int nP, int nH,
                         int min_mw, int min_wil, int min_kru, float* pvals, float* pstats, unsigned* queue,
                         hipStream_t stream) {
  return fm_tick_front_rm(hist, ld_h, T, R, hs, cur, ld_c, n_cur, base, ld_b, n_base, suff, nP, nH, min_mw, min_wil,
                          min_kru, pvals, pstats, queue, nullptr, stream);
}

__global__ __launch_bounds__(256) void window_decide_kernel(
    const float* __restrict__ hs, const float* __restrict__ cur, int64_t ld_c, int n_cur, int64_t R, int M,
    const float* __restrict__ thr, const int* __restrict__ bound, const float* __restrict__ minlb, float pair_factor,
    const int8_t* __restrict__ diff, int min_hist, float* __restrict__ out_stats,
    unsigned long long* __restrict__ out_flags, int NW, int* __restrict__ out_count, float* __restrict__ out_score,
    int* __restrict__ out_valid) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R) return;
  const int lane = lane_id();
  const float mf = hs[row * 3 + 0], sd = hs[row * 3 + 1];
  const int n = (int)hs[row * 3 + 2];
  const int m = (int)(row % M);
  float th = thr[m];
  if (diff != nullptr && diff[row]) th *= pair_factor;
  const int bd = bound[m];
  const float up = mf + th * sd;
  float lo = mf - th * sd;
  if (lo < minlb[m]) lo = minlb[m];
  const bool has_hist = n >= min_hist && n > 0;
  const float inv = sd > 0.f ? __builtin_amdgcn_rcpf(sd) : 0.f;   // z-score scale, 1-ulp rcp
  const float* cr = cur + row * ld_c;
  int acnt = 0, ccnt = 0;
  float best = 0.f;
  for (int i0 = 0; i0 < n_cur; i0 += 64) {
    const int i = i0 + lane;
    bool f = false;
    if (i < n_cur) {
      const float x = cr[i];
      if (isfinite(x)) {
        ++ccnt;
        if (has_hist) {
          const bool hi = (bd & 1) && x > up;
          const bool lw = (bd & 2) && x < lo;
          f = hi || lw;
          if (f) {
            ++acnt;
            const float z = sd > 0.f ? (hi ? x - up : lo - x) * inv : 1e30f;
            best = z > best ? z : best;
          }
        }
      }
    }
    const unsigned long long bal = __ballot(f);
    if (lane == 0 && i0 / 64 < NW) out_flags[row * NW + i0 / 64] = bal;
  }
  acnt = wave_sum(acnt);
  ccnt = wave_sum(ccnt);
  best = wave_max(best);
  if (lane == 0) {
    out_stats[row * 4 + 0] = mf;
    out_stats[row * 4 + 1] = sd;
    out_stats[row * 4 + 2] = up;
    out_stats[row * 4 + 3] = lo;
    out_count[row] = acnt;
    out_score[row] = best;
    out_valid[row] = (has_hist ? 1 : 0) | (ccnt > 0 ? 2 : 0);
  }
}

FM_API int fm_window_decide(const float* hs, const float* cur, int64_t ld_c, int n_cur, int64_t R, int M,
                            const float* thr, const int* bound, const float* minlb, float pair_factor,
                            const int8_t* diff, int min_hist, float* out_stats, unsigned long long* out_flags, int NW,
                            int* out_count, float* out_score, int* out_valid, hipStream_t stream) {
  if (R <= 0) return 0;
  if (NW * 64 < n_cur) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(window_decide_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, hs, cur, ld_c, n_cur,
                     R, M, thr, bound, minlb, pair_factor, diff, min_hist, out_stats, out_flags, NW, out_count,
                     out_score, out_valid);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Decision + pairwise combine + service reduce in ONE launch: one WAVE per
// service, looping over its M <= 16 metric rows.  All global loads of the
// service (current window, p-values) are issued before any arithmetic, so a
// wave pays one memory latency; with 4 services per workgroup a CU keeps up to
// 32 services in flight (a workgroup-per-service layout with a wave per metric
// kept only 4, and the kernel was latency-bound at ~30 us for 10k services).
// Per row: p-values fold into "distribution differs" (lanes 0..N_TESTS-1 +
// two ballots), the threshold is lowered accordingly, the current window is
// flagged against the history band (anomalous / observed counts from ballot
// popcounts), and the service verdict is reduced in registers.  Replaces
// pcombine + window_decide + service_reduce.
// ---------------------------------------------------------------------------
// MAXM: metric slots in registers; EXACT: M == MAXM (no per-metric guards);
// ONE: n_cur <= 64 (the current window is one wave-wide chunk).  The
// specialised forms roughly halve the instruction count of the generic one.
template <int MAXM, bool EXACT, bool ONE>
__global__ __launch_bounds__(256) void decide_service_kernel(
    const float* __restrict__ hs, const float* __restrict__ cur, int64_t ld_c, int n_cur, int64_t S, int M,
    const float* __restrict__ thr, const int* __restrict__ bound, const float* __restrict__ minlb, float pair_factor,
    const float* __restrict__ pvals, int test_mask, int combine_any, float p_thr, int min_hist,
    float* __restrict__ out_stats, unsigned long long* __restrict__ out_flags, int NW, int* __restrict__ out_count,
    float* __restrict__ out_score, int* __restrict__ out_valid, int8_t* __restrict__ out_diff,
    float* __restrict__ packed) {
  if (EXACT) M = MAXM;
  const int64_t svc = (int64_t)blockIdx.x * 4 + wave_id();
  if (svc >= S) return;
  const int lane = lane_id();
  const float NaNf = __builtin_nanf("");
  // phase 1: every load of the service up front (clamped, unpredicated)
  const int li = lane < n_cur ? lane : n_cur - 1;
  const int lp = lane < N_TESTS ? lane : N_TESTS - 1;
  float xs[MAXM], pv[MAXM];
#pragma unroll
  for (int m = 0; m < MAXM; ++m) {
    const int64_t row = svc * M + ((EXACT || m < M) ? m : M - 1);
    xs[m] = cur[row * ld_c + li];
    pv[m] = pvals != nullptr ? pvals[row * N_TESTS + lp] : NaNf;
  }
  // the service's [M, 3] history stats (3M <= 48 floats) as one vector
  // load, lane j holding element j, broadcast per metric with readlane
  const int nh = 3 * M;
  const float hsv = hs[svc * nh + (lane < nh ? lane : nh - 1)];
  int tot = 0, mask = 0;
  bool unknown = false;
  float bestm[MAXM];
  // per-row outputs are collected in lane m (values are wave-uniform per
  // metric) and stored once by lanes 0..M-1: 7 store instructions per
  // service instead of 7 per metric from lane 0
  float4 o_st = make_float4(0.f, 0.f, 0.f, 0.f);
  int o_cnt = 0, o_valid = 0, o_diff = 0;
  unsigned long long o_flag = 0ull;
#pragma unroll
  for (int m = 0; m < MAXM; ++m) {
    bestm[m] = 0.f;
    if (!EXACT && m >= M) continue;
    const int64_t row = svc * M + m;
    bool differs = false;
    if (pvals != nullptr) {
      const bool sel = lane < N_TESTS && ((test_mask >> lane) & 1) && !isnan(pv[m]);
      const unsigned long long app = __ballot(sel), sig = __ballot(sel && pv[m] < p_thr);
      differs = app != 0ull && (combine_any ? sig != 0ull : sig == app);
    }
    const float mf = lane_bcast(hsv, 3 * m);
    const float sd = lane_bcast(hsv, 3 * m + 1);
    const int n = (int)lane_bcast(hsv, 3 * m + 2);
    float th = thr[m];
    if (differs) th *= pair_factor;
    const int bd = bound[m];
    const float up = mf + th * sd;
    float lo = mf - th * sd;
    if (lo < minlb[m]) lo = minlb[m];
    const bool has_hist = n >= min_hist && n > 0;
    const float inv = sd > 0.f ? __builtin_amdgcn_rcpf(sd) : 0.f;   // z-score scale, 1-ulp rcp
    int acnt = 0, ccnt = 0;
    float best = 0.f;
    for (int i0 = 0; i0 < (ONE ? 64 : n_cur); i0 += 64) {
      const int i = i0 + lane;
      const float x = (ONE || i0 == 0) ? xs[m] : cur[row * ld_c + (i < n_cur ? i : n_cur - 1)];
      const bool obs = i < n_cur && isfinite(x);
      const bool hi = has_hist && obs && (bd & 1) && x > up;
      const bool lw = has_hist && obs && (bd & 2) && x < lo;
      const bool f = hi || lw;
      const float z = sd > 0.f ? (hi ? x - up : lo - x) * inv : 1e30f;
      best = f && z > best ? z : best;
      const unsigned long long bal = __ballot(f);
      acnt += __popcll(bal);
      ccnt += __popcll(__ballot(obs));
      if (i0 == 0) {
        if (lane == m) o_flag = bal;
      } else if (lane == 0 && i0 / 64 < NW) {
        out_flags[row * NW + i0 / 64] = bal;
      }
    }
    bestm[m] = best;
    const int valid = (has_hist ? 1 : 0) | (ccnt > 0 ? 2 : 0);
    if (lane == m) {
      o_st = make_float4(mf, sd, up, lo);
      o_cnt = acnt;
      o_valid = valid;
      o_diff = differs ? 1 : 0;
    }
    tot += acnt;
    if (acnt > 0) mask |= 1 << m;
    if ((valid & 3) != 3) unknown = true;
  }
  // the M max-reductions are independent: issued together they overlap
  float sbest = 0.f, o_score = 0.f;
#pragma unroll
  for (int m = 0; m < MAXM; ++m) bestm[m] = wave_max(bestm[m]);
#pragma unroll
  for (int m = 0; m < MAXM; ++m) {
    if (!EXACT && m >= M) break;
    if (lane == m) o_score = bestm[m];
    sbest = bestm[m] > sbest ? bestm[m] : sbest;
  }
  if (lane < M) {
    const int64_t row = svc * M + lane;
    reinterpret_cast<float4*>(out_stats)[row] = o_st;
    out_count[row] = o_cnt;
    out_valid[row] = o_valid;
    out_score[row] = o_score;
    out_flags[row * NW] = o_flag;
    if (out_diff != nullptr && pvals != nullptr) out_diff[row] = (int8_t)o_diff;
  }
  if (lane == 0) {
    packed[svc * 4 + 0] = (float)(tot > 0 ? 1 : (unknown ? 2 : 0));
    packed[svc * 4 + 1] = sbest;
    packed[svc * 4 + 2] = (float)mask;
    packed[svc * 4 + 3] = (float)tot;
  }
}

FM_API int fm_decide_services(const float* hs, const float* cur, int64_t ld_c, int n_cur, int64_t S, int M,
                              const float* thr, const int* bound, const float* minlb, float pair_factor,
                              const float* pvals, int test_mask, int combine_any, float p_thr, int min_hist,
                              float* out_stats, unsigned long long* out_flags, int NW, int* out_count,
                              float* out_score, int* out_valid, int8_t* out_diff, float* packed,
                              hipStream_t stream) {
  if (S <= 0) return 0;
  if (M < 1 || M > 16 || n_cur < 1 || NW * 64 < n_cur) return (int)hipErrorInvalidValue;
  if ((((uintptr_t)out_stats) & 15) != 0) return (int)hipErrorInvalidValue;   // float4 row stores
  const dim3 grid((unsigned)((S + 3) / 4)), block(256);
#define FM_DS(MM, EX, ONE)                                                                                            \
  hipLaunchKernelGGL((decide_service_kernel<MM, EX, ONE>), grid, block, 0, stream, hs, cur, ld_c, n_cur, S, M, thr,    \
                     bound, minlb, pair_factor, pvals, test_mask, combine_any, p_thr, min_hist, out_stats, out_flags,  \
                     NW, out_count, out_score, out_valid, out_diff, packed)
  if (M == 8 && n_cur <= 64) FM_DS(8, true, true);
  else if (M == 4 && n_cur <= 64) FM_DS(4, true, true);
  else if (M <= 8) FM_DS(8, false, false);
  else FM_DS(16, false, false);
#undef FM_DS
  FM_LAUNCH_CHECK();
  return 0;
}

// p-values only (the combine happens in fm_decide_services)
FM_API int fm_pvalues_only(const double* suff, int64_t R, int min_mw, int min_wil, int min_kru, float* pvals,
                           float* stats, hipStream_t stream) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(pvalue_kernel, dim3((unsigned)((R + 255) / 256), N_TESTS), dim3(256), 0, stream, suff, R,
                     min_mw, min_wil, min_kru, pvals, stats, 0);
  FM_LAUNCH_CHECK();
  return 0;
}

// Tests [t0, t1) only (per-test timing in tools/tick_breakdown.py).
FM_API int fm_pvalues_range(const double* suff, int64_t R, int t0, int t1, int min_mw, int min_wil, int min_kru,
                            float* pvals, float* stats, hipStream_t stream) {
  if (R <= 0 || t0 < 0 || t1 > N_TESTS || t1 <= t0) return 0;
  hipLaunchKernelGGL(pvalue_kernel, dim3((unsigned)((R + 255) / 256), t1 - t0), dim3(256), 0, stream, suff, R,
                     min_mw, min_wil, min_kru, pvals, stats, t0);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Service reduce: per service, fold its M metric rows into the packed result
// row [status, score, anomalous-metric mask, anomalous point count] that is
// all-gathered across ranks.  status: 0 = no anomaly, 1 = anomaly, 2 = unknown
// (missing current data or not enough history).
// ---------------------------------------------------------------------------
__global__ void service_reduce_kernel(const int* __restrict__ count, const float* __restrict__ score,
                                      const int* __restrict__ valid, int64_t S, int M, float* __restrict__ packed) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  int tot = 0, mask = 0;
  bool unknown = false;
  float best = 0.f;
  for (int m = 0; m < M; ++m) {
    const int64_t r = s * M + m;
    const int c = count[r];
    tot += c;
    if (c > 0) mask |= 1 << m;
    if ((valid[r] & 3) != 3) unknown = true;
    best = score[r] > best ? score[r] : best;
  }
  const int status = tot > 0 ? 1 : (unknown ? 2 : 0);
  packed[s * 4 + 0] = (float)status;
  packed[s * 4 + 1] = best;
  packed[s * 4 + 2] = (float)mask;
  packed[s * 4 + 3] = (float)tot;
}

FM_API int fm_service_reduce(const int* count, const float* score, const int* valid, int64_t S, int M, float* packed,
                             hipStream_t stream) {
  if (S <= 0) return 0;
  if (M > 24) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(service_reduce_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, count, score,
                     valid, S, M, packed);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Stream compaction of anomalous points: one wave per row, entries
// (row, index, value) appended through one atomic per row with anomalies.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void compact_kernel(const unsigned long long* __restrict__ flags, int NW,
                                                      const float* __restrict__ cur, int64_t ld_c, int n_cur,
                                                      const int* __restrict__ count, int64_t R, int cap,
                                                      int* __restrict__ counter, int* __restrict__ out_idx,
                                                      float* __restrict__ out_val) {
  const int64_t row = (int64_t)blockIdx.x * 4 + wave_id();
  if (row >= R) return;
  const int c = count[row];
  if (c == 0) return;
  const int lane = lane_id();
  int base = 0;
  if (lane == 0) base = atomicAdd(counter, c);
  base = __shfl(base, 0);
  int written = 0;
  for (int w = 0; w < NW; ++w) {
    const unsigned long long word = flags[row * NW + w];
    if (!word) continue;
    const bool mine = (word >> lane) & 1ull;
    const unsigned long long below = lane == 0 ? 0ull : (word & ((1ull << lane) - 1ull));
    const int pos = written + __popcll(below);
    if (mine) {
      const int slot = base + pos;
      const int i = w * 64 + lane;
      if (slot < cap) {
        out_idx[2 * slot + 0] = (int)row;
        out_idx[2 * slot + 1] = i;
        out_val[slot] = cur[row * ld_c + i];
      }
    }
    written += __popcll(word);
  }
}

FM_API int fm_compact_anomalies(const unsigned long long* flags, int NW, const float* cur, int64_t ld_c, int n_cur,
                                const int* count, int64_t R, int cap, int* counter, int* out_idx, float* out_val,
                                hipStream_t stream) {
  if (R <= 0) return 0;
  hipLaunchKernelGGL(compact_kernel, dim3((unsigned)((R + 3) / 4)), dim3(256), 0, stream, flags, NW, cur, ld_c, n_cur,
                     count, R, cap, counter, out_idx, out_val);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// K11: synthetic Prometheus-shaped fleet.  Deterministic in the GLOBAL service
// id so every world size sees the same fleet (docs/BRAIN_SPEC.md, "synthetic
// fleet"); mirrors the daily/weekly seasonality + noise + injected faults of
// examples/spring-boot-demo/src/main/resources/load.txt.
// ---------------------------------------------------------------------------
struct SynthParams {
  float level, amp_d, amp_w, phase, noise;
};

__host__ __device__ __forceinline__ SynthParams synth_params(uint32_t gs, uint32_t m, uint32_t seed) {
  const uint32_t key = gs * 64u + m;
  SynthParams p;
  p.level = 1.0f + 99.0f * u01(hash3(key, 0u, seed));
  p.amp_d = 0.1f + 0.3f * u01(hash3(key, 1u, seed));
  p.amp_w = 0.01f + 0.04f * u01(hash3(key, 2u, seed));
  p.phase = 6.2831853f * u01(hash3(key, 3u, seed));
  p.noise = 0.005f + 0.015f * u01(hash3(key, 4u, seed));
  return p;
}

__device__ __forceinline__ float synth_value(const SynthParams& p, uint32_t key, int64_t t, uint32_t stream_id,
                                             uint32_t seed) {
  const float tf = (float)t;
  const float season = 1.0f + p.amp_d * sinf(6.2831853f * tf / 1440.0f + p.phase) +
                       p.amp_w * sinf(6.2831853f * tf / 10080.0f + p.phase);
  const uint32_t h1 = hash3(key, (uint32_t)t * 2654435761u + stream_id, seed ^ 0xA5A5A5A5u);
  const uint32_t h2 = hash_u32(h1 ^ 0x68E31DA4u);
  const float g = sqrtf(-2.0f * logf(u01(h1))) * cosf(6.2831853f * u01(h2));
  float v = p.level * season * (1.0f + p.noise * g);
  return v > 0.f ? v : 0.f;
}

// kind: 0 = history [R, ld] for t in [0, T); 1 = baseline (P pods x W points,
// t in [T-W, T)); 2 = current (P pods x W points, t in [T, T+W)) with faults
// injected into services whose hash falls under fault_rate.
__global__ void synth_kernel(float* __restrict__ out, int64_t ld, int64_t n_per_row, int64_t S, int M,
                             int64_t svc0, int T, int P, int W, int kind, float fault_rate, float fault_mag,
                             uint32_t seed) {
  const int64_t total = S * M * n_per_row;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = e / n_per_row;
    const int64_t j = e - row * n_per_row;
    const uint32_t gs = (uint32_t)(svc0 + row / M);
    const uint32_t m = (uint32_t)(row % M);
    const SynthParams p = synth_params(gs, m, seed);
    const uint32_t key = gs * 64u + m;
    float v;
    if (kind == 0) {
      v = synth_value(p, key, j, 0u, seed);
    } else {
      const int64_t pod = j / W, w = j - pod * W;
      const int64_t t = (kind == 1) ? (T - W + w) : (T + w);
      v = synth_value(p, key, t, 1000u + (uint32_t)pod + (kind == 2 ? 500u : 0u), seed);
      if (kind == 2) {
        const bool faulty = u01(hash3(gs, 7u, seed)) < fault_rate;
        if (faulty && (m % 4u) == 0u) v = v + p.level * fault_mag * (1.0f + p.amp_d + p.amp_w);
      }
    }
    out[row * ld + j] = v;
  }
  // padding columns of the history are NaN (missing samples)
  if (kind == 0 && ld > n_per_row) {
    const int64_t pad = ld - n_per_row;
    const int64_t tp = S * M * pad;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tp; e += (int64_t)gridDim.x * blockDim.x) {
      const int64_t row = e / pad;
      out[row * ld + n_per_row + (e - row * pad)] = NAN;
    }
  }
}

FM_API int fm_synth_fleet(float* out, int64_t ld, int64_t n_per_row, int64_t S, int M, int64_t svc0, int T, int P,
                          int W, int kind, float fault_rate, float fault_mag, uint32_t seed, hipStream_t stream) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(synth_kernel, dim3(2048), dim3(256), 0, stream, out, ld, n_per_row, S, M, svc0, T, P, W, kind,
                     fault_rate, fault_mag, seed);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------------------
// Self-test of the cross-lane primitives (one wave): the DPP / permlane-swap
// encodings are checked against their definitions by tests/test_canary_ops.py.
// out [12][64]: xor 1,2,4,8,16,32 | incl sum | incl max | suffix min | prev |
// next | wave sum
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void selftest_lanes_kernel(const int* __restrict__ in, int* __restrict__ out) {
  const int l = lane_id();
  const int v = in[l];
  out[0 * 64 + l] = xor_lane<1>(v);
  out[1 * 64 + l] = xor_lane<2>(v);
  out[2 * 64 + l] = xor_lane<4>(v);
  out[3 * 64 + l] = xor_lane<8>(v);
  out[4 * 64 + l] = xor_lane<16>(v);
  out[5 * 64 + l] = xor_lane<32>(v);
  out[6 * 64 + l] = wave_incl_sum(v);
  out[7 * 64 + l] = wave_incl_max(v, (int)0x80000000);
  out[8 * 64 + l] = wave_incl_suffix_min(v, 0x7fffffff);
  out[9 * 64 + l] = lane_prev(v, -1);
  out[10 * 64 + l] = lane_next(v, -2);
  out[11 * 64 + l] = wave_sum(v);
}

FM_API int fm_selftest_lanes(const int* in, int* out, hipStream_t stream) {
  hipLaunchKernelGGL(selftest_lanes_kernel, dim3(1), dim3(64), 0, stream, in, out);
  FM_LAUNCH_CHECK();
  return 0;
}

// Async device -> pinned-host copy of the fleet verdict, issued on the
// caller's stream so it is captured into the tick's HIP graph as a memcpy
// node (the whole step — tick, all-gather, host copy — is one graph launch).
FM_API int fm_front_timing_read(unsigned long long* host, int n) {
#ifdef FM_FRONT_TIMING
  if (n > 2 * 8192) n = 2 * 8192;
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_front_t), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
#else
  (void)host; (void)n;
  return (int)hipErrorNotSupported;
#endif
}

FM_API int fm_copy_d2h_async(void* dst, const void* src, int64_t bytes, hipStream_t stream) {
  if (bytes <= 0) return 0;
  return (int)hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, stream);
}
