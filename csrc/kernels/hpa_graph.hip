// K8: HPA score and K9: downstream-impact propagation.
//
// K8 (docs/dynamic_autoscaling.md:30-130, examples/hpa/images/HPA_Score.png,
// examples/hpa/README.MD:26-64): per service the template metrics are placed
// against their learned [lower, upper] band; load metrics above the band AND an
// SLA metric violated -> score > 50 (scale up); load below the band with the SLA
// met -> score < 50 (scale down); otherwise 50.  Breath-up < breath-down
// hysteresis and a flip counter suppress oscillation.  Exact rules:
// docs/BRAIN_SPEC.md §7.  One thread per service; state is updated in place.
//
// K9 (README.md:24,27; CallerWebMvcTagsProvider.java:22-28): the caller->callee
// graph built from the `caller` tag; downstream impact of u after k hops is
// max over paths of (edge weight product) * anomaly score of the reached callee.
// CSR max-times SpMV, one wave per row, k launches ping-ponging two buffers.
#include "fm_common.h"

using namespace fm;

__global__ __launch_bounds__(256) void hpa_score_kernel(
    const float* __restrict__ cur, const float* __restrict__ upper, const float* __restrict__ lower, int64_t S, int Mt,
    const float* __restrict__ weight, const int8_t* __restrict__ is_increase, const int8_t* __restrict__ is_absolute,
    const int8_t* __restrict__ role, double now, float breath_up, float breath_down, int max_flips,
    float flip_window, int8_t* __restrict__ last_dir_, double* __restrict__ last_time_, int* __restrict__ flips_,
    double* __restrict__ flip_t0_, int* __restrict__ score_out, int8_t* __restrict__ reason_out,
    float* __restrict__ raw_out, const int64_t* __restrict__ slots, int* __restrict__ packed_out) {
  const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= S) return;
  // the hysteresis state of service s: slot slots[s] of the device table
  // (in place, no gather / scatter) or row s of compact state arrays
  const int64_t q = slots != nullptr ? slots[s] : s;
  int8_t* last_dir = last_dir_ + q;
  double* last_time = last_time_ + q;
  int* flips = flips_ + q;
  double* flip_t0 = flip_t0_ + q;
  float up = 0.f, down = 0.f;
  bool has_sla = false, sla_violated = false;
  for (int j = 0; j < Mt; ++j) {
    const float c = cur[s * Mt + j], u = upper[s * Mt + j], l = lower[s * Mt + j];
    if (role[j] == 1) has_sla = true;
    if (!isfinite(c) || !isfinite(u) || !isfinite(l)) continue;
    float scale = is_absolute[j] ? fmaxf(fabsf(u), 1e-12f) : fmaxf(u - l, 1e-12f);
    float dev = 0.f;
    if (c > u) dev = (c - u) / scale;
    else if (c < l) dev = (c - l) / scale;
    if (!is_increase[j]) dev = -dev;
    if (role[j] == 1) {
      if (dev > 0.f) sla_violated = true;
    } else {
      const float w = weight[j];
      if (dev > 0.f) up = fmaxf(up, w * dev);
      if (dev < 0.f) down = fmaxf(down, -w * dev);
    }
  }
  if (!has_sla) sla_violated = up > 0.f;
  int raw = 50;
  if (up > 0.f && sla_violated) raw = 50 + (int)lrintf(50.f * fminf(1.f, up));
  else if (down > 0.f && up == 0.f && !sla_violated) raw = 50 - (int)lrintf(50.f * fminf(1.f, down));
  if (raw_out != nullptr) raw_out[s] = (float)raw;
  int dir = raw > 50 ? 1 : (raw < 50 ? -1 : 0);
  int8_t reason = dir > 0 ? 1 : (dir < 0 ? 2 : 0);
  int score = raw;
  if (now - *flip_t0 > flip_window) { *flips = 0; *flip_t0 = now; }
  if (dir != 0) {
    const int ld = *last_dir;
    const float wait = dir > 0 ? breath_up : breath_down;
    if (ld != 0 && now - *last_time < wait) {
      score = 50; reason = 3;
    } else if (ld != 0 && dir != ld && *flips >= max_flips) {
      score = 50; reason = 4;
    } else {
      if (ld != 0 && dir != ld) *flips += 1;
      *last_dir = (int8_t)dir;
      *last_time = now;
    }
  }
  if (score_out != nullptr) score_out[s] = score;
  if (reason_out != nullptr) reason_out[s] = reason;
  if (packed_out != nullptr) packed_out[s] = score | ((int)reason << 16);
}

FM_API int fm_hpa_score(const float* cur, const float* upper, const float* lower, int64_t S, int Mt, const float* weight,
                        const int8_t* is_increase, const int8_t* is_absolute, const int8_t* role, double now,
                        float breath_up, float breath_down, int max_flips, float flip_window, int8_t* last_dir,
                        double* last_time, int* flips, double* flip_t0, int* score, int8_t* reason, float* raw,
                        hipStream_t stream) {
  if (S <= 0) return 0;
  hipLaunchKernelGGL(hpa_score_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, cur, upper, lower, S,
                     Mt, weight, is_increase, is_absolute, role, now, breath_up, breath_down, max_flips, flip_window,
                     last_dir, last_time, flips, flip_t0, score, reason, raw, nullptr, nullptr);
  FM_LAUNCH_CHECK();
  return 0;
}

// The brain's steady HPA cycle: the services' hysteresis state read and
// updated in place through ``slots`` (the device HPA table), the verdict as
// one int per service (score | reason << 16) for a single device->host copy.
FM_API int fm_hpa_score_slots(const float* cur, const float* upper, const float* lower, int64_t S, int Mt,
                              const float* weight, const int8_t* is_increase, const int8_t* is_absolute,
                              const int8_t* role, double now, float breath_up, float breath_down, int max_flips,
                              float flip_window, int8_t* last_dir, double* last_time, int* flips, double* flip_t0,
                              const int64_t* slots, int* packed, hipStream_t stream) {
  if (S <= 0) return 0;
  if (slots == nullptr || packed == nullptr) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(hpa_score_kernel, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, cur, upper, lower, S,
                     Mt, weight, is_increase, is_absolute, role, now, breath_up, breath_down, max_flips, flip_window,
                     last_dir, last_time, flips, flip_t0, nullptr, nullptr, nullptr, slots, packed);
  FM_LAUNCH_CHECK();
  return 0;
}

__global__ __launch_bounds__(256) void impact_hop_kernel(const int64_t* __restrict__ rowptr,
                                                         const int* __restrict__ col, const float* __restrict__ w,
                                                         const float* __restrict__ a, const float* __restrict__ prev,
                                                         int64_t S, float* __restrict__ out) {
  const int64_t u = (int64_t)blockIdx.x * 4 + wave_id();
  if (u >= S) return;
  const int lane = lane_id();
  const int64_t b = rowptr[u], e = rowptr[u + 1];
  float best = 0.f;
  for (int64_t k = b + lane; k < e; k += 64) {
    const int v = col[k];
    const float val = fmaxf(a[v], prev != nullptr ? prev[v] : 0.f) * w[k];
    best = fmaxf(best, val);
  }
  best = wave_max(best);
  if (lane == 0) out[u] = best;
}

FM_API int fm_downstream_impact(const int64_t* rowptr, const int* col, const float* w, const float* a, int64_t S,
                                int hops, float* buf0, float* buf1, hipStream_t stream) {
  if (S <= 0 || hops <= 0) return 0;
  const dim3 grid((unsigned)((S + 3) / 4)), block(256);
  const float* prev = nullptr;
  float* bufs[2] = {buf0, buf1};
  for (int h = 0; h < hops; ++h) {
    float* out = bufs[h & 1];
    hipLaunchKernelGGL(impact_hop_kernel, grid, block, 0, stream, rowptr, col, w, a, prev, S, out);
    FM_LAUNCH_CHECK();
    prev = out;
  }
  return 0;
}

// ---------------------------------------------------------------------------
// Per-cluster maximum of non-negative scores (the cross-cluster aggregate of
// the downstream-impact step).  Each block folds a grid-stride slice into an
// LDS array of K partial maxima, then merges with K global atomics; a float
// >= 0 orders like its bit pattern, so atomicMax on the int view is exact.
// (A scatter with amax over 4 targets serialises 40k atomics on 4 words.)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void segment_max_kernel(const float* __restrict__ v, const int64_t* __restrict__ seg,
                                                          int64_t S, int K, int* __restrict__ out) {
  extern __shared__ int smax[];
  for (int k = threadIdx.x; k < K; k += blockDim.x) smax[k] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < S; i += (int64_t)gridDim.x * blockDim.x) {
    const float x = v[i];
    const int64_t c = seg[i];
    if (x > 0.f && c >= 0 && c < K) atomicMax(&smax[c], __float_as_int(x));
  }
  __syncthreads();
  for (int k = threadIdx.x; k < K; k += blockDim.x)
    if (smax[k] > 0) atomicMax(&out[k], smax[k]);
}

FM_API int fm_segment_max(const float* v, const int64_t* seg, int64_t S, int K, float* out, hipStream_t stream) {
  if (K <= 0 || K > 16384) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(out, 0, sizeof(float) * (size_t)K, stream);
  if (e != hipSuccess) return (int)e;
  if (S <= 0) return 0;
  int64_t blocks = (S + 2047) / 2048;
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(segment_max_kernel, dim3((unsigned)blocks), dim3(256), sizeof(int) * K, stream, v, seg, S, K,
                     reinterpret_cast<int*>(out));
  FM_LAUNCH_CHECK();
  return 0;
}
