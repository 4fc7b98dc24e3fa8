// K5: bivariate normal detector ("Two Metrics" column of the model table,
// docs/guides/design.md:74-79).  For a metric pair (a, b) of one service the
// history gives the mean vector and 2x2 covariance; each current point pair is
// scored by its Mahalanobis distance d = sqrt(dx' S^-1 dx) and flagged when
// d > threshold (threshold in sigma units, like the univariate models).
//
// One 256-thread workgroup per pair; both history rows are read once with
// 16-B loads and kept in registers for the two-pass moments.
#include "fm_common.h"

using namespace fm;

template <int NV>
__global__ __launch_bounds__(256) void bivariate_kernel(const float* __restrict__ ha, const float* __restrict__ hb,
                                                        int64_t ld_h, int T, const float* __restrict__ ca,
                                                        const float* __restrict__ cb, int64_t ld_c, int n,
                                                        int64_t P, const float* __restrict__ thr,
                                                        float* __restrict__ params /*[P,5]*/,
                                                        float* __restrict__ dist /*[P,n]*/,
                                                        unsigned long long* __restrict__ flags, int NW,
                                                        int* __restrict__ count) {
  __shared__ double red[4];
  __shared__ int redi[4];
  const int64_t p = blockIdx.x;
  const int tid = threadIdx.x;
  const float4* ra = reinterpret_cast<const float4*>(ha + p * ld_h);
  const float4* rb = reinterpret_cast<const float4*>(hb + p * ld_h);
  const int nq = (T + 3) >> 2;
  float4 qa[NV], qb[NV];
  double sa = 0, sb = 0;
  int c = 0;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int qi = tid + j * 256;
    float4 a = make_float4(NAN, NAN, NAN, NAN), b = a;
    if (qi < nq) {
      a = ra[qi]; b = rb[qi];
      const int e0 = qi * 4;
      if (e0 + 1 >= T) { a.y = NAN; b.y = NAN; }
      if (e0 + 2 >= T) { a.z = NAN; b.z = NAN; }
      if (e0 + 3 >= T) { a.w = NAN; b.w = NAN; }
    }
    // a pair counts only when both coordinates are present
    if (!(isfinite(a.x) && isfinite(b.x))) { a.x = NAN; b.x = NAN; }
    if (!(isfinite(a.y) && isfinite(b.y))) { a.y = NAN; b.y = NAN; }
    if (!(isfinite(a.z) && isfinite(b.z))) { a.z = NAN; b.z = NAN; }
    if (!(isfinite(a.w) && isfinite(b.w))) { a.w = NAN; b.w = NAN; }
    qa[j] = a; qb[j] = b;
    if (isfinite(a.x)) { sa += a.x; sb += b.x; ++c; }
    if (isfinite(a.y)) { sa += a.y; sb += b.y; ++c; }
    if (isfinite(a.z)) { sa += a.z; sb += b.z; ++c; }
    if (isfinite(a.w)) { sa += a.w; sb += b.w; ++c; }
  }
  sa = block_sum<256>(sa, red);
  sb = block_sum<256>(sb, red);
  c = block_sum<256>(c, redi);
  const float ma = c > 0 ? (float)(sa / c) : 0.f, mb = c > 0 ? (float)(sb / c) : 0.f;
  float vaa = 0.f, vbb = 0.f, vab = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const float av[4] = {qa[j].x, qa[j].y, qa[j].z, qa[j].w};
    const float bv[4] = {qb[j].x, qb[j].y, qb[j].z, qb[j].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (isfinite(av[e])) {
        const float da = av[e] - ma, db = bv[e] - mb;
        vaa += da * da; vbb += db * db; vab += da * db;
      }
    }
  }
  const double saa = block_sum<256>((double)vaa, red), sbb = block_sum<256>((double)vbb, red),
               sab = block_sum<256>((double)vab, red);
  const double den = c > 1 ? (double)(c - 1) : 1.0;
  const double Caa = saa / den, Cbb = sbb / den, Cab = sab / den;
  double det = Caa * Cbb - Cab * Cab;
  // regularise a (near-)singular covariance
  const double eps = 1e-9 * (Caa + Cbb) + 1e-30;
  if (det < eps * eps) det = (Caa + eps) * (Cbb + eps) - Cab * Cab;
  const float iaa = (float)(Cbb / det), ibb = (float)(Caa / det), iab = (float)(-Cab / det);
  const float th = thr[0];
  int cnt = 0;
  for (int i0 = 0; i0 < n; i0 += 256) {
    const int i = i0 + tid;
    bool f = false;
    if (i < n) {
      const float xa = ca[p * ld_c + i], xb = cb[p * ld_c + i];
      float d = NAN;
      if (isfinite(xa) && isfinite(xb) && c > 1) {
        const float da = xa - ma, db = xb - mb;
        const float q = da * da * iaa + 2.f * da * db * iab + db * db * ibb;
        d = sqrtf(fmaxf(q, 0.f));
        f = d > th;
        cnt += f;
      }
      dist[p * n + i] = d;
    }
    const unsigned long long bal = __ballot(f);
    const int w = i0 / 64 + wave_id();
    if (lane_id() == 0 && w < NW) flags[p * NW + w] = bal;
  }
  cnt = block_sum<256>(cnt, redi);
  if (tid == 0) {
    params[p * 5 + 0] = ma; params[p * 5 + 1] = mb;
    params[p * 5 + 2] = (float)Caa; params[p * 5 + 3] = (float)Cab; params[p * 5 + 4] = (float)Cbb;
    count[p] = cnt;
  }
}

FM_API int fm_bivariate(const float* ha, const float* hb, int64_t ld_h, int T, const float* ca, const float* cb,
                        int64_t ld_c, int n, int64_t P, const float* thr, float* params, float* dist,
                        unsigned long long* flags, int NW, int* count, hipStream_t stream) {
  if (P <= 0) return 0;
  if ((ld_h & 3) || (((uintptr_t)ha) & 15) || (((uintptr_t)hb) & 15) || NW * 64 < n) return (int)hipErrorInvalidValue;
  const int nq = (T + 3) / 4;
  const dim3 grid((unsigned)P), block(256);
#define FM_BV(NVV) hipLaunchKernelGGL(bivariate_kernel<NVV>, grid, block, 0, stream, ha, hb, ld_h, T, ca, cb, ld_c, n, \
                                      P, thr, params, dist, flags, NW, count)
  if (nq <= 256 * 2) FM_BV(2);
  else if (nq <= 256 * 4) FM_BV(4);
  else if (nq <= 256 * 8) FM_BV(8);
  else if (nq <= 256 * 10) FM_BV(10);
  else if (nq <= 256 * 16) FM_BV(16);
  else return (int)hipErrorInvalidValue;
#undef FM_BV
  FM_LAUNCH_CHECK();
  return 0;
}
