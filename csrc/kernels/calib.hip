// Counter calibration: a pure streaming read of a known number of bytes
// (16-B nontemporal loads, one pass, a per-workgroup partial sum written so the
// loads are not dead).  tools/fetch_calib.py runs it under
// ``rocprofv3 --pmc FETCH_SIZE`` next to the tick's history kernel, so the
// tick's counter-based bytes can be stated against a kernel whose bytes are
// exactly known.
#include "fm_common.h"

using namespace fm;

typedef float nt4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void stream_read_kernel(const nt4* __restrict__ x, int64_t n4,
                                                          float* __restrict__ partial) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const nt4 v = __builtin_nontemporal_load(x + i);
    acc += (v.x + v.y) + (v.z + v.w);
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

FM_API int fm_stream_read(const float* x, int64_t n, float* partial, int blocks, hipStream_t stream) {
  if (n <= 0 || (n & 3) || (((uintptr_t)x) & 15) || blocks <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(stream_read_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     reinterpret_cast<const nt4*>(x), n / 4, partial);
  FM_LAUNCH_CHECK();
  return 0;
}
