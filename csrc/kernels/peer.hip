// Peer publish of the per-step fleet verdict:
// every rank's decision rows land straight in rank 0's device buffer over
// xGMI, no collective and no host call on the critical path.
//
// * rank 0 exports a [depth][world * shard][4] fleet buffer and a
//   [depth][world] arrival-flag array through HIP IPC handles; every other
//   rank exports a [depth] ack array the other way round;
// * a rank publishes step k (slot k % depth) with ONE kernel: its shard's
//   rows are copied into rank 0's buffer (vector stores through the peer
//   mapping), then, after a system-scope release fence, its flag for the
//   slot is set to k + 1;
// * rank 0's comm stream waits (one wave polling the flags with acquire
//   loads, bounded by a clock budget) until every rank's flag reached k + 1,
//   copies the fleet verdict to pinned host memory, and acks slot k to every
//   rank; a rank waits for that ack before it reuses the slot (k + depth).
//
// The waits are bounded: a wave that sees no progress for `budget` cycles
// gives up, records it in a status word and exits, so a rank that died never
// leaves a kernel spinning on the GPU.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "fm_common.h"

namespace {

__device__ inline void store_release_sys(unsigned* p, unsigned v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ inline unsigned load_acquire_sys(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Copy n4 float4 rows src -> dst, then publish `value` to *flag.  Blocks
// count their arrival on `arrive` (device-local); the last one fences and
// sets the flag, then re-arms the counter.
__global__ void __launch_bounds__(256) peer_publish_kernel(const float4* __restrict__ src, float4* dst, int64_t n4,
                                                           unsigned* flag, unsigned value, unsigned* arrive) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 == gridDim.x) {
      __threadfence_system();
      store_release_sys(flag, value);
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// One wave: lane r < n waits until flags[r * stride] >= value.  status[0]
// gets 1 if the budget ran out (the caller checks it after the run).
__global__ void __launch_bounds__(64) peer_wait_kernel(const unsigned* flags, int n, int64_t stride, unsigned value,
                                                       long long budget, unsigned* status) {
  const int r = threadIdx.x;
  bool done = r >= n;
  const long long t0 = clock64();
  long long spins = 0;
  while (true) {
    if (!done) done = (int)(load_acquire_sys(flags + (int64_t)r * stride) - value) >= 0;
    // every lane leaves together: the wave exits once all flags arrived or
    // the budget is spent (no lane can keep the wave alive forever)
    const bool all = __all(done);
    if (all) break;
    if (clock64() - t0 > budget) {
      if (!done) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
    ++spins;
  }
  (void)spins;
}

// Release `value` to n remote words (rank 0 -> every rank's ack for a slot).
__global__ void peer_ack_kernel(unsigned* const* dst, int n, unsigned value) {
  const int r = threadIdx.x;
  __threadfence_system();
  if (r < n && dst[r] != nullptr) store_release_sys(dst[r], value);
}

// ---------------------------------------------------------------- device step counter
// The captured-graph form (one graph launch per slot, no host argument that
// changes per step): every rank keeps its step number k in a device word
// `ctr`; the kernels of a step read it, and the step's last kernel stores
// k + 1.  `slot` is fixed per graph (the ring slot k % depth of the steps it
// serves); `slot_status[slot]` records whether this step's wait timed out, so
// the rest of the step skips its writes (no overwrite of a slot rank 0 did
// not consume, no ack of a partial fleet) and the host reads it per retired
// step.

// Wait until every lane's word (base + r * stride, r < n) reached k + 1 - lag
// (lag = depth for the slot-reuse ack wait: nothing to wait for while
// k < lag).  status[0] |= 1 and slot_status[slot] = 1 on timeout, else
// slot_status[slot] = 0.
__global__ void __launch_bounds__(64) peer_wait_ctr_kernel(const unsigned* base, int n, int64_t stride,
                                                           const unsigned* ctr, unsigned lag, long long budget,
                                                           unsigned* status, unsigned* slot_status, int slot) {
  const unsigned k = *ctr;
  const int r = threadIdx.x;
  bool done = r >= n || k < lag;
  const unsigned value = k + 1u - lag;
  const long long t0 = clock64();
  bool timed_out = false;
  while (true) {
    if (!done) done = (int)(load_acquire_sys(base + (int64_t)r * stride) - value) >= 0;
    if (__all(done)) break;
    if (clock64() - t0 > budget) {
      timed_out = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  const bool bad = __any(timed_out && !done);
  if (r == 0) {
    slot_status[slot] = bad ? 1u : 0u;
    if (bad) __hip_atomic_fetch_or(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Publish step k = *ctr: src rows -> dst, then flag = k + 1 (skipped when
// this slot's ack wait timed out).  bump: the last block stores *ctr = k + 1.
__global__ void __launch_bounds__(256) peer_publish_ctr_kernel(const float4* __restrict__ src, float4* dst, int64_t n4,
                                                               unsigned* flag, unsigned* ctr, unsigned* arrive,
                                                               const unsigned* slot_status, int slot, int bump) {
  const unsigned k = *ctr;
  const bool skip = slot_status != nullptr && slot_status[slot] != 0u;
  if (!skip)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
      dst[i] = src[i];
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev + 1 == gridDim.x) {
      __threadfence_system();
      if (!skip) store_release_sys(flag, k + 1u);
      __hip_atomic_store(arrive, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (bump) __hip_atomic_store(ctr, k + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Rank 0: ack step k = *ctr of the slot to every rank (skipped when the
// collect wait timed out: the fleet copy is partial), then *ctr = k + 1.
__global__ void peer_ack_ctr_kernel(unsigned* const* dst, int n, unsigned* ctr, const unsigned* slot_status,
                                    int slot) {
  const unsigned k = *ctr;
  const int r = threadIdx.x;
  __threadfence_system();
  if (r < n && dst[r] != nullptr && slot_status[slot] == 0u) store_release_sys(dst[r], k + 1u);
  __syncthreads();
  if (r == 0) __hip_atomic_store(ctr, k + 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace

// ---------------------------------------------------------------- IPC handles
FM_API int fm_ipc_handle_size() { return (int)sizeof(hipIpcMemHandle_t); }

// The handle names the whole allocation `ptr` lives in (a caching allocator
// sub-allocates tensors from larger blocks): `offset` is ptr's distance from
// the allocation's base, which the importer adds to its mapping.
FM_API int fm_ipc_get_handle(void* ptr, void* out, int64_t* offset) {
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, ptr);
  if (e != hipSuccess) return (int)e;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  e = hipMemGetAddressRange(&base, &size, ptr);
  if (e != hipSuccess) return (int)e;
  std::memcpy(out, &h, sizeof(h));
  *offset = (int64_t)((char*)ptr - (char*)base);
  return 0;
}

FM_API int fm_ipc_open(const void* handle, void** out) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
}

FM_API int fm_ipc_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }

// ---------------------------------------------------------------- kernels
// src / dst 16-byte aligned, bytes a multiple of 16.
FM_API int fm_peer_publish(const void* src, void* dst, int64_t bytes, unsigned* flag, unsigned value,
                           unsigned* arrive, hipStream_t stream) {
  if (bytes < 0 || bytes % 16 != 0 || ((uintptr_t)src | (uintptr_t)dst) % 16 != 0) return (int)hipErrorInvalidValue;
  const int64_t n4 = bytes / 16;
  int blocks = (int)((n4 + 256 * 8 - 1) / (256 * 8));
  blocks = blocks < 1 ? 1 : (blocks > 64 ? 64 : blocks);
  hipLaunchKernelGGL(peer_publish_kernel, dim3(blocks), dim3(256), 0, stream, (const float4*)src, (float4*)dst, n4,
                     flag, value, arrive);
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_peer_wait(const unsigned* flags, int n, int64_t stride, unsigned value, long long budget_cycles,
                        unsigned* status, hipStream_t stream) {
  if (n < 0 || n > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_wait_kernel, dim3(1), dim3(64), 0, stream, flags, n, stride, value, budget_cycles, status);
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_peer_ack(unsigned* const* dst, int n, unsigned value, hipStream_t stream) {
  if (n < 0 || n > 64) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_ack_kernel, dim3(1), dim3(64), 0, stream, dst, n, value);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- device-counter forms (graph-capturable)
FM_API int fm_peer_wait_ctr(const unsigned* base, int n, int64_t stride, const unsigned* ctr, unsigned lag,
                            long long budget_cycles, unsigned* status, unsigned* slot_status, int slot,
                            hipStream_t stream) {
  if (n < 0 || n > 64 || slot < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_wait_ctr_kernel, dim3(1), dim3(64), 0, stream, base, n, stride, ctr, lag, budget_cycles,
                     status, slot_status, slot);
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_peer_publish_ctr(const void* src, void* dst, int64_t bytes, unsigned* flag, unsigned* ctr,
                               unsigned* arrive, const unsigned* slot_status, int slot, int bump, hipStream_t stream) {
  if (bytes < 0 || bytes % 16 != 0 || ((uintptr_t)src | (uintptr_t)dst) % 16 != 0 || slot < 0)
    return (int)hipErrorInvalidValue;
  const int64_t n4 = bytes / 16;
  int blocks = (int)((n4 + 256 * 8 - 1) / (256 * 8));
  blocks = blocks < 1 ? 1 : (blocks > 64 ? 64 : blocks);
  hipLaunchKernelGGL(peer_publish_ctr_kernel, dim3(blocks), dim3(256), 0, stream, (const float4*)src, (float4*)dst,
                     n4, flag, ctr, arrive, slot_status, slot, bump);
  FM_LAUNCH_CHECK();
  return 0;
}

FM_API int fm_peer_ack_ctr(unsigned* const* dst, int n, unsigned* ctr, const unsigned* slot_status, int slot,
                           hipStream_t stream) {
  if (n < 0 || n > 64 || slot < 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(peer_ack_ctr_kernel, dim3(1), dim3(64), 0, stream, dst, n, ctr, slot_status, slot);
  FM_LAUNCH_CHECK();
  return 0;
}

// ---------------------------------------------------------------- board copies
// Copy between any two addresses this process can name (host memory, its own
// device memory, a peer's memory opened through IPC): the brain's
// rank-to-rank board (parallel/board.py) moves gauge vectors and verdict rows
// with the DMA engines over xGMI.  Every copy goes on the board's OWN
// non-blocking stream (one per device, created on first use) and the host
// waits for that stream only: a board copy never queues behind, or holds up,
// work on the null / default stream (an early-launched LSTM forecast, the
// scoring graph), and a seqlock header written after the payload is only
// issued once the payload has landed.
#include <mutex>

namespace {
constexpr int kMaxDevices = 64;
hipStream_t g_board_stream[kMaxDevices] = {};
std::mutex g_board_mu;

hipError_t board_stream(hipStream_t* out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  if (dev < 0 || dev >= kMaxDevices) return hipErrorInvalidDevice;
  std::lock_guard<std::mutex> g(g_board_mu);
  if (g_board_stream[dev] == nullptr) {
    e = hipStreamCreateWithFlags(&g_board_stream[dev], hipStreamNonBlocking);
    if (e != hipSuccess) return e;
  }
  *out = g_board_stream[dev];
  return hipSuccess;
}
}  // namespace

FM_API int fm_board_copy(void* dst, const void* src, int64_t bytes) {
  if (bytes <= 0) return 0;
  hipStream_t s = nullptr;
  hipError_t e = board_stream(&s);
  if (e != hipSuccess) return (int)e;
  e = hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDefault, s);
  if (e != hipSuccess) return (int)e;
  return (int)hipStreamSynchronize(s);
}

// Null-stream form (kept for the A/B in tools/peer_bench.py).
FM_API int fm_memcpy_sync(void* dst, const void* src, int64_t bytes) {
  if (bytes <= 0) return 0;
  return (int)hipMemcpy(dst, src, (size_t)bytes, hipMemcpyDefault);
}
