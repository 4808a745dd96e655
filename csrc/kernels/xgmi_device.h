// Device-side pieces of the xGMI all-reduce protocol (csrc/kernels/xgmi.hip), shared with kernels
// that run an all-reduce in some of their own workgroups (the fused MNIST step).  .hip files only.
#pragma once
#include "kernels/common.h"
#include "kernels/xgmi.h"

namespace tdl {

__device__ __forceinline__ bool xgmi_reached(uint32_t v, uint32_t e) { return (int32_t)(v - e) >= 0; }

// True when a previous exchange on this device already timed out: every later exchange returns at
// once instead of spinning out its own timeout (a dead peer costs ONE timeout, not one per launch).
__device__ __forceinline__ bool xgmi_failed(const uint32_t* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// All stores of this workgroup done -> system-scope release -> epoch e into word [blk][rank] of
// every peer's signal array `round` -> wait for every peer's word [blk][q] in our own array ->
// system-scope acquire.  Returns with the whole workgroup past a barrier: true when every peer
// arrived, false when a bounded wait timed out or the device's error word was already set (the
// caller then writes nothing, so a dead or lagging peer can never leave a half-reduced gradient or
// weight behind).
template <int R>
__device__ __forceinline__ bool xgmi_exchange(const XgmiPeers& p, int rank, int sig_blocks, int64_t timeout,
                                              uint32_t* err, int round, int blk, uint32_t e) {
  const int tid = threadIdx.x;
  int timed_out = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < kWave) {
    // release: writes the XCD's L2 back so the peers' remote reads see this workgroup's stores
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const size_t word = ((size_t)round * sig_blocks + blk) * kXgmiMaxRanks;
    if (tid < R && tid != rank)
      __hip_atomic_store(p.sig[tid] + word + rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (tid < R && tid != rank) {  // one lane per peer; bounded wait
      const uint32_t* f = p.sig[rank] + word + tid;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int polls = 0;
      while (!xgmi_reached(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), e)) {
        __builtin_amdgcn_s_sleep(1);
        // another workgroup's timeout ends this wait too (checked every 64 polls)
        if ((++polls & 63) == 0 && xgmi_failed(err)) {
          timed_out = 1;
          break;
        }
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > timeout) {
          __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          timed_out = 1;
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  return __syncthreads_or(timed_out) == 0;
}

}  // namespace tdl
