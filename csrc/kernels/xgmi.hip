// One-shot all-reduce over the point-to-point xGMI mesh of an MI355X node.
//
// RCCL's ring all-reduce of a small message is latency-bound: 2(R-1) dependent hops, each over
// ONE of the 7 xGMI links of a GPU.  The gradient of the reference model is 900 KB, far below the
// ring's bandwidth regime, so every rank instead pulls every peer's slice directly (7 links in
// parallel, one hop) and reduces locally:
//
//   workgroup b of rank r (1024 f32 elements, 256 lanes x float4):
//     1. copy its slice of the input into r's exchange buffer (parity half e & 1 of call e);
//     2. system-scope release, then write epoch e into peer q's signal word [b][r] for every q;
//     3. wait until every peer's word [b][q] in r's own signal array reaches e (bounded: a peer
//        that never arrives sets the error word instead of hanging the GPU), system-scope acquire;
//     4. load slice b of all R exchange buffers (R-1 of them remote, over xGMI) and add them in
//        rank order, so every rank produces bit-identical sums;
//     5. mode 0 stores the (scaled) sum; mode 1 applies SGD to the parameters directly (the
//        all-reduce and the optimizer update are one kernel).
//
// Reuse safety: call e writes parity half e & 1; a rank can only start call e + 2 on workgroup b
// after every peer's workgroup b published call e + 1, which each peer's stream issues after its
// call e (and with it every read of the half) has completed.  Calls on a channel must therefore be
// stream-ordered on each rank and issued in the same order on every rank (as for any collective).
// The per-workgroup epoch counters live on the device, so the kernel replays inside hipGraphs.
#include "kernels/common.h"
#include "kernels/xgmi.h"

namespace tdl {
namespace {

__device__ __forceinline__ bool reached(uint32_t v, uint32_t e) { return (int32_t)(v - e) >= 0; }

template <int MODE, int R>
__global__ __launch_bounds__(256) void k_xgmi_allreduce(XgmiArgs a) {
  const int blk = blockIdx.x;
  const int tid = threadIdx.x;
  // (no LDS: the kernel must fit beside an LDS-heavy backward kernel it overlaps with)
  const uint32_t e = __builtin_amdgcn_readfirstlane(a.epoch[blk]) + 1u;
  const int64_t half = (int64_t)(e & 1u) * a.cap;
  const int64_t i = (int64_t)blk * kXgmiBlockElems + tid * 4;
  const bool full = i + 3 < a.n;

  // 1. publish
  float* mine = a.p.buf[a.rank] + half;
  if (full) {
    st4(mine + i, ld4(a.src + i));
  } else {
    for (int64_t j = i; j < a.n && j < i + 4; ++j) mine[j] = a.src[j];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid < kWave) {
    // 2. release (writes the XCD's L2 back to HBM for the peers' remote reads), then signal
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (tid < R && tid != a.rank)
      __hip_atomic_store(a.p.sig[tid] + (size_t)blk * kXgmiMaxRanks + a.rank, e, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    // 3. wait for the peers (one lane per peer)
    if (tid < R && tid != a.rank) {
      const uint32_t* f = a.p.sig[a.rank] + (size_t)blk * kXgmiMaxRanks + tid;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (!reached(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), e)) {
        __builtin_amdgcn_s_sleep(1);
        if ((int64_t)(__builtin_amdgcn_s_memrealtime() - t0) > a.timeout) {
          __hip_atomic_fetch_or(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();

  // 4. reduce in rank order (all loads in flight before the adds)
  if (full) {
    f4 v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = ld4(a.p.buf[r] + half + i);
    f4 acc = v[0];
#pragma unroll
    for (int r = 1; r < R; ++r) acc += v[r];
    if (MODE == 0) {
      st4(a.dst + i, a.scale == 1.f ? acc : acc * a.scale);
    } else {
      const float step = *a.lr * a.scale;
      f4 w = ld4(a.w + i);
      w -= step * acc;
      st4(a.w + i, w);
    }
  } else {
    for (int64_t j = i; j < a.n && j < i + 4; ++j) {
      float acc = a.p.buf[0][half + j];
      for (int r = 1; r < R; ++r) acc += a.p.buf[r][half + j];
      if (MODE == 0) {
        a.dst[j] = a.scale == 1.f ? acc : acc * a.scale;
      } else {
        a.w[j] -= (*a.lr * a.scale) * acc;
      }
    }
  }
  // 5. this workgroup's call counter (read back by the next call on this channel)
  if (tid == 0) a.epoch[blk] = e;
}

}  // namespace

template <int R>
void launch_r(const XgmiArgs& a, int mode, int nb, hipStream_t s) {
  if (mode == 0)
    hipLaunchKernelGGL((k_xgmi_allreduce<0, R>), dim3(nb), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((k_xgmi_allreduce<1, R>), dim3(nb), dim3(256), 0, s, a);
}

void xgmi_all_reduce(const XgmiArgs& a, int mode, hipStream_t s) {
  const int nb = xgmi_blocks(a.n);
  if (nb == 0) return;
  switch (a.world) {  // the rank count is a template parameter: straight-line loads, no branches
    case 1: launch_r<1>(a, mode, nb, s); break;
    case 2: launch_r<2>(a, mode, nb, s); break;
    case 3: launch_r<3>(a, mode, nb, s); break;
    case 4: launch_r<4>(a, mode, nb, s); break;
    case 5: launch_r<5>(a, mode, nb, s); break;
    case 6: launch_r<6>(a, mode, nb, s); break;
    case 7: launch_r<7>(a, mode, nb, s); break;
    case 8: launch_r<8>(a, mode, nb, s); break;
    default: break;
  }
}

}  // namespace tdl
