// One-shot and two-shot all-reduce over the point-to-point xGMI mesh of an MI355X node.
//
// RCCL's ring all-reduce of a small message is latency-bound: 2(R-1) dependent hops, each over
// ONE of the 7 xGMI links of a GPU.  The gradient of the reference model is 900 KB, far below the
// ring's bandwidth regime, so ranks read each other's buffers directly, all 7 links in parallel:
//
// ONE-SHOT (small messages): every rank pulls every peer's slice and reduces everything locally
// (one hop; (R-1) x n bytes over the rank's R-1 links).
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
// TWO-SHOT (larger messages at R >= 3): workgroup c publishes chunk c of every rank's shard,
// reduces chunk c of ITS OWN shard from all ranks (reduce-scatter), publishes the result, then
// copies chunk c of every other shard's result (all-gather): two hops, but only 2 (R-1)/R x n
// bytes per rank, n/R per link and phase.  With the SGD epilogue the owner of a shard applies the
// update and the others copy the updated parameters, so replicas stay identical by construction.
//
// Reuse safety: call e writes parity half e & 1; a rank can only start call e + 2 on workgroup b
// after every peer's workgroup b published call e + 1, which each peer's stream issues after its
// call e (and with it every read of the half) has completed.  Calls on a channel must therefore be
// stream-ordered on each rank and issued in the same order on every rank (as for any collective).
// The per-workgroup epoch counters live on the device, so the kernel replays inside hipGraphs.
#include "kernels/xgmi_device.h"

namespace tdl {
namespace {

template <int R>
__device__ __forceinline__ bool exchange(const XgmiArgs& a, int round, int blk, uint32_t e) {
  return xgmi_exchange<R>(a.p, a.rank, a.sig_blocks, a.timeout, a.err, round, blk, e);
}

// rank-order sum of element i (float4) over the R input halves
template <int R>
__device__ __forceinline__ f4 sum_ranks(const XgmiArgs& a, int64_t off) {
  f4 v[R];
#pragma unroll
  for (int r = 0; r < R; ++r) v[r] = ld4(a.p.buf[r] + off);
  f4 acc = v[0];
#pragma unroll
  for (int r = 1; r < R; ++r) acc += v[r];
  return acc;
}

template <int R>
__device__ __forceinline__ float sum_ranks1(const XgmiArgs& a, int64_t off) {
  float acc = a.p.buf[0][off];
#pragma unroll
  for (int r = 1; r < R; ++r) acc += a.p.buf[r][off];
  return acc;
}

// epilogue of a reduced value: mode 0 scaled sum, mode 1 SGD-updated parameter
template <int MODE>
__device__ __forceinline__ f4 finish4(const XgmiArgs& a, int64_t i, f4 acc) {
  if (MODE == 0) return a.scale == 1.f ? acc : acc * a.scale;
  const float step = *a.lr * a.scale;
  f4 w = ld4(a.w + i);
  w -= step * acc;
  return w;
}

template <int MODE>
__device__ __forceinline__ float finish1(const XgmiArgs& a, int64_t j, float acc) {
  if (MODE == 0) return a.scale == 1.f ? acc : acc * a.scale;
  return a.w[j] - (*a.lr * a.scale) * acc;
}

template <int MODE, int R>
__global__ __launch_bounds__(256) void k_xgmi_oneshot(XgmiArgs a) {
  const int blk = blockIdx.x;
  const int tid = threadIdx.x;
  // (no LDS: the kernel must fit beside an LDS-heavy backward kernel it overlaps with)
  const uint32_t e = __builtin_amdgcn_readfirstlane(a.epoch[blk]) + 1u;
  const int64_t half = (int64_t)(e & 1u) * 2 * a.cap;  // [input | result] per parity
  const int64_t i = (int64_t)blk * kXgmiBlockElems + tid * 4;
  const bool full = i + 3 < a.n;
  float* out = MODE == 0 ? a.dst : a.w;
  if (xgmi_failed(a.err)) {  // a peer already failed to arrive: do not wait again
    if (tid == 0) a.epoch[blk] = e;
    return;
  }

  // 1. publish
  float* mine = a.p.buf[a.rank] + half;
  if (full) {
    st4(mine + i, ld4(a.src + i));
  } else {
    for (int64_t j = i; j < a.n && j < i + 4; ++j) mine[j] = a.src[j];
  }
  // 2-3. signal the peers, wait for them
  if (!exchange<R>(a, 0, blk, e)) {
    if (tid == 0) a.epoch[blk] = e;
    return;
  }
  // 4-5. reduce in rank order (all loads in flight before the adds), epilogue
  if (full) {
    st4(out + i, finish4<MODE>(a, i, sum_ranks<R>(a, half + i)));
  } else {
    for (int64_t j = i; j < a.n && j < i + 4; ++j) out[j] = finish1<MODE>(a, j, sum_ranks1<R>(a, half + j));
  }
  if (tid == 0) a.epoch[blk] = e;
}

template <int MODE, int R>
__global__ __launch_bounds__(256) void k_xgmi_twoshot(XgmiArgs a) {
  const int c = blockIdx.x;  // chunk index within every shard
  const int tid = threadIdx.x;
  const uint32_t e = __builtin_amdgcn_readfirstlane(a.epoch[c]) + 1u;
  const int64_t half = (int64_t)(e & 1u) * 2 * a.cap;
  const int64_t res = half + a.cap;  // result region of this parity
  const int64_t within = (int64_t)c * kXgmiBlockElems + tid * 4;
  float* out = MODE == 0 ? a.dst : a.w;
  float* mine = a.p.buf[a.rank];
  if (xgmi_failed(a.err)) {
    if (tid == 0) a.epoch[c] = e;
    return;
  }

  // 1. publish chunk c of every shard (reads all of src before any write of out: in place is safe)
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int64_t i = q * a.shard + within;
    if (i + 3 < a.n) {
      st4(mine + half + i, ld4(a.src + i));
    } else {
      for (int64_t j = i; j < a.n && j < i + 4; ++j) mine[half + j] = a.src[j];
    }
  }
  if (!exchange<R>(a, 0, c, e)) {
    if (tid == 0) a.epoch[c] = e;
    return;
  }
  // 2. reduce-scatter: chunk c of this rank's shard, from every rank, in rank order.  In SGD mode
  // the updated owner shard is staged in the result region only; out (= W) is written after the
  // second exchange, so a timeout leaves W untouched on this rank.
  f4 own4 = zero4();
  {
    const int64_t i = a.rank * a.shard + within;
    if (i + 3 < a.n) {
      own4 = finish4<MODE>(a, i, sum_ranks<R>(a, half + i));
      st4(mine + res + i, own4);
    } else {
      for (int64_t j = i; j < a.n && j < i + 4; ++j) mine[res + j] = finish1<MODE>(a, j, sum_ranks1<R>(a, half + j));
    }
  }
  if (!exchange<R>(a, 1, c, e)) {
    if (tid == 0) a.epoch[c] = e;
    return;
  }
  {
    const int64_t i = a.rank * a.shard + within;
    if (i + 3 < a.n) {
      st4(out + i, own4);
    } else {
      for (int64_t j = i; j < a.n && j < i + 4; ++j) out[j] = mine[res + j];
    }
  }
  // 3. all-gather: chunk c of every other shard, from its owner's result region
#pragma unroll
  for (int q = 0; q < R; ++q) {
    if (q == a.rank) continue;
    const int64_t i = q * a.shard + within;
    const float* theirs = a.p.buf[q] + res;
    if (i + 3 < a.n) {
      st4(out + i, ld4(theirs + i));
    } else {
      for (int64_t j = i; j < a.n && j < i + 4; ++j) out[j] = theirs[j];
    }
  }
  if (tid == 0) a.epoch[c] = e;
}

template <int R>
void launch_r(const XgmiArgs& a, int mode, int algo, hipStream_t s) {
  if (algo == 0) {
    const int nb = xgmi_blocks(a.n);
    if (mode == 0)
      hipLaunchKernelGGL((k_xgmi_oneshot<0, R>), dim3(nb), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((k_xgmi_oneshot<1, R>), dim3(nb), dim3(256), 0, s, a);
  } else {
    const int nb = (int)(a.shard / kXgmiBlockElems);
    if (mode == 0)
      hipLaunchKernelGGL((k_xgmi_twoshot<0, R>), dim3(nb), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((k_xgmi_twoshot<1, R>), dim3(nb), dim3(256), 0, s, a);
  }
}

}  // namespace

void xgmi_all_reduce(const XgmiArgs& a, int mode, int algo, hipStream_t s) {
  if (a.n <= 0) return;
  switch (a.world) {  // the rank count is a template parameter: straight-line loads, no branches
    case 1: launch_r<1>(a, mode, algo, s); break;
    case 2: launch_r<2>(a, mode, algo, s); break;
    case 3: launch_r<3>(a, mode, algo, s); break;
    case 4: launch_r<4>(a, mode, algo, s); break;
    case 5: launch_r<5>(a, mode, algo, s); break;
    case 6: launch_r<6>(a, mode, algo, s); break;
    case 7: launch_r<7>(a, mode, algo, s); break;
    case 8: launch_r<8>(a, mode, algo, s); break;
    default: break;
  }
}

}  // namespace tdl
