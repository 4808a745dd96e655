// One-shot all-reduce over the xGMI mesh of an MI355X node (csrc/kernels/xgmi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

constexpr int kXgmiMaxRanks = 8;
constexpr int kXgmiBlockElems = 1024;  // f32 elements reduced by one 256-thread workgroup

// Device addresses of every rank's exchange buffers, in this process's address space (the
// peers' are IPC-mapped): buf[r] = [input | result] x 2 parity halves of `cap` f32 each,
// sig[r] = [2 rounds][blocks][kXgmiMaxRanks] epoch words written by the peers.
struct XgmiPeers {
  float* buf[kXgmiMaxRanks];
  uint32_t* sig[kXgmiMaxRanks];
};

struct XgmiArgs {
  XgmiPeers p;
  const float* src;  // this rank's contribution [n]
  float* dst;        // mode 0: reduced result [n] (may alias src)
  float* w;          // mode 1: parameters updated w -= lr * scale * sum
  const float* lr;   // mode 1: device learning rate
  uint32_t* epoch;   // this rank's per-workgroup call counters [blocks] (local)
  uint32_t* err;     // this rank's error word (bit 0: a peer did not arrive in time)
  int64_t n;
  int64_t cap;
  int64_t shard;     // two-shot: elements per rank's shard (multiple of kXgmiBlockElems)
  int sig_blocks;    // workgroup capacity of the signal arrays (stride of the second round)
  int64_t timeout;   // 100 MHz s_memrealtime ticks
  float scale;
  int rank;
  int world;
};

inline int xgmi_blocks(int64_t n) { return (int)((n + kXgmiBlockElems - 1) / kXgmiBlockElems); }
inline int64_t xgmi_shard(int64_t n, int world) {
  return (int64_t)xgmi_blocks((n + world - 1) / world) * kXgmiBlockElems;
}

// mode 0: dst = scale * sum_r src_r ; mode 1: w -= lr * scale * sum_r src_r
// algo 0: one-shot (every rank reduces everything: one hop, R-1 full remote reads);
// algo 1: two-shot (reduce-scatter + all-gather: 2 hops, 2 (R-1)/R remote reads per rank)
void xgmi_all_reduce(const XgmiArgs& a, int mode, int algo, hipStream_t s);

}  // namespace tdl
