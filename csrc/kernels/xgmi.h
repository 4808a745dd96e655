// One-shot all-reduce over the xGMI mesh of an MI355X node (csrc/kernels/xgmi.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

constexpr int kXgmiMaxRanks = 8;
constexpr int kXgmiBlockElems = 1024;  // f32 elements reduced by one 256-thread workgroup

// Device addresses of every rank's exchange buffers, in this process's address space (the
// peers' are IPC-mapped): buf[r] = 2 parity halves of `cap` f32, sig[r] = [blocks][kXgmiMaxRanks]
// epoch words written by the peers.
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
  int64_t timeout;   // 100 MHz s_memrealtime ticks
  float scale;
  int rank;
  int world;
};

inline int xgmi_blocks(int64_t n) { return (int)((n + kXgmiBlockElems - 1) / kXgmiBlockElems); }

// mode 0: dst = scale * sum_r src_r ; mode 1: w -= lr * scale * sum_r src_r
void xgmi_all_reduce(const XgmiArgs& a, int mode, hipStream_t s);

}  // namespace tdl
