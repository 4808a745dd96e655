// NHWC max pooling (forward with window-argmax bytes, gather-form backward); see pool.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

struct PoolGeom {
  int N, H, W, C;     // input (C % 8 == 0)
  int OH, OW;         // output
  int kh, kw, sh, sw;
  int pt, pl;         // leading padding (trailing padding is implied by OH/OW)
  int pad_zero;       // padding elements are 0 (fused ZeroPadding2D) instead of -inf
};

// bn_ss (scale[C], shift[C]): x is a batch norm's input and the pool runs over relu(x * scale + shift)
void maxpool_forward(const void* x, void* y, uint8_t* arg, bool bf16, const PoolGeom& g, hipStream_t s,
                     const float* bn_ss = nullptr);
// bn_x / bn_ss / part (with a BN-fused forward): dx := the BN -> ReLU group's masked gradient and
// part[maxpool_backward_blocks][2][C] := per-block channel sums of dx and dx * bn_x
void maxpool_backward(const void* dy, const uint8_t* arg, void* dx, bool bf16, const PoolGeom& g, hipStream_t s,
                      const void* bn_x = nullptr, const float* bn_ss = nullptr, float* part = nullptr);
int maxpool_backward_blocks(const PoolGeom& g);
// A/B hook: the generic window loops (default) or the unrolled kernels for 3x3 stride-2 pooling
void maxpool_force_generic(bool generic);
void maxpool_w2(bool on);  // 2x2 stride-2 backward in scatter form (default on)

}  // namespace tdl
