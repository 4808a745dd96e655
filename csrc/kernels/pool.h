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

void maxpool_forward(const void* x, void* y, uint8_t* arg, bool bf16, const PoolGeom& g, hipStream_t s);
void maxpool_backward(const void* dy, const uint8_t* arg, void* dx, bool bf16, const PoolGeom& g, hipStream_t s);
// A/B hook: the generic window loops (default) or the unrolled kernels for 3x3 stride-2 pooling
void maxpool_force_generic(bool generic);

}  // namespace tdl
