// NHWC bf16 convolution on the gfx950 bf16 matrix cores (v_mfma_f32_16x16x32_bf16), as implicit
// GEMMs: no im2col buffer, the operand loaders gather the receptive fields straight from the NHWC
// activations.  Used by keras.layers.Conv2D for bf16 activations on the GPU (ResNet-50, BASELINE
// configs 4/5) when the per-shape autotuner (keras/conv_select.py) measures it faster than MIOpen.
// f32 accumulation; outputs are rounded to bf16 once, in the epilogue.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace tdl {

struct ConvGeom {
  int N, H, W, C;        // input, NHWC (C % 64 == 0)
  int OH, OW, K;         // output spatial size and channels (K % 64 == 0)
  int KH, KW, SH, SW;    // filter size and strides
  int PT, PL;            // top / left zero padding (bottom / right padding is implied by OH, OW)
};

// Shapes the implicit-GEMM kernels take (the caller falls back to MIOpen otherwise).
bool conv_bf16_supported(const ConvGeom& g);

// y[N,OH,OW,K] = conv(x[N,H,W,C], w[K][KH][KW][C])           (weights OHWI: reduction-contiguous rows)
void conv_fwd_bf16(const void* x, const void* w_ohwi, void* y, const ConvGeom& g, hipStream_t s);
// stride-1 input gradient: dx[N,H,W,C] = conv_transpose(dy[N,OH,OW,K], w[KH][KW][C][K]) (HWIO, the
// Keras layout: for a fixed (kh, kw, c) the K reduction values are contiguous)
void conv_dgrad_bf16(const void* dy, const void* w_hwio, void* dx, const ConvGeom& g, hipStream_t s);

// Tile-sweep hook: 0 = per-shape heuristic (default), 1 = 128x64, 2 = 128x128, 3 = 256x128.
void conv_force_tile(int tile);

}  // namespace tdl
