// NHWC bf16 convolution on the gfx950 bf16 matrix cores (v_mfma_f32_16x16x32_bf16), as implicit
// GEMMs: no im2col buffer, the operand loaders gather the receptive fields straight from the NHWC
// activations.  Used by keras.layers.Conv2D for bf16 activations on the GPU (ResNet-50, BASELINE
// configs 4/5) when the per-shape autotuner (keras/conv_select.py) measures it faster than MIOpen.
// f32 accumulation; outputs are rounded to bf16 once, in the epilogue.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

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
// stats (optional, [ceil(M / conv_fwd_row_tile) row tiles][2][K] f32, M = N*OH*OW): per-row-tile
// channel sums of y and y^2 for a following batch norm (deterministic; bn_forward_train(part=...))
// in_ss (optional, 1x1 stride 1 unpadded only): x is the INPUT of a BN -> ReLU whose output the conv
// reads; the operand loader applies relu(x * scale + shift) (in_ss = scale[C], shift[C]) with the BN
// apply pass's arithmetic -- bit-identical to convolving the materialised group output
void conv_fwd_bf16(const void* x, const void* w_ohwi, void* y, const ConvGeom& g, hipStream_t s,
                   float* stats = nullptr, const float* in_ss = nullptr);
int conv_fwd_row_tile(const ConvGeom& g, bool in_bn = false);
// shapes the input-side BN (in_ss) takes: 1x1 stride 1 unpadded, C <= 512 (its scale / shift in LDS)
bool conv_in_bn_supported(const ConvGeom& g);
// stride-1 input gradient: dx[N,H,W,C] = conv_transpose(dy[N,OH,OW,K], w[KH][KW][C][K]) (HWIO, the
// Keras layout: for a fixed (kh, kw, c) the K reduction values are contiguous)
// residual (optional, shaped like dx): added in the epilogue, dx = dgrad + residual (the other
// gradient contribution of a tensor with two consumers; saves a separate add pass)
// bn_part (with bn_y, bn_x: tensors shaped like dx): fused backward of a BN -> Add -> ReLU group
// whose output is this conv's input bn_y and whose BN input is bn_x: dx := (dgrad + residual) *
// [bn_y > 0] (the group's dz) and bn_part[ceil(M / conv_dgrad_row_tile)][2][C] := per-tile channel
// sums of dz and dz * bn_x (bn_backward(part=...) then skips its reduction pass)
// bn_part2 (with bn_x2, shaped like dx; needs bn_part): the group's residual is the output of a plain
// BN (projection shortcut) with input bn_x2 and no other reader: bn_part2 := per-tile sums of dz and
// dz * bn_x2, that BN's backward reduction
// bn_ss (scale[C], shift[C] of a plain BN -> ReLU group's forward; then bn_y may be null): the mask is
// recomputed as [bn_x * scale + shift > 0] instead of read from bn_y
void conv_dgrad_bf16(const void* dy, const void* w_hwio, void* dx, const ConvGeom& g, hipStream_t s,
                     const void* residual = nullptr, const void* bn_y = nullptr, const void* bn_x = nullptr,
                     float* bn_part = nullptr, const void* bn_x2 = nullptr, float* bn_part2 = nullptr,
                     const float* bn_ss = nullptr);
int conv_dgrad_row_tile(const ConvGeom& g);

// Input gradient of a 1x1, stride-2, unpadded convolution (the strided shortcut / first 1x1 of a
// ResNet-50 stage): dx[n][2i][2j] = dy[n][i][j] . w^T, the other three pixels of every 2x2 block are
// zero (written by the same kernel's epilogue; H <= 2*OH, W <= 2*OW).  residual / bn_*: as for
// conv_dgrad_bf16, over all four pixels of each 2x2 block (the part rows are the row tiles of the
// N*OH*OW dy pixels, conv_dgrad_s2_row_tile)
void conv_dgrad_s2_1x1_bf16(const void* dy, const void* w_hwio, void* dx, const ConvGeom& g, hipStream_t s,
                            const void* residual = nullptr, const void* bn_y = nullptr, const void* bn_x = nullptr,
                            float* bn_part = nullptr, const void* bn_x2 = nullptr, float* bn_part2 = nullptr,
                            const float* bn_ss = nullptr);
int conv_dgrad_s2_row_tile(const ConvGeom& g);

// Weight gradient, split-K over output pixels with a deterministic partial-slab reduction.
struct WgradPlan {
  int wmw, wnw;        // workgroup tile: (64 wmw) output channels x (64 wnw) (kh, kw, c) columns
  int chunk, nsplit;   // pixels per slice, slices
  long long ws_elems;  // f32 partial slab elements (nsplit x KH*KW*C x K)
  // kernel of the 2x2-wave tile: 0 register-staged (k_conv_wgrad), 1 single-stage LDS-DMA at 4 waves
  // per SIMD (k_conv_wgrad_glds<2, 2, 1>); 8-wave tiles are always the 3-stage LDS-DMA ring
  int kind;
};
bool conv_wgrad_supported(const ConvGeom& g);
// the model's best `max_plans` candidates, best first
// in_bn: plans the input-side BN (conv_wgrad_bf16 in_ss) runs with (register-staged tiles only)
std::vector<WgradPlan> conv_wgrad_plans(const ConvGeom& g, int max_plans, bool in_bn = false);
WgradPlan conv_wgrad_make_plan(const ConvGeom& g, int wmw, int wnw, int nsplit, int kind = 0);
// dW (HWIO [KH][KW][C][K]) from x[N,H,W,C] and dy[N,OH,OW,K]: into dw_bf16, or (dw_bf16 == nullptr)
// into the f32 dw_f32 (added to it when accumulate).  ws: plan.ws_elems f32.
// in_ss (optional, 1x1 stride 1 unpadded, kind-0 plans of <= 4 waves): x is a BN -> ReLU's input, as in
// conv_fwd_bf16
void conv_wgrad_bf16(const void* x, const void* dy, float* ws, const WgradPlan& p, void* dw_bf16, float* dw_f32,
                     bool accumulate, const ConvGeom& g, hipStream_t s, const float* in_ss = nullptr);

// Weight gradient of a 3x3 / stride 1 / pad 1 conv with C == 64 (wgrad3x3.hip): whole output rows per
// workgroup, the 9 x 64 x 64 tile in registers, deterministic slice reduction.  ws: ..._ws_elems f32.
bool conv_wgrad3x3_c64_supported(const ConvGeom& g);
long long conv_wgrad3x3_c64_ws_elems(const ConvGeom& g);
void conv_wgrad3x3_c64(const void* x, const void* dy, float* ws, void* dw_bf16, float* dw_f32, bool accumulate,
                       const ConvGeom& g, hipStream_t s);
void conv_wgrad3x3_set_rows(int rows);  // A/B hook: output rows per slice (0 = heuristic)

// Tile-sweep hook: 0 = per-shape heuristic (default), 1 = 128x64, 2 = 128x128, 3 = 256x128.
void conv_force_tile(int tile);
// A/B hook: 1 = the v1 register-staged kernel everywhere, 2 (default) = the LDS-DMA ring kernel where
// it measured faster (>= 32 k-tiles, >= one workgroup per CU), 3 = the ring kernel wherever its
// 256-row tiles give >= one workgroup per CU (tests, sweeps)
void conv_force_impl(int impl);
void conv_force_halo(int on);  // 1: the halo kernel for stride-1 multi-tap convs where its window fits
void conv_force_mfma(int mf);  // dma1 main loop MFMA form: 32 (32x32x16, default) or 16 (16x16x32)
// A/B hook: main loop of the implicit-GEMM kernel: 0 single LDS stage (4 waves per SIMD), 1 / 2
// register prefetch depth (default 2, single stage for 1-2 k-tile reductions), 3 depth 2 always
void conv_force_depth(int depth);
// A/B hook: the register-staged weight-gradient kernel with one LDS stage at 3 waves per SIMD
// or double-buffered with register prefetch at 2 (default)
void conv_wgrad_force_single(bool single);

}  // namespace tdl
