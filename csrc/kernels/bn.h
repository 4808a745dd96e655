// Training-mode batch normalisation over channels-innermost activations [M, C] (NHWC flattened:
// M = N*H*W), bf16 or f32 data, f32 statistics.  Used by keras.layers.BatchNormalization on the
// GPU (ResNet-50, BASELINE configs 4/5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

enum class BnDType { kF32 = 0, kBF16 = 1 };

// rows per workgroup and workgroup count of the partial-sum passes for [M, C]
struct BnPlan {
  int groups;       // C / 8 channel groups (8 channels per thread)
  int rows_iter;    // rows per workgroup iteration = 256 / groups
  int64_t rows_wg;  // rows per workgroup
  int parts;        // workgroups (partial rows in the workspace)
  int part_rows;    // workspace rows ([part_rows][2][C] f32): partials + their first-level reduction
};
BnPlan bn_plan(int64_t M, int C);
// sweep hooks: partial-pass workgroup cap, elementwise-pass grid cap, vectors per thread (1 or 2)
void bn_set_tuning(int max_parts, int elem_blocks, int elem_unroll);
// elementwise kernel family (A/B hook): 0 grid-stride, 1 blocked with 2 / 4 / 8 vectors per thread
void bn_set_elementwise(int kind, int vectors_per_thread);

// forward: part [parts][2][C] scratch; mean/invstd [C] out; scale/shift [C] out (x*scale+shift);
// moving stats updated in place (momentum m: moving = moving*m + batch*(1-m), variance unbiased);
// mean_off (nullable): per-channel bias of a preceding conv folded into this BN (moving mean only).
// given_parts > 0: `part` already holds that many partial rows ([rows][2][C]; space for
// ceil(rows / 64) more behind them), the partial pass is skipped
void bn_forward_stats(const void* x, BnDType dt, int64_t M, int C, float* part, const float* gamma,
                      const float* beta, const float* mean_off, float* mean, float* invstd, float* scale, float* shift,
                      float* moving_mean, float* moving_var, float momentum, float eps, hipStream_t s,
                      int given_parts = 0);
// y = act(x*scale + shift [+ residual])  (relu when relu != 0; residual nullable)
void bn_apply(const void* x, const void* residual, void* y, BnDType dt, int64_t M, int C, const float* scale,
              const float* shift, int relu, hipStream_t s);
// backward; dgamma/dbeta [C] out (acc bit 0/1: added into them), coef [3][C] scratch, dx = A*dz + B*x + D where
//   mode 0: dz = dy                         (plain BN)
//   mode 1: dz = dy * (x*scale+shift > 0)   (BN + ReLU, mask recomputed from x)
//   mode 2: dz = dy * (y > 0), written to dz (BN + Add + ReLU: dz is also the residual's gradient)
void bn_backward(const void* dy, const void* x, const void* y, void* dz, void* dx, BnDType dt, int64_t M, int C,
                 float* part, const float* gamma, const float* mean, const float* invstd, const float* scale,
                 const float* shift, float* dgamma, float* dbeta, float* coef, int mode, int acc, hipStream_t s,
                 int given_parts = 0);  // > 0: dy is the masked dz and part holds its reduction

}  // namespace tdl
