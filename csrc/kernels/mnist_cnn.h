// Host-visible interface of the fused MNIST-CNN train step (see mnist_cnn.hip).
//
// Model (reference tf_dist_example.py:40-48):
//   Conv2D(32,3,relu) -> MaxPool2 -> Conv2D(64,3,relu) -> MaxPool2 -> Flatten
//   -> Dense(128,relu) -> Dense(10), NHWC, f32, TF weight layouts (HWIO / [in,out]).
// Loss SparseCategoricalCrossentropy(from_logits) scaled 1/(b*R) (ex:50), SGD (ex:51),
// SparseCategoricalAccuracy accumulated on device (ex:52).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "kernels/xgmi.h"

namespace tdl {

struct MnistArgs {
  // dataset (device resident) + per-step sample indices for this replica
  const float* X;     // [N, 28, 28, 1]
  const int* Y;       // [N]
  const int* idx;     // [b] sample ids of this replica's slice of the global batch
  // flat parameter / gradient slabs and per-variable offsets (floats)
  float* W;
  float* G;
  int ow1, ob1, ow2, ob2, ow3, ob3, ow4, ob4;
  // activations / saved state
  float* P1;          // [b,13,13,32] pooled relu(conv1)
  uint8_t* A1;        // [b,13,13,32] argmax (dy*2+dx) of each pool window
  float* P2;          // [b,5,5,64] == [b,1600]
  uint8_t* A2;        // [b,1600]
  float* H;           // [b,128] relu(dense1)
  float* dH;          // [b,128] grad of dense1 out (ReLU-masked)
  float* dP2;         // [b,1600] grad of the pooled conv2 output, ReLU-masked (k_fwd_conv)
  float* part2;       // [b][289][64] per-image partials of conv2 wgrad (row 288 = bias); fused_bwd:
                      // [b][kP2Quads][64][4] (see kP2Quads)
  float* part1;       // [2b or 4b][320] partials of conv1 wgrad (+ bias), see mnist_part1_rows
  float* part3;       // [4][b][128] dense1 partials, one per conv2 channel quarter
  float* dL;          // [b][kDLStride] dlogits (already scaled by 1/(b*R)), 10 used per row
  unsigned* cnt;      // [b] per-image arrival counters of k_fwd_conv (re-armed by KC)
  unsigned long long* dHt;  // [b][128] dP2 hand-off: dH bits | tag << 32 (8-B write-through stores)
  unsigned* ep;       // step epoch: k_fwd_conv tags dHt / part3t with *ep + 1, KC advances it
  unsigned long long* part3t;  // [4][b][128] dense1 partials as (value | tag << 32) words: the
                               // hand-off to the image's head in quarter workgroup 3 (dp2_fwd)
  float* metrics;     // [0] loss sum, [1] correct, [2] count
  const float* lr;    // device scalar learning rate
  unsigned long long* stamps;  // optional [grid][8] phase timestamps (s_memrealtime), diagnostics
  int b;              // per-replica batch
  float scale;        // 1 / (b * R)
  int nslab;          // slab length (floats)
  float* logits;      // [b][10] logits output of head mode 2 (null: metrics only)
  int head;           // 1: training loss head (dH, dL, saved activations); 2: evaluation head
                      // (logits, loss / accuracy accumulators, nothing saved); 0: features only
  int dp2_fwd;        // head == 1: dP2 computed at the end of k_fwd_conv (each quarter workgroup
                      // waits for its image's head; only when the launch has the GPU to itself and
                      // every workgroup fits at once), else by k_dense1_bwd
  int fused_bwd;      // dp2_fwd only: the conv backward runs at the end of k_fwd_conv, per (image,
                      // quarter) workgroup from what it already holds in LDS: conv2 wgrad of its 16
                      // output channels, the conv2 dgrad partial over them + pool1/ReLU backward +
                      // conv1 wgrad (part1 rows = image quarters); no k_conv_bwd launch
  unsigned* err;      // bit 1: an in-kernel hand-off (dense1 partials / dH) timed out; that image's
                      // gradient contribution was zeroed (MnistStep.error() raises on the host)
  // fused_bwd finalize with the cross-replica all-reduce built in (xchg): every finalize workgroup
  // publishes the gradient range it just reduced into its slot of a dedicated xGMI channel (slab
  // offsets), exchanges with the same workgroup of every peer, sums the R contributions in rank
  // order and applies SGD to that range -- no separate all-reduce or optimizer launch
  XgmiArgs xa;
  int variant;  // A/B switches of the fused kernel (TDL_MNIST_VARIANT bit flags; 0 = default)
  int fx_grid;  // k_finalize_x grid (0 = one workgroup per range, kFxBlocks); replicas sharing one GPU
                // cap it (TDL_FX_GRID) so every rank's exchange workgroups are resident together
  int xchg;
  int xtwo;  // exchange algorithm: 0 one-shot (every rank sums every range), 1 two-shot (each rank
             // sums and updates 1/R of every range, the others copy its updated weights)
};

// TDL_MNIST_VARIANT bits (A/B switches of k_fwd_conv; the default is what measured fastest):
//   1  s_setprio 1 for waves 4-7 (the younger half of each SIMD pair, the VALU arbitration loser)
//      (measured: 0.3-0.6 % slower, not adopted -- profiles/mnist_step_timeline_r5_v1.txt)
//   2  fused backward: waves 4-7 run their conv2 dgrad before their wgrad (stagger)
//      (measured: the backward's end and the step unchanged at K=20, 1-4 % slower at K=1000 -- the
//      waves' MFMA work is the same either way and the SIMD pairs stay busy; not adopted,
//      profiles/mnist_stagger_ab_r5.txt)
//   4  SGD fused into the finalize (one replica, or the xGMI exchange): the gradient slab G is not
//      written (nothing reads it on those paths; 900 KB fewer dirty lines for the kernel-end write-back)
//   8  XCD-aware workgroup -> (image, quarter) map: the 4 quarter workgroups of an image get block
//      ids of one residue mod 8 (blocks are dealt round-robin over the 8 XCDs, so they share one
//      XCD's L2 for their two hand-offs) instead of 4 consecutive ids (4 XCDs); speed only, the
//      protocol does not depend on placement (needs b % 8 == 0).  Measured: fused span 18.85 ->
//      18.38 us, K=20 2.48-2.49 -> 2.52 M img/s, K=1000 2.59-2.60 -> 2.62-2.63 M (adopted)
constexpr int kMnistVariantPrio = 1;
constexpr int kMnistVariantStagger = 2;
constexpr int kMnistVariantNoG = 4;
constexpr int kMnistVariantXcd = 8;
//   (16, round 6: 5 of conv1's W3 prefetch loads moved into conv2 -- 0.9 % slower at K=1000 and
//   K=20, removed; profiles/mnist_w3_late_rejected_r6.txt)

constexpr int kDefaultMnistVariant = kMnistVariantXcd;  // (measured +1.3 %: profiles/mnist_xcd_map_r6.txt)

constexpr int kMnistPart2Rows = 289;
// fused_bwd layout of part2: [b][73 row quads][64 columns][4 rows] (quad 72 = the bias row + 3 zero
// rows): each lane of the wgrad tiles owns 4 consecutive rows of one column, stored as ONE 16-B
// write-through store
constexpr int kP2Quads = 73, kP2QuadFloats = kP2Quads * 256;

// finalize workgroups of the fused_bwd step (k_finalize_x): 209 dense (dW3 rows 16m..16m+15, columns
// 64h..64h+63 = 16 x 64 slab floats each x 200; db3 in 4 x 32, dW4 in 4 x 32 rows x 10, db4),
// 146 conv2 (row quad, 32-column half) pieces (4 x 32 floats; the last quad: the bias row), 20 conv1
// groups (16).  A dense task issues 32-36 scalar loads (one per lane per row): the dW3 rows go to
// kFxW3 = 200 workgroups of 4 busy waves and db3 / dW4 to 8 workgroups of 2, rather than 8-task
// blocks (a CU with a whole 8-task block queued 256-288 of them behind its texture-address unit:
// those blocks ended last, ~1.9 us of wave life against ~1.0 for a 4-task dW3 block)
constexpr int kFxW3 = 200, kFxSmallDense = 9;
constexpr int kFxDense = kFxW3 + kFxSmallDense, kFxConv2 = 2 * kP2Quads, kFxConv1 = 20;
constexpr int kFxBlocks = kFxDense + kFxConv2 + kFxConv1;
// dlogits row stride: one 128-B line per image.  The head of image r runs on XCD (4r + quarter) % 8,
// so packed 40-B rows put 3-4 images' dlogits from two XCDs into one line, and the finalize's reads
// of such lines right after the boundary write-back were measured at 2.5-7 us (the db4 / dW4 blocks,
// otherwise done in ~0.6 us, then ended the finalize)
constexpr int kDLStride = 32;
constexpr int kDense1Chunks = 4;  // dense1 partials: one per conv2 channel quarter (k_fwd_conv)
constexpr int kMnistPart1Cols = 320;
// conv1 wgrad partial rows: (image, pixel half) of k_conv_bwd, or (image, quarter) of fused_bwd
__host__ __device__ inline int mnist_part1_rows(int b, bool fused_bwd = false) { return fused_bwd ? 4 * b : 2 * b; }

// K5: with `dp2` the dP2 tiles, with `dense` the dense weight gradients dW3/db3/dW4/db4 (R > 1 with
// the overlapped all-reduce: ahead of the conv backward, so their bucket's all-reduce overlaps it)
void mnist_dense1_bwd(const MnistArgs& a, bool dp2, bool dense, hipStream_t s);
void mnist_conv_bwd(const MnistArgs& a, hipStream_t s);
// conv1 + conv2 + dense1 partials per (image, quarter); with a.head the image's last quarter
// workgroup also runs the loss head (dense1 sum + ReLU, dense2, softmax-xent, dlogits, metrics),
// and with a.head == 1 every workgroup then computes its quarter of dP2
void mnist_fwd_conv(const MnistArgs& a, hipStream_t s);
// partial-slab reductions (+ the dense weight gradients when with_dense) (+ SGD when apply_sgd)
void mnist_finalize(const MnistArgs& a, bool apply_sgd, bool with_dense, hipStream_t s);
// fused_bwd finalize: partial-slab reductions + dense weight gradients into G; with apply_sgd the
// SGD update, and with a.xchg (apply_sgd only) the cross-replica sum first (xGMI exchange)
void mnist_finalize_x(const MnistArgs& a, bool apply_sgd, hipStream_t s);

// Plain SGD over a flat slab: w -= lr * g  (lr read from device memory).
// zero_g: g is zeroed after its use (the next step accumulates into it without a fill launch)
void sgd_apply(float* w, const float* g, const float* lr, int64_t n, hipStream_t s, bool zero_g = false);
// Momentum SGD (Keras semantics): v = m*v - lr*g ; w += v  (nesterov: w += m*v - lr*g)
void sgd_momentum_apply(float* w, const float* g, float* v, const float* lr, float momentum,
                        bool nesterov, int64_t n, hipStream_t s, bool zero_g = false);

}  // namespace tdl
