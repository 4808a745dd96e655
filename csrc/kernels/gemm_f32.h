// Generic f32 GEMM / implicit-GEMM convolution for gfx950 on v_mfma_f32_16x16x4_f32 (exact f32
// products, f32 accumulation): the f32 Conv2D and Dense layers of the generic engine -- any kernel
// size, stride, dilation and (asymmetric) padding, any channel count, no library call.  See
// gemm_f32.hip for the tiling.
//
// Every operation is C[M][N] = sum_k A(m, k) B(k, n) (+ bias[n]) (+ C when accumulating), with the
// A / B element fetch chosen by the mode:
//   kF32Gemm       A(m, k) = a[m sam + k sak], B(k, n) = b[k sbk + n sbn]        (Dense fwd / dx / dW)
//   kF32ConvFwd    M = N*OH*OW pixels, N = K out channels, k = (r, s, c):  x NHWC, w HWIO [R S C][K]
//   kF32ConvDgrad  M = N*H*W input pixels, N = C, k = (r, s, k):  dy NHWC, w^T as [R S K][C]
//   kF32ConvWgrad  M = K, N = R*S*C, k = (n, oy, ox): A = dy (channel-contiguous rows), B = x gathered,
//                  stored transposed (trans_out) into dW HWIO [R S C][K]
// Long reductions split over blockIdx.z into a partial-sum workspace reduced in a fixed order by a
// second kernel (deterministic, no atomics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

enum F32GemmMode { kF32Gemm = 0, kF32ConvFwd = 1, kF32ConvDgrad = 2, kF32ConvWgrad = 3 };

struct F32ConvGeom {
  int n, h, w, c;  // input NHWC
  int k;           // output channels
  int r, s;        // filter height / width
  int oh, ow;      // output height / width
  int sh, sw, pt, pl, dh, dw;
};

struct F32GemmArgs {
  const float* a;
  const float* b;
  float* out;
  const float* bias;  // [N] or null
  float* ws;          // [splits][M][N] partial sums (splits > 1)
  int64_t sam, sak, sbk, sbn;
  int M, N, Kred;
  int kchunk, splits;  // reduction slice per blockIdx.z (a multiple of 16) and their count
  int64_t ldo;
  int trans_out;   // out[n * ldo + m] instead of out[m * ldo + n]
  int accumulate;  // out += result
  int vec_a, vec_b;  // 16-B operand loads (set by the host when layouts and alignment allow)
  F32ConvGeom g;
  // Fusions of the layer around the GEMM (the generic engine's f32 Conv2D / Dense with a ReLU):
  int act = 0;                    // epilogue: 0 = none, 1 = ReLU after the bias (forward)
  const float* amask = nullptr;   // A operand *= (amask[same element] > 0): ReLU backward of the
  const float* bmask = nullptr;   // layer's output; B likewise (masks share the operand's layout)
  float* dbias = nullptr;         // bias gradient: a row of ones appended to A (ones_m = M - 1,
  int ones_m = -1, ones_n = -1;   // kF32Gemm) or a column of ones appended to B (ones_n = N - 1,
                                  // kF32ConvWgrad); that output row / column goes to dbias
  int b_hwio = 0;                 // kF32ConvDgrad: b is the forward kernel w HWIO [R][S][C][K] itself
                                  // (B(k = (r, s, kk), n = c) read transposed: no transpose pass)
  // kF32ConvFwd + 2x2 / stride-2 'valid' max pool in the epilogue: rows are ordered (n, ph, pw, q) -- the
  // 4 pixels q = (dy, dx) of each pool window consecutive, i.e. in ONE lane's 4 accumulators -- so
  // M = N * PH * PW * 4 (pixels of an odd last row / column are not computed); y (out, NHWC [N][OH][OW][K])
  // is still written for the backward, plus the pooled maximum pout [N][PH][PW][K] and its window
  // position parg (uint8, ops/pooling.py's argmax format).  Split reductions (< 16 slices) end in
  // k_gemm_f32_reduce_pool, which applies the same epilogue.
  int pool = 0, pool_h = 0, pool_w = 0;
  float* pout = nullptr;
  uint8_t* parg = nullptr;
  int plan_m = 0;  // > 0: the split plan of an M = plan_m problem (the pooled conv takes the unfused conv's
                   // reduction split, so its partial sums -- and outputs -- are bit-identical to it)
  // kF32ConvDgrad / kF32ConvWgrad with the output gradient given POOLED (the backward of that fused
  // forward): a = the pool's output gradient [N][PH][PW][K], amask = the pooled maximum, pin_arg = its
  // window positions; the conv-output gradient the loader forms is, at pixel (oy, ox) of the g.oh x g.ow
  // grid, pooled gradient * [argmax == this pixel] * [maximum > 0] (pixels outside every window: 0)
  // -- the max-pool backward and the ReLU mask without their own pass.  Uses pool_h / pool_w.
  const uint8_t* pin_arg = nullptr;
  // element counts of a / b (and of amask / bmask, shaped alike): when both are set and < 2^29 the kernel
  // reads its operands through buffer resources with 32-bit offsets (out-of-range offsets read 0), so
  // the loaders need no 64-bit address math and no clamped-address selects (0: the generic form)
  int64_t na = 0, nb = 0;
};

constexpr int kF32Tile = 64;

// Reduction split for a (mode-independent) M x N x Kred problem: enough workgroups to fill 256 CUs,
// each with at least `kmin` reduction elements (the kernel keeps 4 slices of 16 in flight, so a
// split of <= 64 is one memory round trip; 128 -- two -- until round 6), at most `cap` splits.
inline void f32_gemm_plan(F32GemmArgs& a, int kmin = 64, int cap = 1024) {
  const int64_t pm = a.plan_m > 0 ? a.plan_m : a.M;
  const int64_t tiles = (int64_t)((pm + kF32Tile - 1) / kF32Tile) * ((a.N + kF32Tile - 1) / kF32Tile);
  int splits = 1;
  if (tiles < 512 && a.Kred > 256) {
    const int64_t want = (1024 + tiles - 1) / tiles;
    const int64_t most = (a.Kred + kmin - 1) / kmin;
    splits = (int)(want < most ? want : most);
    if (splits > cap) splits = cap;
    if (splits < 1) splits = 1;
  }
  int chunk = (a.Kred + splits - 1) / splits;
  chunk = (chunk + 15) / 16 * 16;
  if (chunk < 16) chunk = 16;
  a.kchunk = chunk;
  a.splits = (a.Kred + chunk - 1) / chunk;
  if (a.splits < 1) a.splits = 1;
  if (a.pool && a.splits >= 16) {  // (the pooled reduction replicates the < 16-slice reduce only)
    a.kchunk = (a.Kred + 15) / 16 * 16;
    a.splits = 1;
  }
}

void f32_gemm_launch(int mode, const F32GemmArgs& a, hipStream_t s);
// many-slice reductions over >= 8192 outputs: 16 outputs per wave (default) or one (A/B hook)
void f32_reduce16(bool on);

}  // namespace tdl
