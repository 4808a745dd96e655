// Fused MNIST-CNN training step for gfx950 (MI355X), f32 end to end.
//
// Replaces, for the reference model of tf_dist_example.py:40-52, the ~35 TF/cuDNN/Eigen kernels
// of one replica step by three launches (four when the GPU is
// shared or 4b > CUs, and at R > 1 with the overlapped all-reduce option):
//
//   KA fwd_conv     : per (image, channel quarter), LDS-staged: gather(idx) + conv1 3x3 (1->32)
//                     and conv2 3x3 (32->64) on v_mfma_f32_16x16x4_f32 with bias + ReLU + maxpool2
//                     in registers (a 16-row MFMA tile = 4 pool windows), then this quarter's
//                     dense1 partial [1600/4 features] x W3 (W3 slice prefetched in registers);
//                     the LAST of an image's 4 quarter workgroups (arrival counter) then runs the
//                     head for that image: dense1 partial sum + bias + ReLU, dense2 + softmax-xent
//                     + dlogits*(1/(b*R)) + loss/accuracy accumulators + dH (ReLU mask); with
//                     dp2_fwd every quarter workgroup then waits for its image's dH and computes its 400
//                     features of dP2 = (dH W3^T) * relu-mask from the W3 slice in its registers
//   K5 dense1_bwd   : dP2 = (dH W3^T) * relu-mask when k_fwd_conv did not compute it (the
//                     launch shares the GPU or its workgroups do not all fit at once), and at
//                     R > 1 the dense weight gradients dW3/db3/dW4/db4, so their bucket's
//                     all-reduce overlaps the conv backward
//   KC conv_bwd     : per image (x4 parts), LDS-staged (dC2 expanded from dP2 + pool-2 argmax):
//                     dW2 (+db2 as an extra "ones" row) and
//                     dP1 = dC2 (*) W2^T on MFMA with pool1/ReLU backward AND conv1 wgrad in
//                     the epilogue (dC1 is never materialised); per-image partial slabs
//   KF finalize     : deterministic reduction of the partial slabs into the flat gradient slab and
//                     (unless K5 did) the dense weight gradients dW3 = P2^T dH (+db3), dW4 = H^T dL
//                     (+db4), optionally fused with the SGD update (single replica)
//
// All reductions are slab-based (no float atomics) so every replica computes bit-identical
// updates from identical inputs.
#include <type_traits>

#include "common.h"
#include "mnist_cnn.h"
#include "xgmi_device.h"

namespace tdl {

// --------------------------------------------------------------------------------------------
// Loss head of ONE batch row r, run by one wave (lane l owns hidden features l and l + 64):
// H = relu(b3 + sum of the 4 dense1 quarter partials), logits = dense2 (wave reductions),
// softmax / loss / dlogits computed redundantly by every lane, dH (ReLU-masked) and dL stored,
// loss / accuracy / count accumulated.  The partials come from the other quarter workgroups of
// the same launch: sc1 loads (L2, never a stale L1 line), see k_fwd_conv's hand-off.
// --------------------------------------------------------------------------------------------
struct HeadWeights {  // dense2 kernel rows l and l + 64, dense2 bias, dense1 bias of features l, l + 64
  float wa[10], wb[10], b4[10], b3a, b3b;
};

__device__ __forceinline__ HeadWeights load_head_weights(const MnistArgs& a, int l) {
  HeadWeights hw;
  const float* w4 = a.W + a.ow4;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    hw.wa[c] = w4[l * 10 + c];
    hw.wb[c] = w4[(l + 64) * 10 + c];
    hw.b4[c] = a.W[a.ob4 + c];
  }
  hw.b3a = a.W[a.ob3 + l];
  hw.b3b = a.W[a.ob3 + l + 64];
  return hw;
}

// The head's operands staged in LDS by wave 7 (idle during conv2): hws = [w4 128 x 10][b3 128][b4 10],
// so that wave 0's partial polls do not queue behind 32 head-weight loads per lane (vmcnt is in order)
constexpr int kHeadW = 1280 + 128 + 12;  // floats (b4 padded to 12)

__device__ __forceinline__ HeadWeights lds_head_weights(const float* hws, int l) {
  HeadWeights hw;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    hw.wa[c] = hws[l * 10 + c];
    hw.wb[c] = hws[(l + 64) * 10 + c];
    hw.b4[c] = hws[1408 + c];
  }
  hw.b3a = hws[1280 + l];
  hw.b3b = hws[1280 + l + 64];
  return hw;
}

// phase stamp k of the head, after the per-wave stamps: buf[grid*64 + workgroup*8 + k]
// (diagnostics, stamps != null; the buffer then holds grid * 72 words)
__device__ __forceinline__ void head_stamp(unsigned long long* buf, int k) {
  if (buf != nullptr && (threadIdx.x & 63) == 0)
    buf[(size_t)gridDim.x * 64 + blockIdx.x * 8 + k] = __builtin_amdgcn_s_memrealtime();
}

// Sums of 10 per-lane values over the wave, returned in every lane: a reduce-scatter butterfly
// (lane halves keep 5 / 3 / 2 / 1 of the classes: 13 cross-lane moves instead of 10 x 6) whose
// class sums end in lane groups, then broadcast by v_readlane.
__device__ __forceinline__ void wave_sum10(const float (&v)[10], int l, float (&out)[10]) {
  const bool b8 = l & 8, b4 = l & 4;
  float u[5];  // lanes 0..31 keep v[0..4], lanes 32..63 v[5..9] (v_permlane32_swap)
#pragma unroll
  for (int j = 0; j < 5; ++j) u[j] = rs_swap32(v[j], v[j + 5]);
  float w[3];  // even 16-lane rows keep u[0..2], odd rows u[3..4] (+0) (v_permlane16_swap)
#pragma unroll
  for (int j = 0; j < 3; ++j) w[j] = rs_swap16(u[j], j + 3 < 5 ? u[j + 3] : 0.f);
  float x[2];  // b8 = 0 keeps w[0..1], b8 = 1 keeps w[2] (+0) (DPP row_ror:8)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float hi = j + 2 < 3 ? w[j + 2] : 0.f;
    x[j] = (b8 ? hi : w[j]) + dpp_xor8(b8 ? w[j] : hi);
  }
  // b4 = 0 keeps x[0], b4 = 1 x[1]; the partner is the 8-lane mirror (it has the other b4)
  float y = (b4 ? x[1] : x[0]) + dpp_mirror8(b4 ? x[0] : x[1]);
  y += dpp_xor2(y);
  y += dpp_xor1(y);
  // class c sits in lane 32*hi + 16*b + 8*c8 + 4*d: c = 5*hi + (b ? 3 : 0) + (2*c8 + d)
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    const int hi = c / 5, kk = c % 5, bb = kk >= 3, wi = bb ? kk - 3 : kk;
    const int lane = 32 * hi + 16 * bb + 8 * (wi >> 1) + 4 * (wi & 1);
    out[c] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, y), lane));
  }
}

// Sums over the 32 lanes of each half-wave of N <= 32 per-lane values (v[k], k >= N taken as 0):
// a reduce-scatter butterfly (16 + 8 + 4 + 2 + 1 cross-lane moves); lane l returns the sum of
// value (l & 31) over its half-wave.
// (every step on the VALU: v_permlane16_swap for the 16-lane rows, DPP within a row; the 8-lane
// mirror stands in for xor 4 -- which half a lane keeps is set by its own lane bits, so the lane
// that ends with value k is the same as with a plain xor butterfly)
template <int N>
__device__ __forceinline__ float reduce_scatter32(const float (&v)[N], int l) {
  float s16[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) s16[k] = rs_swap16(k < N ? v[k] : 0.f, k + 16 < N ? v[k + 16] : 0.f);
  float s8[8];
  const bool b8 = l & 8;
#pragma unroll
  for (int k = 0; k < 8; ++k) s8[k] = (b8 ? s16[k + 8] : s16[k]) + dpp_xor8(b8 ? s16[k] : s16[k + 8]);
  float s4[4];
  const bool b4 = l & 4;
#pragma unroll
  for (int k = 0; k < 4; ++k) s4[k] = (b4 ? s8[k + 4] : s8[k]) + dpp_mirror8(b4 ? s8[k] : s8[k + 4]);
  float s2[2];
  const bool b2 = l & 2;
#pragma unroll
  for (int k = 0; k < 2; ++k) s2[k] = (b2 ? s4[k + 2] : s4[k]) + dpp_xor2(b2 ? s4[k] : s4[k + 2]);
  const bool b1 = l & 1;
  return (b1 ? s2[1] : s2[0]) + dpp_xor1(b1 ? s2[0] : s2[1]);
}

constexpr int kHeadQuarter = 3;  // dp2_fwd: the quarter workgroup whose head writes metrics / H / dH / dL

// sown != null (dp2_fwd): EVERY quarter workgroup cq of the image runs this head redundantly (one
// all-to-all exchange of the dense1 partials instead of a partials -> head -> dH round trip): the
// other three quarters' partials arrive as tagged words in part3t, polled here until every tag
// is this step's; its own partial is in LDS.  The sums run in quarter order in every workgroup, so
// all four compute bit-identical dH; only the `primary` one accumulates the metrics and stores
// H / dH / dL for the dense weight gradients.
__device__ __forceinline__ void head_row(const MnistArgs& a, int r, int l, int y, const HeadWeights& hw, float* sdh,
                                         uint32_t tag, const float* sown, int cq = kHeadQuarter,
                                         bool primary = true) {
  const float* wa = hw.wa;
  const float* wb = hw.wb;
  head_stamp(a.stamps, 0);
  float hp0[kDense1Chunks], hp1[kDense1Chunks];
  bool timed_out = false;
  if (sown != nullptr) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = false;
    unsigned npoll = 0;  // (diagnostics: poll rounds, head stamp slot 4)
    for (;;) {
      ++npoll;
      if (!ok) {
        ok = true;
#pragma unroll
        for (int c = 0; c < kDense1Chunks; ++c) {
          if (c == cq) continue;
          const unsigned long long* p = a.part3t + ((size_t)c * a.b + r) * 128 + l;
          const unsigned long long w0 = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const unsigned long long w1 = __hip_atomic_load(p + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = ok && (uint32_t)(w0 >> 32) == tag && (uint32_t)(w1 >> 32) == tag;
          hp0[c] = __uint_as_float((uint32_t)w0);
          hp1[c] = __uint_as_float((uint32_t)w1);
        }
      }
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {  // 20 ms at 100 MHz
        // a quarter's partial never arrived: poison the loss metric, flag the error word, and
        // give this image NO gradient (dH = dL = 0 below) instead of one from stale partials
        if (l == 0) {
          atomicAdd(&a.metrics[0], __builtin_nanf(""));
          if (a.err != nullptr) __hip_atomic_fetch_or(a.err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        timed_out = true;
        break;
      }
    }
    if (a.stamps != nullptr && l == 0) a.stamps[(size_t)gridDim.x * 64 + blockIdx.x * 8 + 4] = npoll;
    const float o0 = sown[l], o1 = sown[l + 64];
#pragma unroll
    for (int c = 0; c < kDense1Chunks; ++c) {  // (static register indices)
      hp0[c] = c == cq ? o0 : hp0[c];
      hp1[c] = c == cq ? o1 : hp1[c];
    }
  } else {
#pragma unroll
    for (int c = 0; c < kDense1Chunks; ++c) {
      hp0[c] = __hip_atomic_load(a.part3 + ((size_t)c * a.b + r) * 128 + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hp1[c] = __hip_atomic_load(a.part3 + ((size_t)c * a.b + r) * 128 + l + 64, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  float h0 = hw.b3a, h1 = hw.b3b;
#pragma unroll
  for (int c = 0; c < kDense1Chunks; ++c) { h0 += hp0[c]; h1 += hp1[c]; }
  h0 = fmaxf(h0, 0.f);
  h1 = fmaxf(h1, 0.f);
  head_stamp(a.stamps, 1);
  float lg[10];
  {
    float v[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) v[c] = fmaf(h0, wa[c], h1 * wb[c]);
    wave_sum10(v, l, lg);
  }
#pragma unroll
  for (int c = 0; c < 10; ++c) lg[c] += hw.b4[c];
  float m = lg[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < 10; ++c)
    if (lg[c] > m) { m = lg[c]; am = c; }
  // softmax on the hardware exp2/log2 (v_exp_f32 / v_log_f32): |logit - max| is small here, so
  // the log2(e) pre-scale costs ~1e-7 relative, far inside the f32 oracle tolerance
  float e[10], se = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    e[c] = __expf(lg[c] - m);
    se += e[c];
  }
  const float lse = m + __logf(se);
  const float inv = 1.f / se;
  head_stamp(a.stamps, 2);
  float ly = lg[0];
#pragma unroll
  for (int c = 1; c < 10; ++c) ly = (c == y) ? lg[c] : ly;
  float dl[10];
#pragma unroll
  for (int c = 0; c < 10; ++c) dl[c] = (e[c] * inv - (c == y ? 1.f : 0.f)) * a.scale;
  float d0 = 0.f, d1 = 0.f, mine = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) {
    d0 = fmaf(dl[c], wa[c], d0);
    d1 = fmaf(dl[c], wb[c], d1);
    mine = (l == c) ? dl[c] : mine;
  }
  const float dh0 = (h0 > 0.f && !timed_out) ? d0 : 0.f, dh1 = (h1 > 0.f && !timed_out) ? d1 : 0.f;
  if (timed_out) mine = 0.f;
  if (a.dp2_fwd) {  // this workgroup's waves read dH from LDS for their dP2
    sdh[l] = dh0;
    sdh[l + 64] = dh1;
  }
  head_stamp(a.stamps, 3);
  if (!primary) return;
  a.dH[r * 128 + l] = dh0;  // plain: read by later launches (dense weight gradients, K5 dP2)
  a.dH[r * 128 + l + 64] = dh1;
  a.H[r * 128 + l] = h0;
  a.H[r * 128 + l + 64] = h1;
  if (l < 10) a.dL[r * kDLStride + l] = mine;
  if (l == 0) {
    atomicAdd(&a.metrics[0], lse - ly);
    atomicAdd(&a.metrics[1], am == y ? 1.f : 0.f);
    atomicAdd(&a.metrics[2], 1.f);
  }
}

// Evaluation / inference head of ONE batch row (head mode 2): logits (optionally stored), loss and
// top-1 accuracy into the metric accumulators; no gradient state.
__device__ __forceinline__ void head_eval(const MnistArgs& a, int r, int l, int y, const HeadWeights& hw) {
  float hp0[kDense1Chunks], hp1[kDense1Chunks];
#pragma unroll
  for (int c = 0; c < kDense1Chunks; ++c) {
    hp0[c] = __hip_atomic_load(a.part3 + ((size_t)c * a.b + r) * 128 + l, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    hp1[c] = __hip_atomic_load(a.part3 + ((size_t)c * a.b + r) * 128 + l + 64, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
  }
  float h0 = hw.b3a, h1 = hw.b3b;
#pragma unroll
  for (int c = 0; c < kDense1Chunks; ++c) { h0 += hp0[c]; h1 += hp1[c]; }
  h0 = fmaxf(h0, 0.f);
  h1 = fmaxf(h1, 0.f);
  float lg[10];
  {
    float v[10];
#pragma unroll
    for (int c = 0; c < 10; ++c) v[c] = fmaf(h0, hw.wa[c], h1 * hw.wb[c]);
    wave_sum10(v, l, lg);
  }
#pragma unroll
  for (int c = 0; c < 10; ++c) lg[c] += hw.b4[c];
  float m = lg[0], ly = lg[0], mine = lg[0];
  int am = 0;
#pragma unroll
  for (int c = 1; c < 10; ++c) {
    if (lg[c] > m) { m = lg[c]; am = c; }
    ly = (c == y) ? lg[c] : ly;
    mine = (c == l) ? lg[c] : mine;
  }
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < 10; ++c) se += __expf(lg[c] - m);
  if (a.logits != nullptr && l < 10) a.logits[(size_t)r * 10 + l] = mine;
  if (l == 0) {
    atomicAdd(&a.metrics[0], m + __logf(se) - ly);
    atomicAdd(&a.metrics[1], am == y ? 1.f : 0.f);
    atomicAdd(&a.metrics[2], 1.f);
  }
}

// --------------------------------------------------------------------------------------------
// K5: dense-layer backward, one 16x16 MFMA output tile per wave task (every task's loads issued
// in one round trip; biases are an extra "ones" row of the weight-gradient GEMMs):
//   tasks [0, 808)        dW3 = P2^T dH (M = 1600 features + db3 row, N = 128, K = b)
//   tasks [808, +100 MT)  dP2 = (dH W3^T) * 1[P2 > 0]  (M = b, N = 1600, K = 128): the pool-2 /
//                         ReLU mask; k_conv_bwd expands it to the conv2-output gradient itself
//   tasks [.., + 9)       dW4 = H^T dL (+ db4 row) (M = 128 + 1, N = 10, K = b)
// Block 0 also re-arms the per-image head counters of k_fwd_conv for the next step.
// --------------------------------------------------------------------------------------------
constexpr int kD1TasksW3 = 101 * 8;

// acc += A^T B over K = b rows of two row-major operands read through buffer resources sized to
// the b valid rows (rows past b load 0, so no clamp or mask): lane (i, g) supplies A[r = r0 + 4s + g]
// at byte ca of the row and B[r] at byte cb, sa / sb the row strides in bytes (the row offset rides
// in the SGPR offset: no per-load 64-bit address arithmetic on the VALU); 64 rows' loads in flight
// per batch
// (E0: A is the unit row e_0 -- lane i == 0 supplies 1 -- instead of a load: the bias columns)
template <bool E0 = false>
__device__ __forceinline__ f4 gemm_tn_buf(int b, int g, __amdgpu_buffer_rsrc_t ra, int sa, int ca,
                                          __amdgpu_buffer_rsrc_t rb, int sb, int cb, float e0 = 0.f) {
  f4 acc0 = zero4(), acc1 = zero4();
  const int va = g * sa + ca, vb = g * sb + cb;
  for (int r0 = 0; r0 < b; r0 += 64) {
    float av[16], bv[16];
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      // (E0: rows past b must add 0: their B loads read 0)
      av[s] = E0 ? e0 : ld1_buf(ra, va, (r0 + 4 * s) * sa);
      bv[s] = ld1_buf(rb, vb, (r0 + 4 * s) * sb);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s & 1) acc1 = mfma16x16x4(av[s], bv[s], acc1);
      else acc0 = mfma16x16x4(av[s], bv[s], acc0);
    }
  }
  return acc0 + acc1;
}

// 4 x 4 transpose within each quad of lanes (q = lane & 3), two xor-butterfly stages on DPP: on entry
// lane q holds M[q][0..3], on exit M[0..3][q] (v[k] of lane q = entry v[q] of lane k).  The whole
// wave must be active.
__device__ __forceinline__ f4 quad_transpose(f4 v, int q) {
  const bool a = (q & 2) != 0, b = (q & 1) != 0;
  // xor 2: the off-diagonal 2 x 2 blocks change lanes
  float r0 = dpp_xor2(a ? v[0] : v[2]), r1 = dpp_xor2(a ? v[1] : v[3]);
  if (a) { v[0] = r0; v[1] = r1; } else { v[2] = r0; v[3] = r1; }
  // xor 1: the off-diagonal elements of every 2 x 2 block
  r0 = dpp_xor1(b ? v[0] : v[1]);
  r1 = dpp_xor1(b ? v[2] : v[3]);
  if (b) { v[0] = r0; v[2] = r1; } else { v[1] = r0; v[3] = r1; }
  return v;
}

// One dense weight-gradient task T in [0, kDenseTasks) for the wave (optionally fused with plain
// SGD of its outputs: nothing else in the launch reads W3 / W4 then).
constexpr int kDenseTasks = kD1TasksW3 + 9;

__device__ __forceinline__ void dense_w_task(const MnistArgs& a, int T, int lane, bool sgd, float lr,
                                             float* xdst = nullptr, bool keep_g = true) {
  const int i = lane & 15, g = lane >> 4;
  const int b = a.b;
  if (T < kD1TasksW3) {
    const int mt = T >> 3, nt = T & 7, n = nt * 16 + i;
    if (mt < 100) {
      const int kf = mt * 16 + i;
      // after the quad transpose lane (i, g) owns row 16 mt + 4 g + (i & 3), columns 16 nt + (i & 12)
      // .. +3: the SGD operand is ONE 16-B load (in the operand loads' round trip) and G / W are ONE
      // 16-B store each (was 4 scalar loads + 4 + 4 scalar stores per lane on the CU's
      // vector-memory queue)
      const int e4 = a.ow3 + (mt * 16 + 4 * g + (i & 3)) * 128 + nt * 16 + (i & 12);
      const f4 wold = sgd ? ld4(a.W + e4) : zero4();
      const f4 acc = quad_transpose(gemm_tn_buf(b, g, buf_rsrc(a.P2, (unsigned)(b * 1600 * 4)), 1600 * 4, kf * 4,
                                                buf_rsrc(a.dH, (unsigned)(b * 128 * 4)), 128 * 4, n * 4), i & 3);
      if (keep_g) st4(a.G + e4, acc);
      if (xdst != nullptr) st4(xdst + e4, acc);
      // W as a 16-B WRITE-THROUGH store: 820 KB fewer dirty L2 lines for the finalize's kernel-end
      // write-back, in front of the next fused kernel (profiles/mnist_fx_w3_writethrough_r5.txt; the
      // 4-B write-through form of the earlier layout lost: profiles/mnist_fx_writethrough_rejected_r5.txt)
      if (sgd) st4_sc1(buf_rsrc(a.W, (unsigned)a.nslab * 4u), e4 * 4, wold - lr * acc);
    } else {  // db3: A = e_0 (row 0 of the tile = column sums of dH)
      const float wold = sgd ? a.W[a.ob3 + n] : 0.f;
      const auto dhr = buf_rsrc(a.dH, (unsigned)(b * 128 * 4));
      const f4 acc = gemm_tn_buf<true>(b, g, dhr, 0, 0, dhr, 128 * 4, n * 4, i == 0 ? 1.f : 0.f);
      if (g == 0) {
        if (keep_g) a.G[a.ob3 + n] = acc[0];
        if (xdst != nullptr) xdst[a.ob3 + n] = acc[0];
        if (sgd) a.W[a.ob3 + n] = wold - lr * acc[0];
      }
    }
    return;
  }
  const int T3 = T - kD1TasksW3;
  if (T3 < 9) {
    // dW4[k][c] = sum_r H[r][k] dL[r][c] (tiles 0..7), db4 (tile 8, A = e_0); N = 10 of 16
    const int c = min(i, 9);
    float wold[4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      wold[r] = sgd ? a.W[T3 < 8 ? a.ow4 + (T3 * 16 + 4 * g + r) * 10 + c : a.ob4 + c] : 0.f;
    // (lanes i >= 10 read past the dL resource: 0)
    const auto dlr = buf_rsrc(a.dL, (unsigned)(b * kDLStride * 4));
    const int dlc = i < 10 ? i * 4 : 0x40000000;
    const f4 acc = T3 < 8 ? gemm_tn_buf(b, g, buf_rsrc(a.H, (unsigned)(b * 128 * 4)), 128 * 4, (T3 * 16 + i) * 4, dlr,
                                        kDLStride * 4, dlc)
                          : gemm_tn_buf<true>(b, g, dlr, 0, 0, dlr, kDLStride * 4, dlc, i == 0 ? 1.f : 0.f);
    if (i < 10) {
      if (T3 < 8) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int e = a.ow4 + (T3 * 16 + 4 * g + r) * 10 + i;
          if (keep_g) a.G[e] = acc[r];
          if (xdst != nullptr) xdst[e] = acc[r];
          if (sgd) a.W[e] = wold[r] - lr * acc[r];
        }
      } else if (g == 0) {
        if (keep_g) a.G[a.ob4 + i] = acc[0];
        if (xdst != nullptr) xdst[a.ob4 + i] = acc[0];
        if (sgd) a.W[a.ob4 + i] = wold[0] - lr * acc[0];
      }
    }
  }
}

// dP2 = (dH W3^T) * 1[P2 > 0] (M = b, N = 1600, K = 128): one 16x16 tile per wave task, the
// pool-2 / ReLU mask in the epilogue (k_conv_bwd expands it to the conv2-output gradient)
__device__ __forceinline__ void dp2_task(const MnistArgs& a, int T, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const int b = a.b;
  const int MT = (b + 15) >> 4;
  const int mt = T % MT, nt = T / MT;
  const int row = mt * 16 + i;
  const bool valid = row < b;
  const float* ap = a.dH + (valid ? row : 0) * 128 + 4 * g;
  const float* bp = a.W + a.ow3 + (size_t)(nt * 16 + i) * 128 + 4 * g;
  f4 av[8], bv[8];
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    av[s] = ld4(ap + s * 16);
    bv[s] = ld4(bp + s * 16);
  }
  float p2v[4];  // the epilogue's ReLU-mask operands in the same round trip
#pragma unroll
  for (int r = 0; r < 4; ++r) p2v[r] = a.P2[(size_t)min(mt * 16 + 4 * g + r, b - 1) * 1600 + nt * 16 + i];
  __builtin_amdgcn_sched_barrier(0);
  const float vm = valid ? 1.f : 0.f;
  f4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    const f4 x = av[s] * vm;
    acc0 = mfma16x16x4(x.x, bv[s].x, acc0);
    acc1 = mfma16x16x4(x.y, bv[s].y, acc1);
    acc0 = mfma16x16x4(x.z, bv[s].z, acc0);
    acc1 = mfma16x16x4(x.w, bv[s].w, acc1);
  }
  const f4 acc = acc0 + acc1;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int rr = mt * 16 + 4 * g + r;
    if (rr < b) a.dP2[(size_t)rr * 1600 + nt * 16 + i] = p2v[r] > 0.f ? acc[r] : 0.f;
  }
}

// K5: tasks [0, ndp2) are dP2 tiles (when k_fwd_conv did not compute dP2), the next kDenseTasks
// (R > 1: `dense`) the dense weight gradients dW3/db3/dW4/db4 of the step, one task per wave, so
// that bucket's all-reduce overlaps the conv backward (at R = 1 k_finalize runs the same tasks
// fused with SGD).
__global__ __launch_bounds__(256) void k_dense1_bwd(MnistArgs a, int ndp2) {
  const int T = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (T < ndp2) {
    dp2_task(a, T, threadIdx.x & 63);
    return;
  }
  if (T - ndp2 < kDenseTasks) dense_w_task(a, T - ndp2, threadIdx.x & 63, false, 0.f);
}

// --------------------------------------------------------------------------------------------
// KC: conv backward per image.  Workgroup = (image, part p in 0..3), 8 waves, LDS-staged:
//   dCs  [15][15][68]  grad of conv2 output, zero border of 2 (no bounds checks in dgrad)
//   P1s  [169][36]     pooled conv1 activations (stride 36: conflict-free ds_read_b128)
//   Xs   [784]         input image
//   Wd   [9][16][16][4] W2 for this part's 16 input channels in MFMA fragment order
// Work of a part: conv2 wgrad for output channels [16p, 16p+16) over the image's 100 positions
// (19 tiles incl. the bias row, 25 k-steps each) + conv2 dgrad for channel half h = p & 1 and
// pixel part p >> 1 (pixels [0, 80) or [80, 169), 16-pixel tiles of up to 9 taps x 16 k-steps)
// whose epilogue does pool1/relu backward and conv1 wgrad.  Kernel rows kh whose taps read only
// the zero border of dC2 for every pixel of a tile are skipped (exact).  Outputs are per-image
// partial slabs, reduced deterministically by KF.
// --------------------------------------------------------------------------------------------
constexpr int kP1Stride = 36;  // forward P1 rows: conflict-free ds_read_b128 in conv2
// conv backward LDS row strides = 16 (mod 64) floats: the wgrad operand reads (16 consecutive
// floats per lane group, lane groups one row apart) hit 4 disjoint 16-bank groups
constexpr int kDcStride = 80, kDcDim = 15, kP1StrideB = 48;
constexpr int kDgSplit = 80;  // pixel split of the dgrad parts: balances their MFMA work after tap skipping
// conv2 wgrad tiles (first, count) per (pixel part, wave): waves w and w+4 share a SIMD, so each
// SIMD's wgrad + dgrad MFMAs come to <= 294 (part 0) / 292 (part 1)
__constant__ int kWgradTiles[2][8][2] = {{{0, 6}, {6, 5}, {11, 6}, {0, 0}, {0, 0}, {0, 0}, {0, 0}, {17, 2}},
                                         {{0, 5}, {5, 5}, {10, 5}, {15, 4}, {0, 0}, {0, 0}, {0, 0}, {0, 0}}};
constexpr int kLdsDc = kDcDim * kDcDim * kDcStride;   // 18000
constexpr int kLdsP1 = 169 * kP1StrideB;             // 8112
constexpr int kLdsWd = 9 * 16 * 16 * 4;              // 9216
constexpr int kLdsConvBwd = kLdsDc + kLdsP1 + 784 + kLdsWd + 8 * 10 * 16;

__global__ __launch_bounds__(512) void k_conv_bwd(MnistArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* dCs = sm;
  float* P1s = dCs + kLdsDc;
  float* Xs = P1s + kLdsP1;
  float* Wd = Xs + 784;
  float* red = Wd + kLdsWd;  // [8 waves][10][16]
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int i = lane & 15, g = lane >> 4;
  const int bi = blockIdx.x >> 2, p = blockIdx.x & 3;
  const int h = p & 1, half = p >> 1;
  if (blockIdx.x == 0) {  // re-arm k_fwd_conv's per-image head counters, next step's dP2 tag
    for (int r = tid; r < a.b; r += 512) a.cnt[r] = 0u;
    if (tid == 0) a.ep[0] += 1u;
  }
  stamp(a.stamps, 0);
  // ---- stage everything in LDS: every global load of the thread is issued first (one memory
  // round trip for the whole staging), then all LDS stores.  Out-of-range slots load a valid
  // address and are zeroed by a multiply (no per-element branch around a load). ----
  constexpr int kIdc = (kLdsDc / 4 + 511) / 512, kIp1 = (169 * 8 + 511) / 512, kIwd = (kLdsWd / 4 + 511) / 512;
  // the conv2-output gradient is expanded here from the pooled gradient dP2 (ReLU-masked by
  // k_dense1_bwd) and the pool-2 argmax bytes: cell (y, x) of window (y/2, x/2) gets the
  // window's value where the argmax is (y&1)*2 + (x&1), else 0 (4x fewer bytes than a dC2 read)
  f4 vdc[kIdc], vp1[kIp1], vwd[kIwd], vx;
  unsigned qdc[kIdc];
  int sel[kIdc];
  const float* dpb = a.dP2 + (size_t)bi * 1600;
  const unsigned* a2b = reinterpret_cast<const unsigned*>(a.A2 + (size_t)bi * 1600);
#pragma unroll
  for (int j = 0; j < kIdc; ++j) {
    const int e4 = tid + j * 512;
    const int cell = e4 / (kDcStride / 4), c4 = e4 - cell * (kDcStride / 4);
    const int y = cell / kDcDim - 2, x = cell - (cell / kDcDim) * kDcDim - 2;
    const bool in = e4 < kLdsDc / 4 && c4 < 16 && y >= 0 && y < 10 && x >= 0 && x < 10;
    const int o = in ? ((y >> 1) * 5 + (x >> 1)) * 64 + c4 * 4 : 0;
    sel[j] = in ? (y & 1) * 2 + (x & 1) : 4;  // 4 = border / pad: no byte matches
    vdc[j] = ld4(dpb + o);
    qdc[j] = a2b[o >> 2];
  }
  const float* p1b = a.P1 + (size_t)bi * 169 * 32;
#pragma unroll
  for (int j = 0; j < kIp1; ++j) {
    const int e4 = min(tid + j * 512, 169 * 8 - 1);
    vp1[j] = ld4(p1b + (e4 >> 3) * 32 + (e4 & 7) * 4);
  }
#pragma unroll
  for (int j = 0; j < kIwd; ++j) {
    const int e4 = min(tid + j * 512, kLdsWd / 4 - 1);
    const int jj = e4 & 15, cq = (e4 >> 4) & 15, tap = e4 >> 8;
    vwd[j] = ld4(a.W + a.ow2 + (size_t)(tap * 32 + 16 * h + jj) * 64 + cq * 4);
  }
  vx = ld4(a.X + (size_t)a.idx[bi] * 784 + min(tid, 195) * 4);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < kIdc; ++j) {
    const int e4 = tid + j * 512;
    if (e4 < kLdsDc / 4) {
      const unsigned q = qdc[j];
      const unsigned s = (unsigned)sel[j];
      const f4 v = vdc[j];
      st4(dCs + e4 * 4, f4{(q & 0xffu) == s ? v.x : 0.f, ((q >> 8) & 0xffu) == s ? v.y : 0.f,
                           ((q >> 16) & 0xffu) == s ? v.z : 0.f, (q >> 24) == s ? v.w : 0.f});
    }
  }
#pragma unroll
  for (int j = 0; j < kIp1; ++j) {
    const int e4 = tid + j * 512;
    if (e4 < 169 * 8) st4(P1s + (e4 >> 3) * kP1StrideB + (e4 & 7) * 4, vp1[j]);
  }
#pragma unroll
  for (int j = 0; j < kIwd; ++j) {
    const int e4 = tid + j * 512;
    if (e4 < kLdsWd / 4) st4(Wd + e4 * 4, vwd[j]);
  }
  if (tid < 196) st4(Xs + tid * 4, vx);
  stamp(a.stamps, 1);
  __syncthreads();
  stamp(a.stamps, 2);

  // ---- conv2 wgrad (19 row tiles of 25 k-steps, columns 16p + i; tile 18 = the bias row), placed
  // per wave by kWgradTiles next to the wave's dgrad work ----
  {
    const int t0 = kWgradTiles[half][wave][0], ntiles = kWgradTiles[half][wave][1];
    for (int j = 0; j < ntiles; ++j) {
      const int mt = t0 + j;
      const bool bias_tile = mt == 18;
      const int k = mt * 16 + i;
      const int tap = bias_tile ? 0 : k >> 5, ci = k & 31;
      const int kh = tap / 3, kw = tap - kh * 3;
      // k-step s covers positions p = 4s + g of the 10x10 grid.  Every operand address is a
      // per-lane base plus a compile-time offset: the 4 positions of a k-step sit in one grid row
      // except for s = 2 mod 5 (p = 10q+8 .. 10q+11), where lanes g >= 2 wrap to the next row and
      // use a second base (+3 P1 cells, +5 dC cells).  The bias row multiplies by the unit vector.
      const float* pa0 = P1s + (kh * 13 + kw + g) * kP1StrideB + ci;
      const float* paS = pa0 + (g >= 2 ? 3 * kP1StrideB : 0);
      const float* pb0 = dCs + (2 * kDcDim + 2 + g) * kDcStride + 16 * p + i;
      const float* pbS = pb0 + (g >= 2 ? 5 * kDcStride : 0);
      const float unit_a = (i == 0) ? 1.f : 0.f;
      auto kloop = [&](auto bias) {
        f4 c0 = zero4(), c1 = zero4();
#pragma unroll
        for (int s0 = 0; s0 < 25; s0 += 5) {
          float av[5], bv[5];
#pragma unroll
          for (int u = 0; u < 5; ++u) {
            const int st = s0 + u, q = (4 * st) / 10, r = (4 * st) % 10;
            const bool strad = r == 8;
            if constexpr (decltype(bias)::value) av[u] = unit_a;
            else av[u] = (strad ? paS : pa0)[(q * 13 + r) * kP1StrideB];
            bv[u] = (strad ? pbS : pb0)[(q * kDcDim + r) * kDcStride];
          }
#pragma unroll
          for (int u = 0; u < 5; ++u) {
            if ((s0 + u) & 1) c1 = mfma16x16x4(av[u], bv[u], c1);
            else c0 = mfma16x16x4(av[u], bv[u], c0);
          }
        }
        return c0 + c1;
      };
      const f4 acc = bias_tile ? kloop(std::true_type{}) : kloop(std::false_type{});
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mt * 16 + 4 * g + r;
        if (row < kMnistPart2Rows) a.part2[((size_t)bi * kMnistPart2Rows + row) * 64 + 16 * p + i] = acc[r];
      }
    }
  }

  stamp(a.stamps, 3);
  // ---- conv2 dgrad (+ pool1/relu backward + conv1 wgrad): waves 7, 6, ... take tiles 0, 1, ... ----
  float dw[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = 0.f;
  const int d = 7 - wave;
  const int pix0 = half ? kDgSplit : 0, pix1 = half ? 169 : kDgSplit;
  if (d < (pix1 - pix0 + 15) / 16) {
    const int P = pix0 + d * 16 + i;
    const bool valid = P < pix1;
    const int Pc = valid ? P : pix0;
    const int ih = Pc / 13, iw = Pc - ih * 13;
    const float* wb = Wd + (g * 16 + i) * 4;
    const int c = 16 * h + i;
    // pool-1 argmax bytes of the epilogue's 4 rows: issued now, consumed after the MFMAs
    unsigned q1v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int Pr = min(pix0 + d * 16 + 4 * g + r, pix1 - 1);
      q1v[r] = a.A1[((size_t)bi * 169 + Pr) * 32 + c];
    }
    // kernel rows kh with 0 <= ih - kh <= 9 for some pixel row ih of the tile (wave-uniform)
    const int ih_lo = (pix0 + d * 16) / 13, ih_hi = min(pix0 + d * 16 + 15, pix1 - 1) / 13;
    const int kh_lo = max(0, ih_lo - 9), kh_hi = min(2, ih_hi);
    f4 acc0 = zero4(), acc1 = zero4();
    for (int kh = kh_lo; kh <= kh_hi; ++kh) {
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int tap = kh * 3 + kw;
        const float* ap = dCs + ((ih - kh + 2) * kDcDim + (iw - kw + 2)) * kDcStride + 4 * g;
#pragma unroll
        for (int c0 = 0; c0 < 64; c0 += 16) {
          const f4 av = ld4(ap + c0);
          const f4 bv = ld4(wb + (tap * 16 + c0 / 4) * 64);
          acc0 = mfma16x16x4(av.x, bv.x, acc0);
          acc1 = mfma16x16x4(av.y, bv.y, acc1);
          acc0 = mfma16x16x4(av.z, bv.z, acc0);
          acc1 = mfma16x16x4(av.w, bv.w, acc1);
        }
      }
    }
    const f4 acc = acc0 + acc1;
    stamp(a.stamps, 6);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int Pr = pix0 + d * 16 + 4 * g + r;
      if (Pr < pix1) {
        const float v = P1s[Pr * kP1StrideB + c] > 0.f ? acc[r] : 0.f;
        const unsigned q1 = q1v[r];
        const int ph = Pr / 13, pw = Pr - ph * 13;
        const float* img = Xs + (2 * ph + (q1 >> 1)) * 28 + 2 * pw + (q1 & 1);
#pragma unroll
        for (int kh = 0; kh < 3; ++kh)
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) dw[kh * 3 + kw] = fmaf(img[kh * 28 + kw], v, dw[kh * 3 + kw]);
        dw[9] += v;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = sum_lane_groups(dw[j]);
  if (g == 0) {
#pragma unroll
    for (int j = 0; j < 10; ++j) red[(wave * 10 + j) * 16 + i] = dw[j];
  }
  stamp(a.stamps, 4);
  __syncthreads();
  stamp(a.stamps, 5);
  if (tid < 160) {
    const int j = tid >> 4, ii = tid & 15;
    float s = 0.f;
#pragma unroll
    for (int w = 2; w < 8; ++w) s += red[(w * 10 + j) * 16 + ii];
    a.part1[((size_t)bi * 2 + half) * kMnistPart1Cols + j * 32 + 16 * h + ii] = s;
  }
}

// --------------------------------------------------------------------------------------------
// KA: forward convolutions per (image, output-channel quarter), 8 waves, LDS-staged:
//   conv1 + bias + relu + maxpool into LDS (P1s, stride 36), then conv2 on MFMA for this
//   quarter's 16 channels over the 100 used positions (7 row tiles of 4 pool windows) with the
//   bias + relu + maxpool epilogue in registers.  Quarter 0 also writes P1 / A1 for backward.
//   Then dense1 for this quarter's 400 of the 1600 features: H_part[cq][bi][:] = P2_q . W3_q,
//   with the 205 KB W3 slice loaded into registers at kernel start (its latency hides behind the
//   convolutions); the head sums the 4 quarter partials + bias + ReLU.
// --------------------------------------------------------------------------------------------
constexpr int kLdsFwd = 784 + 320 + 169 * kP1Stride + 72 * 16 * 4 + 400 + 169 * 32 / 4 + 400 / 4 + 16 * 128 + 4 + 128 +
                        288 * 16 +  // (w2d: the W2 slice again, [k][16 co], for the fused backward's dgrad)
                        kHeadW;     // (hws: the loss head's operands)
// fused_bwd: this quarter's conv2-output gradient dC2 [15][15 cells][16 channels + 4 pad] with a
// zero border of 2 (the dgrad reads cells (ih - kh + 2, iw - kw + 2) without bounds checks).
// Cell stride 20 floats: 16 consecutive cells of a dgrad A read (ds_read_b128) land on 16
// distinct 4-bank groups; the 4 consecutive cells of a wgrad B read (ds_read_b32) on 4 x 16 banks.
constexpr int kDcF = 15, kDcFStride = 20;
constexpr int kLdsFwdFused = kLdsFwd + kDcF * kDcF * kDcFStride;
// conv2 wgrad row tiles (first, count) per wave of the fused backward: waves w and w + 4 share a
// SIMD; with tap skipping the dgrad MFMAs per SIMD are 192 / 168 / 144 / 144, so SIMDs 0..3 take
// 4 / 4 / 5 / 5 of the 18 kernel-row tiles (292 / 268 / 269 / 269 MFMAs per SIMD).  The bias row
// (db2 = the column sums of dC2 = the sums of the masked dP2 over the pool windows) is summed on
// the VALU in the dP2 phase instead of a 19th MFMA tile against a unit vector.
__constant__ int kFusedWgradTiles[8][2] = {{0, 2}, {2, 2}, {4, 3}, {7, 3}, {10, 2}, {12, 2}, {14, 2}, {16, 2}};

// phase stamp k < 4 of the fused backward, per wave, after the head stamps:
// buf[grid*72 + (workgroup*8 + wave)*4 + k] (the buffer then holds grid * 104 words)
__device__ __forceinline__ void bwd_stamp(unsigned long long* buf, int k) {
  if (buf != nullptr && (threadIdx.x & 63) == 0)
    buf[(size_t)gridDim.x * 72 + (blockIdx.x * 8 + (threadIdx.x >> 6)) * 4 + k] = __builtin_amdgcn_s_memrealtime();
}

// N consecutive conv2 wgrad row tiles t0 .. t0+N-1 (kernel rows 16 t .. 16 t + 15) of the fused
// backward, advanced together over the 25 k-steps; stores part2 rows of image bi.
template <int N>
__device__ __forceinline__ void fused_wgrad_tiles(const MnistArgs& a, int bi, int cq, int t0, const float* P1s,
                                                  const float* dCs) {
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const float* pa0[N];
#pragma unroll
  for (int u = 0; u < N; ++u) {
    const int k = (t0 + u) * 16 + i;
    const int tap = k >> 5, ci = k & 31;
    const int kh = tap / 3, kw = tap - kh * 3;
    pa0[u] = P1s + (kh * 13 + kw + g) * kP1Stride + ci;
  }
  // positions p = 10q + r + g; for r = 8 lanes g >= 2 wrap to the next row: +3 P1 cells, +5 dC cells
  const int wrapA = g >= 2 ? 3 * kP1Stride : 0, wrapB = g >= 2 ? 5 * kDcFStride : 0;
  const float* pb0 = dCs + (2 * kDcF + 2 + g) * kDcFStride + i;
  f4 acc[N];
#pragma unroll
  for (int u = 0; u < N; ++u) acc[u] = zero4();
  // software pipeline over blocks of kS k-steps: the operands of block n + 1 are read while the
  // MFMAs of block n issue (sched barriers keep the compiler from sinking the reads back to their
  // first use, which exposed the LDS latency before every MFMA); <= 12 reads in flight
  constexpr int kS = 3, kBlocks = (25 + kS - 1) / kS;
  float bv[2][kS], av[2][kS][N];
  auto load = [&](int buf, int blk) {
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      const int st = blk * kS + j;
      if (st >= 25) break;
      const int q = (4 * st) / 10, r = (4 * st) % 10;
      const bool strad = r == 8;
      bv[buf][j] = pb0[(q * kDcF + r) * kDcFStride + (strad ? wrapB : 0)];
#pragma unroll
      for (int u = 0; u < N; ++u) av[buf][j][u] = pa0[u][(q * 13 + r) * kP1Stride + (strad ? wrapA : 0)];
    }
  };
  load(0, 0);
#pragma unroll
  for (int blk = 0; blk < kBlocks; ++blk) {
    if (blk + 1 < kBlocks) load((blk + 1) & 1, blk + 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < kS; ++j) {
      if (blk * kS + j >= 25) break;
#pragma unroll
      for (int u = 0; u < N; ++u) acc[u] = mfma16x16x4(av[blk & 1][j][u], bv[blk & 1][j], acc[u]);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // lane (i, g) holds rows 4g .. 4g+3 of column 16cq + i: one 16-B write-through (sc1) store into
  // the row-quad layout, so the launch leaves no dirty L2 lines of its 18.7 KB per workgroup for the
  // kernel-end write-back (MI355X_MICROARCH.md: boundary + dirty bytes / 6 TB/s; publish-large)
  const auto rs = buf_rsrc(a.part2 + (size_t)bi * kP2QuadFloats, kP2QuadFloats * 4);
#pragma unroll
  for (int u = 0; u < N; ++u) st4_sc1(rs, ((((t0 + u) * 4 + g) * 64 + 16 * cq + i) * 4) * 4, acc[u]);
}

// ---- fused conv backward of one (image bi, channel quarter cq) workgroup, after its dP2 ----
// dp2s: [25 windows][16] this quarter's masked dP2 (LDS), a2s its pool-2 argmax bytes, P1s/a1s/xs
// the image's pooled conv1 output / pool-1 argmax / input (LDS), dCs the dC2 grid scratch, red
// >= 8*10*16 floats of scratch.  Writes part2 columns 16cq.. of image bi and part1 row 4bi + cq.
// this wave's conv2 dgrad operands W2[tap][16nt + i][16cq + 4g .. +3], nt = wave / 4, from the LDS
// copy w2d ([k][16 co], written at staging beside the forward's fragment-ordered w2s): one
// conflict-free ds_read_b128 per tap (a wave reads 1 KB contiguous).  As global loads (L2) issued
// before the hand-off they were 74 KB per workgroup of vector-memory traffic right when wave 0's
// partial polls need the memory pipe (a poll round then took ~1.8 us); gathered from w2s (4 strided
// ds_read_b32 per tap, 4-way bank conflicts) they cost ~1 us of LDS time.
__device__ __forceinline__ void lds_dgrad_w2(const float* w2d, f4 (&bwd)[9]) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int i = lane & 15, g = lane >> 4, nt = wave >> 2;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) bwd[tap] = ld4(w2d + (tap * 32 + 16 * nt + i) * 16 + 4 * g);
}

__device__ __forceinline__ void fused_conv_bwd(const MnistArgs& a, int bi, int cq, const float* dp2s,
                                               const uint8_t* a2s, const float* P1s, const uint8_t* a1s,
                                               const float* xs, float* dCs, float* red, const f4 (&bwd)[9]) {
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int i = lane & 15, g = lane >> 4;
  // (the dC2 grid dCs is complete: zeroed during conv2, the masked dP2 values scattered to their
  // pool-2 argmax cells by the dP2 phase, behind the caller's barrier)
  bwd_stamp(a.stamps, 0);

  // ---- conv2 wgrad: dW2[k = tap*32 + ci][16cq + co] over the 100 used positions.  k-step s
  // covers positions 4s + g of the 10 x 10 grid (see k_conv_bwd).  All of a wave's row tiles
  // advance together: one dC2 (B) read per k-step serves N MFMAs on N independent accumulators ----
  auto wgrad = [&]() {
    const int t0 = kFusedWgradTiles[wave][0], ntiles = kFusedWgradTiles[wave][1];
    if (ntiles == 2) fused_wgrad_tiles<2>(a, bi, cq, t0, P1s, dCs);
    else fused_wgrad_tiles<3>(a, bi, cq, t0, P1s, dCs);
  };
  // the wgrad and the dgrad of a wave are independent: with kMnistVariantStagger the younger half
  // (waves 4-7, each the SIMD partner of wave w - 4) runs them in the opposite order, so the two
  // waves of a SIMD are not in the same phase at the same time (MI355X_MICROARCH.md item 9)
  const bool swap = (a.variant & kMnistVariantStagger) && wave >= 4;
  if (!swap) wgrad();
  bwd_stamp(a.stamps, 1);

  // ---- conv2 dgrad over this quarter's 16 output channels (a partial sum of dP1; everything after
  // it -- ReLU mask, pool-1 routing, conv1 wgrad -- is linear in dP1, so the four quarters'
  // conv1 weight gradients simply add up in the finalize reduction).  Waves 4nt .. 4nt+3 own input
  // channels ci = 16nt + i and pixel tiles w, w + 4, w + 8 (16 pixels each), advanced together ----
  float dw[10];
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = 0.f;
  {
    const int nt = wave >> 2, wt = wave & 3;
    const int ci = 16 * nt + i;
    constexpr int kT = 3;
    f4 acc[kT][2];
    int ih[kT], iw[kT], khlo[kT], khhi[kT];
#pragma unroll
    for (int u = 0; u < kT; ++u) {
      const int t = wt + 4 * u;  // t = 11 (wave 3's third) is empty: khlo > khhi, no MFMA, no store
      const int Pc = min(t * 16 + i, 168);
      ih[u] = Pc / 13;
      iw[u] = Pc - ih[u] * 13;
      const int ih_lo = min(t * 16, 168) / 13, ih_hi = min(t * 16 + 15, 168) / 13;
      khlo[u] = t < 11 ? max(0, ih_lo - 9) : 3;  // kernel rows with 0 <= ih - kh <= 9 somewhere in the tile
      khhi[u] = min(2, ih_hi);
      acc[u][0] = zero4();
      acc[u][1] = zero4();
    }
    // epilogue operands (ReLU mask source P1, pool-1 argmax) read ahead of the MFMAs
    float p1v[kT][4];
    unsigned q1v[kT][4];
#pragma unroll
    for (int u = 0; u < kT; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int Pr = min((wt + 4 * u) * 16 + 4 * g + r, 168);
        p1v[u][r] = P1s[Pr * kP1Stride + ci];
        q1v[u][r] = a1s[Pr * 32 + ci];
      }
    // taps software-pipelined: the dC2 reads of tap k + 1 are in flight while tap k's MFMAs issue
    f4 av[2][kT];
    auto load = [&](int buf, int tap) {
      const int kh = tap / 3, kw = tap - kh * 3;
#pragma unroll
      for (int u = 0; u < kT; ++u)
        av[buf][u] = ld4(dCs + ((ih[u] - kh + 2) * kDcF + (iw[u] - kw + 2)) * kDcFStride + 4 * g);
    };
    load(0, 0);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      if (tap + 1 < 9) load((tap + 1) & 1, tap + 1);
      __builtin_amdgcn_sched_barrier(0);
      const int kh = tap / 3;
      const f4 bv = bwd[tap];
#pragma unroll
      for (int u = 0; u < kT; ++u) {
        if (kh < khlo[u] || kh > khhi[u]) continue;  // wave-uniform
        const f4 x = av[tap & 1][u];
        acc[u][0] = mfma16x16x4(x.x, bv.x, acc[u][0]);
        acc[u][1] = mfma16x16x4(x.y, bv.y, acc[u][1]);
        acc[u][0] = mfma16x16x4(x.z, bv.z, acc[u][0]);
        acc[u][1] = mfma16x16x4(x.w, bv.w, acc[u][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int u = 0; u < kT; ++u) {
      const int t = wt + 4 * u;
      if (t >= 11) continue;
      const f4 ac = acc[u][0] + acc[u][1];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int Pr = t * 16 + 4 * g + r;
        if (Pr < 169) {
          const float v = p1v[u][r] > 0.f ? ac[r] : 0.f;
          const unsigned q1 = q1v[u][r];
          const int ph = Pr / 13, pw = Pr - ph * 13;
          const float* img = xs + (2 * ph + (q1 >> 1)) * 28 + 2 * pw + (q1 & 1);
#pragma unroll
          for (int kh = 0; kh < 3; ++kh)
#pragma unroll
            for (int kw = 0; kw < 3; ++kw) dw[kh * 3 + kw] = fmaf(img[kh * 28 + kw], v, dw[kh * 3 + kw]);
          dw[9] += v;
        }
      }
    }
  }
  if (swap) wgrad();
  bwd_stamp(a.stamps, 2);
#pragma unroll
  for (int j = 0; j < 10; ++j) dw[j] = sum_lane_groups(dw[j]);
  if (g == 0) {
#pragma unroll
    for (int j = 0; j < 10; ++j) red[(wave * 10 + j) * 16 + i] = dw[j];
  }
  lds_barrier();
  bwd_stamp(a.stamps, 3);
  if (tid < kMnistPart1Cols) {
    const int j = tid >> 5, c = tid & 31, nt = c >> 4, ii = c & 15;
    float sum = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) sum += red[((4 * nt + w) * 10 + j) * 16 + ii];
    a.part1[((size_t)bi * 4 + cq) * kMnistPart1Cols + tid] = sum;
  }
}

// Saved-for-backward activations of one (image, quarter) workgroup, written from LDS AFTER the
// head hand-off (no global store sits in the conv phases, where it would queue behind the W3
// prefetch in the CU's vector-memory pipe): this quarter's share of P1 / A1 (whole image,
// 338 16-B chunks / 338 words) and its 16 channels of P2 / A2 (25 windows).
__device__ __forceinline__ void store_saved_fwd(const MnistArgs& a, int bi, int cq, const float* P1s,
                                                const uint8_t* a1s, const float* p2s, const uint8_t* a2s,
                                                int t, int nt) {
  // fused_bwd: the conv backward runs in this workgroup from LDS; only P2 (dense1 weight gradient)
  // leaves the kernel
  for (int e = (a.fused_bwd ? 676 : 0) + t; e < (a.fused_bwd ? 776 : 2 * 338 + 200); e += nt) {
    if (e < 338) {
      const int e4 = cq * 338 + e, pos = e4 >> 3, c4 = (e4 & 7) * 4;
      st4(a.P1 + (size_t)bi * 5408 + e4 * 4, ld4(P1s + pos * kP1Stride + c4));
    } else if (e < 676) {
      const int w = cq * 338 + (e - 338);
      reinterpret_cast<unsigned*>(a.A1 + (size_t)bi * 5408)[w] = reinterpret_cast<const unsigned*>(a1s)[w];
    } else if (e < 776) {
      const int u = e - 676, wo = u >> 2, q = u & 3;
      st4(a.P2 + (size_t)bi * 1600 + wo * 64 + 16 * cq + 4 * q, ld4(p2s + wo * 16 + 4 * q));
    } else {
      const int u = e - 776, wo = u >> 2, q = u & 3;
      *reinterpret_cast<unsigned*>(a.A2 + (size_t)bi * 1600 + wo * 64 + 16 * cq + 4 * q) =
          reinterpret_cast<const unsigned*>(a2s)[wo * 4 + q];
    }
  }
}

__global__ __launch_bounds__(512) void k_fwd_conv(MnistArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* xs = sm;
  float* w1s = xs + 784;
  float* P1s = w1s + 320;
  float* w2s = P1s + 169 * kP1Stride;  // [kc=72][j=16][t=4]: B[k=4kc+t][16cq+j]
  float* p2s = w2s + 72 * 16 * 4;      // [25 windows][16 channels] pooled conv2 output
  uint8_t* a1s = reinterpret_cast<uint8_t*>(p2s + 400);       // [169][32] pool-1 argmax
  uint8_t* a2s = a1s + 169 * 32;                               // [25][16] pool-2 argmax
  float* red = reinterpret_cast<float*>(a2s + 400);            // [16][128] dense1 row-group partials
  int* s_last = reinterpret_cast<int*>(red + 16 * 128);        // head hand-off: [last?, base count]
  float* w2d = red + 16 * 128 + 4 + 128;  // [k = tap*32 + ci][16 co]: the dgrad B operands, one ds_read_b128 each
  float* hws = w2d + 288 * 16;             // [kHeadW] the loss head's operands (wave 7, during conv2)
  float* dCs = hws + kHeadW;               // fused_bwd: the dC2 grid (kDcF x kDcF cells)
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int i = lane & 15, g = lane >> 4;
  int bi = blockIdx.x >> 2, cq = blockIdx.x & 3;
  if ((a.variant & kMnistVariantXcd) && (a.b & 7) == 0) {
    // block B -> XCD class B % 8, slot B / 8: each class holds b / 8 whole images (4 slots each)
    const int x = blockIdx.x & 7, sl = blockIdx.x >> 3;
    bi = x * (a.b >> 3) + (sl >> 2);
    cq = sl & 3;
  }
  // waves w and w + 4 share a SIMD; the younger half (4-7) loses the VALU issue arbitration in every
  // phase and reaches each barrier last (MI355X_MICROARCH.md, two waves per SIMD, item 4)
  if ((a.variant & kMnistVariantPrio) && __builtin_amdgcn_readfirstlane(wave) >= 4) __builtin_amdgcn_s_setprio(1);
  stamp(a.stamps, 0);
  // ---- staging: all global loads first ----
  const int sample = a.idx[bi];
  const f4 vx = ld4(a.X + (size_t)sample * 784 + min(tid, 195) * 4);
  const int label = a.Y[sample];  // for the head (this image's last quarter workgroup)
  const float vw1 = tid < 288 ? a.W[a.ow1 + tid] : a.W[a.ob1 + min(tid - 288, 31)];
  f4 vw2[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = min(tid + j * 512, 1151);  // (k, q): k = e >> 2, channels 16cq + 4q .. +3
    vw2[j] = ld4(a.W + a.ow2 + (e >> 2) * 64 + 16 * cq + (e & 3) * 4);
  }
  // the conv2 epilogue's bias and this step's hand-off tag, in the staging round trip: loaded where
  // they are used, each was the youngest load of its wave there, and the vmcnt wait for it also
  // waited for every W3 prefetch in flight (then a full global round trip on the critical path)
  const float b2v = a.W[a.ob2 + 16 * cq + (lane & 15)];
  // (a VGPR: a readfirstlane here would wait for the whole staging round trip before the LDS stores)
  const uint32_t tag = a.ep[0] + 1u;  // (advanced by KC / KF)
  __builtin_amdgcn_sched_barrier(0);
  if (tid < 196) st4(xs + tid * 4, vx);
  if (tid < 320) w1s[tid] = vw1;
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int e = tid + j * 512;
    if (e < 1152) {
      const int k = e >> 2, q = e & 3;
      float* d = w2s + ((k >> 2) * 16 + 4 * q) * 4 + (k & 3);
      d[0] = vw2[j].x;
      d[4] = vw2[j].y;
      d[8] = vw2[j].z;
      d[12] = vw2[j].w;
      st4(w2d + k * 16 + 4 * q, vw2[j]);
    }
  }
  stamp(a.stamps, 1);
  __syncthreads();
  stamp(a.stamps, 2);
  // ---- dense1 operand prefetch, overlapping the convolutions: thread (row group rg, 4 columns n4)
  // needs the W3 rows of this quarter's features kk = 16 j + rg, j = 0 .. 24 (feature kk = window
  // j, channel 16cq + rg: W3 row 64 j + 16cq + rg), so its 25 loads sit at ONE per-thread base plus
  // compile-time strides of 64 rows (a feature split by row group, 25 consecutive features per
  // thread, cost ~8 VALU of 64-bit address arithmetic per load: 200 per wave).  The 25 16-B loads
  // per thread (205 KB per workgroup, ~1.3 us of the CU's texture-address rate) are spread over the
  // conv phases in small groups: issued back to back they fill the CU's vector-memory queue and
  // every wave stalls behind them (measured: conv1 3.4-4.4 us instead of ~1 us).
  const int n4 = (tid & 31) * 4, rg = tid >> 5;
  f4 w3v[25];
  // one buffer resource over this quarter's W3 rows; the per-load stride rides in the SGPR offset
  // (a 64-bit global address per load cost ~8 VALU of address arithmetic: 200 per wave)
  const auto w3r = buf_rsrc(a.W + a.ow3 + (size_t)16 * cq * 128, (unsigned)((1600 - 16 * cq) * 128 * 4));
  const int w3vo = (rg * 128 + n4) * 4;
  auto ldw3 = [&](int j) { w3v[j] = ld4_buf(w3r, w3vo, j * 64 * 128 * 4); };
#pragma unroll
  for (int j = 0; j < 6; ++j) ldw3(j);
  // ---- conv1 on MFMA (K = 9 taps padded to 12): rows = 676 conv1 positions in pool-window-major
  // order, so a 16-row tile holds 4 whole 2x2 windows and the maxpool happens in registers.
  // 43 row tiles x 2 channel tiles; bias + relu after the max (they commute with it). ----
  {
    float bw[2][3];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3) {
        const int k = 4 * s3 + g;
        bw[nt][s3] = k < 9 ? w1s[k * 32 + nt * 16 + i] : 0.f;
      }
    int tap_off[3];
#pragma unroll
    for (int s3 = 0; s3 < 3; ++s3) {
      const int k = min(4 * s3 + g, 8);
      tap_off[s3] = (k / 3) * 28 + (k % 3);
    }
    // row tiles mt0 and mt0 + 8 per iteration, both channel tiles each: 4 independent MFMA
    // chains sharing 6 LDS loads (the two channel tiles read the same image values).  The operand
    // reads of iteration it + 1 are issued right behind iteration it's MFMAs, so their LDS latency
    // hides behind the MFMA drain and the epilogue; the conv1 biases live in registers.
    const float bias[2] = {w1s[288 + i], w1s[288 + 16 + i]};
    float xa[2][2][3];
    auto load_x = [&](int buf, int it) {
      const int mt0 = wave + 16 * it;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int mt = min(mt0 + 8 * u, 42);
        const int w = mt * 4 + (i >> 2), q = i & 3;
        const int wc = min(w, 168);
        const int y = 2 * (wc / 13) + (q >> 1), x = 2 * (wc % 13) + (q & 1);
        const float* xb = xs + y * 28 + x;
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) xa[buf][u][s3] = xb[tap_off[s3]];
      }
    };
    load_x(0, 0);
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int mt0 = wave + 16 * it;
      f4 acc[2][2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) acc[u][nt] = zero4();
#pragma unroll
      for (int s3 = 0; s3 < 3; ++s3)
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt) acc[u][nt] = mfma16x16x4(xa[it & 1][u][s3], bw[nt][s3], acc[u][nt]);
      __builtin_amdgcn_sched_barrier(0);
      if (it < 2) load_x((it + 1) & 1, it + 1);
      __builtin_amdgcn_sched_barrier(0);
      if (it < 2) {
#pragma unroll
        for (int j = 6 + 5 * it; j < 11 + 5 * it; ++j) ldw3(j);
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int wo = (mt0 + 8 * u) * 4 + g;
        if (mt0 + 8 * u >= 43 || wo >= 169) continue;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          const f4 ac = acc[u][nt];
          float m = ac.x;
          unsigned am = 0;
          if (ac.y > m) { m = ac.y; am = 1; }
          if (ac.z > m) { m = ac.z; am = 2; }
          if (ac.w > m) { m = ac.w; am = 3; }
          const int co = nt * 16 + i;
          const float v = fmaxf(m + bias[nt], 0.f);
          P1s[wo * kP1Stride + co] = v;
          a1s[wo * 32 + co] = (uint8_t)am;
        }
      }
    }
  }
  stamp(a.stamps, 3);
  lds_barrier();  // P1 / A1 in LDS; the W3 prefetch loads stay in flight
  stamp(a.stamps, 4);
  // ---- conv2 on MFMA: wave w < 7 takes row tile w (windows 4w .. 4w+3); the last 9 W3 loads
  // ride along, one per tap ----
  if (wave < 7) {
    const int wi = wave * 4 + (i >> 2), q = i & 3;
    const bool valid = wi < 25;
    const int wic = valid ? wi : 0;
    const int ph = wic / 5, pw = wic - ph * 5;
    const int oh = 2 * ph + (q >> 1), ow = 2 * pw + (q & 1);
    const float* ab = P1s + (oh * 13 + ow) * kP1Stride + 4 * g;
    const float* bb = w2s + (g * 16 + i) * 4;
    f4 acc0 = zero4(), acc1 = zero4();
#pragma unroll
    for (int kk = 0; kk < 9; ++kk) {
      const int kh = kk / 3, kw = kk % 3;
#pragma unroll
      for (int cb = 0; cb < 32; cb += 16) {
        const f4 av = ld4(ab + (kh * 13 + kw) * kP1Stride + cb);
        const f4 bv = ld4(bb + ((kk * 32 + cb) / 4) * 64);
        acc0 = mfma16x16x4(av.x, bv.x, acc0);
        acc1 = mfma16x16x4(av.y, bv.y, acc1);
        acc0 = mfma16x16x4(av.z, bv.z, acc0);
        acc1 = mfma16x16x4(av.w, bv.w, acc1);
      }
      __builtin_amdgcn_sched_barrier(0);
      ldw3(16 + kk);
      __builtin_amdgcn_sched_barrier(0);
    }
    const f4 acc = acc0 + acc1;
    stamp(a.stamps, 5);
    const int wo = wave * 4 + g;
    if (wo < 25) {
      float m = acc.x;
      unsigned am = 0;
      if (acc.y > m) { m = acc.y; am = 1; }
      if (acc.z > m) { m = acc.z; am = 2; }
      if (acc.w > m) { m = acc.w; am = 3; }
      const float v = fmaxf(m + b2v, 0.f);
      p2s[wo * 16 + i] = v;
      a2s[wo * 16 + i] = (uint8_t)am;
    }
  } else {
#pragma unroll
    for (int j = 16; j < 25; ++j) ldw3(j);
    if (a.head != 0) {
      // the head's operands into LDS: 23 loads per lane, off every critical path
      float hv[23];
#pragma unroll
      for (int u = 0; u < 23; ++u) {
        const int e = min(lane + 64 * u, 1417);
        hv[u] = a.W[e < 1280 ? a.ow4 + e : (e < 1408 ? a.ob3 + (e - 1280) : a.ob4 + (e - 1408))];
      }
#pragma unroll
      for (int u = 0; u < 23; ++u)
        if (lane + 64 * u < 1418) hws[lane + 64 * u] = hv[u];
    }
    if (a.head == 1 && a.dp2_fwd && a.fused_bwd) {
      // wave 7 has no conv2 tile: it zeroes the fused backward's dC2 grid meanwhile (the dP2 phase
      // only scatters the masked dP2 values to their pool-2 argmax cells; every other cell -- the
      // zero border, the non-argmax cells, row / column 10 of the 11 x 11 conv output -- stays 0)
      for (int e4 = lane; e4 < kDcF * kDcF * kDcFStride / 4; e4 += 64) st4(dCs + e4 * 4, zero4());
    }
  }
  __syncthreads();
  // ---- dense1 quarter partial: 25 features x 4 columns per thread, 16 row groups reduced in LDS
  {
    f4 hs = zero4();
#pragma unroll
    for (int j = 0; j < 25; ++j) hs += p2s[j * 16 + rg] * w3v[j];
    st4(red + rg * 128 + n4, hs);
  }
  lds_barrier();
  // dp2_fwd (training): every workgroup resident at once, so every quarter workgroup runs the head
  // itself from the other quarters' tagged partials; otherwise the last to arrive runs it
  const bool tagged = a.head == 1 && a.dp2_fwd;
  float* sown = red + 16 * 128 + 4;   // [128] this quarter's own partial
  if (tid < 32) {
    f4 hsum = zero4();
#pragma unroll
    for (int k = 0; k < 16; ++k) hsum += ld4(red + k * 128 + 4 * tid);
    if (!tagged) {
      // 16-B sc1 store: the image's head may run on another XCD (hand-off below)
      st4_sc1(buf_rsrc(a.part3 + ((size_t)cq * a.b + bi) * 128, 512), tid * 16, hsum);
    } else {
      st4(sown + 4 * tid, hsum);
      // (value, tag) words, 8-B write-through stores, polled by the other three quarters
      unsigned long long* p = a.part3t + ((size_t)cq * a.b + bi) * 128 + 4 * tid;
      const unsigned long long tg = (unsigned long long)tag << 32;
      __hip_atomic_store(p, (unsigned long long)__float_as_uint(hsum.x) | tg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 1, (unsigned long long)__float_as_uint(hsum.y) | tg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 2, (unsigned long long)__float_as_uint(hsum.z) | tg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p + 3, (unsigned long long)__float_as_uint(hsum.w) | tg, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  stamp(a.stamps, 6);
  if (a.head == 0) {
    store_saved_fwd(a, bi, cq, P1s, a1s, p2s, a2s, tid, 512);
    return;
  }
  // the head's weights, loaded by wave 0 of every workgroup now: their latency hides behind the
  // hand-off (5 KB, L2-resident).  (Staged in LDS with the image instead: no faster -- the staging
  // round trip grows by as much, profiles/mnist_head_ab_r5.txt.)
  HeadWeights hw;
  const int uwave = __builtin_amdgcn_readfirstlane(wave);
  if (uwave == 0) hw = lds_head_weights(hws, lane);
  // the fused backward's conv2-dgrad operands, from LDS, while the hand-off is in flight (waves 1-7
  // wait for wave 0's head; wave 0's head waits for its polls: the LDS reads are off both paths)
  f4 bwd[9];
  if (a.head == 1 && a.dp2_fwd && a.fused_bwd) lds_dgrad_w2(w2d, bwd);

  // ---- hand-off to the image's last quarter workgroup (MI355X_MICROARCH.md, inter-workgroup
  // visibility, first table row): the storing wave drains its sc1 stores, a workgroup barrier,
  // ONE agent-scope add per workgroup on the image's counter; the workgroup whose add returns
  // 3 (mod 4) is last and reads the 4 partials with sc1 loads.  The election itself never waits
  // (placement-independent).  k_conv_bwd (in every training step after this launch)
  // zeroes the counters, so a launch that did not add exactly 4 per image cannot shift the
  // election of later steps.
  if (!tagged) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.cnt + bi, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last[0] = (old & 3u) == 3u;
    }
  }
  lds_barrier();  // (tagged: this quarter's own partial in LDS)
  const bool last = tagged || s_last[0] != 0;  // (tagged: every quarter runs the head)
  float* sdh = red;  // [128] dH of this image (the dense1 row-group scratch is free now)
  if (last && uwave == 0) {
    if (a.head == 1) head_row(a, bi, lane, label, hw, sdh, tag, tagged ? sown : nullptr, cq, !tagged || cq == kHeadQuarter);
    else head_eval(a, bi, lane, label, hw);
  }
  if (a.head != 1) return;  // evaluation: nothing is saved for a backward pass
  // saved activations leave LDS only now (off the head's critical path)
  if (!last) store_saved_fwd(a, bi, cq, P1s, a1s, p2s, a2s, tid, 512);
  else if (wave != 0) store_saved_fwd(a, bi, cq, P1s, a1s, p2s, a2s, tid - 64, 448);
  if (!a.dp2_fwd) return;  // dP2 by k_dense1_bwd
  // ---- dP2 = (dH W3^T) * 1[P2 > 0] for this quarter's 400 features, from the W3 slice still in
  // registers (no K5 launch, no second read of W3), dH from this workgroup's own head (LDS) ----
  lds_barrier();
  if (a.fused_bwd) stamp(a.stamps, 7);  // (fused: slot 7 = the dP2 phase's start, after the dH barrier)
  const f4 dh = ld4(sdh + n4);
  float v[25];
  {
    // 4-term dot products on packed f32 math (v_pk_mul_f32 + v_pk_fma_f32 + one add: 3 VALU per
    // feature instead of 5; nothing else competes for the VALU in this phase)
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 dlo = {dh.x, dh.y}, dhi = {dh.z, dh.w};
#pragma unroll
    for (int j = 0; j < 25; ++j) {
      f2 t = f2{w3v[j].x, w3v[j].y} * dlo;
      t = __builtin_elementwise_fma(f2{w3v[j].z, w3v[j].w}, dhi, t);
      v[j] = t.x + t.y;
    }
  }
  // sum over the 32 lanes of the row group (column groups n4): reduce-scatter butterfly, lane
  // (l & 31) ends with feature 16 (l & 31) + rg (j = l & 31 >= 25: zero padding)
  const float d = reduce_scatter32<25>(v, lane);
  const int j = lane & 31;
  if (a.fused_bwd) {
    // the conv2-output gradient dC2 directly: the masked dP2 value of window j, channel rg goes to
    // its pool-2 argmax cell of the (zeroed) dC2 grid; every other cell of the window is 0
    float val = 0.f;
    if (j < 25) {
      const int kk = j * 16 + rg;
      val = p2s[kk] > 0.f ? d : 0.f;
      const unsigned am = a2s[kk];
      const int ph = (j * 13) >> 6, pw = j - 5 * ph;  // j / 5, j % 5 for j < 25
      const int y = 2 * ph + (int)(am >> 1), x = 2 * pw + (int)(am & 1u);
      dCs[((y + 2) * kDcF + x + 2) * kDcFStride + rg] = val;
    }
    // db2 of channel 16cq + rg (the dW2 bias row) = the sum of dC2 over the conv2 positions = the
    // half-wave sum of the masked dP2 values (fixed butterfly order: bit-identical replicas)
    float sb = rs_swap16(val, val);
    sb += dpp_xor8(sb);
    sb += dpp_mirror8(sb);
    sb += dpp_xor2(sb);
    sb += dpp_xor1(sb);
    if (j == 0) {
      const auto rs = buf_rsrc(a.part2 + (size_t)bi * kP2QuadFloats, kP2QuadFloats * 4);
      st4_sc1(rs, (((kP2Quads - 1) * 64 + 16 * cq + rg) * 4) * 4, f4{sb, 0.f, 0.f, 0.f});
    }
    lds_barrier();
    fused_conv_bwd(a, bi, cq, p2s, a2s, P1s, a1s, xs, dCs, red, bwd);
    return;
  }
  if (j < 25) {
    const int kk = j * 16 + rg;
    a.dP2[(size_t)bi * 1600 + j * 64 + 16 * cq + rg] = p2s[kk] > 0.f ? d : 0.f;
  }
  stamp(a.stamps, 7);
}

// --------------------------------------------------------------------------------------------
// KF: reduce the per-image partial slabs into G (+ optional fused SGD).
//   blocks [0, ndb)               : dense weight-gradient tasks (when the step's forward did not
//                                   run them as K5), each fused with SGD of its outputs
//   blocks [ndb, ndb + nbs)       : SGD sweep of the dense range (dense gradients from K5)
//   blocks [.., + nb2)            : conv2 kernel/bias, 4 threads per output (16 images each)
//   blocks [.., + nb1)            : conv1 kernel/bias, 16 threads per output
// --------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_finalize(MnistArgs a, int apply_sgd, int ndb, int nbs, int nb2, int nb1) {
  const float lr = *a.lr;
  int blk = blockIdx.x;
  if (blk < ndb) {
    const int T = blk * 4 + (threadIdx.x >> 6);
    if (T < kDenseTasks) dense_w_task(a, T, threadIdx.x & 63, apply_sgd != 0, lr);
    return;
  }
  blk -= ndb;
  if (blk < nbs) {
    const int e = a.ow3 + blk * 256 + threadIdx.x;
    if (e < a.nslab) a.W[e] -= lr * a.G[e];
    return;
  }
  if (blk < nbs + nb2) {
    const int t = (blk - nbs) * 256 + threadIdx.x;
    const int o = t >> 2, sub = t & 3;  // o in [0, 289*64)
    const int n = kMnistPart2Rows * 64;
    float s = 0.f;
    const int oc = min(o, n - 1);
    const int e = (oc >> 6) < 288 ? a.ow2 + oc : a.ob2 + (oc & 63);
    const float wold = apply_sgd ? a.W[e] : 0.f;  // in the same round trip as the partials
    for (int base = 0; base < a.b; base += 64) {  // 16 independent loads in flight per thread
      float v[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) v[j] = a.part2[(size_t)min(base + sub + 4 * j, a.b - 1) * n + oc];
#pragma unroll
      for (int j = 0; j < 16; ++j) s += (base + sub + 4 * j < a.b) ? v[j] : 0.f;
    }
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    if (sub == 0 && o < n) {
      a.G[e] = s;
      if (apply_sgd) a.W[e] = wold - lr * s;
    }
    return;
  }
  const int t = (blk - nbs - nb2) * 256 + threadIdx.x;
  const int o = t >> 4, sub = t & 15;  // o in [0, 320)
  const int rows = mnist_part1_rows(a.b, a.fused_bwd != 0);
  float s = 0.f;
  const int oc = min(o, kMnistPart1Cols - 1);
  const int e = oc < 288 ? a.ow1 + oc : a.ob1 + (oc - 288);
  const float wold = apply_sgd ? a.W[e] : 0.f;
  for (int base = 0; base < rows; base += 128) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = a.part1[(size_t)min(base + sub + 16 * j, rows - 1) * kMnistPart1Cols + oc];
#pragma unroll
    for (int j = 0; j < 8; ++j) s += (base + sub + 16 * j < rows) ? v[j] : 0.f;
  }
#pragma unroll
  for (int m = 1; m < 16; m <<= 1) s += __shfl_xor(s, m, 64);
  if (sub == 0 && o < kMnistPart1Cols) {
    a.G[e] = s;
    if (apply_sgd) a.W[e] = wold - lr * s;
  }
}

// --------------------------------------------------------------------------------------------
// KF-X: finalize of the fused_bwd step, one workgroup per contiguous slab range (kFxBlocks):
// (512 threads = 8 waves each)
//   [0, 200)    dW3 rows 16m .. 16m+15, columns 64h .. 64h+63 (j = 2m + h): 4 dense tasks, waves 0-3
//   [200, 204)  db3 columns 32 jj .. +31: 2 dense tasks (waves 0-1)
//   [204, 208)  dW4 rows 32 jj .. +31 (x 10): 2 dense tasks (waves 0-1)
//   208         db4 (10 floats): 1 dense task
//   [209, 355)  conv2 (kernel row quad, 32-column half) pieces (the last quad: the bias row)
//   [355, 375)  conv1 kernel / bias outputs 16q .. 16q+15: 4 rows x 16 columns per wave load
// Each writes its gradient range into G.  R = 1 with SGD: W -= lr * G of the range.  R > 1 with
// the exchange (a.xchg): the range is also published into this workgroup's slot of the channel's
// exchange buffer (at its slab offsets), then the xGMI exchange with workgroup j of every peer
// (epoch / parity protocol of csrc/kernels/xgmi.hip, bounded waits), then W -= lr * (sum of the R
// contributions in rank order): bit-identical on every replica, and the all-reduce of one range
// overlaps the reductions of the others inside ONE launch.
// --------------------------------------------------------------------------------------------
// slab range of finalize workgroup j: nseg segments of cnt floats, stride floats apart
__device__ __forceinline__ void fx_range(const MnistArgs& a, int j, int& lo, int& cnt, int& nseg, int& stride) {
  nseg = 1;
  stride = 0;
  if (j < kFxW3) {
    lo = a.ow3 + (j >> 1) * 2048 + (j & 1) * 64;  // rows 16 (j >> 1) .., columns 64 (j & 1) ..
    cnt = 64;
    nseg = 16;
    stride = 128;
  } else if (j < kFxW3 + 4) {
    lo = a.ob3 + 32 * (j - kFxW3);  // db3 columns 32 jj .. (tasks 2 jj, 2 jj + 1)
    cnt = 32;
  } else if (j < kFxW3 + 8) {
    lo = a.ow4 + 320 * (j - kFxW3 - 4);  // dW4 rows 32 jj .. +31, 10 columns each
    cnt = 320;
  } else if (j == kFxW3 + 8) {
    lo = a.ob4;
    cnt = 10;
  } else if (j < kFxDense + kFxConv2) {
    const int qd = (j - kFxDense) >> 1, h = (j - kFxDense) & 1;
    if (qd == kP2Quads - 1) {
      lo = a.ob2 + 32 * h;
      cnt = 32;
    } else {
      lo = a.ow2 + qd * 256 + 32 * h;  // rows 4qd .. 4qd+3, columns 32h .. 32h+31
      cnt = 32;
      nseg = 4;
      stride = 64;
    }
  } else {
    const int q = j - kFxDense - kFxConv2;
    lo = q < 18 ? a.ow1 + q * 16 : a.ob1 + (q - 18) * 16;
    cnt = 16;
  }
}

template <int R>
__device__ __forceinline__ void finalize_x_body(const MnistArgs& a, int apply_sgd, int j);

// phase stamps of KF-X (diagnostics), after the fused kernel's grid*104 words: per wave, start and end
template <int R, bool LOOP>
__global__ __launch_bounds__(512) void k_finalize_x(MnistArgs a, int apply_sgd) {
  unsigned long long* sb = a.stamps == nullptr ? nullptr
      : a.stamps + (size_t)a.b * 4 * 104 + ((size_t)blockIdx.x * 8 + (threadIdx.x >> 6)) * 2;
  if (sb != nullptr && (threadIdx.x & 63) == 0) sb[0] = __builtin_amdgcn_s_memrealtime();
  // workgroup b runs ranges b, b + grid, ... in the same order on every rank: with a capped grid
  // (a.fx_grid, replicas SHARING one GPU) every rank's workgroups are resident together, so range j
  // of each rank always finds range j of its peers running (a full 269-workgroup grid per rank
  // cannot be co-resident for 8 ranks on one GPU: some ranks would fill it while the peers they
  // wait for have no workgroup resident).  One range per workgroup on a GPU of its own.
  // (LOOP = false: the grid is exactly one workgroup per range -- a separate instantiation, because
  // the range loop costs the body its specialisation: 111 VGPRs / 106 SGPRs instead of 72 / 59,
  // i.e. 2 instead of 3 resident workgroups per CU)
  if constexpr (LOOP) {
    for (int j = blockIdx.x; j < kFxBlocks; j += gridDim.x) {
      finalize_x_body<R>(a, apply_sgd, j);
      __syncthreads();  // (LDS scratch reused by the next range)
    }
  } else {
    finalize_x_body<R>(a, apply_sgd, blockIdx.x);
  }
  if (sb != nullptr && (threadIdx.x & 63) == 0) sb[1] = __builtin_amdgcn_s_memrealtime();
}

template <int R>
__device__ __forceinline__ void finalize_x_body(const MnistArgs& a, int apply_sgd, int j) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const float lr = *a.lr;
  const bool xchg = R > 1 && a.xchg && apply_sgd;
  // the next step's hand-off tag (no k_conv_bwd launch), advanced on every path, by a wave with no
  // dense task (range 0 is a dW3 range: waves 0-3 busy): its load -> store round trip in front of a
  // task's operand loads made block 0 the finalize's last
  if (j == 0 && tid == 4 * 64) a.ep[0] += 1u;
  uint32_t e = 0;
  float* xdst = nullptr;
  int64_t half = 0;
  if (xchg) {
    e = __builtin_amdgcn_readfirstlane(a.xa.epoch[j]) + 1u;
    if (xgmi_failed(a.xa.err)) {
      // a peer already failed: no exchange, no update, and G is left as the previous step wrote it.
      // The epoch still advances (as in k_xgmi_oneshot / _twoshot), so that after a reset_error
      // every rank's channel epochs stay in step and no rank reads the other parity half
      if (tid == 0) a.xa.epoch[j] = e;
      return;
    }
    half = (int64_t)(e & 1u) * 2 * a.xa.cap;
    xdst = a.xa.p.buf[a.xa.rank] + half;
  }
  const bool sgd_local = R == 1 && apply_sgd;  // single replica: SGD fused into the reduction
  // (the exchange path applies SGD from the peers' published ranges: G is not read there either)
  const bool keep_g = !((sgd_local || xchg) && (a.variant & kMnistVariantNoG));
  // ---- this workgroup's gradient range ----
  if (j < kFxW3) {
    // dW3 rows 16 (j >> 1) .. +15, column tiles 4 (j & 1) .. +3: one task per wave of waves 0-3
    if (wave < 4) dense_w_task(a, (j >> 1) * 8 + (j & 1) * 4 + wave, lane, sgd_local, lr, xdst, keep_g);
  } else if (j < kFxDense) {
    // db3 (tasks kD1TasksW3 - 8 ..) and dW4 (kD1TasksW3 ..): two tasks per workgroup on waves 0-1;
    // db4 (kD1TasksW3 + 8): wave 0 of the last one
    const int jj = j - kFxW3, t = 2 * jj + wave;
    if (jj < 8 ? wave < 2 : wave == 0)
      dense_w_task(a, jj < 8 ? (t < 8 ? kD1TasksW3 - 8 + t : kD1TasksW3 + t - 8) : kD1TasksW3 + 8, lane, sgd_local, lr,
                   xdst, keep_g);
  } else if (j < kFxDense + kFxConv2) {
    // conv2 row quad qd (kernel rows 4qd .. 4qd+3; the last quad: the bias row), columns 32h ..
    // 32h+31: thread (column c = tid & 31, image group grp = tid >> 5) sums the quad's 4 rows (one
    // 16-B load) over images grp, grp + 16, .. (a wave load: 2 x 512 contiguous bytes); then the
    // two groups of a wave via permlane32 and the 8 waves in LDS (fixed order)
    __shared__ f4 fx_red2[8][32];
    const int qd = (j - kFxDense) >> 1, h = (j - kFxDense) & 1, c = tid & 31, grp = tid >> 5;
    const bool biasq = qd == kP2Quads - 1;
    // the SGD operand of this thread's output (threads < 128) rides in the partials' round trip
    // instead of a second dependent load after the LDS reduction
    const int cc = tid >> 2, rr = tid & 3;
    const bool owner = tid < 128 && (!biasq || rr == 0);
    const int e2 = biasq ? a.ob2 + 32 * h + cc : a.ow2 + (4 * qd + rr) * 64 + 32 * h + cc;
    const float wold = (sgd_local && owner) ? a.W[e2] : 0.f;
    f4 sum = zero4();
    // images past b read 0 (resource sized to the b images); image stride in the SGPR offset
    const auto p2r = buf_rsrc(a.part2, (unsigned)(a.b * kP2QuadFloats * 4));
    const int vo2 = (grp * kP2QuadFloats + (qd * 64 + 32 * h + c) * 4) * 4;
    for (int base = 0; base < a.b; base += 64) {  // 4 images per thread in flight
      f4 v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) v[jj] = ld4_buf(p2r, vo2, (base + 16 * jj) * kP2QuadFloats * 4);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) sum += v[jj];
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sum[r] = rs_swap32(sum[r], sum[r]);
    if (lane < 32) fx_red2[wave][c] = sum;
    __syncthreads();
    if (owner) {
      float s2 = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) s2 += fx_red2[w][cc][rr];
      if (keep_g) a.G[e2] = s2;
      if (xdst != nullptr) xdst[e2] = s2;
      if (sgd_local) a.W[e2] = wold - lr * s2;
    }
  } else {
    // conv1 columns 16q .. 16q+15 over the part1 rows: lane (c = lane & 15, rg = lane >> 4) of wave
    // w reads rows 32 jj + 4 w + rg, so every wave load is 4 rows x one 64-B column segment; then a
    // lane-group sum and the 8 waves' sums in LDS (fixed order)
    __shared__ float fx_red[8][16];
    const int q = j - kFxDense - kFxConv2, c = lane & 15, rg = lane >> 4, o = q * 16 + c;
    const int rows = mnist_part1_rows(a.b, true);
    const int e1 = o < 288 ? a.ow1 + o : a.ob1 + (o - 288);
    const float wold = sgd_local && wave == 0 ? a.W[e1] : 0.f;
    float sum = 0.f;
    // rows past `rows` read 0 (resource sized to them); the row stride rides in the SGPR offset
    const auto p1r = buf_rsrc(a.part1, (unsigned)(rows * kMnistPart1Cols * 4));
    const int vo1 = ((4 * wave + rg) * kMnistPart1Cols + o) * 4;
    for (int b0 = 0; b0 < rows; b0 += 256) {
      float v[8];
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) v[jj] = ld1_buf(p1r, vo1, (b0 + 32 * jj) * kMnistPart1Cols * 4);
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) sum += v[jj];
    }
    sum = sum_lane_groups(sum);
    if (rg == 0) fx_red[wave][c] = sum;
    __syncthreads();
    if (wave == 0 && rg == 0) {
      float s = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) s += fx_red[w][c];
      if (keep_g) a.G[e1] = s;
      if (xdst != nullptr) xdst[e1] = s;
      if (sgd_local) a.W[e1] = wold - lr * s;
    }
  }
  if constexpr (R > 1) {
    if (!xchg) return;
    // ---- exchange with workgroup j of every peer, rank-order sum, SGD of the range ----
    if (!xgmi_exchange<R>(a.xa.p, a.xa.rank, a.xa.sig_blocks, a.xa.timeout, a.xa.err, 0, j, e)) {
      if (tid == 0) a.xa.epoch[j] = e;
      return;
    }
    int lo, cnt, nseg, stride;
    fx_range(a, j, lo, cnt, nseg, stride);
    const int n4 = cnt >> 2;  // (every segment starts 16-B aligned: slab offsets are multiples of 4)
    // updated weights as 16-B write-through stores (no dirty W lines for the kernel-end write-back,
    // as in the single-replica dW3 tasks: profiles/mnist_fx_w3_writethrough_r5.txt)
    const auto wr = buf_rsrc(a.W, (unsigned)a.nslab * 4u);
    const int tot = n4 * nseg;
    auto off_of = [&](int t) { return (int64_t)lo + (int64_t)(t / n4) * stride + 4 * (t % n4); };
    if (a.xtwo) {
      // two-shot: f4 t of the range belongs to rank (t R) / tot.  Reduce-scatter: the owner sums its
      // share in rank order and stages the updated weights in its result region; after the second
      // round every rank copies each share from its owner (bit-identical by construction, and W is
      // written only after both rounds: a timeout leaves it untouched).  2 (R-1)/R of the range
      // crosses the fabric per rank instead of (R-1) x the range.
      const int64_t res = half + a.xa.cap;
      float* mine = a.xa.p.buf[a.xa.rank];
      for (int t = tid; t < tot; t += 512) {
        if ((t * R) / tot != a.xa.rank) continue;
        const int64_t off = off_of(t);
        f4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = ld4(a.xa.p.buf[r] + half + off);
        f4 acc = v[0];
#pragma unroll
        for (int r = 1; r < R; ++r) acc += v[r];
        st4(mine + res + off, ld4(a.W + off) - lr * acc);
      }
      if (!xgmi_exchange<R>(a.xa.p, a.xa.rank, a.xa.sig_blocks, a.xa.timeout, a.xa.err, 1, j, e)) {
        if (tid == 0) a.xa.epoch[j] = e;
        return;
      }
      for (int t = tid; t < tot; t += 512) {
        const int64_t off = off_of(t);
        st4_sc1(wr, (int)off * 4, ld4(a.xa.p.buf[(t * R) / tot] + res + off));
      }
    } else {
      for (int t = tid; t < tot; t += 512) {
        const int64_t off = off_of(t);
        f4 v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = ld4(a.xa.p.buf[r] + half + off);
        f4 acc = v[0];
#pragma unroll
        for (int r = 1; r < R; ++r) acc += v[r];
        st4_sc1(wr, (int)off * 4, ld4(a.W + off) - lr * acc);
      }
    }
    // scalar tail of a range (db4: 10 floats), summed by every rank itself in rank order
    for (int t = 4 * n4 + tid; t < cnt; t += 512) {
      const int64_t off = lo + t;
      float acc = a.xa.p.buf[0][half + off];
#pragma unroll
      for (int r = 1; r < R; ++r) acc += a.xa.p.buf[r][half + off];
      a.W[off] -= lr * acc;
    }
    if (tid == 0) a.xa.epoch[j] = e;
  }
}

// --------------------------------------------------------------------------------------------
// Optimizer kernels over flat slabs.
// --------------------------------------------------------------------------------------------
// gz (optional, = g): the gradient is zeroed after its use, so the next step's backward can accumulate
// into it without a separate fill launch (engine/trainer.py)
// (g is not __restrict__: gz aliases it)
__global__ __launch_bounds__(256) void k_sgd(float* __restrict__ w, const float* g, const float* __restrict__ lrp,
                                             int64_t n, float* gz) {
  const float lr = *lrp;
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    f4 wv = ld4(w + i4);
    const f4 gv = ld4(g + i4);
    wv -= lr * gv;
    st4(w + i4, wv);
    if (gz != nullptr) st4(gz + i4, zero4());
  } else {
    for (int64_t j = i4; j < n; ++j) {
      w[j] -= lr * g[j];
      if (gz != nullptr) gz[j] = 0.f;
    }
  }
}

__global__ __launch_bounds__(256) void k_sgd_momentum(float* __restrict__ w, const float* g,
                                                      float* __restrict__ v, const float* __restrict__ lrp,
                                                      float m, int nesterov, int64_t n, float* gz) {
  const float lr = *lrp;
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i4 + 3 < n) {
    f4 wv = ld4(w + i4), vv = ld4(v + i4);
    const f4 gv = ld4(g + i4);
    vv = m * vv - lr * gv;
    wv += nesterov ? (m * vv - lr * gv) : vv;
    st4(w + i4, wv);
    st4(v + i4, vv);
    if (gz != nullptr) st4(gz + i4, zero4());
  } else {
    for (int64_t j = i4; j < n; ++j) {
      const float gj = g[j];
      const float vj = m * v[j] - lr * gj;
      v[j] = vj;
      w[j] += nesterov ? (m * vj - lr * gj) : vj;
      if (gz != nullptr) gz[j] = 0.f;
    }
  }
}

// --------------------------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------------------------
void mnist_dense1_bwd(const MnistArgs& a, bool dp2, bool dense, hipStream_t s) {
  const int ndp2 = dp2 ? ((a.b + 15) / 16) * 100 : 0;
  const int tasks = ndp2 + (dense ? kDenseTasks : 0);
  if (tasks > 0) hipLaunchKernelGGL(k_dense1_bwd, dim3((tasks + 3) / 4), dim3(256), 0, s, a, ndp2);
}
void mnist_conv_bwd(const MnistArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_conv_bwd, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_conv_bwd, dim3(a.b * 4), dim3(512), kLdsConvBwd * sizeof(float), s, a);
}
void mnist_fwd_conv(const MnistArgs& a, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_fwd_conv, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const bool fused = a.head == 1 && a.dp2_fwd && a.fused_bwd;
  hipLaunchKernelGGL(k_fwd_conv, dim3(a.b * 4), dim3(512), (fused ? kLdsFwdFused : kLdsFwd) * sizeof(float), s, a);
}
void mnist_finalize(const MnistArgs& a, bool apply_sgd, bool with_dense, hipStream_t s) {
  const int ndb = with_dense ? (kDenseTasks + 3) / 4 : 0;
  const int nbs = (apply_sgd && !with_dense) ? (a.nslab - a.ow3 + 255) / 256 : 0;
  const int nb2 = (kMnistPart2Rows * 64 * 4 + 255) / 256;
  const int nb1 = (kMnistPart1Cols * 16 + 255) / 256;
  hipLaunchKernelGGL(k_finalize, dim3(ndb + nbs + nb2 + nb1), dim3(256), 0, s, a, apply_sgd ? 1 : 0, ndb, nbs, nb2,
                     nb1);
}
void mnist_finalize_x(const MnistArgs& a, bool apply_sgd, hipStream_t s) {
  const int R = (a.xchg && apply_sgd) ? a.xa.world : 1;
  const int sgd = apply_sgd ? 1 : 0;
  const int kFxBlocks = (a.fx_grid > 0 && a.fx_grid < tdl::kFxBlocks) ? a.fx_grid : tdl::kFxBlocks;
  auto launch = [&](auto rk, auto loop) {
    constexpr int kR = decltype(rk)::value;
    hipLaunchKernelGGL((k_finalize_x<kR, decltype(loop)::value>), dim3(kFxBlocks), dim3(512), 0, s, a, sgd);
  };
  auto go = [&](auto rk) {
    if (kFxBlocks < tdl::kFxBlocks) launch(rk, std::true_type{});
    else launch(rk, std::false_type{});
  };
  switch (R) {  // the rank count is a template parameter (straight-line rank-order sums)
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 5: go(std::integral_constant<int, 5>{}); break;
    case 6: go(std::integral_constant<int, 6>{}); break;
    case 7: go(std::integral_constant<int, 7>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    default: go(std::integral_constant<int, 1>{}); break;
  }
}
void sgd_apply(float* w, const float* g, const float* lr, int64_t n, hipStream_t s, bool zero_g) {
  const int64_t nt = (n + 3) / 4;
  hipLaunchKernelGGL(k_sgd, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w, g, lr, n,
                     zero_g ? const_cast<float*>(g) : nullptr);
}
void sgd_momentum_apply(float* w, const float* g, float* v, const float* lr, float momentum, bool nesterov,
                        int64_t n, hipStream_t s, bool zero_g) {
  const int64_t nt = (n + 3) / 4;
  hipLaunchKernelGGL(k_sgd_momentum, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, w, g, v, lr, momentum,
                     nesterov ? 1 : 0, n, zero_g ? const_cast<float*>(g) : nullptr);
}

}  // namespace tdl
