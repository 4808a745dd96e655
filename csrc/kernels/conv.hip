// Implicit-GEMM NHWC bf16 convolution for gfx950 (see conv.h).
//
// GEMM view: rows = output pixels (n, oh, ow), columns = output channels, reduction =
// (kh, kw, c) in chunks of 64 channels (C % 64 == 0, so a chunk never straddles a filter tap).
// Workgroup tile BM x BN x 64 (128 x 128; 128 x 64 when K % 128 != 0; 256 x 128 for sweeps), BM/64 x 2 waves, each
// wave 64 x BN/2 built from 16x16x32 MFMAs (4 x BN/32 accumulators).  Operands are register-staged through a double-buffered
// LDS image with 128-byte rows whose 16-byte chunks are XOR-swizzled by row (swz() below: conflict-free
// fragment reads and staging writes; a 16-B row pad instead measured 34 % of LDS cycles in bank
// conflicts, profiles/conv_pmc_r1_padded_rows.txt vs _swizzled.txt).  Global loads of tile t+1 are in flight while the MFMAs of tile t
// run; one barrier per tile.  Out-of-image taps and rows past M load zeros (padding is implicit:
// no padded copy of the activations is ever made).  Epilogue: the f32 tile is rounded to bf16 into
// LDS (8-byte writes: the MFMA takes the weight fragment as its A operand, so each lane's four
// accumulators are four adjacent channels of one pixel) and written back as 16-byte row segments.
//
// The same kernel computes the stride-1 input gradient: dy is the "image", the filter taps are
// mirrored (kh -> KH-1-kh) and the weight rows are HWIO rows (K contiguous for fixed (kh, kw, c)).
//
// blockIdx -> tile mapping is XCD-aware: the 8 XCDs take workgroups round-robin, so the bijective
// remap below hands each XCD a contiguous run of logical tiles (the column tiles of a row block
// are adjacent), and the row block's activations are read into one L2 instead of eight.
#include <algorithm>
#include <array>
#include <cstdlib>
#include <map>
#include <mutex>

#include "kernels/conv.h"
#include "kernels/common.h"

namespace tdl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int kProMaxC = 512;  // input channels the input-side BN (Igemm::in_ss) stages in LDS
constexpr int LDS_ROW = BK;  // bf16 elements per LDS row (128 B, 16-B chunks XOR-swizzled by row)

// 16-B chunk c of tile row r lives at chunk c ^ swz(r): every 16-lane group of a ds_read_b128 fragment
// read (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... on gfx950) and every 8-lane group of a
// ds_write_b128 staging write then touches 16 (8) distinct 4-bank slots.
__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

struct Igemm {
  const uint16_t* x;  // NHWC image [N][H][W][C]
  const uint16_t* w;  // weight rows
  uint16_t* y;        // NHWC output [N][OH][OW][K] == row-major [M][K]
  int N, H, W, C;
  int OH, OW, K;
  int KH, KW, SH, SW, PT, PL;
  int flip;                 // 1: mirrored taps (input gradient)
  long long w_col, w_kh, w_kw;  // weight element strides: per output column, per tap row, per tap column
  int M;
  int scatter;  // 2: output row (n, oh, ow) goes to pixel (2oh, 2ow) of a [N][XH][XW][K] tensor whose
                // other three pixels of each 2x2 block are written as zeros (1x1 stride-2 input gradient)
  int XH, XW;
  const uint16_t* res;  // optional bf16 tensor shaped like y, added in the epilogue (gradient sums)
  float* stats;         // optional [M / BM row tiles][2][K]: per-tile channel sums of y and y^2 (the
                        // batch-norm statistics of the conv output, from the stored bf16 values)
  // optional batch-norm backward fusion (input gradient of a conv whose input is the output
  // relu(bn(x) + r) of a BN -> Add -> ReLU group): the stored gradient is dz = (dgrad + res) * [yb > 0]
  // and bn_part [row tiles][2][K] gets the per-tile channel sums of dz and dz * xb
  const uint16_t* bn_y;  // the conv's input (the group output), for the ReLU mask
  const uint16_t* bn_x;  // the group's BN input
  float* bn_part;
  // optional, with bn_part: the group's residual is the output of a plain BN (a projection
  // shortcut's) whose only reader is the group's Add, so that BN's output gradient is dz as well:
  // bn_part2 [row tiles][2][K] gets the per-tile channel sums of dz and dz * bn_x2 (its input)
  const uint16_t* bn_x2;
  float* bn_part2;
  // optional, with bn_part and no bn_y: the group is a plain BN -> ReLU, and the ReLU mask is
  // recomputed from bn_x as [bn_x * scale + shift > 0] (bn_ss = scale[K], shift[K] of its forward):
  // one tensor read less than loading the group output
  const float* bn_ss;
  // optional input-side BN -> ReLU (forward of a 1x1 stride-1 conv whose input is a plain BN -> ReLU
  // group's output): x is the group's BN INPUT, and the operand loader stores relu(x * scale + shift)
  // (in_ss = scale[C], shift[C]; the BN apply pass's f32 fma and bf16 rounding): the group output is
  // never written
  const float* in_ss;
};

// per-channel sums of 8 packed bf16 values v: s += v, q += v * w (w also 8 packed bf16)
__device__ __forceinline__ void accum_bf16x8(u32x4 v, u32x4 w, float* s, float* q) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float lo = __uint_as_float(v[j] << 16), hi = __uint_as_float(v[j] & 0xffff0000u);
    const float wl = __uint_as_float(w[j] << 16), wh = __uint_as_float(w[j] & 0xffff0000u);
    s[2 * j] += lo;
    q[2 * j] = fmaf(lo, wl, q[2 * j]);
    s[2 * j + 1] += hi;
    q[2 * j + 1] = fmaf(hi, wh, q[2 * j + 1]);
  }
}

// q += v * w for 8 packed bf16 values
__device__ __forceinline__ void dot_bf16x8(u32x4 v, u32x4 w, float* q) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    q[2 * j] = fmaf(__uint_as_float(v[j] << 16), __uint_as_float(w[j] << 16), q[2 * j]);
    q[2 * j + 1] = fmaf(__uint_as_float(v[j] & 0xffff0000u), __uint_as_float(w[j] & 0xffff0000u), q[2 * j + 1]);
  }
}

// v * [y > 0] for 8 packed bf16 (y > 0: sign clear and not +0)
__device__ __forceinline__ u32x4 relu_mask_bf16x8(u32x4 v, u32x4 y) {
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t lo = ((y[i] & 0x8000u) == 0u && (y[i] & 0x7fffu) != 0u) ? 0x0000ffffu : 0u;
    const uint32_t hi = ((y[i] & 0x80000000u) == 0u && (y[i] & 0x7fff0000u) != 0u) ? 0xffff0000u : 0u;
    o[i] = v[i] & (lo | hi);
  }
  return o;
}

// dz lanes where the recomputed group output relu(x * scale + shift) is zero: x 8 packed bf16 of the
// BN input, the same f32 fma as the BN apply pass
__device__ __forceinline__ u32x4 relu_mask_affine_bf16x8(u32x4 v, u32x4 x, const float* sc, const float* sh) {
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = __uint_as_float(x[k] << 16), hi = __uint_as_float(x[k] & 0xffff0000u);
    const uint32_t mlo = fmaf(lo, sc[2 * k], sh[2 * k]) > 0.f ? 0x0000ffffu : 0u;
    const uint32_t mhi = fmaf(hi, sc[2 * k + 1], sh[2 * k + 1]) > 0.f ? 0xffff0000u : 0u;
    o[k] = v[k] & (mlo | mhi);
  }
  return o;
}

// relu(x * sc + sh) for 8 packed bf16 x (the BN apply pass's f32 fma, round to nearest even)
// (v_cvt_pk_bf16_f32 packing: round to nearest even, as the apply pass)
__device__ __forceinline__ u32x4 bn_relu_bf16x8(u32x4 x, f4v sc0, f4v sc1, f4v sh0, f4v sh1) {
  const float sc[8] = {sc0[0], sc0[1], sc0[2], sc0[3], sc1[0], sc1[1], sc1[2], sc1[3]};
  const float sh[8] = {sh0[0], sh0[1], sh0[2], sh0[3], sh1[0], sh1[1], sh1[2], sh1[3]};
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float lo = fmaxf(fmaf(__uint_as_float(x[k] << 16), sc[2 * k], sh[2 * k]), 0.f);
    const float hi = fmaxf(fmaf(__uint_as_float(x[k] & 0xffff0000u), sc[2 * k + 1], sh[2 * k + 1]), 0.f);
    o[k] = pack_bf16x2(lo, hi);
  }
  return o;
}

// a + b for 8 packed bf16 values (f32 add, round to nearest even; HW: v_cvt_pk_bf16_f32, the same bits)
template <bool HW = false>
__device__ __forceinline__ u32x4 add_bf16x8(u32x4 a, u32x4 b) {
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float lo = __uint_as_float(a[i] << 16) + __uint_as_float(b[i] << 16);
    const float hi = __uint_as_float(a[i] & 0xffff0000u) + __uint_as_float(b[i] & 0xffff0000u);
    if constexpr (HW) {
      o[i] = pack_bf16x2(lo, hi);
    } else {
      uint32_t ul = __float_as_uint(lo), uh = __float_as_uint(hi);
      ul += 0x7fffu + ((ul >> 16) & 1u);
      uh += 0x7fffu + ((uh >> 16) & 1u);
      o[i] = (ul >> 16) | (uh & 0xffff0000u);
    }
  }
  return o;
}

// output row m -> (n, oh, ow).  m < 2^24 (every ResNet-50 shape up to b = 5000): one f32 multiply by
// the reciprocal and a +-1 fix-up per quotient (exact: the product's error is < 2 / d), instead of the
// ~30-instruction integer division sequences on the prologue's critical path (the row offsets gate the
// first operand loads)
__device__ __forceinline__ int fdiv_exact(int n, int d, float inv, int& rem) {
  int q = (int)((float)n * inv);
  int r = n - q * d;
  if (r < 0) {
    --q;
    r += d;
  } else if (r >= d) {
    ++q;
    r -= d;
  }
  rem = r;
  return q;
}

__device__ __forceinline__ void split_row(const Igemm& a, int m, float inv_ow, float inv_oh, int& n, int& oh,
                                          int& ow) {
  if (a.M < (1 << 24)) {
    const int t = fdiv_exact(m, a.OW, inv_ow, ow);
    n = fdiv_exact(t, a.OH, inv_oh, oh);
  } else {
    ow = m % a.OW;
    const int t = m / a.OW;
    oh = t % a.OH;
    n = t / a.OH;
  }
}

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even (activations are finite)
  return (uint16_t)(u >> 16);
}

// Epilogue shared by the conv kernels: the f32 accumulators (wave tile WTM x WTN at (wrow0, wcol0) of
// the BM x BN workgroup tile, acc[i][j] = 16x16 subtile, lane = 4 adjacent channels of one pixel) are
// rounded to bf16 into LDS ([BM][BN + 8], the operand LDS is free by now), then written back as 16-byte
// row segments with the variant's fused operations (residual, BN statistics / BN-group backward sums,
// stride-2 scatter).  Every thread of the workgroup must call it (it has workgroup barriers).
// LOWREG (the 4-waves-per-SIMD variants, <= 128 VGPRs): the BN-group backward epilogue loads its
// residual and BN operands in chunks of EPI / 4 segments right before their use instead of all up front.
// EK 3: the BN-group backward of EK 1 with the ReLU mask recomputed from the BN input (bn_ss).
// MF 32: the accumulators are 32x32 blocks of v_mfma_f32_32x32x16_bf16 (ACC = f16v[WTM / 32][WTN / 32]):
// lane l holds channels 8k + 4 (l >> 5) + r (k, r < 4) of pixel l & 31 -- four 8-B LDS writes per block
template <int BM, int BN, int NT, int EK, int WTM, int WTN, int LDS_ELEMS, int LOWREG = 0, int MF = 16, typename ACC>
__device__ __forceinline__ void conv_epilogue(const Igemm& a, const ACC& acc, uint16_t* lds,
                                              int tm, int tn, int wrow0, int wcol0) {
  const int tid = threadIdx.x, lane = tid & 63;
  constexpr int OUT_LD = BN + 8;
  constexpr int SEG = BN / 8;              // 16-B segments per row
  constexpr int EPI = BM * SEG / NT;       // segments per thread
  static_assert(BM * SEG % NT == 0, "epilogue segments must divide evenly");
  // residual (gradient sum): all of this thread's loads issued here, before the LDS round trip, so
  // their latency overlaps it instead of serialising the store loop
  // segments per operand chunk (LOWREG 1: the BN-group backward epilogue only, 2: every epilogue)
  constexpr bool BNB = EK == 1 || EK == 3;  // fused BN-group backward
  constexpr int EC = ((LOWREG == 1 && BNB) || (LOWREG == 2 && EK != 2)) ? (EPI >= 4 ? EPI / 4 : 1) : EPI;
  u32x4 rv[EK == 2 ? 1 : EPI];
  if (EK != 2 && a.res && EC == EPI) {
#pragma unroll
    for (int e = 0; e < EPI; ++e) {
      const int s = tid + e * NT, row = s / SEG, seg = s % SEG, m = tm * BM + row;
      rv[e] = m < a.M ? *reinterpret_cast<const u32x4*>(a.res + (long long)m * a.K + tn * BN + seg * 8)
                      : u32x4{0u, 0u, 0u, 0u};
    }
  }
  static_assert(BM * OUT_LD <= LDS_ELEMS, "epilogue tile must fit the operand LDS");
  // (operands are swapped in the MFMA, so a lane holds 4 consecutive channels of one pixel: one 8-B write)
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < WTM / 16; ++i)
#pragma unroll
      for (int j = 0; j < WTN / 16; ++j) {
        // (hardware packing where it does not raise the VGPR peak: the EK 1 / 2 variants spill with it)
        const uint32_t lo = (EK == 1 || EK == 2) ? (f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16))
                                                 : pack_bf16x2(acc[i][j][0], acc[i][j][1]);
        const uint32_t hi = (EK == 1 || EK == 2) ? (f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16))
                                                 : pack_bf16x2(acc[i][j][2], acc[i][j][3]);
        *reinterpret_cast<uint2*>(lds + (wrow0 + i * 16 + (lane & 15)) * OUT_LD + wcol0 + j * 16 + (lane >> 4) * 4) =
            make_uint2(lo, hi);
      }
  } else {
#pragma unroll
    for (int i = 0; i < WTM / 32; ++i)
#pragma unroll
      for (int j = 0; j < WTN / 32; ++j)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t lo = (EK == 1 || EK == 2) ? (f2bf(acc[i][j][4 * k]) | ((uint32_t)f2bf(acc[i][j][4 * k + 1]) << 16))
                                                   : pack_bf16x2(acc[i][j][4 * k], acc[i][j][4 * k + 1]);
          const uint32_t hi = (EK == 1 || EK == 2)
                                  ? (f2bf(acc[i][j][4 * k + 2]) | ((uint32_t)f2bf(acc[i][j][4 * k + 3]) << 16))
                                  : pack_bf16x2(acc[i][j][4 * k + 2], acc[i][j][4 * k + 3]);
          *reinterpret_cast<uint2*>(lds + (wrow0 + i * 32 + (lane & 31)) * OUT_LD + wcol0 + j * 32 + 8 * k +
                                    (lane >> 5) * 4) = make_uint2(lo, hi);
        }
  }
  // BN-backward fusion operands (the accumulators are dead now: registers to spare)
  constexpr int BNE = BNB ? EPI : 1;
  u32x4 ry[EK == 1 ? EPI : 1], rx[BNE], rx2[BNE];
  // EK 3: this thread's 8 channels (one segment column for all its rows) of the mask's scale / shift
  float msc[EK == 3 ? 8 : 1], msh[EK == 3 ? 8 : 1];
  if constexpr (EK == 3) {
    const int c0 = tn * BN + (tid % SEG) * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      msc[j] = a.bn_ss[c0 + j];
      msh[j] = a.bn_ss[a.K + c0 + j];
    }
  }
  // the BN-group operands of segments [e0, e0 + EC) (all of them up front unless LOWREG)
  auto load_bn = [&](int e0) {
    if constexpr (BNB) {
#pragma unroll
      for (int e = e0; e < e0 + EC; ++e) {
        const int s = tid + e * NT, row = s / SEG, seg = s % SEG, m = tm * BM + row;
        const long long o = (long long)m * a.K + tn * BN + seg * 8;
        const bool in = m < a.M;
        if constexpr (EK == 1) ry[e] = in ? *reinterpret_cast<const u32x4*>(a.bn_y + o) : u32x4{0u, 0u, 0u, 0u};
        rx[e] = in ? *reinterpret_cast<const u32x4*>(a.bn_x + o) : u32x4{0u, 0u, 0u, 0u};
        rx2[e] = (in && a.bn_x2) ? *reinterpret_cast<const u32x4*>(a.bn_x2 + o) : u32x4{0u, 0u, 0u, 0u};
        if (EC != EPI && a.res)
          rv[e] = in ? *reinterpret_cast<const u32x4*>(a.res + o) : u32x4{0u, 0u, 0u, 0u};
      }
    } else if (EC != EPI && EK == 0) {
      if (a.res) {
#pragma unroll
        for (int e = e0; e < e0 + EC; ++e) {
          const int s = tid + e * NT, row = s / SEG, seg = s % SEG, m = tm * BM + row;
          rv[e] = m < a.M ? *reinterpret_cast<const u32x4*>(a.res + (long long)m * a.K + tn * BN + seg * 8)
                          : u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  };
  if (EC == EPI) load_bn(0);
  __syncthreads();
  static_assert(NT % SEG == 0, "a thread keeps one 8-channel segment across its rows");
  // per-tile channel sums: (y, y^2) of the forward output, or (dz, dz * xb) [and dz * xb2] of a fused
  // BN group backward
  float* sums = a.stats ? a.stats : (EK != 0 ? a.bn_part : nullptr);
  float* sums2 = (EK != 0 && a.bn_part) ? a.bn_part2 : nullptr;
  float cs[8], cq[8], cq2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = cq[j] = cq2[j] = 0.f;
  if constexpr (EK != 2) {
#pragma unroll
    for (int e = 0; e < EPI; ++e) {
      if (EC != EPI && e % EC == 0) load_bn(e);
      const int s = tid + e * NT, row = s / SEG, seg = s % SEG;
      const int m = tm * BM + row;
      if (m < a.M) {
        const long long o = (long long)m * a.K + tn * BN + seg * 8;
        u32x4 v = *reinterpret_cast<const u32x4*>(lds + row * OUT_LD + seg * 8);
        if (a.res) v = add_bf16x8<EK == 0 || EK == 3>(v, rv[e]);
        if constexpr (EK == 1) v = relu_mask_bf16x8(v, ry[e]);
        if constexpr (EK == 3) v = relu_mask_affine_bf16x8(v, rx[e], msc, msh);
        *reinterpret_cast<u32x4*>(a.y + o) = v;
        if (sums) accum_bf16x8(v, BNB ? rx[e] : v, cs, cq);
        if constexpr (BNB)
          if (sums2) dot_bf16x8(v, rx2[e], cq2);
      }
    }
  } else {
    for (int s = tid; s < BM * SEG; s += NT) {
      const int row = s / SEG, seg = s % SEG;
      const int m = tm * BM + row;
      if (m >= a.M) continue;
      const int ow = m % a.OW, t = m / a.OW, oh = t % a.OH, n = t / a.OH;
      const int h = 2 * oh, w = 2 * ow;
      const long long off = (((long long)n * a.XH + h) * a.XW + w) * a.K + tn * BN + seg * 8;
      const long long rs = (long long)a.XW * a.K;
      const bool w1 = w + 1 < a.XW, h1 = h + 1 < a.XH;
      // the 2x2 block of dx pixels this output row owns: (2oh, 2ow) gets the computed gradient, the
      // other three only the other contribution (or zeros)
      const bool ok[4] = {true, w1, h1, w1 && h1};
      const long long po[4] = {off, off + a.K, off + rs, off + rs + a.K};
      const u32x4 z{0u, 0u, 0u, 0u};
      u32x4 p[4];
      // every load of the block issued before any math
#pragma unroll
      for (int q = 0; q < 4; ++q) p[q] = (a.res && ok[q]) ? *reinterpret_cast<const u32x4*>(a.res + po[q]) : z;
      u32x4 by[4], bx[4], bx2[4];
      if (a.bn_part) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          by[q] = (ok[q] && a.bn_y) ? *reinterpret_cast<const u32x4*>(a.bn_y + po[q]) : z;
          bx[q] = ok[q] ? *reinterpret_cast<const u32x4*>(a.bn_x + po[q]) : z;
          bx2[q] = (ok[q] && a.bn_x2) ? *reinterpret_cast<const u32x4*>(a.bn_x2 + po[q]) : z;
        }
      }
      const u32x4 v = *reinterpret_cast<const u32x4*>(lds + row * OUT_LD + seg * 8);
      p[0] = a.res ? add_bf16x8(v, p[0]) : v;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!ok[q]) continue;
        if (a.bn_part) {
          if (a.bn_ss) {
            const int c0 = tn * BN + seg * 8;
            float sc[8], sh[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              sc[j] = a.bn_ss[c0 + j];
              sh[j] = a.bn_ss[a.K + c0 + j];
            }
            p[q] = relu_mask_affine_bf16x8(p[q], bx[q], sc, sh);
          } else {
            p[q] = relu_mask_bf16x8(p[q], by[q]);
          }
          accum_bf16x8(p[q], bx[q], cs, cq);
          if (sums2) dot_bf16x8(p[q], bx2[q], cq2);
        }
        *reinterpret_cast<u32x4*>(a.y + po[q]) = p[q];
      }
    }
  }
  if (sums) {
    // fixed-order reduction over the NT / SEG threads of each segment, through the (now free) LDS
    constexpr int TPS = NT / SEG;  // threads per segment
    static_assert(3 * TPS * BN * 4 <= LDS_ELEMS * 2, "stats scratch must fit the operand LDS");
    
    __syncthreads();  // every thread has read its tile rows
    float* red = reinterpret_cast<float*>(lds);
    const int seg = tid % SEG, grp = tid / SEG;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[grp * BN + seg * 8 + j] = cs[j];
      red[TPS * BN + grp * BN + seg * 8 + j] = cq[j];
      if (sums2) red[2 * TPS * BN + grp * BN + seg * 8 + j] = cq2[j];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float S = 0.f, Q = 0.f, Q2 = 0.f;
      for (int g2 = 0; g2 < TPS; ++g2) {
        S += red[g2 * BN + c];
        Q += red[TPS * BN + g2 * BN + c];
        if (sums2) Q2 += red[2 * TPS * BN + g2 * BN + c];
      }
      sums[((long long)tm * 2) * a.K + tn * BN + c] = S;
      sums[((long long)tm * 2 + 1) * a.K + tn * BN + c] = Q;
      if (sums2) {
        sums2[((long long)tm * 2) * a.K + tn * BN + c] = S;
        sums2[((long long)tm * 2 + 1) * a.K + tn * BN + c] = Q2;
      }
    }
  }
}

// EK selects the epilogue a variant carries (registers: the VGPR peak of the heaviest epilogue sets the
// occupancy of the whole kernel, so the plain variant must not pay for the fused ones): 0 plain
// (+ residual, + BN statistics), 1 fused BN-group backward, 2 stride-2 scatter (+ residual, + BN group)
// DEPTH 0 (the default, see launch_tile): one LDS stage, no prefetch, 4 waves per SIMD (four 128x128
// workgroups per CU instead of two: <= 128 VGPRs, 37 KB LDS each); the resident workgroups hide each
// other's load latency and epilogues.
// DEPTH 3: one LDS stage with one tile of register prefetch, 3 waves per SIMD (<= 168 VGPRs; plain
// and scatter epilogues): the next tile's loads fly during this tile's MFMAs, and three workgroups
// per CU instead of the two that double-buffered LDS allows.
template <int BM, int BN, int DEPTH>
constexpr int v1_lds_elems() {
  return (DEPTH == 0 || DEPTH == 3) ? ((BM + BN) * LDS_ROW > BM * (BN + 8) ? (BM + BN) * LDS_ROW : BM * (BN + 8))
                                    : 2 * (BM + BN) * LDS_ROW;
}

// PRO: the input-side BN -> ReLU (Igemm::in_ss) in the operand loader (DEPTH 0, plain epilogue)
template <int BM, int BN, int DEPTH, int EK, bool PRO = false>
__global__ __launch_bounds__(BM * 2, DEPTH == 0 ? 4 : (DEPTH == 3 ? 3 : 2)) void k_conv_igemm(Igemm a) {
  static_assert(!PRO || (DEPTH == 0 && EK == 0), "input-side BN: single-stage plain variant");
  // input-side BN: scale / shift of every input channel staged in LDS once (C <= kProMaxC), read per
  // tile at LDS latency instead of a dependent global round trip after each tile's operand loads
  __shared__ __attribute__((aligned(16))) float lds_ss[PRO ? 2 * kProMaxC : 1];
  constexpr int NT = BM * 2;         // threads: (BM / 64) x 2 waves, each 64 x BN/2
  constexpr int RP = NT / 8;         // tile rows per staging pass (8 x 16-B chunks per 128-B row)
  constexpr int WN = BN / 2;         // columns per wave
  constexpr int NS = WN / 16;        // 16-wide column subtiles per wave
  constexpr int A_LD = BM * BK / 8 / NT;  // 16-B A chunks per thread per tile (4)
  constexpr int B_LD = BN * BK / 8 / NT;  // 16-B B chunks per thread per tile
  __shared__ __attribute__((aligned(16))) uint16_t lds[v1_lds_elems<BM, BN, DEPTH>()];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // XCD-aware bijective remap of the 1-D grid
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntn = a.K / BN;
  const int tn = wg % ntn, tm = wg / ntn;

  // Operands are read with raw buffer loads: byte voffset per thread (fixed for the whole k loop),
  // wave-uniform soffset per k-tile, and the buffer's range check supplies the zeros of padding
  // taps (voffset 0x80000000 is past any tensor this kernel takes: conv_bf16_supported keeps both
  // under 2 GiB).  The image resource starts `bias` elements before x, so that every in-image
  // offset (kh, kw >= 0 added to a row's top-left tap, which may lie in the padding) is >= 0.
  // per-thread A rows: chunk j = tid + 256 i -> row j >> 3, 16-B column j & 7
  const int col8 = (tid & 7) * 8;
  const long long bias = ((long long)a.PT * a.W + a.PL) * a.C;
  const auto x_rsrc = buf_rsrc(a.x - bias, (unsigned)(((long long)a.N * a.H * a.W * a.C + bias) * 2));
  const auto w_rsrc = buf_rsrc(a.w, (unsigned)((long long)a.KH * a.KW * a.C * a.K * 2));
  int a_vo[A_LD];
  uint32_t a_tap[A_LD];  // bit (kh * KW + kw): that tap of this row lies inside the image
  // 1x1 stride 1 unpadded (same image and output grid): output row m reads image pixel m
  const bool direct = a.KH == 1 && a.KW == 1 && a.SH == 1 && a.SW == 1 && a.PT == 0 && a.PL == 0 && a.H == a.OH &&
                      a.W == a.OW;
  const float inv_ow = 1.0f / (float)a.OW, inv_oh = 1.0f / (float)a.OH;
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int m = tm * BM + (tid >> 3) + RP * i;
    a_tap[i] = 0u;
    a_vo[i] = 0;
    if (m < a.M && direct) {
      a_vo[i] = (int)(((long long)m * a.C + col8) * 2);
      a_tap[i] = 1u;
    } else if (m < a.M) {
      int n, oh, ow;
      split_row(a, m, inv_ow, inv_oh, n, oh, ow);
      const int ih = oh * a.SH - a.PT, iw = ow * a.SW - a.PL;
      a_vo[i] = (int)(((((long long)n * a.H + ih) * a.W + iw) * a.C + col8 + bias) * 2);
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih + kh) < (unsigned)a.H && (unsigned)(iw + kw) < (unsigned)a.W) a_tap[i] |= 1u << (kh * a.KW + kw);
    }
  }
  int b_vo[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) b_vo[i] = (int)(((long long)(tn * BN + (tid >> 3) + RP * i) * a.w_col + col8) * 2);

  // register staging sets: DEPTH 2 keeps two tiles of global loads in flight (tile t+2 is issued
  // while tile t computes and tile t+1's registers are written to LDS), DEPTH 1 one tile
  u32x4 ra[2][A_LD], rb[2][B_LD];
  const int ctiles = a.C / BK;
  const int ntiles = a.KH * a.KW * ctiles;

  // reduction position of the next tile to load (advanced incrementally: no per-tile div/mod)
  int n_c = 0, n_kw = 0, n_kh = 0;
  int ld_c0 = 0;  // channel base of the last loaded tile (input-side BN)
  auto gload = [&](u32x4* pa, u32x4* pb) {
    const int c0 = n_c * BK, kw = n_kw, kh = n_kh;
    ld_c0 = c0;
    if (++n_c == ctiles) {
      n_c = 0;
      if (++n_kw == a.KW) {
        n_kw = 0;
        ++n_kh;
      }
    }
    const int tap = kh * a.KW + kw;
    const int soff_a = (int)((((long long)kh * a.W + kw) * a.C + c0) * 2);
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int vo = ((a_tap[i] >> tap) & 1u) ? a_vo[i] : (int)0x80000000;
      pa[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(x_rsrc, vo, soff_a, 0));
    }
    const int wkh = a.flip ? a.KH - 1 - kh : kh, wkw = a.flip ? a.KW - 1 - kw : kw;
    const int soff_b = (int)((wkh * a.w_kh + wkw * a.w_kw + c0) * 2);
#pragma unroll
    for (int i = 0; i < B_LD; ++i)
      pb[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(w_rsrc, b_vo[i], soff_b, 0));
  };
  const int scol = ((tid & 7) ^ swz(tid >> 3)) * 8;  // swizzled LDS column of this thread's chunk (RP % 16 == 0)
  auto sstore = [&](int buf, const u32x4* pa, const u32x4* pb) {
    uint16_t* la = lds + buf * (BM + BN) * LDS_ROW;
    uint16_t* lb = la + BM * LDS_ROW;
    if constexpr (PRO) {
      // B first: its staging registers die before the scale / shift ones are loaded
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        *reinterpret_cast<u32x4*>(lb + ((tid >> 3) + RP * i) * LDS_ROW + scol) = pb[i];
      // every chunk of this thread holds channels ld_c0 + col8 .. + 7 (1x1 stride 1: no padding taps;
      // rows past M are transformed too and their outputs never stored)
      const f4v* ss = reinterpret_cast<const f4v*>(lds_ss + ld_c0 + col8);
      const f4v sc0 = ss[0], sc1 = ss[1], sh0 = ss[a.C / 4], sh1 = ss[a.C / 4 + 1];
#pragma unroll
      for (int i = 0; i < A_LD; ++i)
        *reinterpret_cast<u32x4*>(la + ((tid >> 3) + RP * i) * LDS_ROW + scol) = bn_relu_bf16x8(pa[i], sc0, sc1, sh0, sh1);
    } else {
#pragma unroll
      for (int i = 0; i < A_LD; ++i)
        *reinterpret_cast<u32x4*>(la + ((tid >> 3) + RP * i) * LDS_ROW + scol) = pa[i];
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        *reinterpret_cast<u32x4*>(lb + ((tid >> 3) + RP * i) * LDS_ROW + scol) = pb[i];
    }
  };

  f4v acc[4][NS];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NS; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  const int frow = lane & 15;
  const int fk0 = (((lane >> 4)) ^ swz(frow)) * 8, fk1 = (((lane >> 4) | 4) ^ swz(frow)) * 8;  // k 0-31, 32-63
  auto compute = [&](int buf) {
    const uint16_t* la = lds + buf * (BM + BN) * LDS_ROW + (wm * 64 + frow) * LDS_ROW;
    const uint16_t* lb = lds + buf * (BM + BN) * LDS_ROW + BM * LDS_ROW + (wn * WN + frow) * LDS_ROW;
#pragma unroll
    for (int kk = 0; kk < BK; kk += 32) {
      const int fk = kk ? fk1 : fk0;
      bf16x8 fa[4], fb[NS];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(la + i * 16 * LDS_ROW + fk);
#pragma unroll
      for (int j = 0; j < NS; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(lb + j * 16 * LDS_ROW + fk);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NS; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
    }
  };

  if (DEPTH == 0) {
    for (int t = 0; t < ntiles; ++t) {
      gload(ra[0], rb[0]);
      if constexpr (PRO) {
        if (t == 0) {  // stage scale / shift while the first tile's operand loads fly
          for (int i = tid * 4; i < 2 * a.C; i += NT * 4)
            *reinterpret_cast<f4v*>(lds_ss + i) = *reinterpret_cast<const f4v*>(a.in_ss + i);
        }
      }
      if (PRO || t) __syncthreads();  // every wave done reading the previous tile (PRO: lds_ss written)
      sstore(0, ra[0], rb[0]);
      __syncthreads();
      compute(0);
    }
    __syncthreads();  // the epilogue reuses the operand LDS
  } else if (DEPTH == 3) {
    gload(ra[0], rb[0]);
    for (int t = 0; t < ntiles; ++t) {
      if (t) __syncthreads();  // every wave done reading tile t - 1
      sstore(0, ra[0], rb[0]);
      __syncthreads();
      if (t + 1 < ntiles) gload(ra[0], rb[0]);  // in flight during this tile's MFMAs
      compute(0);
    }
    __syncthreads();
  } else if (DEPTH == 1) {
    gload(ra[0], rb[0]);
    sstore(0, ra[0], rb[0]);
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
      const int buf = t & 1;
      if (t + 1 < ntiles) gload(ra[0], rb[0]);
      compute(buf);
      if (t + 1 < ntiles) sstore(buf ^ 1, ra[0], rb[0]);
      __syncthreads();
    }
  } else {
    gload(ra[0], rb[0]);
    if (ntiles > 1) gload(ra[1], rb[1]);
    sstore(0, ra[0], rb[0]);
    __syncthreads();
    for (int t = 0; t < ntiles; t += 2) {
      // even tile t in LDS buffer 0; set 0 is free, set 1 holds tile t + 1
      if (t + 2 < ntiles) gload(ra[0], rb[0]);
      compute(0);
      if (t + 1 < ntiles) sstore(1, ra[1], rb[1]);
      __syncthreads();
      if (t + 1 >= ntiles) break;
      // odd tile t + 1 in LDS buffer 1; set 1 is free, set 0 holds tile t + 2
      if (t + 3 < ntiles) gload(ra[1], rb[1]);
      compute(1);
      if (t + 2 < ntiles) sstore(0, ra[0], rb[0]);
      __syncthreads();
    }
  }

  // epilogue: bf16 tile into LDS ([BM][BN + 8]), then 16-B row segments to global
  conv_epilogue<BM, BN, NT, EK, 64, WN, v1_lds_elems<BM, BN, DEPTH>(), DEPTH == 0 ? 1 : 0>(a, acc, lds, tm, tn,
                                                                                         wm * 64, wn * WN);
}

// ---------------------------------------------------------------------------------------------
// v2 main loop: 8 waves (512 threads), BM x BN x 64 tiles, a 3-stage LDS ring filled by LDS-DMA
// (buffer_load_dwordx4 ... lds: no register staging, no ds_write pass), tile t+2's loads in flight
// while tile t computes, ONE raw barrier per k-tile (counted vmcnt, never 0 in the loop).  The
// LDS image is the v1 one (128-B rows, 16-B chunks XOR-swizzled by row): an LDS-DMA writes 64 lanes x
// 16 B linearly, so the swizzle goes on the SOURCE address -- lane L of a wave-instruction covering
// rows 8g .. 8g+7 writes slot L % 8 of row 8g + L / 8 and therefore fetches chunk (L % 8) ^ swz(row)
// (cdna_hip_programming.md rule 21).  Out-of-image taps read voffset 0x80000000: the buffer's
// range check lands zeros in LDS, exactly as the v1 loader's register zeros.
template <int N>
__device__ __forceinline__ void wait_vmcnt_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// STAGES 1 (the "dma1" variant): 4 waves, one LDS stage, no prefetch, 4 waves per SIMD -- the v1
// DEPTH 0 schedule with the operands landing in LDS by DMA instead of registers + ds_write_b128.
template <int BM, int BN, int STAGES>
constexpr int v2_lds_elems() {
  return STAGES * (BM + BN) * LDS_ROW > BM * (BN + 8) ? STAGES * (BM + BN) * LDS_ROW : BM * (BN + 8);
}

typedef float f16v __attribute__((ext_vector_type(16)));

// MF 32: the same main loop on v_mfma_f32_32x32x16_bf16 (2 x 2 blocks of 32 x 32 per 64 x 64 wave tile,
// four 16-deep k-steps per 64-deep tile; the same LDS bytes per MFMA FLOP as the 16x16x32 form)
template <int BM, int BN, int WGM, int WGN, int EK, int STAGES, int MINW, int MF = 16>
__global__ __launch_bounds__(64 * WGM * WGN, MINW) void k_conv_glds(Igemm a) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;  // wave tile
  constexpr int MI = WTM / 16, NJ = WTN / 16;
  constexpr int STAGE = (BM + BN) * LDS_ROW;      // bf16 elements per ring stage
  constexpr int A_LD = BM / (8 * NW);             // LDS-DMA wave-instructions (8 rows each) per thread, A
  constexpr int B_LD = BN / (8 * NW);             //                                              ..., B
  static_assert((STAGES == 3 || STAGES == 1) && BM % (8 * NW) == 0 && BN % (8 * NW) == 0 && MI >= 1 && NJ >= 1,
                "v2 geometry");
  __shared__ __attribute__((aligned(16))) uint16_t lds[v2_lds_elems<BM, BN, STAGES>()];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntn = a.K / BN;
  const int tn = wg % ntn, tm = wg / ntn;

  const long long bias = ((long long)a.PT * a.W + a.PL) * a.C;
  const auto x_rsrc = buf_rsrc(a.x - bias, (unsigned)(((long long)a.N * a.H * a.W * a.C + bias) * 2));
  const auto w_rsrc = buf_rsrc(a.w, (unsigned)((long long)a.KH * a.KW * a.C * a.K * 2));
  // this lane's row inside each of its row groups, and the (source-swizzled) chunk it fetches
  const int lrow = lane >> 3;
  int a_vo[A_LD];
  uint32_t a_tap[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int row = (i * NW + wave) * 8 + lrow;  // row group i*NW + wave
    const int chunk = (lane & 7) ^ swz(row);
    const int m = tm * BM + row;
    a_tap[i] = 0u;
    a_vo[i] = 0;
    if (m < a.M) {  // (integer division: the reciprocal form of split_row raises this kernel's prologue spills)
      const int ow = m % a.OW, t = m / a.OW, oh = t % a.OH, n = t / a.OH;
      const int ih = oh * a.SH - a.PT, iw = ow * a.SW - a.PL;
      a_vo[i] = (int)(((((long long)n * a.H + ih) * a.W + iw) * a.C + chunk * 8 + bias) * 2);
      for (int kh = 0; kh < a.KH; ++kh)
        for (int kw = 0; kw < a.KW; ++kw)
          if ((unsigned)(ih + kh) < (unsigned)a.H && (unsigned)(iw + kw) < (unsigned)a.W) a_tap[i] |= 1u << (kh * a.KW + kw);
    }
  }
  int b_vo[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int row = (i * NW + wave) * 8 + lrow;
    const int chunk = (lane & 7) ^ swz(row);
    b_vo[i] = (int)(((long long)(tn * BN + row) * a.w_col + chunk * 8) * 2);
  }

  const int ctiles = a.C / BK;
  const int ntiles = a.KH * a.KW * ctiles;
  int n_c = 0, n_kw = 0, n_kh = 0;
  auto issue = [&](int stage) {
    const int c0 = n_c * BK, kw = n_kw, kh = n_kh;
    if (++n_c == ctiles) {
      n_c = 0;
      if (++n_kw == a.KW) {
        n_kw = 0;
        ++n_kh;
      }
    }
    const int tap = kh * a.KW + kw;
    const int soff_a = (int)((((long long)kh * a.W + kw) * a.C + c0) * 2);
    uint16_t* base = lds + stage * STAGE;
#pragma unroll
    for (int i = 0; i < A_LD; ++i) {
      const int vo = ((a_tap[i] >> tap) & 1u) ? a_vo[i] : (int)0x80000000;
      lds_dma16(x_rsrc, base + (i * NW + wave) * 8 * LDS_ROW, vo, soff_a);
    }
    const int wkh = a.flip ? a.KH - 1 - kh : kh, wkw = a.flip ? a.KW - 1 - kw : kw;
    const int soff_b = (int)((wkh * a.w_kh + wkw * a.w_kw + c0) * 2);
#pragma unroll
    for (int i = 0; i < B_LD; ++i)
      lds_dma16(w_rsrc, base + (BM + (i * NW + wave) * 8) * LDS_ROW, b_vo[i], soff_b);
  };

  constexpr int MI32 = WTM / 32, NJ32 = WTN / 32;
  static_assert(MF == 16 || (WTM % 32 == 0 && WTN % 32 == 0), "32x32 blocks need 32-multiple wave tiles");
  f4v acc[MF == 16 ? MI : 1][MF == 16 ? NJ : 1];
  f16v acc32[MF == 32 ? MI32 : 1][MF == 32 ? NJ32 : 1];
  if constexpr (MF == 16) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
  } else {
#pragma unroll
    for (int i = 0; i < MI32; ++i)
#pragma unroll
      for (int j = 0; j < NJ32; ++j)
#pragma unroll
        for (int q = 0; q < 16; ++q) acc32[i][j][q] = 0.f;
  }

  const int frow = lane & 15;
  const int fk0 = ((lane >> 4) ^ swz(frow)) * 8, fk1 = (((lane >> 4) | 4) ^ swz(frow)) * 8;
  // 32x32x16: lane l reads row l & 31, 16-B chunk 2 step + (l >> 5) of the 64-deep tile (swizzled by row;
  // swz is the same for rows r and r + 16 m)
  const int frow32 = lane & 31;
  auto compute = [&](int stage) {
    if constexpr (MF == 16) {
      const uint16_t* la = lds + stage * STAGE + (wm * WTM + frow) * LDS_ROW;
      const uint16_t* lb = lds + stage * STAGE + (BM + wn * WTN + frow) * LDS_ROW;
#pragma unroll
      for (int kk = 0; kk < BK; kk += 32) {
        const int fk = kk ? fk1 : fk0;
        bf16x8 fa[MI], fb[NJ];
#pragma unroll
        for (int i = 0; i < MI; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(la + i * 16 * LDS_ROW + fk);
#pragma unroll
        for (int j = 0; j < NJ; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(lb + j * 16 * LDS_ROW + fk);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[i][j], 0, 0, 0);
      }
    } else {
      const uint16_t* la = lds + stage * STAGE + (wm * WTM + frow32) * LDS_ROW;
      const uint16_t* lb = lds + stage * STAGE + (BM + wn * WTN + frow32) * LDS_ROW;
#pragma unroll
      for (int st = 0; st < BK / 16; ++st) {
        const int fk = ((2 * st + (lane >> 5)) ^ swz(frow32)) * 8;
        bf16x8 fa[MI32], fb[NJ32];
#pragma unroll
        for (int i = 0; i < MI32; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(la + i * 32 * LDS_ROW + fk);
#pragma unroll
        for (int j = 0; j < NJ32; ++j) fb[j] = *reinterpret_cast<const bf16x8*>(lb + j * 32 * LDS_ROW + fk);
#pragma unroll
        for (int i = 0; i < MI32; ++i)
#pragma unroll
          for (int j = 0; j < NJ32; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j], fa[i], acc32[i][j], 0, 0, 0);
      }
    }
  };

  if constexpr (STAGES == 1) {
    for (int t = 0; t < ntiles; ++t) {
      if (t) __syncthreads();  // every wave done reading tile t - 1
      issue(0);
      wait_vmcnt_barrier<0>();  // tile t landed, for every wave
      compute(0);
    }
  } else {
    issue(0);
    if (ntiles > 1) issue(1);
    int st = 0;
    for (int t = 0; t < ntiles; ++t) {
      // tile t landed (this thread's loads: all but tile t+1's), every wave past tile t-1's reads
      if (t + 1 < ntiles)
        wait_vmcnt_barrier<A_LD + B_LD>();
      else
        wait_vmcnt_barrier<0>();
      if (t + 2 < ntiles) issue(st == 0 ? 2 : st - 1);  // stage (t + 2) % 3 == stage (t - 1) % 3
      compute(st);
      st = st == 2 ? 0 : st + 1;
    }
  }
  __syncthreads();  // every wave done reading the ring: the epilogue reuses it
  if constexpr (MF == 16)
    conv_epilogue<BM, BN, NT, EK, WTM, WTN, v2_lds_elems<BM, BN, STAGES>(), STAGES == 1 ? 2 : 0>(a, acc, lds, tm, tn,
                                                                                               wm * WTM, wn * WTN);
  else
    conv_epilogue<BM, BN, NT, EK, WTM, WTN, v2_lds_elems<BM, BN, STAGES>(), STAGES == 1 ? 2 : 0, 32>(
        a, acc32, lds, tm, tn, wm * WTM, wn * WTN);
}

// ---- halo (input-reuse) main loop: stride-1 KH x KW convolutions ----
// The im2col loaders above fetch every input pixel once per filter tap (9x for a 3x3), which makes the
// 3x3 shapes L2 -> LDS bound (28x28 3x3: ~12.8 TB/s chip-wide into LDS at 0.8 PF/s; the LDS-DMA
// gather ceiling is ~70 GB/s per CU, MI355X_MICROARCH.md 'gather into LDS').  Here a BM-row output
// tile loads its input window ONCE per 64-channel chunk and every tap reads shifted rows of it:
// with the input viewed as zero-padded to Hp = OH + KH - 1 by Wp = OW + KW - 1 (padding is virtual:
// out-of-image slots are LDS-DMA range-check zeros), output pixel (n, oh, ow) of tap (kh, kw) reads
// padded pixel pidx(n, oh, ow) + kh * Wp + kw, pidx = (n * Hp + oh) * Wp + ow.  A tile of consecutive
// output rows therefore needs ONE contiguous run of padded pixels, [pidx(m0), pidx(m_last) + (KH-1) Wp
// + KW - 1] -- its "slots" (128 B = 64 channels each, 16-B chunks XOR-swizzled by slot) -- plus the
// BN x 64 weight tile of the current tap.  Per 64-channel chunk a 256 x 128 tile then moves ~64 KB of
// input + 9 x 16 KB of weights instead of 9 x (32 + 16) KB.  Single LDS stage for the weights, 8 waves
// (4 x 2 of 64 x WTN on v_mfma_f32_32x32x16_bf16), two workgroups per CU; rows are still the linear
// (n, oh, ow) order, so the conv_epilogue variants (BN statistics, residual, BN-group backward) apply
// unchanged.  The same kernel runs the stride-1 input gradient (dy as the image, mirrored taps).
template <int BM, int BN, int WGM, int WGN, int NSLOT, int EK>
__global__ __launch_bounds__(64 * WGM * WGN, 4) void k_conv_halo(Igemm a, int Hp, int Wp, int diag) {
  constexpr int NW = WGM * WGN, NT = 64 * NW;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int MI32 = WTM / 32, NJ32 = WTN / 32;
  constexpr int A_ELEMS = NSLOT * LDS_ROW, B_ELEMS = BN * LDS_ROW;
  constexpr int LDS_E = (A_ELEMS + B_ELEMS) > BM * (BN + 8) ? (A_ELEMS + B_ELEMS) : BM * (BN + 8);
  constexpr int A_LD = NSLOT / (8 * NW);  // 8-slot LDS-DMA wave-instructions per wave, input window
  constexpr int B_LD = BN / (8 * NW);     // ..., weight tile
  static_assert(NSLOT % (8 * NW) == 0 && BN % (8 * NW) == 0 && MI32 >= 1 && NJ32 >= 1 && WTM % 32 == 0 &&
                    WTN % 32 == 0,
                "halo geometry");
  __shared__ __attribute__((aligned(16))) uint16_t lds[LDS_E];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int ntn = a.K / BN;
  const int tn = wg % ntn, tm = wg / ntn;

  const int HWp = Hp * Wp;
  auto pidx = [&](int m) {
    const int ow = m % a.OW, t = m / a.OW, oh = t % a.OH, n = t / a.OH;
    return (n * Hp + oh) * Wp + ow;
  };
  const int m0 = tm * BM, mlast = min(m0 + BM, a.M) - 1;
  const int pbase = pidx(m0);
  const int nslot = pidx(mlast) + (a.KH - 1) * Wp + a.KW - pbase;  // <= NSLOT (host-checked)

  const auto x_rsrc = buf_rsrc(a.x, (unsigned)((long long)a.N * a.H * a.W * a.C * 2));
  const auto w_rsrc = buf_rsrc(a.w, (unsigned)((long long)a.KH * a.KW * a.C * a.K * 2));
  // input window: lane L of wave-instruction i fills slot 8 (i NW + wave) + L / 8, position L % 8, i.e.
  // fetches chunk (L % 8) ^ swz(slot) of that padded pixel (zeros outside the image / past the window)
  int a_vo[A_LD];
#pragma unroll
  for (int i = 0; i < A_LD; ++i) {
    const int s = (i * NW + wave) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(s);
    const int P = pbase + s;
    const int n = P / HWp, rem = P - n * HWp, ph = rem / Wp, pw = rem - ph * Wp;
    const int ih = ph - a.PT, iw = pw - a.PL;
    const bool ok = s < nslot && n < a.N && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    a_vo[i] = ok ? (int)(((((long long)n * a.H + ih) * a.W + iw) * a.C + chunk * 8) * 2) : (int)0x80000000;
  }
  int b_vo[B_LD];
#pragma unroll
  for (int i = 0; i < B_LD; ++i) {
    const int row = (i * NW + wave) * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ swz(row);
    b_vo[i] = (int)(((long long)(tn * BN + row) * a.w_col + chunk * 8) * 2);
  }
  // this lane's fragment rows (32x32x16: row l & 31 of each 32-row block) as window slots of tap (0, 0);
  // rows past M read a valid slot (their results are never stored)
  const int frow32 = lane & 31, kq = lane >> 5;
  int sb[MI32];
#pragma unroll
  for (int i = 0; i < MI32; ++i) sb[i] = pidx(min(m0 + wm * WTM + i * 32 + frow32, mlast)) - pbase;

  f16v acc32[MI32][NJ32];
#pragma unroll
  for (int i = 0; i < MI32; ++i)
#pragma unroll
    for (int j = 0; j < NJ32; ++j)
#pragma unroll
      for (int z = 0; z < 16; ++z) acc32[i][j][z] = 0.f;

  uint16_t* const la = lds;
  uint16_t* const lb = lds + A_ELEMS;
  const int ctiles = a.C / BK, taps = a.KH * a.KW;
  for (int c = 0; c < ctiles; ++c) {
    int kh = 0, kw = 0;
    for (int tap = 0; tap < taps; ++tap) {
      if (c | tap) __syncthreads();  // every wave done reading the previous weight tile (and window)
      const bool ld = !(diag & 1) || (c == 0 && tap == 0);  // diag 1: loads of the first step only
      if (tap == 0 && ld) {
#pragma unroll
        for (int i = 0; i < A_LD; ++i)
          if ((i * NW + wave) * 8 < nslot)  // (wave-uniform)
            lds_dma16(x_rsrc, la + (i * NW + wave) * 8 * LDS_ROW, a_vo[i], c * BK * 2);
      }
      const int wkh = a.flip ? a.KH - 1 - kh : kh, wkw = a.flip ? a.KW - 1 - kw : kw;
      const int soff_b = (int)((wkh * a.w_kh + wkw * a.w_kw + c * BK) * 2);
#pragma unroll
      for (int i = 0; i < B_LD; ++i)
        if (ld) lds_dma16(w_rsrc, lb + (i * NW + wave) * 8 * LDS_ROW, b_vo[i], soff_b);
      wait_vmcnt_barrier<0>();
      const int toff = kh * Wp + kw;
#pragma unroll
      for (int st = 0; st < ((diag & 2) ? 0 : BK / 16); ++st) {  // diag 2: no MFMA work
        bf16x8 fa[MI32], fb[NJ32];
#pragma unroll
        for (int i = 0; i < MI32; ++i) {
          const int sl = sb[i] + toff;
          fa[i] = *reinterpret_cast<const bf16x8*>(la + sl * LDS_ROW + (((2 * st + kq) ^ swz(sl)) * 8));
        }
#pragma unroll
        for (int j = 0; j < NJ32; ++j) {
          const int row = wn * WTN + j * 32 + frow32;
          fb[j] = *reinterpret_cast<const bf16x8*>(lb + row * LDS_ROW + (((2 * st + kq) ^ swz(row)) * 8));
        }
#pragma unroll
        for (int i = 0; i < MI32; ++i)
#pragma unroll
          for (int j = 0; j < NJ32; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[j], fa[i], acc32[i][j], 0, 0, 0);
      }
      if (++kw == a.KW) {
        kw = 0;
        ++kh;
      }
    }
  }
  __syncthreads();  // every wave done reading the window: the epilogue reuses the LDS
  conv_epilogue<BM, BN, NT, EK, WTM, WTN, LDS_E, 2, 32>(a, acc32, lds, tm, tn, wm * WTM, wn * WTN);
}

constexpr int kHaloBM = 256, kHaloSlots = 512;

// padded geometry of the halo kernel and the longest window over its row tiles (host; cached per shape)
int halo_window(const Igemm& a, int& Hp, int& Wp) {
  Hp = a.OH + a.KH - 1;
  Wp = a.OW + a.KW - 1;
  static std::mutex mu;
  static std::map<std::array<int, 6>, int> cache;
  const std::array<int, 6> key{a.N, a.OH, a.OW, a.KH, a.KW, a.M};
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  auto pidx = [&](long long m) {
    const long long ow = m % a.OW, t = m / a.OW, oh = t % a.OH, n = t / a.OH;
    return (n * Hp + oh) * Wp + ow;
  };
  long long worst = 0;
  for (long long m0 = 0; m0 < a.M; m0 += kHaloBM) {
    const long long ml = std::min<long long>(m0 + kHaloBM, a.M) - 1;
    worst = std::max(worst, pidx(ml) + (long long)(a.KH - 1) * Wp + a.KW - pidx(m0));
  }
  const int w = (int)std::min<long long>(worst, 1 << 30);
  std::lock_guard<std::mutex> g(mu);
  cache[key] = w;
  return w;
}

int g_depth = 2;  // main-loop variant; conv_force_depth for A/B sweeps
bool g_single = true;  // default: the single-stage, 4-waves-per-SIMD variant for every reduction length

template <int BM, int BN, int DEPTH>
void launch_epi(const Igemm& a, hipStream_t s) {
  const dim3 grid((a.M + BM - 1) / BM * (a.K / BN)), block(BM * 2);
  {
    if (a.scatter)  // (the scatter epilogue spills at 128 VGPRs: depth 0 takes the 3-waves-per-SIMD variant)
      hipLaunchKernelGGL((k_conv_igemm<BM, BN, DEPTH == 0 ? 3 : DEPTH, 2>), grid, block, 0, s, a);
    else if (a.bn_part && a.bn_ss)  // (DEPTH 3's fused BN-group backward epilogue spills at 168 VGPRs: depth 2)
      hipLaunchKernelGGL((k_conv_igemm<BM, BN, DEPTH == 3 ? 2 : DEPTH, 3>), grid, block, 0, s, a);
    else if (a.bn_part)
      hipLaunchKernelGGL((k_conv_igemm<BM, BN, DEPTH == 3 ? 2 : DEPTH, 1>), grid, block, 0, s, a);
    else
      hipLaunchKernelGGL((k_conv_igemm<BM, BN, DEPTH, 0>), grid, block, 0, s, a);
  }
}

// Main-loop variant, from the A/B over the Keras ResNet-50 b=256 convolutions
// (profiles/conv_main_loop_ab_r4.txt): four resident 128x128 workgroups per CU without any
// software pipelining (DEPTH 0) beat two double-buffered ones with two tiles of register prefetch
// (DEPTH 2) on every shape, 1x1 and 3x3, short and long reductions (e.g. 28x28 3x3 fwd 95.6 -> 73.4
// us, 14x14 1024->256 1x1 fwd 46.2 -> 40.3): the other workgroups' MFMAs hide a workgroup's load
// latency and its epilogue better than its own prefetch does.  The single LDS stage with register
// prefetch at three per CU (DEPTH 3) lands in between.
template <int BM, int BN>
void launch_tile(const Igemm& a, hipStream_t s) {
  if (g_depth == 0 || (g_depth == 2 && g_single))
    launch_epi<BM, BN, 0>(a, s);
  else if (g_depth == 3)
    launch_epi<BM, BN, 3>(a, s);
  else if (g_depth == 1)
    launch_epi<BM, BN, 1>(a, s);
  else
    launch_epi<BM, BN, 2>(a, s);
}

int g_forced_tile = 0;  // 0: heuristic below; 1: 128 x 64, 2: 128 x 128, 3: 256 x 128 (tile sweeps)
// MFMA form of the dma1 main loop: 32 (v_mfma_f32_32x32x16_bf16) or 16 (v_mfma_f32_16x16x32_bf16).
// TDL_CONV_MFMA overrides (A/B); conv_force_mfma too.
int g_mf = [] {
  const char* e = std::getenv("TDL_CONV_MFMA");
  return (e != nullptr && std::atoi(e) == 16) ? 16 : 32;
}();
int g_impl = [] {  // (TDL_CONV_IMPL: the conv_force_impl A/B hook from the environment)
  const char* e = std::getenv("TDL_CONV_IMPL");
  const int v = e != nullptr ? std::atoi(e) : 2;
  return (v == 1 || (v >= 3 && v <= 7)) ? v : 2;
}();  // 1: v1 only; 2: the LDS-DMA ring kernel where it measured faster; 3: wherever it fits;
                 // 4 / 5: the single-stage LDS-DMA kernel (dma1) at 4 / 3 waves per SIMD wherever v1 runs;
                 // 7: the halo kernel wherever it fits, else the default selection

template <int BM, int BN, int WGM, int WGN, int STAGES = 3, int MINW = 1, int MF = 16>
void launch_v2(const Igemm& a, hipStream_t s) {
  const dim3 grid((a.M + BM - 1) / BM * (a.K / BN)), block(64 * WGM * WGN);
  if (a.scatter)
    hipLaunchKernelGGL((k_conv_glds<BM, BN, WGM, WGN, 2, STAGES, MINW, MF>), grid, block, 0, s, a);
  else if (a.bn_part && a.bn_ss)
    hipLaunchKernelGGL((k_conv_glds<BM, BN, WGM, WGN, 3, STAGES, MINW, MF>), grid, block, 0, s, a);
  else if (a.bn_part)
    hipLaunchKernelGGL((k_conv_glds<BM, BN, WGM, WGN, 1, STAGES, MINW, MF>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((k_conv_glds<BM, BN, WGM, WGN, 0, STAGES, MINW, MF>), grid, block, 0, s, a);
}

// v2 (256-row tiles, one 8-wave workgroup per CU, 3-stage LDS-DMA ring): only when forced (impl 3)
// or under the pre-round-4 selection (conv_force_depth(3): >= 32 k-tiles).  The default never takes
// it: dma1 and the single-stage v1 beat it on every shape (profiles/conv_dma1_ab_r4.txt).
bool use_v2(int M, int K, int ktiles, int taps) {
  (void)taps;
  if (g_forced_tile != 0 || !(g_impl == 3 || (g_impl == 2 && !g_single && ktiles >= 32))) return false;
  const long long wgs = (long long)(M + 255) / 256 * (K % 128 == 0 ? K / 128 : K / 64);
  return wgs >= 256;
}

// dma1 (the single-stage LDS-DMA kernel, 4 waves of 64x64, 4 waves per SIMD) for the 3x3 convs and
// the stride-2 scatter dgrads with >= 9 k-tiles and 128-column tiles: 6-11 % faster there in the
// ResNet-50 step than the register-staged single-stage v1 (no VGPR staging, no ds_write pass: the
// operands land in LDS by DMA).  The per-shape bench also favoured it for 1x1 convs with >= 16
// k-tiles, but inside the step (fused BN epilogues, neighbouring kernels) those and the 64-column
// tiles ran 2-7 % slower (profiles/conv_dma1_ab_r4.txt, resnet50_steady_state_breakdown_r4_dma1.txt).
// Bit-identical either way.
bool use_dma1(const Igemm& a) {
  if (g_forced_tile != 0) return false;
  if (g_impl >= 4) return true;
  const int ktiles = a.KH * a.KW * (a.C / BK);
  return g_impl == 2 && g_single && ktiles >= 9 && a.K % 128 == 0 && (a.KH * a.KW > 1 || a.scatter);
}

// halo kernel (k_conv_halo) for stride-1 multi-tap convolutions whose longest input window fits
// kHaloSlots: forced by impl 7 or g_halo 1; by default (g_halo 2) only where the per-shape A/B
// favoured it (profiles/conv_halo_r6.txt, b=256 Keras ResNet-50 3x3 shapes, three boxes):
//   14x14x256 3x3  fwd 72.6 -> 67.1 us, dgrad 71.4 -> 67.2 (the 256-row tile spans 1.3 images)
//   56x56x64 (+-3 %, noise), 28x28x128 (+3-10 % slower), 7x7x512 (+10-14 % slower): default kernels
// Both kernels sit at the ~0.85-0.9 PF/s ceiling of a one-barrier-per-k-tile loop: with the loads
// removed (TDL_CONV_HALO_DIAG=1) the halo kernel still needs 58-88 us, so the im2col re-reads were not
// the limiter; a two-window / two-stage ring at one workgroup per CU measured 30-50 % slower.
// TDL_CONV_HALO=0/1/2 overrides.
int g_halo = [] {
  const char* e = std::getenv("TDL_CONV_HALO");
  return e != nullptr ? std::atoi(e) : 2;
}();

bool halo_default_shape(const Igemm& a) {
  const int hw = a.OH * a.OW;
  return a.KH == 3 && a.KW == 3 && hw > 128 && hw <= 256 && a.C >= 256 && a.K >= 256;
}

int g_halo_diag = [] {  // timing diagnostics (wrong results): 1 compute only, 2 loads only
  const char* e = std::getenv("TDL_CONV_HALO_DIAG");
  return e != nullptr ? std::atoi(e) : 0;
}();

bool use_halo(const Igemm& a, int& Hp, int& Wp) {
  if (g_forced_tile != 0 || !(g_impl == 7 || (g_impl == 2 && g_halo != 0))) return false;
  if (g_impl != 7 && g_halo == 2 && !halo_default_shape(a)) return false;
  if (a.SH != 1 || a.SW != 1 || a.scatter || a.in_ss || a.KH * a.KW < 2 || a.K % 64 != 0 || a.C % BK != 0)
    return false;
  return halo_window(a, Hp, Wp) <= kHaloSlots;
}

template <int BN>
void launch_halo(const Igemm& a, int Hp, int Wp, hipStream_t s) {
  const dim3 grid((a.M + kHaloBM - 1) / kHaloBM * (a.K / BN)), block(512);
  if (a.bn_part && a.bn_ss)
    hipLaunchKernelGGL((k_conv_halo<kHaloBM, BN, 4, 2, kHaloSlots, 3>), grid, block, 0, s, a, Hp, Wp, g_halo_diag);
  else if (a.bn_part)
    hipLaunchKernelGGL((k_conv_halo<kHaloBM, BN, 4, 2, kHaloSlots, 1>), grid, block, 0, s, a, Hp, Wp, g_halo_diag);
  else
    hipLaunchKernelGGL((k_conv_halo<kHaloBM, BN, 4, 2, kHaloSlots, 0>), grid, block, 0, s, a, Hp, Wp, g_halo_diag);
}

// Tile choice, from the sweep over the ResNet-50 b=256 convolutions (profiles/conv_tile_sweep_r1.jsonl):
// 128 x 128 wins every shape with K % 128 == 0, including the 7x7 ones whose grid is under two
// workgroups per CU (the 64-column tile's extra LDS traffic per MFMA costs more than the idle CUs);
// 256 x 128 loses 5-20 % everywhere.  The 64-column tile only serves K == 64 * odd.
void launch(const Igemm& a, hipStream_t s) {
  if (a.in_ss) {  // input-side BN -> ReLU: the register-staged loader, single stage, plain epilogue
    if (a.C > kProMaxC) return;  // (conv_fwd_bf16's callers check conv_in_bn_supported)
    if (a.K % 128 == 0) {
      hipLaunchKernelGGL((k_conv_igemm<128, 128, 0, 0, true>), dim3((a.M + 127) / 128 * (a.K / 128)), dim3(256), 0, s, a);
    } else {
      hipLaunchKernelGGL((k_conv_igemm<128, 64, 0, 0, true>), dim3((a.M + 127) / 128 * (a.K / 64)), dim3(256), 0, s, a);
    }
    return;
  }
  {
    int Hp, Wp;
    if (use_halo(a, Hp, Wp)) {
      if (a.K % 128 == 0 && g_halo != 3) return launch_halo<128>(a, Hp, Wp, s);
      return launch_halo<64>(a, Hp, Wp, s);  // (g_halo 3: 64-column tiles everywhere, an A/B arm)
    }
  }
  if (use_v2(a.M, a.K, a.KH * a.KW * (a.C / BK), a.KH * a.KW)) {
    if (a.K % 128 == 0) return launch_v2<256, 128, 4, 2>(a, s);
    return launch_v2<256, 64, 4, 2>(a, s);
  }
  if (use_dma1(a)) {
    // dma1 at 4 waves per SIMD on 32x32x16 (default; impl 6 forces it everywhere) or 16x16x32 MFMAs
    // (impl 4 / TDL_CONV_MFMA=16), or at 3 waves per SIMD (impl 5)
    const bool mf32 = g_impl == 6 || (g_mf == 32 && g_impl != 4 && g_impl != 5);
    if (a.K % 128 == 0) {
      if (mf32) return launch_v2<128, 128, 2, 2, 1, 4, 32>(a, s);
      return g_impl != 5 ? launch_v2<128, 128, 2, 2, 1, 4>(a, s) : launch_v2<128, 128, 2, 2, 1, 3>(a, s);
    }
    if (mf32) return launch_v2<128, 64, 2, 2, 1, 4, 32>(a, s);
    return g_impl != 5 ? launch_v2<128, 64, 2, 2, 1, 4>(a, s) : launch_v2<128, 64, 2, 2, 1, 3>(a, s);
  }
  if (g_forced_tile == 3 && a.K % 128 == 0) return launch_tile<256, 128>(a, s);
  if (g_forced_tile == 1 || a.K % 128 != 0) return launch_tile<128, 64>(a, s);
  launch_tile<128, 128>(a, s);
}

}  // namespace

void conv_force_tile(int tile) { g_forced_tile = tile; }
void conv_force_impl(int impl) { g_impl = (impl == 1 || (impl >= 3 && impl <= 7)) ? impl : 2; }
void conv_force_halo(int on) { g_halo = on; }
void conv_force_mfma(int mf) { g_mf = mf == 16 ? 16 : 32; }
void conv_force_depth(int depth) {
  // 0: single stage everywhere, 1 / 2: register prefetch depth 1 / the default selection (single
  // stage), 3: depth 2 everywhere (the selection before round 4's A/B, v2 for every long reduction),
  // 4: single LDS stage + register prefetch everywhere
  g_depth = depth == 0 ? 0 : (depth == 1 ? 1 : (depth == 4 ? 3 : 2));
  g_single = depth != 3;
}

bool conv_in_bn_supported(const ConvGeom& g) {
  return g.KH == 1 && g.KW == 1 && g.SH == 1 && g.SW == 1 && g.PT == 0 && g.PL == 0 && g.C <= kProMaxC;
}

bool conv_bf16_supported(const ConvGeom& g) {
  // byte offsets of every operand and output within 2 GiB (32-bit buffer offsets), <= 32 taps
  // (the per-row tap-validity bitmask of the operand loader), padding < the filter size (the
  // image resource's base offset is non-negative in both directions)
  const long long two_gib_elems = 1ll << 30;
  return g.C % 64 == 0 && g.K % 64 == 0 && g.N > 0 && g.OH > 0 && g.OW > 0 && g.KH * g.KW <= 32 &&
         g.PT >= 0 && g.PL >= 0 && g.PT < g.KH && g.PL < g.KW &&
         (long long)g.N * g.H * g.W * g.C + ((long long)g.PT * g.W + g.PL) * g.C < two_gib_elems &&
         (long long)g.N * g.OH * g.OW * g.K + ((long long)(g.KH - 1 - g.PT) * g.OW + (g.KW - 1 - g.PL)) * g.K <
             two_gib_elems &&
         (long long)g.KH * g.KW * g.C * g.K < two_gib_elems;
}

static Igemm fwd_args(const ConvGeom& g, const void* x, const void* w_ohwi, void* y) {
  return Igemm{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(w_ohwi), static_cast<uint16_t*>(y),
               g.N, g.H, g.W, g.C, g.OH, g.OW, g.K, g.KH, g.KW, g.SH, g.SW, g.PT, g.PL, 0,
               (long long)g.KH * g.KW * g.C, (long long)g.KW * g.C, (long long)g.C, g.N * g.OH * g.OW, 0, 0, 0,
               nullptr, nullptr};
}

// image = dy [N][OH][OW][K] (reduction channels K), output = dx [N][H][W][C] (columns C), stride 1,
// mirrored taps with padding KH-1-PT / KW-1-PL
static Igemm dgrad_args(const ConvGeom& g, const void* dy, const void* w_hwio, void* dx) {
  return Igemm{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w_hwio), static_cast<uint16_t*>(dx),
               g.N, g.OH, g.OW, g.K, g.H, g.W, g.C, g.KH, g.KW, 1, 1, g.KH - 1 - g.PT, g.KW - 1 - g.PL, 1,
               (long long)g.K, (long long)g.KW * g.C * g.K, (long long)g.C * g.K, g.N * g.H * g.W, 0, 0, 0,
               nullptr, nullptr};
}

// the row tile launch() picks (the BN partial-sum rows of an epilogue are per row tile)
int conv_fwd_row_tile(const ConvGeom& g, bool in_bn) {
  if (in_bn) return 128;
  {
    int Hp, Wp;
    const Igemm a = fwd_args(g, nullptr, nullptr, nullptr);
    if (use_halo(a, Hp, Wp)) return kHaloBM;
  }
  if (use_v2(g.N * g.OH * g.OW, g.K, g.KH * g.KW * (g.C / BK), g.KH * g.KW)) return 256;
  return (g_forced_tile == 3 && g.K % 128 == 0) ? 256 : 128;
}

int conv_dgrad_row_tile(const ConvGeom& g) {
  {
    int Hp, Wp;
    const Igemm a = dgrad_args(g, nullptr, nullptr, nullptr);
    if (use_halo(a, Hp, Wp)) return kHaloBM;
  }
  if (use_v2(g.N * g.H * g.W, g.C, g.KH * g.KW * (g.K / BK), g.KH * g.KW)) return 256;
  return (g_forced_tile == 3 && g.C % 128 == 0) ? 256 : 128;
}

int conv_dgrad_s2_row_tile(const ConvGeom& g) {
  if (use_v2(g.N * g.OH * g.OW, g.C, g.K / BK, 1)) return 256;
  return (g_forced_tile == 3 && g.C % 128 == 0) ? 256 : 128;
}

void conv_fwd_bf16(const void* x, const void* w_ohwi, void* y, const ConvGeom& g, hipStream_t s, float* stats,
                   const float* in_ss) {
  Igemm a = fwd_args(g, x, w_ohwi, y);
  a.stats = stats;
  a.in_ss = in_ss;
  launch(a, s);
}

void conv_dgrad_bf16(const void* dy, const void* w_hwio, void* dx, const ConvGeom& g, hipStream_t s,
                     const void* residual, const void* bn_y, const void* bn_x, float* bn_part, const void* bn_x2,
                     float* bn_part2, const float* bn_ss) {
  // image = dy [N][OH][OW][K] (reduction channels K), output = dx [N][H][W][C] (columns C), stride 1,
  // mirrored taps with padding KH-1-PT / KW-1-PL
  Igemm a = dgrad_args(g, dy, w_hwio, dx);
  a.res = static_cast<const uint16_t*>(residual);
  a.bn_y = static_cast<const uint16_t*>(bn_y);
  a.bn_x = static_cast<const uint16_t*>(bn_x);
  a.bn_part = bn_part;
  a.bn_x2 = static_cast<const uint16_t*>(bn_x2);
  a.bn_part2 = bn_part2;
  a.bn_ss = bn_ss;
  launch(a, s);
}

void conv_dgrad_s2_1x1_bf16(const void* dy, const void* w_hwio, void* dx, const ConvGeom& g, hipStream_t s,
                            const void* residual, const void* bn_y, const void* bn_x, float* bn_part,
                            const void* bn_x2, float* bn_part2, const float* bn_ss) {
  // a 1x1 stride-1 "convolution" of dy [N][OH][OW][K] with the HWIO rows [C][K] (columns C, reduction K),
  // scattered to the even pixels of dx [N][H][W][C]
  Igemm a{static_cast<const uint16_t*>(dy), static_cast<const uint16_t*>(w_hwio), static_cast<uint16_t*>(dx),
          g.N, g.OH, g.OW, g.K, g.OH, g.OW, g.C, 1, 1, 1, 1, 0, 0, 0,
          (long long)g.K, 0, 0, g.N * g.OH * g.OW, 2, g.H, g.W, static_cast<const uint16_t*>(residual), nullptr,
          static_cast<const uint16_t*>(bn_y), static_cast<const uint16_t*>(bn_x), bn_part,
          static_cast<const uint16_t*>(bn_x2), bn_part2, bn_ss};
  launch(a, s);
}

}  // namespace tdl
