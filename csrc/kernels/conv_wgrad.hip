// Weight gradient of the NHWC bf16 convolution on the gfx950 bf16 matrix cores (see conv.h).
//
// GEMM view: dW[tc][k] (HWIO: tc = (kh * KW + kw) * C + c) = sum over output pixels m of
// x(m, tc) * dy[m][k], with x(m, tc) = x[n][oh*SH - PT + kh][ow*SW - PL + kw][c] (zero outside the
// image).  The reduction runs over PIXELS, and both operands are channel-contiguous in HBM, so the
// tiles are staged into LDS exactly as they arrive (64 pixels x 64 channels = 128-B rows, 16-B
// chunks) and the MFMA fragments, which need 8 consecutive pixels of one channel per lane, are
// read with the gfx950 hardware transpose read ds_read_b64_tr_b16 (4 pixels x 16 channels per
// 16-lane group; two reads make one bf16x8 operand).  No im2col copy, no transposed copy.
//
// LDS image: 16-B chunk ch of pixel row r lives at chunk ch ^ f(r), f(r) = 2*bit1(r) + 4*bit3(r).
// A 32-lane half of a transposed read touches rows {8g+4h+q} (q = 0..3, g = 2 adjacent groups) and
// one 32-B column pair; under f the 8 row/chunk combinations land on 16 distinct 4-bank slots of
// the 64-bank modulus (conflict-free), and a staging write (8 lanes = one full 128-B row) is a
// permutation of one row, also conflict-free.
//
// Split-K: the pixel range is cut into S slices; each workgroup writes its f32 tile to a partial
// slab ws[s][tc][k] and k_wgrad_reduce sums the S partials in slice order (deterministic: the same
// bits on every run and every replica) into bf16 HWIO dW or adds them into an f32 gradient.
// The tile shape and S come from a roofline/tail model (conv_wgrad_plans); the Python autotuner
// times its first candidates against MIOpen on the first call of every shape.
//
// Every wave owns a 64 (k) x 64 (tc) tile of 16x16x32 MFMAs with dy as the A operand, so each lane
// holds 4 consecutive k of one tc (16-B partial stores); a workgroup is 1 x 1 .. 4 x 1 such waves.
// blockIdx -> (slice, tile) is XCD-aware: the tiles of one slice (which read the same dy and x
// pixels) run on one XCD and share its L2.
#include "kernels/conv.h"
#include "kernels/common.h"

#include <algorithm>
#include <cmath>
#include <vector>

namespace tdl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int RB = 64;        // pixels per reduction stage
constexpr int SUB = RB * 64;  // bf16 elements of one 64-pixel x 64-channel sub-image (8 KiB)

__device__ __forceinline__ int fswz(int r) { return (((r >> 1) & 1) << 1) | (((r >> 3) & 1) << 2); }

struct Wgrad {
  const uint16_t* x;   // NHWC [N][H][W][C]
  const uint16_t* dy;  // NHWC [N][OH][OW][K] == [M][K]
  float* ws;           // partial slab [S][TC][K]
  int N, H, W, C;
  int OH, OW, K;
  int KH, KW, SH, SW, PT, PL;
  int M, TC;
  int chunk;     // pixels per split slice (multiple of RB)
  int nsplit;    // S
  int direct;    // 1x1, stride 1, no padding: x(m, c) = x[m][c]
  float inv_ow, inv_oh;
  // optional (direct only): x is a BN -> ReLU's input; the staging stores relu(x * scale + shift)
  // (in_ss = scale[C], shift[C]), the BN apply pass's arithmetic
  const float* in_ss;
};

// relu(x * sc + sh) for 8 packed bf16 x (f32 fma, round to nearest even)
__device__ __forceinline__ u32x4 bn_relu_bf16x8(u32x4 x, const float* sc, const float* sh) {
  typedef float f2v __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f2v v = {__uint_as_float(x[k] << 16), __uint_as_float(x[k] & 0xffff0000u)};
    const f2v r = __builtin_elementwise_max(
        __builtin_elementwise_fma(v, f2v{sc[2 * k], sc[2 * k + 1]}, f2v{sh[2 * k], sh[2 * k + 1]}), f2v{0.f, 0.f});
    o[k] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, bf16x2));  // v_cvt_pk_bf16_f32 (RNE)
  }
  return o;
}

// q = n / d for 0 <= n < 2^24 via one f32 multiply and a +-1 fix-up
__device__ __forceinline__ int fdiv(int n, int d, float inv, int& rem) {
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

// Workgroup = WMW x WNW waves, each wave a 64 (k) x 64 (tc) tile of 4 x 4 16x16x32 MFMAs; the
// workgroup tile is (64 WMW) x (64 WNW) and its LDS stage is WMW + WNW sub-images of 64 pixels x
// 64 channels.  Columns past TC (a partial last tc tile) are staged as zeros and not stored.
// SINGLE: one LDS stage and no register prefetch, 3 waves per SIMD (<= 168 VGPRs; at 4 the staging
// registers spill): the other
// resident workgroups hide a workgroup's load latency (the conv.hip DEPTH 0 finding).
// PRO: the input-side BN -> ReLU (Wgrad::in_ss) on the staged x chunks; the per-thread channel
// scale / shift stay in registers (double-buffered variant: 2 waves per SIMD, room for them)
template <int WMW, int WNW, bool SINGLE, bool PRO = false>
__global__ __launch_bounds__(64 * WMW * WNW) __attribute__((amdgpu_waves_per_eu(SINGLE ? 3 : 2))) void k_conv_wgrad(
    Wgrad a) {
  static_assert(!(PRO && SINGLE), "input-side BN: double-buffered variant");
  constexpr int NW = WMW * WNW, NT = 64 * NW;
  constexpr int SA = WMW, SBn = WNW;
  constexpr int RPT = 8 / NW;                 // staged rows per thread per sub-image
  constexpr int RSTEP = 8 * NW;               // row stride between a thread's staged rows
  constexpr int STAGE = (SA + SBn) * SUB;     // bf16 elements per LDS stage
  static_assert(8 % NW == 0, "1, 2, 4 or 8 waves");
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  // XCD-aware bijective remap, then (slice, tile) with the tiles of one slice adjacent
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int ntk = a.K / (64 * WMW), ntc = (a.TC + 64 * WNW - 1) / (64 * WNW), ntiles = ntk * ntc;
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tk = tile % ntk, ttc = tile / ntk;
  const int k0 = tk * 64 * WMW, tc0 = ttc * 64 * WNW;
  const int mbeg = split * a.chunk;
  const int mend = min(a.M, mbeg + a.chunk);
  const int nst = (mend - mbeg + RB - 1) / RB;

  const int srow = tid >> 3, sch = tid & 7;
  int soff[RPT];
#pragma unroll
  for (int i = 0; i < RPT; ++i) {
    const int r = srow + RSTEP * i;
    soff[i] = r * 64 + ((sch ^ fswz(r)) << 3);
  }
  // B sub-images: tap and channel base are fixed for the workgroup
  int b_kh[SBn], b_kw[SBn], b_off[SBn];
  bool b_live[SBn];
#pragma unroll
  for (int j = 0; j < SBn; ++j) {
    const int tc = tc0 + 64 * j;
    b_live[j] = tc < a.TC;
    const int tap = tc / a.C, c0 = tc - tap * a.C;
    b_kh[j] = tap / a.KW;
    b_kw[j] = tap - b_kh[j] * a.KW;
    b_off[j] = (b_kh[j] * a.W + b_kw[j]) * a.C + c0 + sch * 8;
  }

  float isc[PRO ? SBn : 1][8], ish[PRO ? SBn : 1][8];
  if constexpr (PRO) {
#pragma unroll
    for (int j = 0; j < SBn; ++j) {
      const int c = tc0 + 64 * j + sch * 8;  // direct: tc == c
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f4v s4 = b_live[j] ? *reinterpret_cast<const f4v*>(a.in_ss + c + 4 * h) : f4v{0.f, 0.f, 0.f, 0.f};
        const f4v t4 = b_live[j] ? *reinterpret_cast<const f4v*>(a.in_ss + a.C + c + 4 * h) : f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          isc[j][4 * h + e] = s4[e];
          ish[j][4 * h + e] = t4[e];
        }
      }
    }
  }
  u32x4 ra[RPT][SA], rb[RPT][SBn];
  auto gload = [&](int st) {
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
      const int m = mbeg + st * RB + srow + RSTEP * i;
      const bool live = m < mend;
#pragma unroll
      for (int j = 0; j < SA; ++j)
        ra[i][j] = live ? *reinterpret_cast<const u32x4*>(a.dy + (long long)m * a.K + k0 + 64 * j + sch * 8)
                        : u32x4{0u, 0u, 0u, 0u};
      if (a.direct) {
#pragma unroll
        for (int j = 0; j < SBn; ++j)
          rb[i][j] = (live && b_live[j]) ? *reinterpret_cast<const u32x4*>(a.x + (long long)m * a.C + b_off[j])
                                         : u32x4{0u, 0u, 0u, 0u};
      } else {
        int ow, oh;
        const int t = fdiv(live ? m : 0, a.OW, a.inv_ow, ow);
        const int n = fdiv(t, a.OH, a.inv_oh, oh);
        const int ih0 = oh * a.SH - a.PT, iw0 = ow * a.SW - a.PL;
        const long long base = (((long long)n * a.H + ih0) * a.W + iw0) * a.C;
#pragma unroll
        for (int j = 0; j < SBn; ++j) {
          const int ih = ih0 + b_kh[j], iw = iw0 + b_kw[j];
          const bool ok = live && b_live[j] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          rb[i][j] = ok ? *reinterpret_cast<const u32x4*>(a.x + base + b_off[j]) : u32x4{0u, 0u, 0u, 0u};
        }
      }
    }
  };
  auto sstore = [&](int buf) {
    uint16_t* base = lds + buf * STAGE;
#pragma unroll
    for (int i = 0; i < RPT; ++i) {
#pragma unroll
      for (int j = 0; j < SA; ++j) *reinterpret_cast<u32x4*>(base + j * SUB + soff[i]) = ra[i][j];
#pragma unroll
      for (int j = 0; j < SBn; ++j) {
        // (rows past the slice are transformed too: their dy rows are zeros)
        u32x4 v = rb[i][j];
        if constexpr (PRO) v = bn_relu_bf16x8(v, isc[j], ish[j]);
        *reinterpret_cast<u32x4*>(base + (SA + j) * SUB + soff[i]) = v;
      }
    }
  };

  // transposed-read addresses: group g = lane >> 4, lane 4q + p of the group reads pixel row
  // 8g + 4h + q (h = 0, 1), channels col0 + 4p .. 4p + 3 of its 16-column block
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int trow = 8 * g + qq;  // + 4h + 32 kk
  const int tsw = fswz(trow);   // bits 1 and 3 of the row do not change with h or kk
  auto tr_off = [&](int col0) { return trow * 64 + (((col0 >> 3) + (pp >> 1)) ^ tsw) * 8 + (pp & 1) * 4; };
  const int a_sub = wm * SUB, b_sub = (SA + wn) * SUB;

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (!SINGLE && nst > 0) {
    gload(0);
    sstore(0);
  }
  if (!SINGLE) __syncthreads();
  for (int st = 0; st < nst; ++st) {
    const int buf = SINGLE ? 0 : st & 1;
    if (SINGLE) {
      gload(st);
      if (st) __syncthreads();  // every wave done reading stage st - 1
      sstore(0);
      __syncthreads();
    } else if (st + 1 < nst) {
      gload(st + 1);
    }
    const uint16_t* base = lds + buf * STAGE;
#pragma unroll
    for (int kk = 0; kk < RB; kk += 32) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint16_t* p = base + a_sub + tr_off(16 * i) + kk * 64;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 64));
        fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t* p = base + b_sub + tr_off(16 * j) + kk * 64;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 64));
        fb[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if (!SINGLE) {
      if (st + 1 < nst) sstore(buf ^ 1);
      __syncthreads();
    }
  }

  // partial tile: lane holds k = 4 * (lane >> 4) .. + 3 of column tc = lane & 15 in each 16 x 16 block
  if (tc0 + 64 * wn >= a.TC) return;
  float* ws = a.ws + (long long)split * a.TC * a.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wm * 64 + i * 16 + 4 * g;
      const int tc = tc0 + wn * 64 + j * 16 + (lane & 15);
      *reinterpret_cast<f4v*>(ws + (long long)tc * a.K + k) = acc[i][j];
    }
}

// v2: 8 waves (2 per SIMD, one workgroup per CU), a 3-stage LDS ring filled by LDS-DMA
// (buffer_load_dwordx4 ... lds), stage st+2's loads in flight while stage st computes, one raw
// barrier per stage.  Wave w stages pixel rows 8w .. 8w+7 of EVERY sub-image (one 1-KiB LDS-DMA
// wave-instruction each), so a lane decomposes its pixel once per stage for all of its loads.  The
// LDS image is the v1 one (fswz-swizzled 128-B rows), produced by swizzling the SOURCE chunk: lane L
// writes slot L % 8 of its row, so it fetches chunk (L % 8) ^ fswz(row).  Padding taps and pixels
// past the slice read voffset 0x80000000: the buffer range check lands zeros.
template <int N>
__device__ __forceinline__ void wg_wait_vmcnt_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// STAGES 1 (wgrad "dma1"): 4-wave tiles, one LDS stage, no prefetch, 4 waves per SIMD -- the conv
// dma1 schedule (four resident workgroups per CU hide each other's DMA latency).
template <int WMW, int WNW, int STAGES = 3>
__global__ __launch_bounds__(64 * WMW * WNW, STAGES == 1 ? 4 : 1) void k_conv_wgrad_glds(Wgrad a) {
  constexpr int SA = WMW, SBn = WNW, NSUB = SA + SBn;
  constexpr int STAGE = NSUB * SUB;
  constexpr int NWV = WMW * WNW;
  constexpr int RPW = 8 / NWV;  // 8-row LDS-DMA pieces per sub-image per wave
  static_assert((NWV == 8 && STAGES == 3) || (WMW == 2 && WNW == 2 && STAGES == 1), "8 waves ring / 2x2 single stage");
  __shared__ __attribute__((aligned(16))) uint16_t lds[STAGES * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WNW, wn = wave % WNW;

  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q8 = nwg >> 3, r8 = nwg & 7, xcd = orig & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (orig >> 3);
  const int ntk = a.K / (64 * WMW), ntc = (a.TC + 64 * WNW - 1) / (64 * WNW), ntiles = ntk * ntc;
  const int split = wg / ntiles, tile = wg % ntiles;
  const int tk = tile % ntk, ttc = tile / ntk;
  const int k0 = tk * 64 * WMW, tc0 = ttc * 64 * WNW;
  const int mbeg = split * a.chunk;
  const int mend = min(a.M, mbeg + a.chunk);
  const int nst = (mend - mbeg + RB - 1) / RB;

  const auto dy_rsrc = buf_rsrc(a.dy, (unsigned)((long long)a.M * a.K * 2));
  const auto x_rsrc = buf_rsrc(a.x, (unsigned)((long long)a.N * a.H * a.W * a.C * 2));
  // this lane's pixel rows of every sub-image: (r * NWV + wave) * 8 + lane / 8; fswz depends on row bits
  // 1 and 3 only, which r * NWV * 8 does not change: one source-swizzled chunk for all of them
  const int row = wave * 8 + (lane >> 3);
  const int chunk8 = ((lane & 7) ^ fswz(row)) * 8;
  int b_kh[SBn], b_kw[SBn], b_off[SBn];
  bool b_live[SBn];
#pragma unroll
  for (int j = 0; j < SBn; ++j) {
    const int tc = tc0 + 64 * j;
    b_live[j] = tc < a.TC;
    const int tap = tc / a.C, c0 = tc - tap * a.C;
    b_kh[j] = tap / a.KW;
    b_kw[j] = tap - b_kh[j] * a.KW;
    b_off[j] = (b_kh[j] * a.W + b_kw[j]) * a.C + c0 + chunk8;
  }
  auto issue = [&](int st, int stage) {
#pragma unroll
   for (int r = 0; r < RPW; ++r) {
    const int m = mbeg + st * RB + row + r * NWV * 8;
    const bool live = m < mend;
    uint16_t* base = lds + stage * STAGE + (wave + r * NWV) * 8 * 64;
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      const int vo = live ? (int)(((long long)m * a.K + k0 + 64 * j + chunk8) * 2) : (int)0x80000000;
      lds_dma16(dy_rsrc, base + j * SUB, vo, 0);
    }
    if (a.direct) {
#pragma unroll
      for (int j = 0; j < SBn; ++j) {
        const int vo = (live && b_live[j]) ? (int)(((long long)m * a.C + b_off[j]) * 2) : (int)0x80000000;
        lds_dma16(x_rsrc, base + (SA + j) * SUB, vo, 0);
      }
    } else {
      int ow, oh;
      const int t = fdiv(live ? m : 0, a.OW, a.inv_ow, ow);
      const int n = fdiv(t, a.OH, a.inv_oh, oh);
      const int ih0 = oh * a.SH - a.PT, iw0 = ow * a.SW - a.PL;
      const int pbase = ((n * a.H + ih0) * a.W + iw0) * a.C;
#pragma unroll
      for (int j = 0; j < SBn; ++j) {
        const int ih = ih0 + b_kh[j], iw = iw0 + b_kw[j];
        const bool ok = live && b_live[j] && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const int vo = ok ? (pbase + b_off[j]) * 2 : (int)0x80000000;
        lds_dma16(x_rsrc, base + (SA + j) * SUB, vo, 0);
      }
    }
   }
  };

  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  const int trow = 8 * g + qq;
  const int tsw = fswz(trow);
  auto tr_off = [&](int col0) { return trow * 64 + (((col0 >> 3) + (pp >> 1)) ^ tsw) * 8 + (pp & 1) * 4; };
  const int a_sub = wm * SUB, b_sub = (SA + wn) * SUB;

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  if (STAGES == 3 && nst > 0) issue(0, 0);
  if (STAGES == 3 && nst > 1) issue(1, 1);
  int stg = 0;
  for (int st = 0; st < nst; ++st) {
    if constexpr (STAGES == 1) {
      if (st) __syncthreads();  // every wave done reading stage st - 1
      issue(st, 0);
      wg_wait_vmcnt_barrier<0>();
    } else {
      if (st + 1 < nst)
        wg_wait_vmcnt_barrier<NSUB>();
      else
        wg_wait_vmcnt_barrier<0>();
      if (st + 2 < nst) issue(st + 2, stg == 0 ? 2 : stg - 1);
    }
    const uint16_t* base = lds + stg * STAGE;
#pragma unroll
    for (int kk = 0; kk < RB; kk += 32) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint16_t* p = base + a_sub + tr_off(16 * i) + kk * 64;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 64));
        fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint16_t* p = base + b_sub + tr_off(16 * j) + kk * 64;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p + 4 * 64));
        fb[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    if constexpr (STAGES == 3) stg = stg == 2 ? 0 : stg + 1;
  }

  if (tc0 + 64 * wn >= a.TC) return;
  float* ws = a.ws + (long long)split * a.TC * a.K;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + wm * 64 + i * 16 + 4 * g;
      const int tc = tc0 + wn * 64 + j * 16 + (lane & 15);
      *reinterpret_cast<f4v*>(ws + (long long)tc * a.K + k) = acc[i][j];
    }
}

// dW = sum of the S partial slabs in a fixed order: wave w of the block sums slices w, w + G, ...
// (4 independent chains), then wave 0 adds the G wave sums in order.  Out: HWIO bf16, or f32
// (+= when accumulate).
__global__ __launch_bounds__(1024) void k_wgrad_reduce(const float* ws, long long n4, int S, uint16_t* out_bf16,
                                                       float* out_f32, int accumulate) {
  __shared__ f4v red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = blockDim.x >> 6;
  const long long i = (long long)blockIdx.x * 64 + lane;
  f4v s = f4v{0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    const f4v* p = reinterpret_cast<const f4v*>(ws) + i;
    f4v s0 = s, s1 = s, s2 = s, s3 = s;
    int k = w;
    for (; k + 3 * G < S; k += 4 * G) {
      s0 += p[(long long)k * n4];
      s1 += p[(long long)(k + G) * n4];
      s2 += p[(long long)(k + 2 * G) * n4];
      s3 += p[(long long)(k + 3 * G) * n4];
    }
    for (; k < S; k += G) s0 += p[(long long)k * n4];
    s = (s0 + s1) + (s2 + s3);
  }
  red[w][lane] = s;
  __syncthreads();
  if (w != 0 || i >= n4) return;
  s = red[0][lane];
  for (int k = 1; k < G; ++k) s += red[k][lane];
  if (out_f32) {
    f4v* o = reinterpret_cast<f4v*>(out_f32) + i;
    *o = accumulate ? *o + s : s;
  } else {
    uint32_t u0 = __float_as_uint(s[0]), u1 = __float_as_uint(s[1]), u2 = __float_as_uint(s[2]),
             u3 = __float_as_uint(s[3]);
    u0 += 0x7fffu + ((u0 >> 16) & 1u);
    u1 += 0x7fffu + ((u1 >> 16) & 1u);
    u2 += 0x7fffu + ((u2 >> 16) & 1u);
    u3 += 0x7fffu + ((u3 >> 16) & 1u);
    reinterpret_cast<uint2*>(out_bf16)[i] = make_uint2((u0 >> 16) | (u1 & 0xffff0000u), (u2 >> 16) | (u3 & 0xffff0000u));
  }
}

bool g_wgrad_single = false;  // conv_wgrad_force_single (A/B hook)

template <int WMW, int WNW, bool SINGLE, bool PRO = false>
void launch_wgrad_t(const Wgrad& a, hipStream_t s) {
  constexpr int lds = (SINGLE ? 1 : 2) * (WMW + WNW) * SUB * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)k_conv_wgrad<WMW, WNW, SINGLE, PRO>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int tiles = (a.K / (64 * WMW)) * ((a.TC + 64 * WNW - 1) / (64 * WNW));
  hipLaunchKernelGGL((k_conv_wgrad<WMW, WNW, SINGLE, PRO>), dim3(tiles * a.nsplit), dim3(64 * WMW * WNW), lds, s, a);
}

template <int WMW, int WNW>
void launch_wgrad(const Wgrad& a, int kind, hipStream_t s) {
  if (a.in_ss) return launch_wgrad_t<WMW, WNW, false, true>(a, s);
  if constexpr (WMW == 2 && WNW == 2) {
    if (kind == 1) {
      const int tiles = (a.K / (64 * WMW)) * ((a.TC + 64 * WNW - 1) / (64 * WNW));
      hipLaunchKernelGGL((k_conv_wgrad_glds<WMW, WNW, 1>), dim3(tiles * a.nsplit), dim3(256), 0, s, a);
      return;
    }
  }
  if (g_wgrad_single)
    launch_wgrad_t<WMW, WNW, true>(a, s);
  else
    launch_wgrad_t<WMW, WNW, false>(a, s);
}

template <int WMW, int WNW>
void launch_wgrad_glds(const Wgrad& a, hipStream_t s) {
  const int tiles = (a.K / (64 * WMW)) * ((a.TC + 64 * WNW - 1) / (64 * WNW));
  hipLaunchKernelGGL((k_conv_wgrad_glds<WMW, WNW>), dim3(tiles * a.nsplit), dim3(512), 0, s, a);
}

// tile shapes (waves along k, waves along tc); the 8-wave ones are the LDS-DMA ring kernel
constexpr int kTiles[][2] = {{1, 1}, {1, 2}, {2, 1}, {2, 2}, {1, 4}, {4, 1}, {2, 4}, {4, 2}};

}  // namespace

void conv_wgrad_force_single(bool single) { g_wgrad_single = single; }

bool conv_wgrad_supported(const ConvGeom& g) {
  return conv_bf16_supported(g) && (long long)g.N * g.OH * g.OW < (1ll << 24);
}

WgradPlan conv_wgrad_make_plan(const ConvGeom& g, int wmw, int wnw, int nsplit, int kind) {
  WgradPlan p{};
  p.wmw = wmw;
  p.wnw = wnw;
  p.kind = wmw == 2 && wnw == 2 ? kind : 0;
  const long long M = (long long)g.N * g.OH * g.OW;
  const int stages = (int)((M + RB - 1) / RB);
  const int S = std::max(1, std::min(nsplit, stages));
  const int per = (stages + S - 1) / S;
  p.chunk = per * RB;
  p.nsplit = (int)((M + p.chunk - 1) / p.chunk);
  p.ws_elems = (long long)p.nsplit * g.KH * g.KW * g.C * g.K;
  return p;
}

// Candidate plans, best first, from a roofline-style model: per tile shape and slice count,
// time = max(MFMA time at ~1 PF/s, HBM time for the operand bytes the tiles re-read at ~5 TB/s)
// stretched by the grid's tail (resident workgroups per CU from LDS and VGPRs), plus the partial
// slab written and re-read by the reduce.  The caller times the first few and keeps the fastest.
std::vector<WgradPlan> conv_wgrad_plans(const ConvGeom& g, int max_plans, bool in_bn) {
  struct Cand {
    double t;
    WgradPlan p;
  };
  std::vector<Cand> c;
  const long long M = (long long)g.N * g.OH * g.OW;
  const int TC = g.KH * g.KW * g.C;
  const int stages = (int)((M + RB - 1) / RB);
  for (int ti = 0; ti < (int)(sizeof(kTiles) / sizeof(kTiles[0])) * 2; ++ti) {
    const int wmw = kTiles[ti >> 1][0], wnw = kTiles[ti >> 1][1], bmk = 64 * wmw, btc = 64 * wnw;
    const int kind = ti & 1;  // 1: the single-stage LDS-DMA kernel (4-wave tiles only)
    if (kind && (wmw != 2 || wnw != 2)) continue;  // 1x4 / 4x1 spill at 128 VGPRs
    if (in_bn && (kind || wmw * wnw == 8)) continue;  // the input-side BN runs in the register staging
    if (g.K % bmk) continue;
    const int ntc = (TC + btc - 1) / btc;
    if ((ntc * btc - TC) * 4 > ntc * btc) continue;  // > 25 % of the tc columns padding
    const int tiles = (g.K / bmk) * ntc;
    const bool ring = wmw * wnw == 8;  // LDS-DMA ring kernel: one 144-KiB workgroup per CU
    const bool dma1 = kind == 1;
    const bool single = !ring && ((g_wgrad_single && !in_bn) || dma1);
    const int lds_kb = (ring ? 3 : (single ? 1 : 2)) * (wmw + wnw) * 8;
    // <= 2 waves per SIMD (3 for the single-stage v1 kernel, 4 for the single-stage DMA one)
    const int per_cu = std::max(1, std::min(160 / lds_kb, (dma1 ? 16 : single ? 12 : 8) / (wmw * wnw)));
    const double macs = (double)M * tiles * bmk * btc;
    // measured (profiles/conv_v2_r4.txt, wgrad_dma1_r4.txt): the LDS-DMA kernels win on 3x3 and
    // strided 1x1 shapes (the single-stage one most on 3x3) and lose on stride-1 1x1 ones (the v1
    // 2x2-wave tile), where their rates are scaled down
    const bool direct = g.KH == 1 && g.KW == 1 && g.SH == 1 && g.SW == 1 && g.PT == 0 && g.PL == 0;
    const double rate = ring ? (direct ? 0.85e15 : 1.3e15) : dma1 ? (direct ? 0.85e15 : 1.4e15) : 1.0e15;
    const double t_mma = macs * 2.0 / rate * 1e6;
    // dy re-read per tc tile, x per k tile (taps of one pixel neighbourhood hit L2: count once per tile)
    const double bytes = (double)M * 2.0 * ((double)g.K * ntc + (double)std::min(TC, btc) * ntc * (g.K / bmk));
    const double t_mem = bytes / 5.0e12 * 1e6;
    for (int S = 1; S <= std::min(stages, 8192); S = S < 8 ? S + 1 : S * 5 / 4) {
      const int per = (stages + S - 1) / S;
      const int Sr = (stages + per - 1) / per;
      const long long wgs = (long long)tiles * Sr;
      const double slots = 256.0 * per_cu;
      const double fill = std::min(1.0, wgs / slots);
      const double rounds = std::ceil(wgs / slots);
      const double eff = wgs / (rounds * slots);  // tail efficiency
      double t = std::max(t_mma, t_mem) / std::max(1e-3, fill * eff);
      t += rounds * 1.0;  // per-round prologue / epilogue
      if (Sr > 1) t += (double)Sr * TC * g.K * 8.0 / 4.0e12 * 1e6 + 2.0;
      c.push_back({t, conv_wgrad_make_plan(g, wmw, wnw, Sr, kind)});
    }
  }
  std::sort(c.begin(), c.end(), [](const Cand& x, const Cand& y) { return x.t < y.t; });
  // best first, but every kernel family (v1 register-staged, single-stage LDS-DMA, 8-wave LDS-DMA
  // ring) among the first candidates, round-robin in the order of each family's best plan: the model
  // ranks them only roughly, the autotuner's timing decides
  std::vector<WgradPlan> fam[3];
  int order[3], nf = 0;
  for (const auto& e : c) {
    const int fi = e.p.wmw * e.p.wnw == 8 ? 2 : e.p.kind;
    auto& f = fam[fi];
    if (f.empty()) order[nf++] = fi;
    bool dup = false;
    for (const auto& o : f) dup |= (o.wmw == e.p.wmw && o.wnw == e.p.wnw && o.nsplit == e.p.nsplit);
    if (!dup) f.push_back(e.p);
  }
  std::vector<WgradPlan> out;
  size_t idx[3] = {0, 0, 0};
  for (bool any = true; any && (int)out.size() < max_plans;) {
    any = false;
    for (int j = 0; j < nf && (int)out.size() < max_plans; ++j) {
      const int fi = order[j];
      if (idx[fi] < fam[fi].size()) {
        out.push_back(fam[fi][idx[fi]++]);
        any = true;
      }
    }
  }
  return out;
}

void conv_wgrad_bf16(const void* x, const void* dy, float* ws, const WgradPlan& p, void* dw_bf16, float* dw_f32,
                     bool accumulate, const ConvGeom& g, hipStream_t s, const float* in_ss) {
  Wgrad a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(dy), ws,
          g.N, g.H, g.W, g.C, g.OH, g.OW, g.K, g.KH, g.KW, g.SH, g.SW, g.PT, g.PL,
          g.N * g.OH * g.OW, g.KH * g.KW * g.C, p.chunk, p.nsplit,
          (g.KH == 1 && g.KW == 1 && g.SH == 1 && g.SW == 1 && g.PT == 0 && g.PL == 0 && g.H == g.OH && g.W == g.OW)
              ? 1 : 0,
          1.0f / (float)g.OW, 1.0f / (float)g.OH};
  a.in_ss = in_ss;
  if (in_ss && (!a.direct || p.kind != 0 || p.wmw * p.wnw > 4)) return;  // (the caller checks)
  const int t = p.wmw * 8 + p.wnw;
  switch (t) {
    case 9: launch_wgrad<1, 1>(a, p.kind, s); break;
    case 10: launch_wgrad<1, 2>(a, p.kind, s); break;
    case 17: launch_wgrad<2, 1>(a, p.kind, s); break;
    case 18: launch_wgrad<2, 2>(a, p.kind, s); break;
    case 12: launch_wgrad<1, 4>(a, p.kind, s); break;
    case 33: launch_wgrad<4, 1>(a, p.kind, s); break;
    case 20: launch_wgrad_glds<2, 4>(a, s); break;
    case 34: launch_wgrad_glds<4, 2>(a, s); break;
    default: return;
  }
  const long long n4 = (long long)a.TC * a.K / 4;
  const int G = std::min(16, p.nsplit);
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((n4 + 63) / 64)), dim3(64 * G), 0, s, ws, n4, p.nsplit,
                     static_cast<uint16_t*>(dw_bf16), dw_f32, accumulate ? 1 : 0);
}

}  // namespace tdl
