// Weight gradient of a 3x3, stride-1, pad-1 NHWC bf16 convolution with 64 input channels (the
// ResNet-50 stage-1 3x3 conv, 56x56x64 -> 64), on the gfx950 bf16 matrix cores (see conv.h).
//
// The split-K kernel of conv_wgrad.hip tiles the (kh, kw, c) axis in 64-column chunks per tap and
// re-stages the shifted image for every tap; with only 64 channels its partial slab (one 576 x 64
// f32 tile per pixel slice) outweighs the GEMM, and MIOpen ran this shape 2x faster.  Here a
// workgroup walks whole OUTPUT ROWS: per row it stages dy[row][0..OW) (64 channels) and the three
// input rows oh-1 .. oh+1 with one zero pixel on each side (zeros for rows outside the image), so
// every one of the nine taps is the same LDS image read at a row / pixel offset -- no im2col, no
// per-tap restaging.  MFMA (16x16x32, reduction = 32 pixels of the row): A = dy^T (rows = output
// channels k), B = x^T (columns = input channels c of one tap); both fragments need 8 consecutive
// pixels of one channel per lane: gfx950 transpose reads (ds_read_b64_tr_b16) of the pixel-major
// images, the tap shift being a plain row offset.  The whole 9 x 64 x 64 tile stays in the
// accumulators of the 4 waves (wave w: column blocks w, w + 4, ... of the 36 (tap, c-block) blocks,
// all 4 k blocks) across the workgroup's rows; slice partials go to a slab reduced in slice order
// by a second kernel (deterministic).
#include "kernels/conv.h"

#include "kernels/common.h"

#include <algorithm>

namespace tdl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kMaxOW = 64;          // output row length the images hold (padded to 2 k-steps of 32)
constexpr int kXW = kMaxOW + 8;     // input pixels per staged row: 1 zero pixel left, OW + 1, padding
constexpr int kLd = 64 + 8;         // bf16 per pixel row of the LDS images (16-B pad)
constexpr int kBlocks = 9 * 4;      // (tap, 16-channel c block) column blocks
constexpr int kPerWave = kBlocks / 4;

struct W3 {
  const uint16_t* x;   // [N][H][W][64]
  const uint16_t* dy;  // [N][H][W][K] (stride 1, same size)
  float* ws;           // [slices][9 * 64][K] partials
  int N, H, W, K;
  int rows_per_slice, slices;
};

// lane's transposed fragment: pixels p0 .. p0+7 (rows of the pixel-major image) of columns
// c16 .. c16 + 15; lane i of each 16-lane group receives column c16 + i (every lane active)
__device__ __forceinline__ bf16x8 tr8(const uint16_t* img, int p0, int c16, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const uint16_t* a0 = img + (p0 + q) * kLd + c16 + 4 * p;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0 + 4 * kLd));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// grid: (slices, K / 64); 256 threads
__global__ __launch_bounds__(256, 1) void k_wgrad3x3_c64(W3 a) {
  __shared__ __attribute__((aligned(16))) uint16_t dl[kMaxOW * kLd];     // dy row: [pixel][k]
  __shared__ __attribute__((aligned(16))) uint16_t xl[3 * kXW * kLd];     // 3 input rows: [r][pixel][c]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int qq = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
  const int sl = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
  const int tn = blockIdx.y;
  const int OW = a.W;
  const long long row0 = (long long)sl * a.rows_per_slice;
  const long long row1 = min((long long)a.N * a.H, row0 + a.rows_per_slice);

  f4v acc[kPerWave][4];  // [this wave's column block j][k block i]
#pragma unroll
  for (int j = 0; j < kPerWave; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f4v{0.f, 0.f, 0.f, 0.f};

  // staging roles: dy: 64 px x 8 chunks = 512 (2 per thread); x: 3 rows x kXW px x 8 chunks; the
  // next row's global loads are in flight in registers while this row's MFMAs run
  constexpr int kXChunks = 3 * kXW * 8;
  constexpr int kXPer = (kXChunks + 255) / 256;
  u32x4 pd[2], pxv[kXPer];
  auto gload = [&](long long row) {
    const int oh = (int)(row % a.H);
    const long long n = row / a.H;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int s = tid + 256 * u, px = s >> 3, ch = s & 7;
      pd[u] = px < OW ? *reinterpret_cast<const u32x4*>(a.dy + ((n * a.H + oh) * a.W + px) * a.K + tn * 64 + ch * 8)
                      : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
      const int s = tid + 256 * u;
      const int ch = s & 7, px = (s >> 3) % kXW, r = (s >> 3) / kXW;
      const int ih = oh + r - 1, iw = px - 1;
      pxv[u] = (s < kXChunks && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W)
                   ? *reinterpret_cast<const u32x4*>(a.x + ((n * a.H + ih) * a.W + iw) * 64 + ch * 8)
                   : u32x4{0u, 0u, 0u, 0u};
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int s = tid + 256 * u, px = s >> 3, ch = s & 7;
      *reinterpret_cast<u32x4*>(dl + px * kLd + ch * 8) = pd[u];
    }
#pragma unroll
    for (int u = 0; u < kXPer; ++u) {
      const int s = tid + 256 * u;
      if (s < kXChunks) {
        const int ch = s & 7, px = (s >> 3) % kXW, r = (s >> 3) / kXW;
        *reinterpret_cast<u32x4*>(xl + (r * kXW + px) * kLd + ch * 8) = pxv[u];
      }
    }
  };
  if (row0 < row1) gload(row0);
  for (long long row = row0; row < row1; ++row) {
    sstore();
    __syncthreads();
    if (row + 1 < row1) gload(row + 1);
#pragma unroll
    for (int kk = 0; kk < kMaxOW; kk += 32) {
      if (kk >= OW) break;  // workgroup-uniform
      const int p0 = kk + 8 * (lane >> 4);  // this lane group's 8 output pixels
      bf16x8 fd[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fd[i] = tr8(dl, p0, i * 16, lane);
#pragma unroll
      for (int j = 0; j < kPerWave; ++j) {
        const int blk = wave + 4 * j, tap = blk >> 2, cb = blk & 3;
        const int kh = tap / 3, kw = tap % 3;
        // output pixel ow reads input pixel ow + kw - 1 = staged pixel ow + kw of row kh
        const bf16x8 fx = tr8(xl + kh * kXW * kLd, p0 + kw, cb * 16, lane);
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx, acc[j][i], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // acc[j][i]: output channels k = 16 i + 4 (lane >> 4) .. +3 (MFMA result rows) of input channel
  // c = 16 cb + (lane & 15) of tap `tap`; slab layout [slice][tap * 64 + c][K] (HWIO order)
  float* w = a.ws + (long long)sl * 9 * 64 * a.K;
#pragma unroll
  for (int j = 0; j < kPerWave; ++j) {
    const int blk = wave + 4 * j, tap = blk >> 2, cb = blk & 3;
    const int tc = tap * 64 + cb * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<f4v*>(w + (long long)tc * a.K + tn * 64 + i * 16 + (lane >> 4) * 4) = acc[j][i];
  }
}

// out[e] (= [tc][K], HWIO) = sum of the slice partials in slice order; 4 interleaved phases per
// element combined in a fixed order.  bf16 out, or f32 (added to when acc)
__global__ __launch_bounds__(256) void k_wgrad3x3_reduce(const float* __restrict__ ws, int slices, int n,
                                                         float* __restrict__ out_f32, uint16_t* __restrict__ out_bf16,
                                                         int acc) {
  __shared__ float red[4][64];
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  float s = 0.f;
  if (e < n) {
#pragma unroll 4
    for (int sl = ph; sl < slices; sl += 4) s += ws[(long long)sl * n + e];
  }
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph != 0 || e >= n) return;
  const int t = threadIdx.x;
  s = ((red[0][t] + red[1][t]) + red[2][t]) + red[3][t];
  if (out_f32) {
    out_f32[e] = acc ? out_f32[e] + s : s;
  } else {
    uint32_t u = __float_as_uint(s);
    u += 0x7fffu + ((u >> 16) & 1u);
    out_bf16[e] = (uint16_t)(u >> 16);
  }
}

int g_w3_rows = 0;  // rows per slice override (A/B sweeps); 0: heuristic

}  // namespace

bool conv_wgrad3x3_c64_supported(const ConvGeom& g) {
  return g.C == 64 && g.K % 64 == 0 && g.KH == 3 && g.KW == 3 && g.SH == 1 && g.SW == 1 && g.PT == 1 &&
         g.PL == 1 && g.OH == g.H && g.OW == g.W && g.W <= kMaxOW && g.W >= 1 &&
         (long long)g.N * g.H * g.W * g.K < (1LL << 31);
}

void conv_wgrad3x3_set_rows(int rows) { g_w3_rows = rows; }

static int w3_rows(const ConvGeom& g) {
  if (g_w3_rows > 0) return g_w3_rows;
  // one workgroup per CU (1 resident each: the 9x64x64 partial tile lives in registers)
  const long long rows = (long long)g.N * g.H;
  const long long target = 256LL / (g.K / 64);  // one slice per CU: 56 rows at b=256 (rows 28: +8 %, 112: +70 %)
  return (int)std::max<long long>(1, (rows + target - 1) / target);
}

long long conv_wgrad3x3_c64_ws_elems(const ConvGeom& g) {
  const long long rows = (long long)g.N * g.H;
  const long long slices = (rows + w3_rows(g) - 1) / w3_rows(g);
  return slices * 9 * 64 * g.K;
}

void conv_wgrad3x3_c64(const void* x, const void* dy, float* ws, void* dw_bf16, float* dw_f32, bool accumulate,
                       const ConvGeom& g, hipStream_t s) {
  W3 a{static_cast<const uint16_t*>(x), static_cast<const uint16_t*>(dy), ws, g.N, g.H, g.W, g.K, w3_rows(g), 0};
  const long long rows = (long long)g.N * g.H;
  a.slices = (int)((rows + a.rows_per_slice - 1) / a.rows_per_slice);
  hipLaunchKernelGGL(k_wgrad3x3_c64, dim3(a.slices, g.K / 64), dim3(256), 0, s, a);
  const int n = 9 * 64 * g.K;
  hipLaunchKernelGGL(k_wgrad3x3_reduce, dim3((n + 63) / 64), dim3(256), 0, s, ws, a.slices, n, dw_f32,
                     static_cast<uint16_t*>(dw_bf16), accumulate ? 1 : 0);
}

}  // namespace tdl
