// Small-channel stride-2 convolution (the ResNet-50 stem: 7x7, stride 2, 3 input channels) on the
// gfx950 bf16 matrix cores (see stem.h).
//
// The implicit-GEMM kernels of conv.hip reduce over 64-channel chunks of one filter tap, which a
// 3-channel image cannot fill (MIOpen's igemm_fwd ran this layer at ~170 TFLOP/s, 358 us per step at
// b=256).  Here the image is first packed into a zero-bordered NHWC4 copy xp (channel 3 = 0; the
// preceding ZeroPadding2D is folded into the border), so that for one output pixel and one filter
// row kh the receptive field of 8 taps x 4 channels is 32 CONTIGUOUS bf16 = 64 bytes, 16-B aligned
// whenever the column stride is even.  The GEMM reduction then runs in KH steps of exactly one
// v_mfma_f32_16x16x32_bf16 k-depth (taps 7..KW and channel 3 carry zero weights), and every lane
// loads its MFMA operand fragment (2 pixels x 4 channels = 16 B) straight from global memory: no
// LDS staging of the image at all.  The packed weights (K x KH x 32, 28 KiB for the stem) live in
// LDS for the whole workgroup.
//
// Workgroup: 4 waves x 64 output pixels, all K (= 64 per column tile) output channels; each wave
// 4 x 4 MFMA tiles (the weight fragment is the A operand, so a lane's 4 accumulators are 4
// adjacent channels of one pixel).  Epilogue: bf16 tile through LDS, 16-B row segments to y, and
// the following batch norm's per-tile channel sums of y and y^2 (the same [tiles][2][K] partial
// layout as conv_fwd_bf16's, bn_forward_train(part=...)).
//
// Weight gradient: dW[k][kh][t] = sum over pixels of dy[m][k] * xp(m, kh, t), the reduction over
// pixels.  A workgroup takes a slice of pixels: dy (64 channels) and the 8 x 4 receptive-field
// rows are staged into LDS as they arrive and the MFMA operands (8 consecutive pixels of one
// channel / tap) are read back with the gfx950 transpose read ds_read_b64_tr_b16; the f32 slice
// partials are summed in slice order by a second kernel (deterministic).
#include "kernels/stem.h"

#include "kernels/common.h"

namespace tdl {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int kTaps = 32;  // 8 filter columns x 4 channels per filter row

__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even (finite values)
  return (uint16_t)(u >> 16);
}

// x [N][H][W][C] (f32 or bf16) -> xp [N][HP][WP][4] bf16: pixel (h, w) of x at (h + PT, w + PL),
// zeros elsewhere and in channels C..3.  One thread per xp pixel (one 8-byte store).
template <typename T>
__global__ __launch_bounds__(256) void k_stem_pack(const T* __restrict__ x, uint2* __restrict__ xp, int N, int H,
                                                   int W, int C, int HP, int WP, int PT, int PL) {
  const long long total = (long long)N * HP * WP;
  for (long long p = (long long)blockIdx.x * 256 + threadIdx.x; p < total; p += (long long)gridDim.x * 256) {
    const int wp = (int)(p % WP);
    const long long t = p / WP;
    const int hp = (int)(t % HP), n = (int)(t / HP);
    const int h = hp - PT, w = wp - PL;
    uint16_t v[4] = {0, 0, 0, 0};
    if ((unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W) {
      const T* s = x + (((long long)n * H + h) * W + w) * C;
      for (int c = 0; c < C; ++c) {
        if constexpr (sizeof(T) == 2)
          v[c] = reinterpret_cast<const uint16_t*>(s)[c];
        else
          v[c] = f2bf((float)s[c]);
      }
    }
    xp[p] = make_uint2(v[0] | ((uint32_t)v[1] << 16), v[2] | ((uint32_t)v[3] << 16));
  }
}

// w_hwio [KH][KW][C][K] bf16 -> wp [K][KH][32] bf16 (tap t = kw * 4 + c; zeros for kw >= KW, c >= C)
__global__ __launch_bounds__(256) void k_stem_wpack(const uint16_t* __restrict__ w, uint16_t* __restrict__ wp, int KH,
                                                    int KW, int C, int K) {
  const int total = K * KH * kTaps;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int t = i % kTaps, kh = (i / kTaps) % KH, k = i / (kTaps * KH);
    const int kw = t >> 2, c = t & 3;
    wp[i] = (kw < KW && c < C) ? w[((kh * KW + kw) * C + c) * K + k] : (uint16_t)0;
  }
}

struct StemArgs {
  const uint16_t* xp;  // [N][HP][WP][4]
  const uint16_t* wp;  // [K][KH][32]
  uint16_t* y;         // [N][OH][OW][K]
  float* stats;        // optional [tiles][2][K]
  int N, HP, WP, OH, OW, K, KH, SH;
  int M;
};

constexpr int kMaxKH = 8;
constexpr int kRows = 256;  // output pixels per workgroup (4 waves x 64)
constexpr int kOutLd = 64 + 8;

// grid: (ceil(M / 256), K / 64)
__global__ __launch_bounds__(256, 2) void k_stem_fwd(StemArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t wl[64 * kMaxKH * kTaps];  // this column tile's weights
  __shared__ __attribute__((aligned(16))) uint16_t tile[kRows * kOutLd];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware remap of the row tiles (a row tile's neighbours share input rows: keep them on one L2)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7;
  const int tm = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
  const int tn = blockIdx.y;
  const int KH = a.KH;

  {  // weights of output channels [64 tn, 64 tn + 64)
    const u32x4* src = reinterpret_cast<const u32x4*>(a.wp + (long long)tn * 64 * KH * kTaps);
    u32x4* dst = reinterpret_cast<u32x4*>(wl);
    for (int i = tid; i < 64 * KH * kTaps / 8; i += 256) dst[i] = src[i];
  }

  // this lane's 4 operand rows (pixels): element offset of their receptive field's top-left tap
  const int kg = lane >> 4;  // k group: taps 8 kg .. 8 kg + 7 = filter columns 2 kg, 2 kg + 1
  long long base[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    int m = tm * kRows + wave * 64 + i * 16 + (lane & 15);
    m = m < a.M ? m : a.M - 1;  // rows past M: read a valid pixel, never stored
    const int ow = m % a.OW, t = m / a.OW, oh = t % a.OH, n = t / a.OH;
    base[i] = (((long long)n * a.HP + (long long)oh * a.SH) * a.WP + 2LL * ow) * 4 + kg * 8;
  }
  // every filter row's fragments issued up front (KH x 4 independent 16-B loads in flight)
  u32x4 fa[kMaxKH][4];
#pragma unroll
  for (int kh = 0; kh < kMaxKH; ++kh)
    if (kh < KH)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        fa[kh][i] = *reinterpret_cast<const u32x4*>(a.xp + base[i] + (long long)kh * a.WP * 4);
  __syncthreads();  // weights in LDS

  f4v acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kh = 0; kh < kMaxKH; ++kh) {
    if (kh >= KH) break;
    bf16x8 fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(wl + ((j * 16 + (lane & 15)) * KH + kh) * kTaps + kg * 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16x8 av = __builtin_bit_cast(bf16x8, fa[kh][i]);
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], av, acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: lane holds channels 16 j + 4 kg .. +3 of pixel row 16 i + (lane & 15)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      const uint32_t hi = f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
      *reinterpret_cast<uint2*>(tile + (wave * 64 + i * 16 + (lane & 15)) * kOutLd + j * 16 + kg * 4) =
          make_uint2(lo, hi);
    }
  __syncthreads();
  // 8 16-B segments per 64-channel row; thread: segment tid & 7 of rows tid >> 3 + 32 e
  const int seg = tid & 7, r0 = tid >> 3;
  float cs[8], cq[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) cs[j] = cq[j] = 0.f;
#pragma unroll
  for (int e = 0; e < kRows / 32; ++e) {
    const int row = r0 + 32 * e, m = tm * kRows + row;
    if (m < a.M) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(tile + row * kOutLd + seg * 8);
      *reinterpret_cast<u32x4*>(a.y + (long long)m * a.K + tn * 64 + seg * 8) = v;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float lo = __uint_as_float(v[j] << 16), hi = __uint_as_float(v[j] & 0xffff0000u);
        cs[2 * j] += lo;
        cq[2 * j] = fmaf(lo, lo, cq[2 * j]);
        cs[2 * j + 1] += hi;
        cq[2 * j + 1] = fmaf(hi, hi, cq[2 * j + 1]);
      }
    }
  }
  if (a.stats == nullptr) return;
  // fixed-order reduction over the 32 threads of each segment (deterministic), through LDS
  __syncthreads();
  float* red = reinterpret_cast<float*>(tile);  // [2][32][64]
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[r0 * 64 + seg * 8 + j] = cs[j];
    red[32 * 64 + r0 * 64 + seg * 8 + j] = cq[j];
  }
  __syncthreads();
  if (tid < 64) {
    float S = 0.f, Q = 0.f;
    for (int g = 0; g < 32; ++g) {
      S += red[g * 64 + tid];
      Q += red[32 * 64 + g * 64 + tid];
    }
    a.stats[((long long)tm * 2) * a.K + tn * 64 + tid] = S;
    a.stats[((long long)tm * 2 + 1) * a.K + tn * 64 + tid] = Q;
  }
}

// ---- weight gradient ----
// Workgroup: one slice of kWgPix pixels in chunks of kChunk; 4 waves.  Per chunk, LDS holds
// dy [kChunk px][64 ch] and the receptive-field rows xr [kChunk px][KH][32 taps] as loaded
// (pixel-major; the next chunk's global loads are in flight in registers while this one computes).
// MFMA (16x16x32, reduction = 32 pixels): A = dy^T (rows = output channels), B = xr (columns =
// (kh, tap)); both fragments need 8 consecutive pixels of one channel / tap: transposed reads.
// Output tile per workgroup: 64 channels x KH*32 columns; wave w takes column blocks w, w+4, ...
// (KH*2 blocks of 16 columns: 14 for KH = 7, so waves 0-1 take 4 and waves 2-3 take 3).
constexpr int kWgPix = 4096;
constexpr int kChunk = 64;
constexpr int kXrLd = kMaxKH * kTaps + 8;  // bf16 per pixel row of the xr image (pad: 16 B)
constexpr int kDyLd = 64 + 8;
constexpr int kXrLoads = (kChunk * kMaxKH * 4 + 255) / 256;  // 16-B xr chunks per thread (max)
constexpr int kDyLoads = kChunk * 8 / 256;

struct StemWgrad {
  const uint16_t* xp;
  const uint16_t* dy;  // [M][K]
  float* ws;           // [slices][K][KH*32] partials
  int N, HP, WP, OH, OW, K, KH, SH;
  int M, slices;
};

// transposed fragment: 8 consecutive rows (pixels) r0 .. r0+7 of columns c16 .. c16+15 of a
// row-major bf16 image with row stride ld (elements), as two 4-row ds_read_b64_tr_b16 blocks: lane
// 4q+p of each 16-lane group addresses row r0 + q (+4), columns c16 + 4p .. +3; lane i of the group
// receives column c16 + i (every lane active: the gather crosses lanes)
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* img, int ld, int r0, int c16, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const uint16_t* a0 = img + (r0 + q) * ld + c16 + 4 * p;
  const uint16_t* a1 = a0 + 4 * ld;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a0));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(a1));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// grid: (slices, K / 64)
__global__ __launch_bounds__(256, 2) void k_stem_wgrad(StemWgrad a) {
  __shared__ __attribute__((aligned(16))) uint16_t xr[kChunk * kXrLd];
  __shared__ __attribute__((aligned(16))) uint16_t dl[kChunk * kDyLd];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware: consecutive slices (neighbouring image rows) on one XCD
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int qq = nwg >> 3, rr = nwg & 7, xcd = orig & 7;
  const int sl = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (orig >> 3);
  const int tn = blockIdx.y;
  const int KH = a.KH, NB = KH * 2;  // 16-column blocks of the (kh, tap) axis
  const int nx = kChunk * KH * 4;    // xr 16-B chunks per pixel chunk
  const long long p0 = (long long)sl * kWgPix;
  const long long p1 = min((long long)a.M, p0 + kWgPix);

  // each thread stages fixed (pixel-in-chunk, kh, part) items; its pixels' (n, oh, ow) advance by
  // kChunk per chunk without divisions (kChunk < OW wraps at most once... or loops)
  int xpx[kXrLoads], xoff[kXrLoads], xn[kXrLoads], xoh[kXrLoads], xow[kXrLoads];
#pragma unroll
  for (int u = 0; u < kXrLoads; ++u) {
    const int s = tid + 256 * u;
    const int px = s < nx ? s / (KH * 4) : 0, rem = s < nx ? s - px * (KH * 4) : 0;
    xpx[u] = s < nx ? px : -1;
    xoff[u] = ((rem >> 2) * a.WP) * 4 + (rem & 3) * 8;  // kh rows down, part * 8 elements across
    const long long m = p0 + px;
    xow[u] = (int)(m % a.OW);
    const long long t = m / a.OW;
    xoh[u] = (int)(t % a.OH);
    xn[u] = (int)(t / a.OH);
  }
  u32x4 rd[kDyLoads], rx[kXrLoads];
  auto gload = [&](long long c0) {
#pragma unroll
    for (int u = 0; u < kDyLoads; ++u) {
      const int s = tid + 256 * u, px = s >> 3, ch = s & 7;
      const long long m = c0 + px;
      rd[u] = m < p1 ? *reinterpret_cast<const u32x4*>(a.dy + m * a.K + tn * 64 + ch * 8) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < kXrLoads; ++u) {
      rx[u] = u32x4{0u, 0u, 0u, 0u};
      if (xpx[u] >= 0 && c0 + xpx[u] < p1) {
        const long long off = (((long long)xn[u] * a.HP + (long long)xoh[u] * a.SH) * a.WP + 2LL * xow[u]) * 4 + xoff[u];
        rx[u] = *reinterpret_cast<const u32x4*>(a.xp + off);
      }
      // advance this item's pixel by one chunk
      xow[u] += kChunk;
      while (xow[u] >= a.OW) {
        xow[u] -= a.OW;
        if (++xoh[u] == a.OH) {
          xoh[u] = 0;
          ++xn[u];
        }
      }
    }
  };
  auto sstore = [&]() {
#pragma unroll
    for (int u = 0; u < kDyLoads; ++u) {
      const int s = tid + 256 * u, px = s >> 3, ch = s & 7;
      *reinterpret_cast<u32x4*>(dl + px * kDyLd + ch * 8) = rd[u];
    }
#pragma unroll
    for (int u = 0; u < kXrLoads; ++u) {
      const int s = tid + 256 * u;
      if (s < nx) {
        const int px = xpx[u], rem = s - px * (KH * 4);
        *reinterpret_cast<u32x4*>(xr + px * kXrLd + rem * 8) = rx[u];  // rem * 8 = kh * 32 + part * 8
      }
    }
  };

  f4v acc[4][4];  // [channel block i][this wave's column block jj]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4v{0.f, 0.f, 0.f, 0.f};

  gload(p0);
  for (long long c0 = p0; c0 < p1; c0 += kChunk) {
    sstore();
    __syncthreads();
    if (c0 + kChunk < p1) gload(c0 + kChunk);  // next chunk in flight during the MFMAs
#pragma unroll
    for (int kk = 0; kk < kChunk; kk += 32) {
      const int pr = kk + 8 * (lane >> 4);  // this lane group's 8 pixels
      bf16x8 fd[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fd[i] = tr_frag(dl, kDyLd, pr, i * 16, lane);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int jb = wave + 4 * jj;
        if (jb < NB) {  // wave-uniform
          const bf16x8 fx = tr_frag(xr, kXrLd, pr, jb * 16, lane);
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fd[i], fx, acc[i][jj], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  // partial tile: acc[i][jj] holds output channels 16 i + 4 (lane >> 4) .. +3 (the MFMA result
  // rows) of column jb * 16 + (lane & 15)
  const int TC = KH * kTaps;
  float* w = a.ws + ((long long)sl * a.K + tn * 64) * TC;
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    const int jb = wave + 4 * jj;
    if (jb >= NB) continue;
    const int col = jb * 16 + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) w[(long long)(i * 16 + (lane >> 4) * 4 + e) * TC + col] = acc[i][jj][e];
  }
}

// dW: sum the slice partials in slice order (4 interleaved phases per column, combined in a fixed
// order: deterministic).  Workgroup: 64 consecutive (k, col) entries of the [K][KH*32] layout.
// out: HWIO [KH][KW][C][K], f32 (added to when acc) or bf16; columns with kw >= KW or c >= C dropped.
__global__ __launch_bounds__(256) void k_stem_wgrad_reduce(const float* __restrict__ ws, int slices, int K, int KH,
                                                           int KW, int C, float* __restrict__ out_f32,
                                                           uint16_t* __restrict__ out_bf16, int acc) {
  __shared__ float red[4][64];
  const int TC = KH * kTaps;
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), ph = threadIdx.x >> 6;
  const long long stride = (long long)K * TC;
  float s = 0.f;
  if (e < K * TC) {
#pragma unroll 4
    for (int sl = ph; sl < slices; sl += 4) s += ws[sl * stride + e];
  }
  red[ph][threadIdx.x & 63] = s;
  __syncthreads();
  if (ph != 0 || e >= K * TC) return;
  s = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) + red[3][threadIdx.x];
  const int k = e / TC, col = e % TC, kh = col / kTaps, kw = (col % kTaps) >> 2, c = col & 3;
  if (kw >= KW || c >= C) return;
  const long long o = (((long long)kh * KW + kw) * C + c) * K + k;
  if (out_f32)
    out_f32[o] = acc ? out_f32[o] + s : s;
  else
    out_bf16[o] = f2bf(s);
}

}  // namespace

bool stem_supported(int C, int KH, int KW, int SW, int K) {
  return C >= 1 && C <= 4 && KH >= 1 && KH <= kMaxKH && KW >= 1 && KW <= 8 && SW == 2 && K % 64 == 0;
}

void stem_pack(const void* x, bool x_bf16, void* xp, int N, int H, int W, int C, int HP, int WP, int PT, int PL,
               hipStream_t s) {
  const long long total = (long long)N * HP * WP;
  const int grid = (int)std::min<long long>((total + 255) / 256, 256LL * 32);
  if (x_bf16)
    hipLaunchKernelGGL(k_stem_pack<uint16_t>, dim3(grid), dim3(256), 0, s, static_cast<const uint16_t*>(x),
                       static_cast<uint2*>(xp), N, H, W, C, HP, WP, PT, PL);
  else
    hipLaunchKernelGGL(k_stem_pack<float>, dim3(grid), dim3(256), 0, s, static_cast<const float*>(x),
                       static_cast<uint2*>(xp), N, H, W, C, HP, WP, PT, PL);
}

void stem_wpack(const void* w_hwio, void* wp, int KH, int KW, int C, int K, hipStream_t s) {
  const int total = K * KH * kTaps;
  hipLaunchKernelGGL(k_stem_wpack, dim3((total + 255) / 256), dim3(256), 0, s, static_cast<const uint16_t*>(w_hwio),
                     static_cast<uint16_t*>(wp), KH, KW, C, K);
}

int stem_fwd_row_tile() { return kRows; }

void stem_fwd(const void* xp, const void* wp, void* y, float* stats, int N, int HP, int WP, int OH, int OW, int K,
              int KH, int SH, hipStream_t s) {
  StemArgs a{static_cast<const uint16_t*>(xp), static_cast<const uint16_t*>(wp), static_cast<uint16_t*>(y), stats,
             N, HP, WP, OH, OW, K, KH, SH, N * OH * OW};
  hipLaunchKernelGGL(k_stem_fwd, dim3((a.M + kRows - 1) / kRows, K / 64), dim3(256), 0, s, a);
}

long long stem_wgrad_ws_elems(int M, int K, int KH) {
  const long long slices = (M + kWgPix - 1) / kWgPix;
  return slices * K * KH * kTaps;
}

void stem_wgrad(const void* xp, const void* dy, float* ws, int N, int HP, int WP, int OH, int OW, int K, int KH, int KW,
                int C, int SH, float* dw_f32, void* dw_bf16, bool accumulate, hipStream_t s) {
  StemWgrad a{static_cast<const uint16_t*>(xp), static_cast<const uint16_t*>(dy), ws, N, HP, WP, OH, OW, K, KH, SH,
              N * OH * OW, 0};
  a.slices = (a.M + kWgPix - 1) / kWgPix;
  hipLaunchKernelGGL(k_stem_wgrad, dim3(a.slices, K / 64), dim3(256), 0, s, a);
  const int n = K * KH * kTaps;
  hipLaunchKernelGGL(k_stem_wgrad_reduce, dim3((n + 63) / 64), dim3(256), 0, s, ws, a.slices, K, KH, KW, C, dw_f32,
                     static_cast<uint16_t*>(dw_bf16), accumulate ? 1 : 0);
}

}  // namespace tdl
