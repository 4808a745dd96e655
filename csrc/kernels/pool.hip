// NHWC max pooling on gfx950, bf16 / f32, 8 channels (16 B of bf16) per thread.
//
// forward : y = max over the window; arg = window position of the (first) maximum per element
//           (255 when an implicit zero-padding element won).  Padding is either -inf (TF 'same'
//           max pool) or zero (a fused ZeroPadding2D in front, the ResNet stem).
// backward: gather form — each input element sums dy over the <= ceil(k/s)^2 windows whose
//           argmax points at it: no atomics, deterministic, one pass over dx.
#include <cstdlib>

#include "common.h"
#include "pool.h"

namespace tdl {
namespace {

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

template <bool BF>
__device__ __forceinline__ void ld8(const void* p, int64_t e, float* o) {
  if (BF) {
    const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + e);
    o[0] = bf_lo(u.x); o[1] = bf_hi(u.x); o[2] = bf_lo(u.y); o[3] = bf_hi(u.y);
    o[4] = bf_lo(u.z); o[5] = bf_hi(u.z); o[6] = bf_lo(u.w); o[7] = bf_hi(u.w);
  } else {
    const f4* q = reinterpret_cast<const f4*>(static_cast<const float*>(p) + e);
    const f4 a = q[0], b = q[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
}

template <bool BF>
__device__ __forceinline__ void st8(void* p, int64_t e, const float* v) {
  if (BF) {
    uint4 u;
    u.x = f2bf(v[0]) | (f2bf(v[1]) << 16);
    u.y = f2bf(v[2]) | (f2bf(v[3]) << 16);
    u.z = f2bf(v[4]) | (f2bf(v[5]) << 16);
    u.w = f2bf(v[6]) | (f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + e) = u;
  } else {
    f4* q = reinterpret_cast<f4*>(static_cast<float*>(p) + e);
    q[0] = f4{v[0], v[1], v[2], v[3]};
    q[1] = f4{v[4], v[5], v[6], v[7]};
  }
}

// K3S2: the 3x3 stride-2 window of ResNet (compile-time loops: every tap's load issued before the
// compares, and at most 2 x 2 windows per input element in the backward, all four loads at once).
// Same compare / sum order as the generic loops: bit-identical results.
// BNF: the input is a batch norm's input x and the pooled values are relu(x * scale + shift) rounded to
// bf16 (bn_ss = scale[C], shift[C]): the BN -> ReLU pass and its output tensor are skipped.
template <bool BF>
__device__ __forceinline__ void bn_relu8(float* v, const float* sc, const float* sh) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float o = fmaxf(fmaf(v[j], sc[j], sh[j]), 0.f);
    v[j] = BF ? __uint_as_float(f2bf(o) << 16) : o;  // the value the BN pass would have stored
  }
}

template <bool BF, bool K3S2, bool BNF = false>
__global__ __launch_bounds__(256) void k_maxpool_fwd(const void* __restrict__ x, void* __restrict__ y,
                                                     uint8_t* __restrict__ arg, PoolGeom g,
                                                     const float* __restrict__ bn_ss = nullptr) {
  const int G = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.OH * g.OW * G;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int cg = (int)(t % G);
    int64_t r = t / G;
    const int ow = (int)(r % g.OW);
    r /= g.OW;
    const int oh = (int)(r % g.OH);
    const int n = (int)(r / g.OH);
    float best[8];
    uint32_t am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = -INFINITY;
      am[j] = 255;
    }
    float bsc[BNF ? 8 : 1], bsh[BNF ? 8 : 1];  // this channel group's BN scale / shift (once per element)
    if constexpr (BNF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bsc[j] = bn_ss[cg * 8 + j];
        bsh[j] = bn_ss[g.C + cg * 8 + j];
      }
    }
    if constexpr (K3S2) {
      float v[9][8];
      bool in[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int h = oh * 2 - g.pt + i, w = ow * 2 - g.pl + k, q = i * 3 + k;
          in[q] = h >= 0 && h < g.H && w >= 0 && w < g.W;
          if (in[q]) {
            ld8<BF>(x, (((int64_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v[q]);
            if constexpr (BNF) bn_relu8<BF>(v[q], bsc, bsh);
          } else {
#pragma unroll
            for (int j = 0; j < 8; ++j) v[q][j] = g.pad_zero ? 0.f : -INFINITY;
          }
        }
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        if (!in[q] && !g.pad_zero) continue;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[q][j] > best[j]) {
            best[j] = v[q][j];
            am[j] = in[q] ? (uint32_t)q : 255u;
          }
      }
    }
    for (int i = 0; i < (K3S2 ? 0 : g.kh); ++i) {
      const int h = oh * g.sh - g.pt + i;
      for (int k = 0; k < g.kw; ++k) {
        const int w = ow * g.sw - g.pl + k;
        const uint32_t pos = (uint32_t)(i * g.kw + k);
        float v[8];
        if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
          ld8<BF>(x, (((int64_t)n * g.H + h) * g.W + w) * g.C + cg * 8, v);
          if constexpr (BNF) bn_relu8<BF>(v, bsc, bsh);
        } else if (g.pad_zero) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = 0.f;
        } else {
          continue;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (v[j] > best[j]) {
            best[j] = v[j];
            am[j] = (h >= 0 && h < g.H && w >= 0 && w < g.W) ? pos : 255u;
          }
      }
    }
    const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + cg * 8;
    st8<BF>(y, o, best);
    uint2 a;
    a.x = am[0] | (am[1] << 8) | (am[2] << 16) | (am[3] << 24);
    a.y = am[4] | (am[5] << 8) | (am[6] << 16) | (am[7] << 24);
    *reinterpret_cast<uint2*>(arg + o) = a;
  }
}

// BNF: the pooled tensor was relu(bn(bn_x)) (forward BNF): dx is that group's masked gradient dz =
// dgrad * [bn_x * scale + shift > 0], and part[block][2][C] gets the block's channel sums of dz and
// dz * bn_x (the BN backward's reduction: bn_backward(part=...) skips its pass).  Needs gridDim * 256
// to be a multiple of C / 8 (each thread keeps one 8-channel group).
template <bool BF, bool K3S2, bool BNF = false>
__global__ __launch_bounds__(256) void k_maxpool_bwd(const void* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                     void* __restrict__ dx, PoolGeom g,
                                                     const void* __restrict__ bn_x = nullptr,
                                                     const float* __restrict__ bn_ss = nullptr,
                                                     float* __restrict__ part = nullptr) {
  const int G = g.C >> 3;
  const int64_t total = (int64_t)g.N * g.H * g.W * G;
  float bs[BNF ? 8 : 1], bq[BNF ? 8 : 1], msc[BNF ? 8 : 1], msh[BNF ? 8 : 1];
#pragma unroll
  for (int j = 0; j < (BNF ? 8 : 1); ++j) bs[j] = bq[j] = 0.f;
  if constexpr (BNF) {  // a thread's channel group never changes (gridDim * 256 % G == 0)
    const int cg0 = (int)(((int64_t)blockIdx.x * 256 + threadIdx.x) % G);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      msc[j] = bn_ss[cg0 * 8 + j];
      msh[j] = bn_ss[g.C + cg0 * 8 + j];
    }
  }
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int cg = (int)(t % G);
    int64_t r = t / G;
    const int w = (int)(r % g.W);
    r /= g.W;
    const int h = (int)(r % g.H);
    const int n = (int)(r / g.H);
    const int64_t xo = (((int64_t)n * g.H + h) * g.W + w) * g.C + cg * 8;
    float xv[BNF ? 8 : 1];
    if constexpr (BNF) ld8<BF>(bn_x, xo, xv);  // issued before the window loads: its latency overlaps theirs
    const int hp = h + g.pt, wp = w + g.pl;
    const int oh0 = hp - g.kh + 1 <= 0 ? 0 : (hp - g.kh + g.sh) / g.sh;
    const int oh1 = min(g.OH - 1, hp / g.sh);
    const int ow0 = wp - g.kw + 1 <= 0 ? 0 : (wp - g.kw + g.sw) / g.sw;
    const int ow1 = min(g.OW - 1, wp / g.sw);
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if constexpr (K3S2) {  // oh1 - oh0 <= 1 and ow1 - ow0 <= 1
      uint2 a[4];
      float d[4][8];
      bool ok[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int oh = oh0 + (q >> 1), ow = ow0 + (q & 1);
        ok[q] = oh <= oh1 && ow <= ow1;
        if (ok[q]) {
          const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + cg * 8;
          a[q] = *reinterpret_cast<const uint2*>(arg + o);
          ld8<BF>(dy, o, d[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (!ok[q]) continue;
        const int oh = oh0 + (q >> 1), ow = ow0 + (q & 1);
        const uint32_t pos = (uint32_t)((hp - oh * 2) * 3 + (wp - ow * 2));
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t aj = ((j < 4 ? a[q].x : a[q].y) >> (8 * (j & 3))) & 0xffu;
          if (aj == pos) acc[j] += d[q][j];
        }
      }
    }
    for (int oh = oh0; oh <= (K3S2 ? -1 : oh1); ++oh)
      for (int ow = ow0; ow <= ow1; ++ow) {
        const uint32_t pos = (uint32_t)((hp - oh * g.sh) * g.kw + (wp - ow * g.sw));
        const int64_t o = (((int64_t)n * g.OH + oh) * g.OW + ow) * g.C + cg * 8;
        const uint2 a = *reinterpret_cast<const uint2*>(arg + o);
        float d[8];
        ld8<BF>(dy, o, d);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t aj = ((j < 4 ? a.x : a.y) >> (8 * (j & 3))) & 0xffu;
          if (aj == pos) acc[j] += d[j];
        }
      }
    if constexpr (BNF) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // the stored dz is the bf16 value; the sums are over exactly what is stored
        const float d = fmaf(xv[j], msc[j], msh[j]) > 0.f ? (BF ? __uint_as_float(f2bf(acc[j]) << 16) : acc[j]) : 0.f;
        acc[j] = d;
        bs[j] += d;
        bq[j] = fmaf(d, xv[j], bq[j]);
      }
    }
    st8<BF>(dx, xo, acc);
  }
  if constexpr (BNF) {
    // fixed-order block reduction: thread t holds channel group t % G (gridDim * 256 % G == 0)
    __shared__ float red[2][2048];
    const int R = 256 / G, cg = threadIdx.x % G, rr = threadIdx.x / G;
    if (rr < R) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        red[0][rr * g.C + cg * 8 + j] = bs[j];
        red[1][rr * g.C + cg * 8 + j] = bq[j];
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < g.C; c += 256) {
      float S = 0.f, Q = 0.f;
      for (int k = 0; k < R; ++k) {
        S += red[0][k * g.C + c];
        Q += red[1][k * g.C + c];
      }
      part[((int64_t)blockIdx.x * 2) * g.C + c] = S;
      part[((int64_t)blockIdx.x * 2 + 1) * g.C + c] = Q;
    }
  }
}

// 2x2 stride-2 windows without padding (every input element in at most one window): scatter form, one
// thread per (window, channel group) writes the window's four input pixels (dy at the argmax, zero
// elsewhere) and, on the last window of an odd row / column, the zeros of the uncovered edge pixels.
// 32-bit index math (total < 2^31, checked on the host); a quarter of the generic form's threads and no
// per-input-pixel window search.  Same values as the gather form: 0 + dy at the argmax, 0 elsewhere.
template <bool BF>
__global__ __launch_bounds__(256) void k_maxpool_bwd_w2(const void* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                        void* __restrict__ dx, PoolGeom g) {
  const int G = g.C >> 3;
  const int total = g.N * g.OH * g.OW * G;
  const bool edge_w = g.W > 2 * g.OW, edge_h = g.H > 2 * g.OH;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const int cg = t % G;
    int r = t / G;
    const int ow = r % g.OW;
    r /= g.OW;
    const int oh = r % g.OH;
    const int n = r / g.OH;
    const int o = t * 8;  // ((n * OH + oh) * OW + ow) * C + cg * 8
    const uint2 a = *reinterpret_cast<const uint2*>(arg + o);
    float d[8];
    ld8<BF>(dy, o, d);
    const int x0 = ((n * g.H + 2 * oh) * g.W + 2 * ow) * g.C + cg * 8;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t aj = ((j < 4 ? a.x : a.y) >> (8 * (j & 3))) & 0xffu;
        v[j] = aj == (uint32_t)q ? 0.f + d[j] : 0.f;
      }
      st8<BF>(dx, x0 + ((q >> 1) * g.W + (q & 1)) * g.C, v);
    }
    const bool lw = edge_w && ow == g.OW - 1, lh = edge_h && oh == g.OH - 1;
    if (lw || lh) {
      float z[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) z[j] = 0.f;
      if (lw) {
        st8<BF>(dx, x0 + 2 * g.C, z);
        st8<BF>(dx, x0 + (g.W + 2) * g.C, z);
      }
      if (lh) {
        st8<BF>(dx, x0 + 2 * g.W * g.C, z);
        st8<BF>(dx, x0 + (2 * g.W + 1) * g.C, z);
      }
      if (lw && lh) st8<BF>(dx, x0 + (2 * g.W + 2) * g.C, z);
    }
  }
}

// TDL_POOL_W2=0 / maxpool_w2(false): the gather form for these windows too (A/B hook)
bool g_pool_w2 = [] {
  const char* e = std::getenv("TDL_POOL_W2");
  return e == nullptr || std::atoi(e) != 0;
}();

bool w2(const PoolGeom& g) {
  return g_pool_w2 && g.kh == 2 && g.kw == 2 && g.sh == 2 && g.sw == 2 && g.pt == 0 && g.pl == 0 &&
         g.OH == g.H / 2 && g.OW == g.W / 2 && (int64_t)g.N * g.H * g.W * g.C < (int64_t(1) << 31);
}

int grid_for(int64_t n) { return (int)std::min<int64_t>((n + 255) / 256, 256 * 32); }

// maxpool_force_generic (A/B hook).  Default: the generic loops -- the unrolled 3x3 stride-2 kernels
// measured slower in the ResNet-50 step (fwd 143 -> 237 us, bwd 226 -> 266 us: 9 loads of 16 B per
// thread in flight cost occupancy, resnet50_steady_state_breakdown_r4_dma1.txt)
bool g_pool_k3s2 = false;

bool k3s2(const PoolGeom& g) { return g_pool_k3s2 && g.kh == 3 && g.kw == 3 && g.sh == 2 && g.sw == 2; }

}  // namespace

void maxpool_force_generic(bool generic) { g_pool_k3s2 = !generic; }

void maxpool_w2(bool on) { g_pool_w2 = on; }

void maxpool_forward(const void* x, void* y, uint8_t* arg, bool bf16, const PoolGeom& g, hipStream_t s,
                     const float* bn_ss) {
  const int64_t n = (int64_t)g.N * g.OH * g.OW * (g.C / 8);
  const dim3 gr(grid_for(n)), b(256);
  if (bn_ss != nullptr) {
    if (bf16)
      hipLaunchKernelGGL((k_maxpool_fwd<true, false, true>), gr, b, 0, s, x, y, arg, g, bn_ss);
    else
      hipLaunchKernelGGL((k_maxpool_fwd<false, false, true>), gr, b, 0, s, x, y, arg, g, bn_ss);
    return;
  }
  if (k3s2(g)) {
    if (bf16)
      hipLaunchKernelGGL((k_maxpool_fwd<true, true>), gr, b, 0, s, x, y, arg, g);
    else
      hipLaunchKernelGGL((k_maxpool_fwd<false, true>), gr, b, 0, s, x, y, arg, g);
  } else if (bf16) {
    hipLaunchKernelGGL((k_maxpool_fwd<true, false>), gr, b, 0, s, x, y, arg, g);
  } else {
    hipLaunchKernelGGL((k_maxpool_fwd<false, false>), gr, b, 0, s, x, y, arg, g);
  }
}

int maxpool_backward_blocks(const PoolGeom& g) { return grid_for((int64_t)g.N * g.H * g.W * (g.C / 8)); }

void maxpool_backward(const void* dy, const uint8_t* arg, void* dx, bool bf16, const PoolGeom& g, hipStream_t s,
                      const void* bn_x, const float* bn_ss, float* part) {
  const int64_t n = (int64_t)g.N * g.H * g.W * (g.C / 8);
  const dim3 gr(grid_for(n)), b(256);
  if (bn_x != nullptr) {
    if (bf16)
      hipLaunchKernelGGL((k_maxpool_bwd<true, false, true>), gr, b, 0, s, dy, arg, dx, g, bn_x, bn_ss, part);
    else
      hipLaunchKernelGGL((k_maxpool_bwd<false, false, true>), gr, b, 0, s, dy, arg, dx, g, bn_x, bn_ss, part);
    return;
  }
  if (w2(g)) {
    const dim3 gw(grid_for((int64_t)g.N * g.OH * g.OW * (g.C / 8)));
    if (bf16)
      hipLaunchKernelGGL((k_maxpool_bwd_w2<true>), gw, b, 0, s, dy, arg, dx, g);
    else
      hipLaunchKernelGGL((k_maxpool_bwd_w2<false>), gw, b, 0, s, dy, arg, dx, g);
    return;
  }
  if (k3s2(g)) {
    if (bf16)
      hipLaunchKernelGGL((k_maxpool_bwd<true, true>), gr, b, 0, s, dy, arg, dx, g);
    else
      hipLaunchKernelGGL((k_maxpool_bwd<false, true>), gr, b, 0, s, dy, arg, dx, g);
  } else if (bf16) {
    hipLaunchKernelGGL((k_maxpool_bwd<true, false>), gr, b, 0, s, dy, arg, dx, g);
  } else {
    hipLaunchKernelGGL((k_maxpool_bwd<false, false>), gr, b, 0, s, dy, arg, dx, g);
  }
}

}  // namespace tdl
