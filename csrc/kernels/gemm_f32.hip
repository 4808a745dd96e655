// Generic f32 GEMM / implicit-GEMM convolution on v_mfma_f32_16x16x4_f32 (see gemm_f32.h).
//
// Workgroup: 256 threads = 4 waves, a 64 x 64 output tile, reduction in slices of 16 staged through
// LDS.  Wave w owns the 32 x 32 quadrant (w & 1, w >> 1): 2 x 2 MFMA 16x16 blocks, 16 MFMAs per
// slice.  Operands are fetched into registers one slice ahead (the next slice's global loads are in
// flight while the MFMAs of this one issue), then written to LDS k-major:
//   As[k][m]: thread t loads 4 consecutive k of row m = t & 63 (one 16-B load when the 4 values are
//             contiguous in memory, e.g. 4 channels of one pixel); lanes of a wave write 64
//             consecutive m -> conflict-free scalar LDS writes.
//   Bs[k][n]: thread t loads 4 consecutive n of row k = t >> 4, one 16-B LDS write.
// Row pitch 80 floats: the MFMA operand reads (16 consecutive m or n, 4 consecutive k across the
// lane groups) hit 64 distinct banks.
//
// The convolution index decodes run on mixed-radix counters advanced by 16 per slice (a division
// only on wrap-around), not per-element integer divisions.
#include "common.h"
#include "gemm_f32.h"

namespace tdl {
namespace {

constexpr int kLd = 80;

// (hi, mid, lo) counter, lo fastest, radices (., nmid, nlo)
struct Ctr {
  int hi, mid, lo;
  __device__ void set(int v, int nmid, int nlo) {
    const int q = v / nlo;
    lo = v - q * nlo;
    mid = q % nmid;
    hi = q / nmid;
  }
  __device__ void step(int d, int nmid, int nlo) {
    lo += d;
    if (lo >= nlo) {
      const int q = lo / nlo;
      lo -= q * nlo;
      mid += q;
      if (mid >= nmid) {
        const int q2 = mid / nmid;
        mid -= q2 * nmid;
        hi += q2;
      }
    }
  }
};

__device__ __forceinline__ void out_store(const F32GemmArgs& a, int m, int n, float v) {
  if (a.bias != nullptr) v += a.bias[n];
  const int64_t i = a.trans_out ? (int64_t)n * a.ldo + m : (int64_t)m * a.ldo + n;
  if (a.accumulate) v += a.out[i];
  a.out[i] = v;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_gemm_f32(F32GemmArgs a) {
  __shared__ float As[16 * kLd];
  __shared__ float Bs[16 * kLd];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int m0 = blockIdx.x * kF32Tile, n0 = blockIdx.y * kF32Tile;
  const int kbeg = blockIdx.z * a.kchunk;
  const int kend = min(a.Kred, kbeg + a.kchunk);
  const F32ConvGeom& g = a.g;

  // A: row ml, reduction quad kqa; B: reduction row kl, column quad nqb
  const int ml = lane, kqa = wave * 4;
  const int kl = t >> 4, nqb = (t & 15) * 4;
  const int am = m0 + ml, bn = n0 + nqb;
  const bool arow = am < a.M;

  // per-thread fixed decodes
  int an = 0, ay = 0, ax = 0;  // conv fwd: image, top-left input row / col; dgrad: image, y + pt, x + pl
  if constexpr (MODE == kF32ConvFwd) {
    const int hw = g.oh * g.ow;
    an = am / hw;
    const int p = am - an * hw, oy = p / g.ow;
    ay = oy * g.sh - g.pt;
    ax = (p - oy * g.ow) * g.sw - g.pl;
  } else if constexpr (MODE == kF32ConvDgrad) {
    const int hw = g.h * g.w;
    an = am / hw;
    const int p = am - an * hw, y = p / g.w;
    ay = y + g.pt;
    ax = p - y * g.w + g.pl;
  }
  int wr[4] = {0, 0, 0, 0}, ws_[4] = {0, 0, 0, 0}, wc[4] = {0, 0, 0, 0};  // wgrad: (r, s, c) of the B columns
  if constexpr (MODE == kF32ConvWgrad) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int n = bn + i, rs = n / g.c;
      wc[i] = n - rs * g.c;
      ws_[i] = rs % g.s;
      wr[i] = rs / g.s;
    }
  }
  // reduction counters: fwd (r, s, c) / dgrad (r, s, k) of this thread's A quad; wgrad (img, oy, ox) of its B row
  Ctr ka{0, 0, 0}, kb{0, 0, 0};
  if constexpr (MODE == kF32ConvFwd) ka.set(kbeg + kqa, g.s, g.c);
  if constexpr (MODE == kF32ConvDgrad) ka.set(kbeg + kqa, g.s, g.k);
  if constexpr (MODE == kF32ConvWgrad) kb.set(kbeg + kl, g.oh, g.ow);

  const bool s1 = g.sh == 1 && g.sw == 1;
  float ra[4], rb[4];
  auto load = [&](int k0) {
    const int kk = k0 + kqa;  // A: reduction index of ra[0]
    if constexpr (MODE == kF32Gemm) {
      if (a.vec_a && arow && kk < kend) {
        const f4 v = ld4(a.a + (int64_t)am * a.sam + kk);
#pragma unroll
        for (int i = 0; i < 4; ++i) ra[i] = v[i];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          ra[i] = (arow && kk + i < kend) ? a.a[(int64_t)am * a.sam + (int64_t)(kk + i) * a.sak] : 0.f;
      }
    } else if constexpr (MODE == kF32ConvFwd || MODE == kF32ConvDgrad) {
      const int nlo = MODE == kF32ConvFwd ? g.c : g.k;
      Ctr c = ka;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
        if (a.vec_a && i > 0) {
          v = ra[i];  // (filled by the vector load below)
        } else if (arow && kk + i < kend) {
          int iy, ix;
          bool ok;
          if constexpr (MODE == kF32ConvFwd) {
            iy = ay + c.hi * g.dh;
            ix = ax + c.mid * g.dw;
            ok = iy >= 0 && iy < g.h && ix >= 0 && ix < g.w;
          } else {
            const int ty = ay - c.hi * g.dh, tx = ax - c.mid * g.dw;
            iy = s1 ? ty : ty / g.sh;  // (stride 1: no integer division per element)
            ix = s1 ? tx : tx / g.sw;
            ok = ty >= 0 && tx >= 0 && (s1 || (iy * g.sh == ty && ix * g.sw == tx)) && iy < g.oh && ix < g.ow;
          }
          if (ok) {
            const int64_t base = MODE == kF32ConvFwd ? (((int64_t)an * g.h + iy) * g.w + ix) * g.c
                                                     : (((int64_t)an * g.oh + iy) * g.ow + ix) * g.k;
            if (a.vec_a) {
              const f4 q = ld4(a.a + base + c.lo);
              v = q[0];
              ra[1] = q[1];
              ra[2] = q[2];
              ra[3] = q[3];
            } else {
              v = a.a[base + c.lo];
            }
          } else if (a.vec_a) {
            ra[1] = ra[2] = ra[3] = 0.f;
          }
        } else if (a.vec_a) {
          ra[1] = ra[2] = ra[3] = 0.f;
        }
        ra[i] = v;
        if (!a.vec_a && i < 3) c.step(1, g.s, nlo);
      }
    } else {  // wgrad: A(m = out channel, j) = dy[j][m]
#pragma unroll
      for (int i = 0; i < 4; ++i) ra[i] = (arow && kk + i < kend) ? a.a[(int64_t)(kk + i) * g.k + am] : 0.f;
    }

    const int kr = k0 + kl;  // B: reduction index of this thread's row
    const bool brow = kr < kend;
    if constexpr (MODE == kF32ConvWgrad) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float v = 0.f;
        if (a.vec_b && i > 0) {
          v = rb[i];
        } else if (brow && bn + i < a.N) {
          const int iy = kb.mid * g.sh - g.pt + wr[i] * g.dh, ix = kb.lo * g.sw - g.pl + ws_[i] * g.dw;
          if (iy >= 0 && iy < g.h && ix >= 0 && ix < g.w) {
            const int64_t base = (((int64_t)kb.hi * g.h + iy) * g.w + ix) * g.c + wc[i];
            if (a.vec_b) {
              const f4 q = ld4(a.b + base);
              v = q[0];
              rb[1] = q[1];
              rb[2] = q[2];
              rb[3] = q[3];
            } else {
              v = a.b[base];
            }
          } else if (a.vec_b) {
            rb[1] = rb[2] = rb[3] = 0.f;
          }
        } else if (a.vec_b) {
          rb[1] = rb[2] = rb[3] = 0.f;
        }
        rb[i] = v;
      }
    } else {
      const int64_t sbk = MODE == kF32Gemm ? a.sbk : (int64_t)a.N;
      const int64_t sbn = MODE == kF32Gemm ? a.sbn : 1;
      if (a.vec_b && brow && bn < a.N) {
        const f4 v = ld4(a.b + (int64_t)kr * sbk + bn);
#pragma unroll
        for (int i = 0; i < 4; ++i) rb[i] = v[i];
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) rb[i] = (brow && bn + i < a.N) ? a.b[(int64_t)kr * sbk + (int64_t)(bn + i) * sbn] : 0.f;
      }
    }
  };

  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero4();

  const int wm = (wave & 1) * 32, wn = (wave >> 1) * 32;
  const int lr = lane & 15, lk = lane >> 4;
  load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) As[(kqa + i) * kLd + ml] = ra[i];
    st4(&Bs[kl * kLd + nqb], f4{rb[0], rb[1], rb[2], rb[3]});
    __syncthreads();
    if (k0 + 16 < kend) {
      if constexpr (MODE == kF32ConvFwd) ka.step(16, g.s, g.c);
      if constexpr (MODE == kF32ConvDgrad) ka.step(16, g.s, g.k);
      if constexpr (MODE == kF32ConvWgrad) kb.step(16, g.oh, g.ow);
      load(k0 + 16);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int kr = (4 * ks + lk) * kLd;
      const float a0 = As[kr + wm + lr], a1 = As[kr + wm + 16 + lr];
      const float b0 = Bs[kr + wn + lr], b1 = Bs[kr + wn + 16 + lr];
      acc[0][0] = mfma16x16x4(a0, b0, acc[0][0]);
      acc[0][1] = mfma16x16x4(a0, b1, acc[0][1]);
      acc[1][0] = mfma16x16x4(a1, b0, acc[1][0]);
      acc[1][1] = mfma16x16x4(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }

  // D[(lane >> 4) * 4 + r][lane & 15] of each 16x16 block
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm + 16 * i + 4 * lk + r, n = n0 + wn + 16 * j + lr;
        if (m >= a.M || n >= a.N) continue;
        if (a.splits > 1)
          a.ws[((int64_t)blockIdx.z * a.M + m) * a.N + n] = acc[i][j][r];
        else
          out_store(a, m, n, acc[i][j][r]);
      }
}

__device__ __forceinline__ void out_index(const F32GemmArgs& a, int64_t e, int& m, int& n) {
  if (a.trans_out) {
    n = (int)(e / a.M);
    m = (int)(e - (int64_t)n * a.M);
  } else {
    m = (int)(e / a.N);
    n = (int)(e - (int64_t)m * a.N);
  }
}

// Split-reduction epilogue: the slices summed in a fixed order, then bias / accumulate / store.
// Outputs are walked in storage order (coalesced stores, strided partial reads when transposed).
// Few slices: one thread per output, 8 independent partial loads in flight.
__global__ __launch_bounds__(256) void k_gemm_f32_reduce(F32GemmArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mn = (int64_t)a.M * a.N;
  if (e >= mn) return;
  int m, n;
  out_index(a, e, m, n);
  const float* src = a.ws + (int64_t)m * a.N + n;
  float v = 0.f;
  int z = 0;
  for (; z + 8 <= a.splits; z += 8) {
    float p[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) p[u] = src[(z + u) * mn];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += p[u];
  }
  for (; z < a.splits; ++z) v += src[z * mn];
  out_store(a, m, n, v);
}

// Many slices over few outputs (a small weight gradient over a long reduction): one wave per output,
// lane l sums slices l, l + 64, .. in order, then a fixed xor butterfly over the wave (deterministic).
__global__ __launch_bounds__(256) void k_gemm_f32_reduce_wave(F32GemmArgs a) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int64_t mn = (int64_t)a.M * a.N;
  if (e >= mn) return;
  int m, n;
  out_index(a, e, m, n);
  const float* src = a.ws + (int64_t)m * a.N + n;
  float v = 0.f;
  for (int z = lane; z < a.splits; z += 64) v += src[z * mn];
  v = wave_sum(v);
  if (lane == 0) out_store(a, m, n, v);
}

}  // namespace

void f32_gemm_launch(int mode, const F32GemmArgs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  const dim3 grid((a.M + kF32Tile - 1) / kF32Tile, (a.N + kF32Tile - 1) / kF32Tile, a.splits);
  switch (mode) {
    case kF32Gemm: hipLaunchKernelGGL(k_gemm_f32<kF32Gemm>, grid, dim3(256), 0, s, a); break;
    case kF32ConvFwd: hipLaunchKernelGGL(k_gemm_f32<kF32ConvFwd>, grid, dim3(256), 0, s, a); break;
    case kF32ConvDgrad: hipLaunchKernelGGL(k_gemm_f32<kF32ConvDgrad>, grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(k_gemm_f32<kF32ConvWgrad>, grid, dim3(256), 0, s, a); break;
  }
  if (a.splits > 1) {
    const int64_t mn = (int64_t)a.M * a.N;
    if (a.splits >= 32 && mn <= 16384)
      hipLaunchKernelGGL(k_gemm_f32_reduce_wave, dim3((unsigned)((mn + 3) / 4)), dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(k_gemm_f32_reduce, dim3((unsigned)((mn + 255) / 256)), dim3(256), 0, s, a);
  }
}

}  // namespace tdl
