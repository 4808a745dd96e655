// Training-mode batch normalisation for NHWC activations on gfx950 (see bn.h).
//
// HBM-bound work; the design minimises passes and keeps every wave streaming 16-byte loads:
//   forward : [partial sums x, x^2 per channel]  -> [finalize: mean/invstd, scale/shift, moving
//             stats]  -> [apply y = act(x*scale + shift)]                (2 reads + 1 write of x)
//   backward: [partial sums dy, dy*x]  -> [finalize: dgamma, dbeta, dx coefficients]
//             -> [dx = A*dy + B*x + D]                                    (2x2 reads + 1 write)
// A thread owns 8 consecutive channels (one 16-byte bf16 vector); a 256-thread workgroup covers
// 256/(C/8) rows per iteration, unrolled 4 deep so each wave keeps 4 independent loads in flight.
// Partials are per workgroup ([parts][2][C]) and reduced in a fixed order (deterministic).
#include "bn.h"
#include "common.h"

namespace tdl {
namespace {

constexpr int kUnroll = 4;
// workgroups of the partial-sum pass and of the elementwise passes, and vectors per thread in the
// latter, tunable at run time (bn_set_tuning) for the sweep in scripts/bench_bn.py: the defaults
// measured best (the large shapes run at 4.7-5.7 TB/s, the device copy at 5.3-6.7 TB/s)
int g_max_parts = 512;
int g_elem_blocks = 256 * 16;
int g_elem_unroll = 1;  // 2 measured 1-4 % slower (scripts/bench_bn.py, profiles/bn_tuning_sweep_r2.jsonl)
// elementwise kernel family: 0 grid-stride (one vector per thread per tensor in flight, LDS channel
// tables), 1 blocked (g_elem_vpt vectors per thread per tensor in flight, channels in registers)
int g_elem_kind = 1;
int g_elem_vpt = 4;
int g_blk_blocks = 8192;  // grid cap of the blocked kernels (measured best, profiles/bn_blocked_sweep_r4.jsonl)
constexpr int kFinPhases = 16;  // partial-row phases per channel in the finalize kernels (1024 threads)

__device__ __forceinline__ float bf_lo(uint32_t u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(uint32_t u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ uint32_t f2bf(float f) {  // round to nearest even
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

template <BnDType D>
struct Io;

template <>
struct Io<BnDType::kF32> {
  static __device__ __forceinline__ void load(const void* p, int64_t e, float* o) {
    const f4* q = reinterpret_cast<const f4*>(static_cast<const float*>(p) + e);
    const f4 a = q[0], b = q[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void store(void* p, int64_t e, const float* v) {
    f4* q = reinterpret_cast<f4*>(static_cast<float*>(p) + e);
    q[0] = f4{v[0], v[1], v[2], v[3]};
    q[1] = f4{v[4], v[5], v[6], v[7]};
  }
};

template <>
struct Io<BnDType::kBF16> {
  static __device__ __forceinline__ void load(const void* p, int64_t e, float* o) {
    const uint4 u = *reinterpret_cast<const uint4*>(static_cast<const uint16_t*>(p) + e);
    o[0] = bf_lo(u.x); o[1] = bf_hi(u.x); o[2] = bf_lo(u.y); o[3] = bf_hi(u.y);
    o[4] = bf_lo(u.z); o[5] = bf_hi(u.z); o[6] = bf_lo(u.w); o[7] = bf_hi(u.w);
  }
  static __device__ __forceinline__ void store(void* p, int64_t e, const float* v) {
    uint4 u;
    u.x = f2bf(v[0]) | (f2bf(v[1]) << 16);
    u.y = f2bf(v[2]) | (f2bf(v[3]) << 16);
    u.z = f2bf(v[4]) | (f2bf(v[5]) << 16);
    u.w = f2bf(v[6]) | (f2bf(v[7]) << 16);
    *reinterpret_cast<uint4*>(static_cast<uint16_t*>(p) + e) = u;
  }
};

// Partial per-channel sums over a workgroup's rows.
//   MODE 0 (forward)      : (sum x, sum x*x)                     a = x
//   MODE 1 (backward)     : (sum dy, sum dy*x)                   a = dy, b = x
//   MODE 2 (bwd, relu)    : dz = dy masked by x*scale+shift > 0  (the fused ReLU, recomputed from x)
//   MODE 3 (bwd, add+relu): dz = dy masked by y > 0, written to dz_out (the residual's gradient)
template <BnDType D, int MODE>
__global__ __launch_bounds__(256) void k_bn_partial(const void* __restrict__ a, const void* __restrict__ b,
                                                    const void* __restrict__ y, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, void* __restrict__ dz_out,
                                                    int64_t M, int C, int64_t rows_wg, float* __restrict__ part) {
  __shared__ float red[2][2048];
  const int G = C >> 3, R = 256 / G;
  const int t = threadIdx.x, cg = t % G, rr = t / G;
  const int64_t r0 = (int64_t)blockIdx.x * rows_wg;
  const int64_t r1 = min(M, r0 + rows_wg);
  float s[8], q[8], sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s[j] = q[j] = 0.f;
    sc[j] = MODE == 2 ? scale[cg * 8 + j] : 0.f;
    sh[j] = MODE == 2 ? shift[cg * 8 + j] : 0.f;
  }
  if (rr < R) {
    int64_t r = r0 + rr;
    for (; r + (kUnroll - 1) * R < r1; r += kUnroll * R) {
      float va[kUnroll][8], vb[kUnroll][8], vy[kUnroll][8];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
        Io<D>::load(a, (r + u * R) * C + cg * 8, va[u]);
        if (MODE != 0) Io<D>::load(b, (r + u * R) * C + cg * 8, vb[u]);
        if (MODE == 3) Io<D>::load(y, (r + u * R) * C + cg * 8, vy[u]);
      }
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (MODE == 2 && !(fmaf(vb[u][j], sc[j], sh[j]) > 0.f)) va[u][j] = 0.f;
          if (MODE == 3 && !(vy[u][j] > 0.f)) va[u][j] = 0.f;
          s[j] += va[u][j];
          q[j] = fmaf(va[u][j], MODE == 0 ? va[u][j] : vb[u][j], q[j]);
        }
        if (MODE == 3) Io<D>::store(dz_out, (r + u * R) * C + cg * 8, va[u]);
      }
    }
    for (; r < r1; r += R) {
      float va[8], vb[8], vy[8];
      Io<D>::load(a, r * C + cg * 8, va);
      if (MODE != 0) Io<D>::load(b, r * C + cg * 8, vb);
      if (MODE == 3) Io<D>::load(y, r * C + cg * 8, vy);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MODE == 2 && !(fmaf(vb[j], sc[j], sh[j]) > 0.f)) va[j] = 0.f;
        if (MODE == 3 && !(vy[j] > 0.f)) va[j] = 0.f;
        s[j] += va[j];
        q[j] = fmaf(va[j], MODE == 0 ? va[j] : vb[j], q[j]);
      }
      if (MODE == 3) Io<D>::store(dz_out, r * C + cg * 8, va);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][rr * C + cg * 8 + j] = s[j];
      red[1][rr * C + cg * 8 + j] = q[j];
    }
  }
  __syncthreads();
  for (int c = t; c < C; c += 256) {
    float S = 0.f, Q = 0.f;
    for (int k = 0; k < R; ++k) {
      S += red[0][k * C + c];
      Q += red[1][k * C + c];
    }
    part[((int64_t)blockIdx.x * 2) * C + c] = S;
    part[((int64_t)blockIdx.x * 2 + 1) * C + c] = Q;
  }
}

// Sum the partial rows of channel c: 64 channels x kFinPhases phases per 1024-thread workgroup, f64.
__device__ __forceinline__ bool reduce_parts(const float* __restrict__ part, int P, int C, double& S, double& Q) {
  __shared__ double rs[kFinPhases][64], rq[kFinPhases][64];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  double s = 0.0, q = 0.0;
  if (c < C) {
#pragma unroll 4
    for (int p = ph; p < P; p += kFinPhases) {
      s += part[((int64_t)p * 2) * C + c];
      q += part[((int64_t)p * 2 + 1) * C + c];
    }
  }
  rs[ph][lane] = s;
  rq[ph][lane] = q;
  __syncthreads();
  if (ph != 0 || c >= C) return false;
  S = 0.0;
  Q = 0.0;
#pragma unroll
  for (int k = 0; k < kFinPhases; ++k) {
    S += rs[k][lane];
    Q += rq[k][lane];
  }
  return true;
}

// First level of the partial reduction when there are many partial rows: block (cb, pb) sums rows
// [64 pb, 64 pb + 64) of channels [64 cb, 64 cb + 64) in a fixed order into out[pb][2][C] (the
// finalize then reduces ceil(P / 64) rows: a single 1024-thread block per 64 channels reading
// thousands of rows was latency-bound).
__global__ __launch_bounds__(1024) void k_bn_prereduce(const float* __restrict__ part, int P, int C,
                                                       float* __restrict__ out) {
  __shared__ float rs[kFinPhases][64], rq[kFinPhases][64];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const int p0 = blockIdx.y * 64, p1 = min(P, p0 + 64);
  float s = 0.f, q = 0.f;
  if (c < C)
    for (int p = p0 + ph; p < p1; p += kFinPhases) {
      s += part[((int64_t)p * 2) * C + c];
      q += part[((int64_t)p * 2 + 1) * C + c];
    }
  rs[ph][lane] = s;
  rq[ph][lane] = q;
  __syncthreads();
  if (ph != 0 || c >= C) return;
  s = 0.f;
  q = 0.f;
#pragma unroll
  for (int k = 0; k < kFinPhases; ++k) {
    s += rs[k][lane];
    q += rq[k][lane];
  }
  out[((int64_t)blockIdx.y * 2) * C + c] = s;
  out[((int64_t)blockIdx.y * 2 + 1) * C + c] = q;
}

// P > 1024 partial rows in `part` -> ceil(P / 64) rows at part + P*2*C
static const float* prereduce(const float* part, int& P, int C, hipStream_t s) {
  if (P <= 1024) return part;
  float* out = const_cast<float*>(part) + (int64_t)P * 2 * C;
  const int P2 = (P + 63) / 64;
  hipLaunchKernelGGL(k_bn_prereduce, dim3((C + 63) / 64, P2), dim3(64 * kFinPhases), 0, s, part, P, C, out);
  P = P2;
  return out;
}

__global__ __launch_bounds__(1024) void k_bn_fwd_finalize(const float* __restrict__ part, int P, int64_t M, int C,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta,
                                                         const float* __restrict__ mean_off, float* __restrict__ mean,
                                                         float* __restrict__ invstd, float* __restrict__ scale,
                                                         float* __restrict__ shift, float* __restrict__ mm,
                                                         float* __restrict__ mv, float momentum, float eps) {
  double S, Q;
  if (!reduce_parts(part, P, C, S, Q)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double mu = S / (double)M;
  const double var = fmax(Q / (double)M - mu * mu, 0.0);
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  mean[c] = (float)mu;
  invstd[c] = inv;
  scale[c] = g * inv;
  shift[c] = be - (float)mu * g * inv;
  if (mm != nullptr) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    // mean_off: bias of a preceding conv folded into this BN (it shifts only the batch mean)
    const float mu_o = (float)mu + (mean_off ? mean_off[c] : 0.f);
    mm[c] = mm[c] * momentum + mu_o * (1.f - momentum);
    mv[c] = mv[c] * momentum + (float)unb * (1.f - momentum);
  }
}

__global__ __launch_bounds__(1024) void k_bn_bwd_finalize(const float* __restrict__ part, int P, int64_t M, int C,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ invstd, float* __restrict__ dgamma,
                                                         float* __restrict__ dbeta, float* __restrict__ coef, int acc) {
  double S, Q;
  if (!reduce_parts(part, P, C, S, Q)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double mu = mean[c], inv = invstd[c];
  const double g = gamma ? gamma[c] : 1.0;
  const double dg = (Q - mu * S) * inv;  // sum dy * xhat
  const double db = S;                   // sum dy
  // acc bit 0 / 1: add into dgamma / dbeta (a trainer's gradient slab) instead of overwriting
  if (dgamma) dgamma[c] = (acc & 1) ? dgamma[c] + (float)dg : (float)dg;
  if (dbeta) dbeta[c] = (acc & 2) ? dbeta[c] + (float)db : (float)db;
  // dx = g*inv/M * (M*dy - db - xhat*dg) = A*dy + B*x + D
  const double A = g * inv, B = -g * inv * inv * dg / (double)M;
  coef[c] = (float)A;
  coef[C + c] = (float)B;
  coef[2 * C + c] = (float)(-A * db / (double)M - B * mu);
}

template <BnDType D, int U>
__global__ __launch_bounds__(256) void k_bn_apply(const void* __restrict__ x, const void* __restrict__ res,
                                                  void* __restrict__ y, int64_t n8, int C,
                                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                                  int relu) {
  __shared__ float sc[2048], sh[2048];
  for (int c = threadIdx.x; c < C; c += 256) {
    sc[c] = scale[c];
    sh[c] = shift[c];
  }
  __syncthreads();
  // U vectors per thread per iteration (all loads issued before any math): U x 16 B in flight
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int cstep = (int)((stride * 8) % C);  // channel advance per grid stride (no 64-bit modulo per vector)
  int c0 = (int)((v0 * 8) % C);
  auto adv = [&](int c) { return c + cstep >= C ? c + cstep - C : c + cstep; };
  for (int64_t v = v0; v < n8; v += U * stride) {
    float xv[U][8], rv[U][8];
    int cu[U];
    cu[0] = c0;
#pragma unroll
    for (int u = 1; u < U; ++u) cu[u] = adv(cu[u - 1]);
    c0 = adv(cu[U - 1]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v + u * stride < n8) {
        Io<D>::load(x, (v + u * stride) * 8, xv[u]);
        if (res != nullptr) Io<D>::load(res, (v + u * stride) * 8, rv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v + u * stride >= n8) break;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float o = fmaf(xv[u][j], sc[cu[u] + j], sh[cu[u] + j]);
        if (res != nullptr) o += rv[u][j];
        xv[u][j] = relu ? fmaxf(o, 0.f) : o;
      }
      Io<D>::store(y, (v + u * stride) * 8, xv[u]);
    }
  }
}

// dx = A*dz + B*x + D with dz = dy (modes 1, 3: dy is the masked dz) or dy masked by the
// recomputed relu condition x*scale + shift > 0 (mode 2)
template <BnDType D, bool MASK, int U>
__global__ __launch_bounds__(256) void k_bn_dx(const void* __restrict__ dy, const void* __restrict__ x,
                                               void* __restrict__ dx, int64_t n8, int C, const float* __restrict__ coef,
                                               const float* __restrict__ scale, const float* __restrict__ shift) {
  __shared__ float cA[2048], cB[2048], cD[2048], cS[MASK ? 2048 : 1], cT[MASK ? 2048 : 1];
  for (int c = threadIdx.x; c < C; c += 256) {
    cA[c] = coef[c];
    cB[c] = coef[C + c];
    cD[c] = coef[2 * C + c];
    if (MASK) {
      cS[c] = scale[c];
      cT[c] = shift[c];
    }
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t v0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int cstep = (int)((stride * 8) % C);
  int c0 = (int)((v0 * 8) % C);
  auto adv = [&](int c) { return c + cstep >= C ? c + cstep - C : c + cstep; };
  for (int64_t v = v0; v < n8; v += U * stride) {
    float g[U][8], xv[U][8];
    int cu[U];
    cu[0] = c0;
#pragma unroll
    for (int u = 1; u < U; ++u) cu[u] = adv(cu[u - 1]);
    c0 = adv(cu[U - 1]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v + u * stride < n8) {
        Io<D>::load(dy, (v + u * stride) * 8, g[u]);
        Io<D>::load(x, (v + u * stride) * 8, xv[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v + u * stride >= n8) break;
      const int cc = cu[u];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MASK && !(fmaf(xv[u][j], cS[cc + j], cT[cc + j]) > 0.f)) g[u][j] = 0.f;
        g[u][j] = fmaf(cA[cc + j], g[u][j], fmaf(cB[cc + j], xv[u][j], cD[cc + j]));
      }
      Io<D>::store(dx, (v + u * stride) * 8, g[u]);
    }
  }
}

// Blocked elementwise passes (bf16, C a power of two <= 2048).  A workgroup streams chunks of 256*V
// consecutive 16-B vectors, thread t owning vectors t, t + 256, ... of a chunk: the V loads per
// tensor are all issued before any math (2V x 16 B in flight per thread), and since C divides
// 2048 = 256 vectors x 8 channels a thread's 8 channels are the same in every chunk, so its
// scale/shift (dx coefficients) sit in registers instead of an LDS table read per vector.  bf16
// packing is v_cvt_pk_bf16_f32 (round to nearest even, as f2bf).
__device__ __forceinline__ uint32_t pk_bf16(float lo, float hi) {
  uint32_t r;
  asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(lo), "v"(hi));
  return r;
}

__device__ __forceinline__ void unpack8(const uint4& u, float* o) {
  o[0] = bf_lo(u.x); o[1] = bf_hi(u.x); o[2] = bf_lo(u.y); o[3] = bf_hi(u.y);
  o[4] = bf_lo(u.z); o[5] = bf_hi(u.z); o[6] = bf_lo(u.w); o[7] = bf_hi(u.w);
}

__device__ __forceinline__ uint4 pack8(const float* v) {
  return uint4{pk_bf16(v[0], v[1]), pk_bf16(v[2], v[3]), pk_bf16(v[4], v[5]), pk_bf16(v[6], v[7])};
}

template <int V>
__global__ __launch_bounds__(256) void k_bn_apply_blk(const uint4* __restrict__ x, const uint4* __restrict__ res,
                                                      uint4* __restrict__ y, int64_t n8, int C,
                                                      const float* __restrict__ scale,
                                                      const float* __restrict__ shift, int relu) {
  const int c0 = (threadIdx.x * 8) & (C - 1);
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    sc[j] = scale[c0 + j];
    sh[j] = shift[c0 + j];
  }
  const int64_t nch = (n8 + 256 * V - 1) / (256 * V);
  for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t v0 = ch * (256 * V) + threadIdx.x;
    uint4 xu[V], ru[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (v0 + u * 256 < n8) {
        xu[u] = x[v0 + u * 256];
        if (res != nullptr) ru[u] = res[v0 + u * 256];
      }
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (v0 + u * 256 >= n8) break;
      float o[8], r[8];
      unpack8(xu[u], o);
      if (res != nullptr) unpack8(ru[u], r);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = fmaf(o[j], sc[j], sh[j]);
        if (res != nullptr) o[j] += r[j];
        if (relu) o[j] = fmaxf(o[j], 0.f);
      }
      y[v0 + u * 256] = pack8(o);
    }
  }
}

template <bool MASK, int V>
__global__ __launch_bounds__(256) void k_bn_dx_blk(const uint4* __restrict__ dy, const uint4* __restrict__ x,
                                                   uint4* __restrict__ dx, int64_t n8, int C,
                                                   const float* __restrict__ coef, const float* __restrict__ scale,
                                                   const float* __restrict__ shift) {
  const int c0 = (threadIdx.x * 8) & (C - 1);
  float cA[8], cB[8], cD[8], cS[8], cT[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    cA[j] = coef[c0 + j];
    cB[j] = coef[C + c0 + j];
    cD[j] = coef[2 * C + c0 + j];
    cS[j] = MASK ? scale[c0 + j] : 0.f;
    cT[j] = MASK ? shift[c0 + j] : 0.f;
  }
  const int64_t nch = (n8 + 256 * V - 1) / (256 * V);
  for (int64_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {
    const int64_t v0 = ch * (256 * V) + threadIdx.x;
    uint4 gu[V], xu[V];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (v0 + u * 256 < n8) {
        gu[u] = dy[v0 + u * 256];
        xu[u] = x[v0 + u * 256];
      }
    }
#pragma unroll
    for (int u = 0; u < V; ++u) {
      if (v0 + u * 256 >= n8) break;
      float g[8], xv[8];
      unpack8(gu[u], g);
      unpack8(xu[u], xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (MASK && !(fmaf(xv[j], cS[j], cT[j]) > 0.f)) g[j] = 0.f;
        g[j] = fmaf(cA[j], g[j], fmaf(cB[j], xv[j], cD[j]));
      }
      dx[v0 + u * 256] = pack8(g);
    }
  }
}

bool blocked_ok(BnDType dt, int C) { return g_elem_kind == 1 && dt == BnDType::kBF16 && C >= 8 && C <= 2048 && (C & (C - 1)) == 0; }

int blocked_grid(int64_t n8) {
  const int64_t nch = (n8 + 256 * g_elem_vpt - 1) / (256 * g_elem_vpt);
  return (int)std::min<int64_t>(std::max<int64_t>(nch, 1), g_blk_blocks);
}

template <int V>
void launch_apply_blk(const void* x, const void* res, void* y, int64_t n8, int C, const float* scale,
                      const float* shift, int relu, hipStream_t s) {
  hipLaunchKernelGGL((k_bn_apply_blk<V>), dim3(blocked_grid(n8)), dim3(256), 0, s, static_cast<const uint4*>(x),
                     static_cast<const uint4*>(res), static_cast<uint4*>(y), n8, C, scale, shift, relu);
}

template <bool MASK, int V>
void launch_dx_blk(const void* dy, const void* x, void* dx, int64_t n8, int C, const float* coef, const float* scale,
                   const float* shift, hipStream_t s) {
  hipLaunchKernelGGL((k_bn_dx_blk<MASK, V>), dim3(blocked_grid(n8)), dim3(256), 0, s, static_cast<const uint4*>(dy),
                     static_cast<const uint4*>(x), static_cast<uint4*>(dx), n8, C, coef, scale, shift);
}

// dispatch on the per-thread depth (2, 4 or 8 vectors per tensor)
void apply_blk(const void* x, const void* res, void* y, int64_t n8, int C, const float* scale, const float* shift,
               int relu, hipStream_t s) {
  if (g_elem_vpt == 2)
    launch_apply_blk<2>(x, res, y, n8, C, scale, shift, relu, s);
  else if (g_elem_vpt == 8)
    launch_apply_blk<8>(x, res, y, n8, C, scale, shift, relu, s);
  else
    launch_apply_blk<4>(x, res, y, n8, C, scale, shift, relu, s);
}

template <bool MASK>
void dx_blk(const void* dy, const void* x, void* dx, int64_t n8, int C, const float* coef, const float* scale,
            const float* shift, hipStream_t s) {
  if (g_elem_vpt == 2)
    launch_dx_blk<MASK, 2>(dy, x, dx, n8, C, coef, scale, shift, s);
  else if (g_elem_vpt == 8)
    launch_dx_blk<MASK, 8>(dy, x, dx, n8, C, coef, scale, shift, s);
  else
    launch_dx_blk<MASK, 4>(dy, x, dx, n8, C, coef, scale, shift, s);
}

int elementwise_grid(int64_t n8) {
  const int64_t b = (n8 + 255) / 256;
  return (int)std::min<int64_t>(b, g_elem_blocks);
}

}  // namespace

void bn_set_tuning(int max_parts, int elem_blocks, int elem_unroll) {
  if (max_parts > 0) g_max_parts = max_parts;
  if (elem_blocks > 0) g_elem_blocks = g_blk_blocks = elem_blocks;
  if (elem_unroll == 1 || elem_unroll == 2) g_elem_unroll = elem_unroll;
}

void bn_set_elementwise(int kind, int vectors_per_thread) {
  g_elem_kind = kind == 0 ? 0 : 1;
  if (vectors_per_thread == 2 || vectors_per_thread == 4 || vectors_per_thread == 8) g_elem_vpt = vectors_per_thread;
}

BnPlan bn_plan(int64_t M, int C) {
  BnPlan p;
  p.groups = C / 8;
  p.rows_iter = 256 / p.groups;
  const int64_t chunk = (int64_t)p.rows_iter * kUnroll;
  const int64_t nchunks = (M + chunk - 1) / chunk;
  const int64_t parts = std::min<int64_t>(std::max<int64_t>(nchunks, 1), g_max_parts);
  p.rows_wg = ((nchunks + parts - 1) / parts) * chunk;
  p.parts = (int)std::max<int64_t>(1, (M + p.rows_wg - 1) / p.rows_wg);
  // scratch rows: the partials, plus the pre-reduced rows when there are more than 256
  p.part_rows = p.parts + (p.parts > 1024 ? (p.parts + 63) / 64 : 0);
  return p;
}

void bn_forward_stats(const void* x, BnDType dt, int64_t M, int C, float* part, const float* gamma, const float* beta,
                      const float* mean_off, float* mean, float* invstd, float* scale, float* shift,
                      float* moving_mean, float* moving_var, float momentum, float eps, hipStream_t s,
                      int given_parts) {
  const BnPlan p = bn_plan(M, C);
  if (given_parts > 0) {  // partial sums already produced (by the conv epilogue that wrote x)
    int P = given_parts;
    const float* pr = prereduce(part, P, C, s);
    hipLaunchKernelGGL(k_bn_fwd_finalize, dim3((C + 63) / 64), dim3(64 * kFinPhases), 0, s, pr, P, M, C, gamma, beta,
                       mean_off, mean, invstd, scale, shift, moving_mean, moving_var, momentum, eps);
    return;
  }
  if (dt == BnDType::kBF16)
    hipLaunchKernelGGL((k_bn_partial<BnDType::kBF16, 0>), dim3(p.parts), dim3(256), 0, s, x, nullptr, nullptr, nullptr,
                       nullptr, nullptr, M, C, p.rows_wg, part);
  else
    hipLaunchKernelGGL((k_bn_partial<BnDType::kF32, 0>), dim3(p.parts), dim3(256), 0, s, x, nullptr, nullptr, nullptr,
                       nullptr, nullptr, M, C, p.rows_wg, part);
  int P = p.parts;
  const float* pr = prereduce(part, P, C, s);
  hipLaunchKernelGGL(k_bn_fwd_finalize, dim3((C + 63) / 64), dim3(64 * kFinPhases), 0, s, pr, P, M, C, gamma, beta,
                     mean_off, mean, invstd, scale, shift, moving_mean, moving_var, momentum, eps);
}

void bn_apply(const void* x, const void* residual, void* y, BnDType dt, int64_t M, int C, const float* scale,
              const float* shift, int relu, hipStream_t s) {
  const int64_t n8 = M * C / 8;
  if (blocked_ok(dt, C)) {
    apply_blk(x, residual, y, n8, C, scale, shift, relu, s);
    return;
  }
  const dim3 g(elementwise_grid(n8)), b(256);
  if (dt == BnDType::kBF16) {
    if (g_elem_unroll == 2)
      hipLaunchKernelGGL((k_bn_apply<BnDType::kBF16, 2>), g, b, 0, s, x, residual, y, n8, C, scale, shift, relu);
    else
      hipLaunchKernelGGL((k_bn_apply<BnDType::kBF16, 1>), g, b, 0, s, x, residual, y, n8, C, scale, shift, relu);
  } else {
    hipLaunchKernelGGL((k_bn_apply<BnDType::kF32, 1>), g, b, 0, s, x, residual, y, n8, C, scale, shift, relu);
  }
}

template <BnDType D>
static void bn_backward_t(const void* dy, const void* x, const void* y, void* dz, void* dx, int64_t M, int C,
                          float* part, const float* gamma, const float* mean, const float* invstd, const float* scale,
                          const float* shift, float* dgamma, float* dbeta, float* coef, int mode, int acc,
                          hipStream_t s, int given_parts) {
  const BnPlan p = bn_plan(M, C);
  const dim3 gp(p.parts), blk(256);
  if (given_parts > 0) {
    // dy is already the group's dz and `part` its reduction (the producing conv's epilogue)
    int P = given_parts;
    const float* pr = prereduce(part, P, C, s);
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(64 * kFinPhases), 0, s, pr, P, M, C, gamma, mean,
                       invstd, dgamma, dbeta, coef, acc);
    const int64_t n8 = M * C / 8;
    if (blocked_ok(D, C))
      dx_blk<false>(dy, x, dx, n8, C, coef, nullptr, nullptr, s);
    else
      hipLaunchKernelGGL((k_bn_dx<D, false, 1>), dim3(elementwise_grid(n8)), blk, 0, s, dy, x, dx, n8, C, coef,
                         nullptr, nullptr);
    return;
  }
  if (mode == 0)
    hipLaunchKernelGGL((k_bn_partial<D, 1>), gp, blk, 0, s, dy, x, nullptr, nullptr, nullptr, nullptr, M, C, p.rows_wg,
                       part);
  else if (mode == 1)
    hipLaunchKernelGGL((k_bn_partial<D, 2>), gp, blk, 0, s, dy, x, nullptr, scale, shift, nullptr, M, C, p.rows_wg,
                       part);
  else
    hipLaunchKernelGGL((k_bn_partial<D, 3>), gp, blk, 0, s, dy, x, y, nullptr, nullptr, dz, M, C, p.rows_wg, part);
  int P = p.parts;
  const float* pr = prereduce(part, P, C, s);
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(64 * kFinPhases), 0, s, pr, P, M, C, gamma, mean, invstd,
                     dgamma, dbeta, coef, acc);
  const int64_t n8 = M * C / 8;
  if (blocked_ok(D, C)) {
    if (mode == 1)
      dx_blk<true>(dy, x, dx, n8, C, coef, scale, shift, s);
    else
      dx_blk<false>(mode == 2 ? dz : dy, x, dx, n8, C, coef, nullptr, nullptr, s);
    return;
  }
  const dim3 ge(elementwise_grid(n8));
  const bool u2 = g_elem_unroll == 2 && D == BnDType::kBF16;
  if (mode == 1) {
    if (u2)
      hipLaunchKernelGGL((k_bn_dx<D, true, 2>), ge, blk, 0, s, dy, x, dx, n8, C, coef, scale, shift);
    else
      hipLaunchKernelGGL((k_bn_dx<D, true, 1>), ge, blk, 0, s, dy, x, dx, n8, C, coef, scale, shift);
  } else {
    if (u2)
      hipLaunchKernelGGL((k_bn_dx<D, false, 2>), ge, blk, 0, s, mode == 2 ? dz : dy, x, dx, n8, C, coef, nullptr,
                         nullptr);
    else
      hipLaunchKernelGGL((k_bn_dx<D, false, 1>), ge, blk, 0, s, mode == 2 ? dz : dy, x, dx, n8, C, coef, nullptr,
                         nullptr);
  }
}

void bn_backward(const void* dy, const void* x, const void* y, void* dz, void* dx, BnDType dt, int64_t M, int C,
                 float* part, const float* gamma, const float* mean, const float* invstd, const float* scale,
                 const float* shift, float* dgamma, float* dbeta, float* coef, int mode, int acc, hipStream_t s,
                 int given_parts) {
  if (dt == BnDType::kBF16)
    bn_backward_t<BnDType::kBF16>(dy, x, y, dz, dx, M, C, part, gamma, mean, invstd, scale, shift, dgamma, dbeta,
                                   coef, mode, acc, s, given_parts);
  else
    bn_backward_t<BnDType::kF32>(dy, x, y, dz, dx, M, C, part, gamma, mean, invstd, scale, shift, dgamma, dbeta, coef,
                                  mode, acc, s, given_parts);
}

}  // namespace tdl
