// Flat-slab optimizer updates (see optim.h).  The formulas are those of keras/optimizers.py (Keras
// semantics, the ones the eager torch fallback applies), element for element in f32: one pass over
// the slab, 16-B vector accesses, every state tensor read and written once.  Adam's bias correction
// uses the step t = *t0 + t_add + 1: the host refreshes t0 before each execution and a captured
// graph bakes each step's offset t_add in, so no host sync per step and no device counter race.
#include "common.h"
#include "optim.h"

namespace tdl {
namespace {

template <bool AMS>
__global__ __launch_bounds__(256) void k_adam(OptimArgs a) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const float lr = *a.lr;
  const float t = *a.t0 + (float)(a.t_add + 1);
  const float lr_t = lr * sqrtf(1.f - powf(a.b2, t)) / (1.f - powf(a.b1, t));
  const float decay = 1.f - lr * a.wd;
  auto one = [&](float& w, float g, float& m, float& v, float* vh) {
    if (a.wd != 0.f) w *= decay;
    m = m * a.b1 + g * (1.f - a.b1);
    v = v * a.b2 + g * g * (1.f - a.b2);
    float vv = v;
    if constexpr (AMS) {
      *vh = fmaxf(*vh, v);
      vv = *vh;
    }
    w = w - lr_t * m / (sqrtf(vv) + a.eps);
  };
  if (i4 + 3 < a.n) {
    f4 w = ld4(a.w + i4), m = ld4(a.s0 + i4), v = ld4(a.s1 + i4);
    const f4 g = ld4(a.g + i4);
    f4 vh = AMS ? ld4(a.s2 + i4) : zero4();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float wk = w[k], mk = m[k], vk = v[k], hk = vh[k];
      one(wk, g[k], mk, vk, &hk);
      w[k] = wk;
      m[k] = mk;
      v[k] = vk;
      vh[k] = hk;
    }
    st4(a.w + i4, w);
    st4(a.s0 + i4, m);
    st4(a.s1 + i4, v);
    if constexpr (AMS) st4(a.s2 + i4, vh);
  } else {
    for (int64_t j = i4; j < a.n; ++j) one(a.w[j], a.g[j], a.s0[j], a.s1[j], AMS ? a.s2 + j : nullptr);
  }
}

__global__ __launch_bounds__(256) void k_rmsprop(OptimArgs a) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const float lr = *a.lr;
  const bool mom = a.flags & 1, centered = a.flags & 2;
  for (int64_t j = i0; j < i0 + 4 && j < a.n; ++j) {
    const float g = a.g[j];
    const float rms = a.s0[j] * a.b1 + g * g * (1.f - a.b1);
    a.s0[j] = rms;
    float denom = rms;
    if (centered) {
      const float mg = a.s2[j] * a.b1 + g * (1.f - a.b1);
      a.s2[j] = mg;
      denom = rms - mg * mg;
    }
    const float step = g / (sqrtf(denom) + a.eps);
    if (mom) {
      const float m = a.s1[j] * a.b2 + lr * step;
      a.s1[j] = m;
      a.w[j] -= m;
    } else {
      a.w[j] -= lr * step;
    }
  }
}

__global__ __launch_bounds__(256) void k_adagrad(OptimArgs a) {
  const int64_t i4 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const float lr = *a.lr;
  if (i4 + 3 < a.n) {
    const f4 g = ld4(a.g + i4);
    const f4 acc = ld4(a.s0 + i4) + g * g;
    f4 w = ld4(a.w + i4);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = w[k] - lr * g[k] / (sqrtf(acc[k]) + a.eps);
    st4(a.s0 + i4, acc);
    st4(a.w + i4, w);
  } else {
    for (int64_t j = i4; j < a.n; ++j) {
      const float g = a.g[j];
      const float acc = a.s0[j] + g * g;
      a.s0[j] = acc;
      a.w[j] -= lr * g / (sqrtf(acc) + a.eps);
    }
  }
}

inline dim3 grid_of(int64_t n) { return dim3((unsigned)(((n + 3) / 4 + 255) / 256)); }

}  // namespace

void adam_apply(const OptimArgs& a, hipStream_t s) {
  if (a.n <= 0) return;
  if (a.flags & 1)
    hipLaunchKernelGGL(k_adam<true>, grid_of(a.n), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_adam<false>, grid_of(a.n), dim3(256), 0, s, a);
}
void rmsprop_apply(const OptimArgs& a, hipStream_t s) {
  if (a.n > 0) hipLaunchKernelGGL(k_rmsprop, grid_of(a.n), dim3(256), 0, s, a);
}
void adagrad_apply(const OptimArgs& a, hipStream_t s) {
  if (a.n > 0) hipLaunchKernelGGL(k_adagrad, grid_of(a.n), dim3(256), 0, s, a);
}

}  // namespace tdl
