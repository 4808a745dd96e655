// Flat-slab optimizer updates for gfx950 (see optim.hip): Keras Adam / AdamW (+AMSGrad), RMSprop
// (+momentum, centered) and Adagrad over a whole parameter slab in ONE launch, learning rate and step
// counter read from device memory so a captured execution graph replays them correctly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tdl {

struct OptimArgs {
  float* w;
  const float* g;
  float* s0;          // Adam m / RMSprop rms / Adagrad accumulator
  float* s1;          // Adam v / RMSprop momentum (or null)
  float* s2;          // Adam vhat (AMSGrad) / RMSprop mean gradient (centered) (or null)
  const float* lr;    // device learning rate
  const float* t0;    // Adam: device step count of the execution's first step (float, exact to 2^24)
  int64_t n;
  float b1, b2, eps;  // Adam beta_1 / beta_2 / epsilon; RMSprop rho / momentum / epsilon
  float wd;           // AdamW decoupled weight decay (0: none)
  int t_add;          // Adam: this step's offset from t0 (the step's index inside a captured execution)
  int flags;          // Adam: 1 AMSGrad; RMSprop: 1 momentum, 2 centered
};

void adam_apply(const OptimArgs& a, hipStream_t s);
void rmsprop_apply(const OptimArgs& a, hipStream_t s);
void adagrad_apply(const OptimArgs& a, hipStream_t s);

}  // namespace tdl
