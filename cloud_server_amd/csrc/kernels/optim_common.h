// Per-element optimizer updates shared by the standalone optimizer launch (optim.hip) and
// the kernels that apply the update in their own epilogue (dense_update.hip), so a
// parameter sees bit-identical arithmetic whichever kernel updates it.
//
// Reference: tf.train.AdagradOptimizer(1e-4) (construct_distribute.py:372-373) plus the
// GD / Adam / Adadelta choices of apps/construction/util/options.py:26-37, with TF's
// defaults (Adam b1 0.9 b2 0.999 eps 1e-8; Adadelta rho 0.95 eps 1e-8; Adagrad
// accumulators start at 0.1, set by the host).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace csa {

enum Opt : int { OPT_SGD = 0, OPT_ADAGRAD = 1, OPT_ADAM = 2, OPT_ADADELTA = 3 };

// Effective learning rate of this step.  ``step`` is the device step counter AFTER this
// step's increment (the head kernel advances it before any update runs): Adam's 1-based t.
__device__ __forceinline__ float opt_step_lr(int opt, float lr, const int64_t* step) {
  if (opt != OPT_ADAM) return lr;
  const float t = (float)(*step);
  return lr * sqrtf(1.f - powf(0.999f, t)) / (1.f - powf(0.9f, t));
}

// w, s0, s1 updated in place from gradient g (s1 only for Adam / Adadelta).
__device__ __forceinline__ void opt_update(int opt, float lr, float& w, float g, float& s0, float& s1) {
  if (opt == OPT_SGD) {
    w -= lr * g;
  } else if (opt == OPT_ADAGRAD) {
    s0 += g * g;
    w -= lr * g * rsqrtf(s0);
  } else if (opt == OPT_ADAM) {
    s0 = 0.9f * s0 + 0.1f * g;
    s1 = 0.999f * s1 + 0.001f * g * g;
    w -= lr * s0 / (sqrtf(s1) + 1e-8f);
  } else {  // Adadelta
    s0 = 0.95f * s0 + 0.05f * g * g;
    const float upd = sqrtf(s1 + 1e-8f) / sqrtf(s0 + 1e-8f) * g;
    s1 = 0.95f * s1 + 0.05f * upd * upd;
    w -= lr * upd;
  }
}

__host__ __device__ __forceinline__ int opt_nslots(int opt) {
  return opt == OPT_SGD ? 0 : (opt == OPT_ADAGRAD ? 1 : 2);
}

}  // namespace csa
