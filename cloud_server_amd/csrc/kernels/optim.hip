// Fused multi-tensor optimizer over the flat parameter buffer (gfx950 / CDNA4).
//
// Reference: tf.train.AdagradOptimizer(1e-4).minimize (construct_distribute.py:372-373)
// running ApplyAdagrad on the parameter server, plus the GD / Adam / Adadelta choices of
// the option catalog (apps/construction/util/options.py:26-37).  All 2.28 M parameters of
// the sample model live in one contiguous buffer, so the whole update is ONE launch of a
// float4-vectorised streaming kernel (memory-bound: w, g, slots read, w, slots written).
//
// Side jobs folded into the same launch (each would otherwise be its own tiny launch):
//   * zero the split-K / atomic accumulators the NEXT step's kernels add into,
//   * update BatchNorm running statistics from this step's forward partial slabs.
#include "common.h"

namespace csa {

enum Opt : int { OPT_SGD = 0, OPT_ADAGRAD = 1, OPT_ADAM = 2, OPT_ADADELTA = 3 };

constexpr int MAXZ = 16;
constexpr int MAXBN = 8;

struct ZeroList { float* p[MAXZ]; long n[MAXZ]; int count; };

struct BNRun {
  const float* slab; int nslab; int C; float count; float* rmean; float* rvar; float momentum;
};
struct BNRunList { BNRun r[MAXBN]; int count; };

struct OptArgs {
  int opt; float* w; const float* g; float* s0; float* s1; long n;
  float lr; const int64_t* step;   // 1-based step AFTER the head kernel's increment
  ZeroList z; BNRunList bn;
  int64_t* cursor;                 // batch-stream cursor: += 1 at the end of the step
};

__global__ __launch_bounds__(256) void optim_kernel(OptArgs a) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nth = (long)gridDim.x * blockDim.x;
  float lr = a.lr;
  if (a.opt == OPT_ADAM) {
    const float t = (float)(*a.step);
    lr = a.lr * sqrtf(1.f - powf(0.999f, t)) / (1.f - powf(0.9f, t));
  }
  const long n4 = a.n >> 2;
  float4* w4 = (float4*)a.w;
  const float4* g4 = (const float4*)a.g;
  float4* s04 = (float4*)a.s0;
  float4* s14 = (float4*)a.s1;
  for (long i = tid; i < n4; i += nth) {
    float4 w = w4[i];
    const float4 g = g4[i];
    float* wp = (float*)&w;
    const float* gp = (const float*)&g;
    if (a.opt == OPT_SGD) {
#pragma unroll
      for (int j = 0; j < 4; ++j) wp[j] -= lr * gp[j];
    } else if (a.opt == OPT_ADAGRAD) {
      float4 s = s04[i];
      float* sp = (float*)&s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sp[j] += gp[j] * gp[j];
        wp[j] -= lr * gp[j] * rsqrtf(sp[j]);
      }
      s04[i] = s;
    } else if (a.opt == OPT_ADAM) {
      float4 m = s04[i], v = s14[i];
      float* mp = (float*)&m;
      float* vp = (float*)&v;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        mp[j] = 0.9f * mp[j] + 0.1f * gp[j];
        vp[j] = 0.999f * vp[j] + 0.001f * gp[j] * gp[j];
        wp[j] -= lr * mp[j] / (sqrtf(vp[j]) + 1e-8f);
      }
      s04[i] = m;
      s14[i] = v;
    } else {  // Adadelta (TF: rho 0.95, eps 1e-8)
      float4 acc = s04[i], au = s14[i];
      float* ap = (float*)&acc;
      float* up = (float*)&au;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        ap[j] = 0.95f * ap[j] + 0.05f * gp[j] * gp[j];
        const float upd = sqrtf(up[j] + 1e-8f) / sqrtf(ap[j] + 1e-8f) * gp[j];
        up[j] = 0.95f * up[j] + 0.05f * upd * upd;
        wp[j] -= lr * upd;
      }
      s04[i] = acc;
      s14[i] = au;
    }
    w4[i] = w;
  }
  // zero accumulators for the next step
  for (int z = 0; z < a.z.count; ++z) {
    float* p = a.z.p[z];
    const long n = a.z.n[z];
    for (long i = tid; i < n; i += nth) p[i] = 0.f;
  }
  if (a.cursor && blockIdx.x == 0 && threadIdx.x == 0) *a.cursor += 1;
  // BN running statistics (one block)
  if (blockIdx.x == gridDim.x - 1) {
    for (int r = 0; r < a.bn.count; ++r) {
      const BNRun& b = a.bn.r[r];
      for (int c = threadIdx.x; c < b.C; c += blockDim.x) {
        float s1 = 0.f, s2 = 0.f;
        for (int i = 0; i < b.nslab; ++i) {
          s1 += b.slab[(size_t)i * 2 * b.C + c];
          s2 += b.slab[(size_t)i * 2 * b.C + b.C + c];
        }
        const float mean = s1 / b.count;
        const float var = fmaxf(s2 / b.count - mean * mean, 0.f);
        b.rmean[c] = (1.f - b.momentum) * b.rmean[c] + b.momentum * mean;
        b.rvar[c] = (1.f - b.momentum) * b.rvar[c] + b.momentum * var;
      }
    }
  }
}

}  // namespace csa

using namespace csa;

// zero_ptrs/zero_ns: count <= 16 regions; bn_*: count <= 8 descriptors, arrays of length count.
CSA_API int csa_optimizer(int opt, float* w, const float* g, float* s0, float* s1, long n, float lr,
                          const int64_t* step, float* const* zero_ptrs, const long* zero_ns,
                          int nzero, const float* const* bn_slabs, const int* bn_nslab,
                          const int* bn_C, const float* bn_count, float* const* bn_rmean,
                          float* const* bn_rvar, float momentum, int nbn, int64_t* cursor,
                          hipStream_t st) {
  if (n % 4 || nzero > MAXZ || nbn > MAXBN) return -1;
  OptArgs a{};
  a.cursor = cursor;
  a.opt = opt; a.w = w; a.g = g; a.s0 = s0; a.s1 = s1; a.n = n; a.lr = lr; a.step = step;
  a.z.count = nzero;
  for (int i = 0; i < nzero; ++i) { a.z.p[i] = zero_ptrs[i]; a.z.n[i] = zero_ns[i]; }
  a.bn.count = nbn;
  for (int i = 0; i < nbn; ++i)
    a.bn.r[i] = BNRun{bn_slabs[i], bn_nslab[i], bn_C[i], bn_count[i], bn_rmean[i], bn_rvar[i], momentum};
  long n4 = n / 4;
  int blocks = (int)((n4 + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(optim_kernel, dim3(blocks), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// Zero a list of regions (used once at init and by tests).
__global__ void zero_kernel(ZeroList z) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nth = (long)gridDim.x * blockDim.x;
  for (int k = 0; k < z.count; ++k)
    for (long i = tid; i < z.n[k]; i += nth) z.p[k][i] = 0.f;
}

CSA_API int csa_zero(float* const* ptrs, const long* ns, int count, hipStream_t st) {
  if (count > MAXZ) return -1;
  ZeroList z{};
  z.count = count;
  for (int i = 0; i < count; ++i) { z.p[i] = ptrs[i]; z.n[i] = ns[i]; }
  hipLaunchKernelGGL(zero_kernel, dim3(256), dim3(256), 0, st, z);
  return (int)hipGetLastError();
}
