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
//   * fold striped gradient accumulators: a conv weight gradient is accumulated by
//     hundreds of workgroups into S stripes (S x fewer atomics per cache line, see
//     conv.hip); the update of those parameters reads g = sum of the S stripes,
//   * advance the batch-stream cursor.
#include "common.h"

namespace csa {

enum Opt : int { OPT_SGD = 0, OPT_ADAGRAD = 1, OPT_ADAM = 2, OPT_ADADELTA = 3 };

constexpr int MAXZ = 16;
constexpr int MAXF = 8;

struct ZeroList { float* p[MAXZ]; long n[MAXZ]; int count; };

// g[off + e] = sum_s src[s * ld + e] for e < n (flat-buffer offsets; off % 4 == 0);
// the stripes are re-zeroed by the thread that folds them (their only reader)
struct Fold { long off, n, ld; float* src; int S; };
struct FoldList { Fold f[MAXF]; int count; long lo, hi; };

constexpr int MAXK = 8;
// Gradient ranges whose producer STORES every element each step (e.g. a dense weight
// gradient computed without split-K): the update need not re-zero them — for the sample
// model that is fc1's 8 MB, ~15 % of the optimizer's memory traffic.
struct KeepList { long lo[MAXK], hi[MAXK]; int count; };

struct OptArgs {
  int opt; float* w; const float* g; float* s0; float* s1; long n;
  float* gz;                       // if set (== g): each thread zeroes the gradient it read
  KeepList keep;                   // ... except inside these ranges (float4-aligned)
  float lr; const int64_t* step;   // 1-based step AFTER the head kernel's increment
  ZeroList z; FoldList fold;
  int64_t* cursor;                 // batch-stream cursor: += 1 (mod cursor_wrap) per step
  long cursor_wrap;
};

constexpr int MAXS = 16;   // stripes per folded gradient

__device__ __forceinline__ float4 fold_grad(const FoldList& fl, long e, float4 g) {
  float gs[4] = {g.x, g.y, g.z, g.w};
  for (int k = 0; k < fl.count; ++k) {
    const Fold& f = fl.f[k];
    if (e + 3 < f.off || e >= f.off + f.n) continue;
    const long i0 = e - f.off;
    if (i0 >= 0 && i0 + 4 <= f.n && (f.ld & 3) == 0) {
      // whole float4 inside the segment: all stripes' loads in flight together
      float4 v[MAXS];
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2)
        v[s2] = s2 < f.S ? *reinterpret_cast<const float4*>(f.src + s2 * f.ld + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) {
        acc.x += v[s2].x; acc.y += v[s2].y; acc.z += v[s2].z; acc.w += v[s2].w;
        if (s2 < f.S) *reinterpret_cast<float4*>(f.src + s2 * f.ld + i0) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      gs[0] = acc.x; gs[1] = acc.y; gs[2] = acc.z; gs[3] = acc.w;
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // segment edge: per element
      const long i = i0 + j;
      if (i < 0 || i >= f.n) continue;
      float v[MAXS];
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) v[s2] = s2 < f.S ? f.src[s2 * f.ld + i] : 0.f;
      float acc = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) {
        acc += v[s2];
        if (s2 < f.S) f.src[s2 * f.ld + i] = 0.f;
      }
      gs[j] = acc;
    }
  }
  return make_float4(gs[0], gs[1], gs[2], gs[3]);
}

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
    float4 g = g4[i];
    // Zeroing the accumulators the next step adds into must not race with this read:
    // a zero-list pass over flat-gradient ranges run by OTHER threads could clear an
    // element before its owner read it, so the owner clears what it read.
    if (a.gz) {
      bool keep = false;
      for (int k = 0; k < a.keep.count; ++k) keep |= (i * 4 >= a.keep.lo[k]) & (i * 4 < a.keep.hi[k]);
      if (!keep) reinterpret_cast<float4*>(a.gz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (i * 4 + 3 >= a.fold.lo && i * 4 < a.fold.hi) g = fold_grad(a.fold, i * 4, g);
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
  if (a.cursor && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t c = *a.cursor + 1;
    *a.cursor = (a.cursor_wrap > 0 && c >= a.cursor_wrap) ? 0 : c;
  }
}

}  // namespace csa

using namespace csa;

// zero_ptrs/zero_ns: count <= 16 regions; fold_*: count <= 8 striped-gradient descriptors.
// zero_grad != 0: the update clears g[i] after reading it (g is then an accumulator that
// must start the next step at zero); zero_ptrs must NOT overlap g or the fold stripes.
CSA_API int csa_optimizer(int opt, float* w, float* g, float* s0, float* s1, long n, int zero_grad,
                          float lr, const int64_t* step, float* const* zero_ptrs, const long* zero_ns,
                          int nzero, const long* fold_off, const long* fold_n, float* const* fold_src,
                          const int* fold_S, const long* fold_ld, int nfold, const long* keep_lo,
                          const long* keep_hi, int nkeep, int64_t* cursor, long cursor_wrap,
                          hipStream_t st) {
  if (n % 4 || nzero > MAXZ || nfold > MAXF || nkeep > MAXK) return -1;
  OptArgs a{};
  a.keep.count = nkeep;
  for (int i = 0; i < nkeep; ++i) {
    if (keep_lo[i] % 4 || keep_hi[i] % 4) return -1;
    a.keep.lo[i] = keep_lo[i];
    a.keep.hi[i] = keep_hi[i];
  }
  a.cursor = cursor;
  a.cursor_wrap = cursor_wrap;
  a.opt = opt; a.w = w; a.g = g; a.s0 = s0; a.s1 = s1; a.n = n; a.lr = lr; a.step = step;
  a.gz = zero_grad ? g : nullptr;
  a.z.count = nzero;
  for (int i = 0; i < nzero; ++i) { a.z.p[i] = zero_ptrs[i]; a.z.n[i] = zero_ns[i]; }
  a.fold.count = nfold;
  a.fold.lo = nfold ? fold_off[0] : 0;
  a.fold.hi = 0;
  for (int i = 0; i < nfold; ++i) {
    if (fold_off[i] % 4 || fold_S[i] > MAXS || fold_S[i] < 1) return -1;
    a.fold.f[i] = Fold{fold_off[i], fold_n[i], fold_ld[i], fold_src[i], fold_S[i]};
    a.fold.lo = fold_off[i] < a.fold.lo ? fold_off[i] : a.fold.lo;
    a.fold.hi = fold_off[i] + fold_n[i] > a.fold.hi ? fold_off[i] + fold_n[i] : a.fold.hi;
  }
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
