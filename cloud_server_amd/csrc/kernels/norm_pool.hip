// Standalone BatchNorm(+activation) and max-pool units (gfx950) — the general DSL layer
// orders the fused lowering cannot fold into a consumer:
//   * a norm after a dense layer (2-D BatchNorm over features, C up to thousands),
//   * a norm over more than 128 channels, a norm directly before the head,
//   * a pool that does not directly follow a conv (e.g. conv -> norm -> act -> pool),
//   * activation / norm sequences the consumer transform cannot express.
// The reference builds all of these with tf.nn.moments + tf.nn.batch_normalization and
// tf.nn.max_pool wherever the layer list puts them (construct_distribute.py:155-165,
// 208-265).  Here each becomes a materialised unit of the HIP step:
//
//   forward : bn_stats (per-channel {sum, sumsq} -> atomic slab rows)
//             bn_finalize (one tiny launch: mean/rstd/a/b tables + running-stat update,
//                          or the running statistics themselves in eval)
//             bn_apply   (y = act(x * a[c] + b[c]))
//   backward: bn_bwd_reduce (dz = act'(.) dy; {sum dz, sum dz*xhat} -> slab)
//             bn_bwd_finalize (dscale, doffset, the two dx coefficients)
//             bn_bwd_apply  (dx = a (dz - m1 - xhat m2))
//   pool    : maxpool_fwd (value + uint8 window argmax), maxpool_bwd (GATHER form: each
//             input sums the windows whose argmax points at it — no atomics, any
//             overlap, deterministic).
// Layouts: x is [N][C] row-major with C fastest (NHWC flattened: N = B*H*W; 2-D: N = B).
#include "common.h"

namespace csa {

constexpr int NP_THREADS = 256;
constexpr int NP_ROWS = 64;            // rows per stats / reduce block

// Per-channel sums of f(row, c) over this block's rows, folded atomically into
// slab row (blockIdx.x % nslab): out[0][c] += sum f0, out[1][c] += sum f1.  The in-block
// fold is fixed-order; with det (deterministic mode, nslab = gridDim.x) the block STORES
// its exclusive row blockIdx.x (the finalize kernels sum the rows in row order).
template <class F>
__device__ __forceinline__ void np_col_sums(long N, int C, float* slab, int nslab, int det, F f) {
  __shared__ float s_acc[2 * NP_THREADS];
  const int t = threadIdx.x;
  const long r0 = (long)blockIdx.x * NP_ROWS, r1 = r0 + NP_ROWS < N ? r0 + NP_ROWS : N;
  float* row = slab + (size_t)(det ? blockIdx.x : blockIdx.x % nslab) * 2 * C;
  if (C <= NP_THREADS) {
    const int per = NP_THREADS / C, sub = t / C, c = t - sub * C;
    float a0 = 0.f, a1 = 0.f;
    if (sub < per)
      for (long r = r0 + sub; r < r1; r += per) {
        float v0, v1;
        f(r, c, v0, v1);
        a0 += v0;
        a1 += v1;
      }
    // fold the `per` row groups of each channel through LDS, in row-group order
    s_acc[t] = a0;
    s_acc[NP_THREADS + t] = a1;
    __syncthreads();
    if (t < C) {
      float s0 = 0.f, s1 = 0.f;
      for (int u = 0; u < per; ++u) { s0 += s_acc[u * C + t]; s1 += s_acc[NP_THREADS + u * C + t]; }
      if (det) { row[t] = s0; row[C + t] = s1; }
      else { atomicAdd(&row[t], s0); atomicAdd(&row[C + t], s1); }
    }
  } else {
    for (int c = t; c < C; c += NP_THREADS) {
      float a0 = 0.f, a1 = 0.f;
      for (long r = r0; r < r1; ++r) {
        float v0, v1;
        f(r, c, v0, v1);
        a0 += v0;
        a1 += v1;
      }
      if (det) { row[c] = a0; row[C + c] = a1; }
      else { atomicAdd(&row[c], a0); atomicAdd(&row[C + c], a1); }
    }
  }
}

__global__ __launch_bounds__(NP_THREADS) void bn_stats_kernel(const float* __restrict__ x, long N, int C,
                                                             float* slab, int nslab, int det) {
  np_col_sums(N, C, slab, nslab, det, [&](long r, int c, float& v0, float& v1) {
    const float v = x[r * C + c];
    v0 = v;
    v1 = v * v;
  });
}

// tab = [mean | rstd | a | b] x C.  mode 0: batch statistics from the slab (+ running
// update when rm != null);  mode 1: the running statistics (eval).
__global__ __launch_bounds__(NP_THREADS) void bn_finalize_kernel(const float* slab, int nslab, int C, float count,
                                                                float eps, const float* scale, const float* offset,
                                                                float* rm, float* rv, float momentum, int mode,
                                                                float* tab) {
  const int c = blockIdx.x * NP_THREADS + threadIdx.x;
  if (c >= C) return;
  float mean, var;
  if (mode == 1) {
    mean = rm[c];
    var = rv[c];
  } else {
    float s0 = 0.f, s1 = 0.f;
    for (int r = 0; r < nslab; ++r) {
      s0 += slab[(size_t)r * 2 * C + c];
      s1 += slab[(size_t)r * 2 * C + C + c];
    }
    mean = s0 / count;
    var = fmaxf(s1 / count - mean * mean, 0.f);
    if (rm != nullptr) {
      rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
      rv[c] = (1.f - momentum) * rv[c] + momentum * var;
    }
  }
  const float rstd = rsqrtf(var + eps);
  const float a = (scale ? scale[c] : 1.f) * rstd;
  tab[c] = mean;
  tab[C + c] = rstd;
  tab[2 * C + c] = a;
  tab[3 * C + c] = (offset ? offset[c] : 0.f) - mean * a;
}

// y = act(x * a[c] + b[c]);  tab == null: y = act(x) (activation-only unit)
__global__ __launch_bounds__(NP_THREADS) void bn_apply_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                             long n, int C, const float* __restrict__ tab, int act,
                                                             float alpha) {
  for (long i = (long)blockIdx.x * NP_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * NP_THREADS) {
    float v = x[i];
    if (tab) {
      const int c = (int)(i % C);
      v = v * tab[2 * C + c] + tab[3 * C + c];
    }
    y[i] = act_fwd(v, act, alpha);
  }
}

__device__ __forceinline__ float np_dz(const float* x, const float* y, const float* dy, long i, int c, int C,
                                       const float* tab, int act, float alpha) {
  const float xv = x[i];
  const float z = tab ? xv * tab[2 * C + c] + tab[3 * C + c] : xv;
  return act_bwd(dy[i], z, y[i], act, alpha);
}

__global__ __launch_bounds__(NP_THREADS) void bn_bwd_reduce_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                  const float* __restrict__ dy, long N, int C,
                                                                  const float* __restrict__ tab, int act, float alpha,
                                                                  float* slab, int nslab, int det) {
  np_col_sums(N, C, slab, nslab, det, [&](long r, int c, float& v0, float& v1) {
    const long i = r * C + c;
    const float dz = np_dz(x, y, dy, i, c, C, tab, act, alpha);
    const float xhat = (x[i] - tab[c]) * tab[C + c];
    v0 = dz;
    v1 = dz * xhat;
  });
}

// dscale[c] = sum dz*xhat * gscale, doffset[c] = sum dz * gscale;  k = [m1 | m2] x C with
// m1 = sum dz / count, m2 = sum dz*xhat / count (the dx coefficients)
__global__ __launch_bounds__(NP_THREADS) void bn_bwd_finalize_kernel(const float* slab, int nslab, int C, float count,
                                                                    float gscale, float* dscale, float* doffset,
                                                                    float* k) {
  const int c = blockIdx.x * NP_THREADS + threadIdx.x;
  if (c >= C) return;
  float s0 = 0.f, s1 = 0.f;
  for (int r = 0; r < nslab; ++r) {
    s0 += slab[(size_t)r * 2 * C + c];
    s1 += slab[(size_t)r * 2 * C + C + c];
  }
  if (dscale) dscale[c] = s1 * gscale;
  if (doffset) doffset[c] = s0 * gscale;
  k[c] = s0 / count;
  k[C + c] = s1 / count;
}

// dx = a (dz - m1 - xhat m2) with norm;  dx = dz for an activation-only unit (tab null)
__global__ __launch_bounds__(NP_THREADS) void bn_bwd_apply_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                                                 const float* __restrict__ dy, float* __restrict__ dx,
                                                                 long n, int C, const float* __restrict__ tab,
                                                                 const float* __restrict__ k, int act, float alpha) {
  for (long i = (long)blockIdx.x * NP_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * NP_THREADS) {
    const int c = tab ? (int)(i % C) : 0;
    const float dz = np_dz(x, y, dy, i, c, C, tab, act, alpha);
    if (!tab) {
      dx[i] = dz;
      continue;
    }
    const float xhat = (x[i] - tab[c]) * tab[C + c];
    dx[i] = tab[2 * C + c] * (dz - k[c] - xhat * k[C + c]);
  }
}

// ---------------------------------------------------------------- max pool (NHWC)
struct PoolGeom { int B, H, W, C, kh, kw, sh, sw, pt, pl, OH, OW; };

__global__ __launch_bounds__(NP_THREADS) void maxpool_fwd_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                uint8_t* __restrict__ am, PoolGeom g) {
  const long n = (long)g.B * g.OH * g.OW * g.C;
  for (long i = (long)blockIdx.x * NP_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * NP_THREADS) {
    const int c = (int)(i % g.C);
    long r = i / g.C;
    const int ox = (int)(r % g.OW);
    r /= g.OW;
    const int oy = (int)(r % g.OH);
    const int b = (int)(r / g.OH);
    float best = -INFINITY;
    int arg = 0;
    for (int dy = 0; dy < g.kh; ++dy) {
      const int yy = oy * g.sh - g.pt + dy;
      if (yy < 0 || yy >= g.H) continue;
      for (int dx = 0; dx < g.kw; ++dx) {
        const int xx = ox * g.sw - g.pl + dx;
        if (xx < 0 || xx >= g.W) continue;
        const float v = x[(((long)b * g.H + yy) * g.W + xx) * g.C + c];
        if (v > best) {                  // first maximum wins (tf.nn.max_pool gradient)
          best = v;
          arg = dy * g.kw + dx;
        }
      }
    }
    y[i] = best;
    am[i] = (uint8_t)arg;
  }
}

__global__ __launch_bounds__(NP_THREADS) void maxpool_bwd_kernel(const float* __restrict__ dy,
                                                                const uint8_t* __restrict__ am,
                                                                float* __restrict__ dx, PoolGeom g) {
  const long n = (long)g.B * g.H * g.W * g.C;
  for (long i = (long)blockIdx.x * NP_THREADS + threadIdx.x; i < n; i += (long)gridDim.x * NP_THREADS) {
    const int c = (int)(i % g.C);
    long r = i / g.C;
    const int xx = (int)(r % g.W);
    r /= g.W;
    const int yy = (int)(r % g.H);
    const int b = (int)(r / g.H);
    // output windows covering (yy, xx): oy*sh - pt <= yy <= oy*sh - pt + kh - 1
    const int ty = yy + g.pt, tx = xx + g.pl;
    const int oy0 = ty - g.kh + 1 > 0 ? (ty - g.kh + 1 + g.sh - 1) / g.sh : 0;
    const int oy1 = min(ty / g.sh, g.OH - 1);
    const int ox0 = tx - g.kw + 1 > 0 ? (tx - g.kw + 1 + g.sw - 1) / g.sw : 0;
    const int ox1 = min(tx / g.sw, g.OW - 1);
    float acc = 0.f;
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const long o = (((long)b * g.OH + oy) * g.OW + ox) * g.C + c;
        const int arg = (ty - oy * g.sh) * g.kw + (tx - ox * g.sw);
        if (am[o] == arg) acc += dy[o];
      }
    dx[i] = acc;
  }
}

static unsigned np_grid(long n) {
  long g = (n + NP_THREADS - 1) / NP_THREADS;
  return (unsigned)(g < 1 ? 1 : (g > 8192 ? 8192 : g));
}

}  // namespace csa

using namespace csa;

// Slab rows a stats / backward-reduce launch folds into (the caller allocates
// [rows][2][C] and zeroes it before every step).
CSA_API int csa_bn_slab_rows() { return 16; }

// Statistic-slab rows for N rows of input: 16 atomically-folded rows, or in deterministic
// mode one exclusive row per stats / reduce workgroup.
CSA_API int csa_bn_stat_rows(long N) { return g_csa_det ? (int)((N + NP_ROWS - 1) / NP_ROWS) : 16; }

CSA_API int csa_bn_stats(const float* x, long N, int C, float* slab, int nslab, hipStream_t st) {
  if (N <= 0 || C <= 0 || nslab <= 0) return -1;
  const long nb = (N + NP_ROWS - 1) / NP_ROWS;
  if (g_csa_det && nslab < nb) return -3;          // det: one exclusive row per workgroup
  hipLaunchKernelGGL(bn_stats_kernel, dim3((unsigned)nb), dim3(NP_THREADS), 0, st, x, N, C, slab, nslab,
                     g_csa_det);
  return (int)hipGetLastError();
}

CSA_API int csa_bn_finalize(const float* slab, int nslab, int C, float count, float eps, const float* scale,
                            const float* offset, float* rm, float* rv, float momentum, int mode, float* tab,
                            hipStream_t st) {
  if (C <= 0) return -1;
  hipLaunchKernelGGL(bn_finalize_kernel, dim3((unsigned)((C + NP_THREADS - 1) / NP_THREADS)), dim3(NP_THREADS), 0,
                     st, slab, nslab, C, count, eps, scale, offset, rm, rv, momentum, mode, tab);
  return (int)hipGetLastError();
}

CSA_API int csa_bn_apply(const float* x, float* y, long n, int C, const float* tab, int act, float alpha,
                         hipStream_t st) {
  if (n <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(np_grid(n)), dim3(NP_THREADS), 0, st, x, y, n, C, tab, act, alpha);
  return (int)hipGetLastError();
}

CSA_API int csa_bn_bwd_reduce(const float* x, const float* y, const float* dy, long N, int C, const float* tab,
                              int act, float alpha, float* slab, int nslab, hipStream_t st) {
  if (N <= 0 || C <= 0 || !tab) return -1;
  const long nb = (N + NP_ROWS - 1) / NP_ROWS;
  if (g_csa_det && nslab < nb) return -3;
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3((unsigned)nb), dim3(NP_THREADS), 0, st, x, y, dy, N, C, tab, act,
                     alpha, slab, nslab, g_csa_det);
  return (int)hipGetLastError();
}

CSA_API int csa_bn_bwd_finalize(const float* slab, int nslab, int C, float count, float gscale, float* dscale,
                                float* doffset, float* k, hipStream_t st) {
  if (C <= 0) return -1;
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((unsigned)((C + NP_THREADS - 1) / NP_THREADS)), dim3(NP_THREADS),
                     0, st, slab, nslab, C, count, gscale, dscale, doffset, k);
  return (int)hipGetLastError();
}

CSA_API int csa_bn_bwd_apply(const float* x, const float* y, const float* dy, float* dx, long n, int C,
                             const float* tab, const float* k, int act, float alpha, hipStream_t st) {
  if (n <= 0 || C <= 0) return -1;
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(np_grid(n)), dim3(NP_THREADS), 0, st, x, y, dy, dx, n, C, tab, k,
                     act, alpha);
  return (int)hipGetLastError();
}

// g = {B, H, W, C, kh, kw, sh, sw, pad_top, pad_left, OH, OW}; kh * kw <= 256
CSA_API int csa_maxpool_fwd(const float* x, float* y, uint8_t* argmax, const int* g, hipStream_t st) {
  PoolGeom p{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11]};
  if (p.kh * p.kw > 256 || p.kh < 1 || p.kw < 1 || p.sh < 1 || p.sw < 1) return -1;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(np_grid((long)p.B * p.OH * p.OW * p.C)), dim3(NP_THREADS), 0, st,
                     x, y, argmax, p);
  return (int)hipGetLastError();
}

CSA_API int csa_maxpool_bwd(const float* dy, const uint8_t* argmax, float* dx, const int* g, hipStream_t st) {
  PoolGeom p{g[0], g[1], g[2], g[3], g[4], g[5], g[6], g[7], g[8], g[9], g[10], g[11]};
  if (p.kh * p.kw > 256 || p.kh < 1 || p.kw < 1 || p.sh < 1 || p.sw < 1) return -1;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(np_grid((long)p.B * p.H * p.W * p.C)), dim3(NP_THREADS), 0, st,
                     dy, argmax, dx, p);
  return (int)hipGetLastError();
}
