// Dense-layer backward + optimizer update in ONE launch (gfx950 / CDNA4).
//
// Reference: the train op minimize() of construct_distribute.py:372-373 — gradients of
// the dense layers (:168-182) followed by ApplyAdagrad on the parameter server.  On one
// GPU nothing needs the dense weight gradient except the optimizer, so it is never
// written to memory: every workgroup owns FT = 16 rows of W ([K][N], input features x
// output features) and, for those rows,
//
//   1. stages dY [M][N] (the whole output gradient, L2-resident) and its W rows in LDS;
//   2. wgrad   dW[f][n] = sum_m Xw[m][f] dY[m][n]       (v_mfma_f32_16x16x4_f32, K = M);
//   3. dgrad   dX[m][f] = sum_n dY[m][n] W[f][n]        (same MFMA, K = N, split over the
//              4 waves, folded in LDS), through the forward input transform's backward
//              (activation, BatchNorm partial statistics) exactly like csa_dense_dgrad;
//   4. update  W[f][:] and its optimizer slots with the shared per-element rule
//              (optim_common.h), reading the OLD W from LDS — no other workgroup reads
//              these rows, so updating in place inside the backward is race-free.
//
// Block 0 also forms the bias gradient (column sums of dY) and updates the bias.
// Memory per step for the sample fc1 (3920 x 512): W and the Adagrad accumulator read
// once and written once (32 MB) instead of the separate backward pair + optimizer pass
// (dW written, re-read, W/acc read and written, ~56 MB, two launches).
//
// LDS layout: row stride S = N + 2 (S/2 odd) makes the dgrad operand reads — lanes
// spanning 16 rows x 2 columns — hit 32 distinct banks.
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15], D[4*(l>>4)+r][l&15].
#include "common.h"
#include "optim_common.h"

namespace csa {

typedef float du_f32x4 __attribute__((ext_vector_type(4)));

constexpr int DU_FT = 16;          // W rows per workgroup
constexpr int DU_THREADS = 256;
constexpr int DU_MAXTILES = 8;     // 16-wide output-feature tiles per wave (N <= 512)
constexpr int DU_MAXKS = 16;       // batch k-steps of 4 (M <= 64)
constexpr size_t DU_LDS_MAX = 160 * 1024;
constexpr int MAXC_DU = 128;       // BatchNorm channels handled in LDS

struct DUArgs {
  int M, K, N;
  const float* dY;          // [M][N]
  float* W;                 // [K][N] parameters (updated in place)
  float* bias;              // [N] or null
  float* dX;                // [M][K] input gradient (null: first layer, no dgrad)
  const float* x_fwd;       // [M][K] pre-transform forward input (act / BN backward)
  int act; float alpha;
  BNRef bn; int bn_on;      // forward BatchNorm of the input, channel = f % C
  float* bwd_slab;          // [gridDim.x][2][C]: {sum dz, sum dz*xhat} per workgroup
  const float* Xw;          // [M][K] weight-gradient operand (transform applied)
  int opt; float lr; const int64_t* step;
  float* s0w; float* s1w;   // optimizer slots of W (same [K][N] layout) ...
  float* s0b; float* s1b;   // ... and of the bias
  float scale;
};

__host__ __device__ inline size_t du_lds_floats(int M, int N) {
  const int S = N + 2;
  const size_t part = 4 * 4 * 256;                      // dgrad fold (aliases dY)
  const size_t dy = (size_t)M * S > part ? (size_t)M * S : part;
  return dy + (size_t)DU_FT * S + 4 * MAXC_DU + 2 * MAXC_DU;
}

__global__ __launch_bounds__(DU_THREADS) void dense_bwd_update_kernel(DUArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int M = a.M, K = a.K, N = a.N;
  const int S = N + 2;
  const size_t dyf = (size_t)M * S > 4096 ? (size_t)M * S : 4096;
  float* s_dy = smem;                  // [M][S]; after the MFMAs: dgrad fold [4][4][256]
  float* s_w = smem + dyf;             // [16][S] this block's (old) W rows
  float* s_bn = s_w + DU_FT * S;       // [mean | rstd | a | b] x MAXC_DU
  float* s_st = s_bn + 4 * MAXC_DU;    // [2][MAXC_DU] BN-backward sums / slab scratch
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, q = lane >> 4;
  const int f0 = blockIdx.x * DU_FT;
  const int nf = min(DU_FT, K - f0);
  const int ntile = N >> 4;
  const int ksteps = (M + 3) >> 2;

  // ---- weight-gradient B operand (Xw[m][f], m = 4s + q) and this lane's optimizer
  // slots: global loads issued first, they land under the staging / MFMAs
  float xb[DU_MAXKS];
#pragma unroll
  for (int s = 0; s < DU_MAXKS; ++s) {
    const int m = 4 * s + q;
    const bool ok = s < ksteps && m < M && i16 < nf;
    const float v = a.Xw[ok ? (long)m * K + f0 + i16 : 0];
    xb[s] = ok ? v : 0.f;
  }
  const int nslot = a.opt == OPT_SGD ? 0 : (a.opt == OPT_ADAGRAD ? 1 : 2);
  float4 p0[DU_MAXTILES], p1[DU_MAXTILES];
#pragma unroll
  for (int tt = 0; tt < DU_MAXTILES; ++tt) {
    const int nt = wave + 4 * tt;
    const bool ok = nt < ntile && i16 < nf;
    const long gi = ok ? (long)(f0 + i16) * N + nt * 16 + 4 * q : 0;
    p0[tt] = (nslot >= 1 && ok) ? *reinterpret_cast<const float4*>(a.s0w + gi) : make_float4(0.f, 0.f, 0.f, 0.f);
    p1[tt] = (nslot >= 2 && ok) ? *reinterpret_cast<const float4*>(a.s1w + gi) : make_float4(0.f, 0.f, 0.f, 0.f);
  }

  // ---- staging: dY and this block's W rows -> LDS (float4 loads, all in flight per
  // batch; float2 stores since S is even but not a multiple of 4)
  {
    const int n4 = N >> 2;
    const int tot_dy = M * n4, tot = tot_dy + nf * n4;
    const float4* gdy = reinterpret_cast<const float4*>(a.dY);
    const float4* gw = reinterpret_cast<const float4*>(a.W + (long)f0 * N);
    const FastDiv dn4(n4);
    constexpr int U = 8;
    for (int base = 0; base < tot; base += DU_THREADS * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(base + u * DU_THREADS + tid, tot - 1);
        v[u] = e < tot_dy ? gdy[e] : gw[e - tot_dy];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * DU_THREADS + tid;
        if (e >= tot) break;
        int r, c;
        float* dst;
        if (e < tot_dy) { dn4.divmod(e, r, c); dst = s_dy + r * S + 4 * c; }
        else { dn4.divmod(e - tot_dy, r, c); dst = s_w + r * S + 4 * c; }
        reinterpret_cast<float2*>(dst)[0] = make_float2(v[u].x, v[u].y);
        reinterpret_cast<float2*>(dst)[1] = make_float2(v[u].z, v[u].w);
      }
    }
    for (int e = nf * S + tid; e < DU_FT * S; e += DU_THREADS) s_w[e] = 0.f;   // tail rows
  }
  if (a.dX && a.bn_on) bn_reduce_to_lds(a.bn, s_bn, s_bn + MAXC_DU, s_bn + 2 * MAXC_DU, s_bn + 3 * MAXC_DU, s_st);
  __syncthreads();
  // bias gradient (block 0): column sums of dY while it is in LDS
  float bg[2] = {0.f, 0.f};
  if (blockIdx.x == 0 && a.bias) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int n = tid + u * DU_THREADS;
      if (n < N)
        for (int m = 0; m < M; ++m) bg[u] += s_dy[m * S + n];
    }
  }

  // ---- weight gradient: rows = output features n (16-wide tiles, round-robin over the
  // waves), cols = this block's 16 input features, K = batch
  du_f32x4 wacc[DU_MAXTILES];
#pragma unroll
  for (int tt = 0; tt < DU_MAXTILES; ++tt) wacc[tt] = du_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < DU_MAXKS; ++s) {
    if (s >= ksteps) break;
    const int m = 4 * s + q;
    const bool okm = m < M;
    const float* row = s_dy + (okm ? m : 0) * S + i16;
    float av[DU_MAXTILES];
#pragma unroll
    for (int tt = 0; tt < DU_MAXTILES; ++tt) {
      const int nt = wave + 4 * tt;
      av[tt] = (okm && nt < ntile) ? row[nt * 16] : 0.f;
    }
#pragma unroll
    for (int tt = 0; tt < DU_MAXTILES; ++tt)
      if (wave + 4 * tt < ntile) wacc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[tt], xb[s], wacc[tt], 0, 0, 0);
  }

  // ---- input gradient: 4 batch tiles of 16 rows x 16 features, K = N split over waves
  if (a.dX) {
    du_f32x4 dacc[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) dacc[t] = du_f32x4{0.f, 0.f, 0.f, 0.f};
    const int nq = N >> 2;                 // multiple of 4
    const int nb = wave * nq;
    const float* wrow = s_w + i16 * S + nb + q;
    const float* drow[4];
    bool okr[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int m = 16 * t + i16;
      okr[t] = m < M;
      drow[t] = s_dy + (okr[t] ? m : 0) * S + nb + q;
    }
#pragma unroll 4
    for (int s = 0; s < nq; s += 4) {
      const float bv = wrow[s];
      float av[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) av[t] = okr[t] ? drow[t][s] : 0.f;
#pragma unroll
      for (int t = 0; t < 4; ++t) dacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv, dacc[t], 0, 0, 0);
    }
    __syncthreads();                       // every wave done with s_dy: fold area reuses it
    float* s_part = s_dy;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_part[(wave * 4 + t) * 256 + (4 * q + r) * 16 + i16] = dacc[t][r];
    for (int c = tid; c < 2 * MAXC_DU && a.bn_on; c += DU_THREADS) s_st[c] = 0.f;
    __syncthreads();
    // epilogue: thread -> feature j = tid & 15 (fixed), 4 batch rows
    const int j = tid & 15;
    const int f = f0 + j;
    const int C = a.bn.C > 0 ? a.bn.C : 1;
    const int ch = f % C;
    const bool tf = a.act != ACT_NONE || a.bn_on;
    float sd = 0.f, sdx = 0.f;
    float xv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + DU_THREADS * u;
      const int m = 16 * (e >> 8) + ((e & 255) >> 4);
      const bool ok = tf && m < M && j < nf;
      const float v = a.x_fwd ? a.x_fwd[ok ? (long)m * K + f : 0] : 0.f;
      xv[u] = v;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + DU_THREADS * u;
      const int t = e >> 8, rem = e & 255;
      const int m = 16 * t + (rem >> 4);
      if (m >= M || j >= nf) continue;
      float g = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) g += s_part[(w * 4 + t) * 256 + rem];
      if (tf) {
        const float x = xv[u];
        const float z = a.bn_on ? x * s_bn[2 * MAXC_DU + ch] + s_bn[3 * MAXC_DU + ch] : x;
        const float y = act_fwd(z, a.act, a.alpha);
        g = act_bwd(g, z, y, a.act, a.alpha);
        if (a.bn_on) {
          sd += g;
          sdx += g * (x - s_bn[ch]) * s_bn[MAXC_DU + ch];
        }
      }
      a.dX[(long)m * K + f] = g;
    }
    if (a.bn_on && a.bwd_slab) {
      if (j < nf) { atomicAdd(&s_st[ch], sd); atomicAdd(&s_st[MAXC_DU + ch], sdx); }
      __syncthreads();
      float* row = a.bwd_slab + (size_t)blockIdx.x * 2 * C;
      for (int c = tid; c < 2 * C; c += DU_THREADS) row[c] = c < C ? s_st[c] : s_st[MAXC_DU + c - C];
    }
  }

  // ---- optimizer update of this block's W rows (old W from LDS), slots prefetched
  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  if (i16 < nf) {
#pragma unroll
    for (int tt = 0; tt < DU_MAXTILES; ++tt) {
      const int nt = wave + 4 * tt;
      if (nt >= ntile) break;
      const int n = nt * 16 + 4 * q;
      const float* wl = s_w + i16 * S + n;
      const float2 w01 = *reinterpret_cast<const float2*>(wl);
      const float2 w23 = *reinterpret_cast<const float2*>(wl + 2);
      float w[4] = {w01.x, w01.y, w23.x, w23.y};
      float s0[4] = {p0[tt].x, p0[tt].y, p0[tt].z, p0[tt].w};
      float s1[4] = {p1[tt].x, p1[tt].y, p1[tt].z, p1[tt].w};
#pragma unroll
      for (int r = 0; r < 4; ++r) opt_update(a.opt, lr, w[r], wacc[tt][r] * a.scale, s0[r], s1[r]);
      const long gi = (long)(f0 + i16) * N + n;
      *reinterpret_cast<float4*>(a.W + gi) = make_float4(w[0], w[1], w[2], w[3]);
      if (nslot >= 1) *reinterpret_cast<float4*>(a.s0w + gi) = make_float4(s0[0], s0[1], s0[2], s0[3]);
      if (nslot >= 2) *reinterpret_cast<float4*>(a.s1w + gi) = make_float4(s1[0], s1[1], s1[2], s1[3]);
    }
  }
  // ---- bias update (block 0)
  if (blockIdx.x == 0 && a.bias) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int n = tid + u * DU_THREADS;
      if (n >= N) continue;
      const float g = bg[u];
      float w = a.bias[n];
      float s0 = nslot >= 1 ? a.s0b[n] : 0.f, s1 = nslot >= 2 ? a.s1b[n] : 0.f;
      opt_update(a.opt, lr, w, g * a.scale, s0, s1);
      a.bias[n] = w;
      if (nslot >= 1) a.s0b[n] = s0;
      if (nslot >= 2) a.s1b[n] = s1;
    }
  }
}

}  // namespace csa

using namespace csa;

// Shape family of the fused kernel (0 = outside: the caller uses the separate backward
// kernels + the flat optimizer).  Needs M <= 64, N % 16 == 0, N <= 512, the LDS budget.
CSA_API int csa_dense_bwd_update_ok(int M, int K, int N, int bn_C) {
  if (M < 1 || M > 4 * DU_MAXKS || K < 1 || N < 16 || N % 16 || N > 16 * 4 * DU_MAXTILES) return 0;
  if (bn_C > MAXC_DU) return 0;
  return du_lds_floats(M, N) * sizeof(float) <= DU_LDS_MAX ? 1 : 0;
}

// BN-backward slab rows the kernel writes (one per workgroup).
CSA_API int csa_dense_bwd_update_slabs(int K) { return (K + DU_FT - 1) / DU_FT; }

CSA_API int csa_dense_bwd_update(const float* dY, float* W, float* bias, float* dX, int M, int K, int N,
                                 const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                 int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                 const float* bn_offset, float* bwd_slab, const float* Xw, int opt, float lr,
                                 const int64_t* step, float* s0w, float* s1w, float* s0b, float* s1b,
                                 float scale, hipStream_t st) {
  if (!csa_dense_bwd_update_ok(M, K, N, bn_slab ? bn_C : 0)) return -1;
  if (!Xw || !W || !dY) return -2;
  DUArgs a{};
  a.M = M; a.K = K; a.N = N; a.dY = dY; a.W = W; a.bias = bias; a.dX = dX; a.x_fwd = x_fwd;
  a.act = act; a.alpha = alpha;
  a.bn = BNRef{bn_slab, bn_nslab, bn_slab ? bn_C : 1, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr; a.bwd_slab = bwd_slab; a.Xw = Xw;
  a.opt = opt; a.lr = lr; a.step = step; a.s0w = s0w; a.s1w = s1w; a.s0b = s0b; a.s1b = s1b; a.scale = scale;
  static bool attr = hipFuncSetAttribute((const void*)dense_bwd_update_kernel,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  const size_t shm = du_lds_floats(M, N) * sizeof(float);
  hipLaunchKernelGGL(dense_bwd_update_kernel, dim3((unsigned)((K + DU_FT - 1) / DU_FT)), dim3(DU_THREADS), shm,
                     st, a);
  return (int)hipGetLastError();
}
