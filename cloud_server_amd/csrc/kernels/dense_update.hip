// Dense-layer backward + optimizer update in ONE launch (gfx950 / CDNA4).
//
// Reference: the train op minimize() of construct_distribute.py:372-373 — gradients of
// the dense layers (:168-182) followed by ApplyAdagrad on the parameter server.  On one
// GPU nothing needs a dense weight gradient except the optimizer, so it is never written
// to memory.
//
// Decomposition (round 2, v4).  W is [K][N] (input x output features).  One 1024-thread
// workgroup per ROW GROUP of 16 input features (f0 .. f0+15) owns those W rows across ALL
// N columns, so the input gradient of its features is complete inside the workgroup (no
// split-K, no cross-workgroup hand-off) and every W element has exactly one owner (the
// in-place update is race-free).  fc1 of the sample config: 245 workgroups = one round
// on 256 CUs; everything is issued as ONE batch of loads at kernel start:
//
//   dY           the whole [M][N] batch gradient -> LDS (row stride N + 4);
//   W / slots    lane (i = lane & 15, q = lane >> 4) of wave w, column sub-tile
//                j in {w, w + 16} (16 columns each): W[f0 + i][16j + 4q .. +3] as one float4
//                straight into registers (the "update layout");
//   Xw           the weight-gradient operand Xw[4s + q][f0 + i] (13 k-steps at M = 50);
//   x_fwd, BN    the epilogue's forward input and BatchNorm tables (precomputed by
//                csa_bn_act_apply, so the epilogue needs no slab reduction).
//
// Per sub-tile: wgrad  dW[f][n] = sum_m dY[m][n] Xw[m][f]  (v_mfma_f32_16x16x4_f32,
// A = dY[4s + q][16j + i] from LDS, B = Xw) lands in the update layout, so the optimizer
// update is register-local; dgrad partial  dX[m][f] += sum_n dY[m][n] W[f][n]  (A = one
// LDS float4 dY[16t + i][16j + 4q ..], B = the OLD W float4, consumed before the update).
// The 16 waves' partials fold in LDS in fixed order, then the forward input transform's
// backward (activation; BatchNorm partial statistics into the backward slab) and dX.
// Bias gradients (column sums of dY) are spread over the workgroups, a few columns each.
//
// Earlier designs measured slower (profiles/r2_dense_fused.md): one 256-thread workgroup
// per row group walking N in 8 dependent chunks (23 us for fc1), and 16 x 64 tiles with a
// write-through partial hand-off to the row group's last arriving tile (31 us: 1960 tiles
// queue for slots and the elected tile's epilogue is a second chain).
//
// HBM per step for the sample fc1 (3920 x 512): W and the Adagrad accumulator read once
// and written once (32 MB) — instead of the split-K backward pair (dW written) plus the
// flat optimizer pass (dW, W, acc re-read).
#include "common.h"
#include "optim_common.h"
#include <cstdlib>

namespace csa {

typedef float du_f32x4 __attribute__((ext_vector_type(4)));

constexpr int DU_FT = 16;            // W rows per workgroup
constexpr int DU_WAVES = 16;
constexpr int DU_THREADS = 64 * DU_WAVES;
constexpr int DU_SUB = 2;            // 16-column sub-tiles per wave (N <= 16 * 16 * 2 = 512)
constexpr int DU_MAXM = 64;          // batch rows (4 tiles of 16)
constexpr int DU_KS = DU_MAXM / 4;   // wgrad MFMA k-steps (4 batch rows each)
constexpr int MAXC_DU = 128;         // BatchNorm channels handled in LDS
constexpr int DU_SLAB = 16;          // BN-backward slab rows (atomically folded)
constexpr size_t DU_LDS_MAX = 150 * 1024;

struct DUArgs {
  int M, K, N;
  const float* dY;          // [M][N]
  float* W;                 // [K][N] parameters (updated in place)
  float* bias;              // [N] or null
  float* dX;                // [M][K] input gradient (null: first layer, no dgrad)
  const float* x_fwd;       // [M][K] pre-transform forward input (act / BN backward)
  int act; float alpha;
  BNRef bn; int bn_on;      // forward BatchNorm of the input, channel = f % C
  const float* bn_tab;      // [4][C] mean | rstd | a | b (null: reduce bn.slab here)
  float* bwd_slab;          // [DU_SLAB][2][C]: {sum dz, sum dz*xhat}, atomically folded
  const float* Xw;          // [M][K] weight-gradient operand (transform applied)
  int opt; float lr; const int64_t* step;
  float* s0w; float* s1w;   // optimizer slots of W (same [K][N] layout) ...
  float* s0b; float* s1b;   // ... and of the bias
  float scale;
  int bias_per;             // bias columns per workgroup
};

// diagnostics: s_memrealtime stamps (100 MHz, one clock for all XCDs) of EVERY block,
// [block][8] = start, dY staged, W landed, MFMA + update done, fold done, dX stored, end
// (scripts/microbench.py MB_DU)
__constant__ long long* g_du_dbg = nullptr;
#define DU_STAMP(i)                                                                          \
  do {                                                                                       \
    if (g_du_dbg && threadIdx.x == 0) g_du_dbg[blockIdx.x * 8 + (i)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)

__host__ __device__ inline int du_sn(int N) { return N + 4; }            // dY LDS row stride
__host__ __device__ inline int du_tiles(int M) { return (M + 15) / 16; } // batch tiles of 16
__host__ __device__ inline size_t du_lds_floats(int M, int N) {
  const size_t a = (size_t)M * du_sn(N), b = (size_t)DU_WAVES * 4 * 16 * DU_FT;   // dY | the fold
  return (a > b ? a : b) + DU_MAXM * DU_FT + 6 * MAXC_DU;
}

// Write back the updated W / slot float4s of a lane's sub-tiles (rows < nf, columns < N).
template <int NSLOT>
__device__ __forceinline__ void du_store_w(const DUArgs& a, const float4 (&wv)[DU_SUB], const float4 (&s0v)[DU_SUB],
                                           const float4 (&s1v)[DU_SUB], const long (&wofs)[DU_SUB], int wave, int i,
                                           int nf, int N, bool bown, int bn0, float bw, float bs0, float bs1) {
  if (bown && (threadIdx.x & 63) == 0) {     // the wave's first bias column
    a.bias[bn0] = bw;
    if (NSLOT >= 1) a.s0b[bn0] = bs0;
    if (NSLOT >= 2) a.s1b[bn0] = bs1;
  }
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    if (16 * (wave + DU_WAVES * j) >= N || i >= nf) continue;
    *reinterpret_cast<float4*>(a.W + wofs[j]) = wv[j];
    if (NSLOT >= 1) *reinterpret_cast<float4*>(a.s0w + wofs[j]) = s0v[j];
    if (NSLOT >= 2) *reinterpret_cast<float4*>(a.s1w + wofs[j]) = s1v[j];
  }
}

// NSLOT = optimizer slots (0 SGD, 1 Adagrad, 2 Adam / Adadelta): unused slot registers
// are not allocated (the 1024-thread workgroup has 128 VGPRs per lane)
template <int NSLOT>
__global__ __launch_bounds__(DU_THREADS) void dense_bwd_update_kernel(DUArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int M = a.M, K = a.K, N = a.N, SN = du_sn(N);
  float* sdy = smem;                                       // [M][SN] dY, later the fold
  float* s_bn = smem + du_lds_floats(M, N) - 6 * MAXC_DU;  // [mean | rstd | a | b] x MAXC_DU
  float* sxw = s_bn - DU_MAXM * DU_FT;                     // [64 m][16 f] Xw slice, later BN partials
  float* s_st = s_bn + 4 * MAXC_DU;                        // [2][MAXC_DU] slab-reduction scratch
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int grp = blockIdx.x, f0 = grp * DU_FT, nf = min(DU_FT, K - f0);
  const bool dgrad = a.dX != nullptr;
  const bool tf = dgrad && (a.act != ACT_NONE || a.bn_on);
  constexpr int nslot = NSLOT;
  DU_STAMP(0);

  // ---- every load, issued in the order it is consumed (vmcnt retires in order).  Two
  // column halves: half j = columns [256 j, 256 j + 256) = every wave's sub-tile j, so the
  // MFMAs of half 0 run while half 1's dY and W are still in flight.
  // (0) the weight-gradient operand slice Xw[m][f0 .. f0+15], one element per thread
  float xw1 = a.Xw[(long)min(tid >> 4, M - 1) * K + f0 + min(tid & 15, nf - 1)];
  const int n4 = N >> 2;
  int h4[DU_SUB];
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) h4[j] = max(min(N - 256 * j, 256), 0) >> 2;
  const float* b0 = nslot >= 1 ? a.s0w : a.W;              // address select: loads stay unconditional
  const float* b1 = nslot >= 2 ? a.s1w : a.W;
  const int frow = f0 + min(i, nf - 1);
  float4 dyv[DU_SUB][4], wv[DU_SUB], s0v[DU_SUB], s1v[DU_SUB];
  long wofs[DU_SUB];
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    // (1) dY half j: float4 e = u * 1024 + tid -> row e / h4, column 256 j + 4 (e % h4)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * DU_THREADS + tid;
      int row = 0, c4 = 0;
      if (h4[j] == 64) { row = e >> 6; c4 = e & 63; }
      else if (h4[j] > 0) { row = e / h4[j]; c4 = e - row * h4[j]; }
      dyv[j][u] = reinterpret_cast<const float4*>(a.dY)[min(row, M - 1) * n4 + (h4[j] > 0 ? 64 * j + c4 : 0)];
    }
    // (2) W and slot float4s of sub-tile j
    const int col = min(16 * (wave + DU_WAVES * j), N - 16) + 4 * q;
    wofs[j] = (long)frow * N + col;
    wv[j] = *reinterpret_cast<const float4*>(a.W + wofs[j]);
    s0v[j] = s1v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (nslot >= 1) s0v[j] = *reinterpret_cast<const float4*>(b0 + wofs[j]);
    if (nslot >= 2) s1v[j] = *reinterpret_cast<const float4*>(b1 + wofs[j]);
  }
  // (3) bias: wave w owns column grp * bias_per + w (+16 r); its first operands prefetched
  //     (unconditional loads from selected addresses: a load inside a branch is waited
  //     for right there, and vmcnt is in order — it would wait for W too)
  const int bn0 = grp * a.bias_per + wave;
  const bool bown = a.bias && wave < a.bias_per && bn0 < N;
  const int bnc = bown ? bn0 : 0;
  float bw = (a.bias ? a.bias : a.dY)[bnc];
  float bs0 = (nslot >= 1 && a.bias ? a.s0b : a.dY)[bnc];
  float bs1 = (nslot >= 2 && a.bias ? a.s1b : a.dY)[bnc];
  // (4) epilogue operands: thread -> (batch row em = tid / 16, feature ef = tid % 16)
  const int em = tid >> 4, ef = tid & 15;
  const bool eok = dgrad && em < M && ef < nf;
  const bool tabs = a.bn_on && a.bn_tab;
  const int C = a.bn.C > 0 ? a.bn.C : 1;
  const int ch = (f0 + ef) % C;
  const float* xsrc = tf && a.x_fwd ? a.x_fwd : a.Xw;     // address select (same [M][K] shape)
  float xf = xsrc[(long)min(em, M - 1) * K + f0 + min(ef, nf - 1)];
  const float* tsrc = tabs ? a.bn_tab : a.Xw;
  const int tc = tabs ? ch : 0, tC = tabs ? C : 0;
  float tmean = tsrc[tc], trstd = tsrc[tC + tc], ta = tsrc[2 * tC + tc], tb = tsrc[3 * tC + tc];

  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  du_f32x4 dacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dacc[t] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  float xb[DU_KS];                                         // weight-gradient B: Xw[4s + q][f0 + i]
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    if (j == 0) {
      pin(xw1);
      sxw[tid] = ((tid >> 4) < M && (tid & 15) < nf) ? xw1 : 0.f;
    }
    // stage dY half j (rows < M only: dgrad rows >= M are clamped reads whose outputs are
    // dropped, wgrad rows >= M meet Xw = 0); its columns are disjoint from half 0's, which
    // other waves may still be reading
#pragma unroll
    for (int u = 0; u < 4; ++u) pin(dyv[j][u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * DU_THREADS + tid;
      if (h4[j] > 0 && e < M * h4[j]) {
        const int row = h4[j] == 64 ? e >> 6 : e / h4[j];
        const int c4 = e - row * h4[j];
        *reinterpret_cast<float4*>(sdy + row * SN + 256 * j + 4 * c4) = dyv[j][u];
      }
    }
    if (j == 0 && a.bn_on && dgrad && !tabs)              // no precomputed tables: reduce here
      bn_reduce_to_lds(a.bn, s_bn, s_bn + MAXC_DU, s_bn + 2 * MAXC_DU, s_bn + 3 * MAXC_DU, s_st);
    __syncthreads();
    if (j == 0) {
      DU_STAMP(1);
#pragma unroll
      for (int s = 0; s < DU_KS; ++s) xb[s] = sxw[(4 * s + q) * DU_FT + i];
    }
    pin(wv[j]); pin(s0v[j]); pin(s1v[j]);
    if (j == 0) DU_STAMP(2);
    const int n0 = 16 * (wave + DU_WAVES * j);
    if (n0 >= N) continue;                                 // wave-uniform
    // input-gradient partial (OLD weights): 4 batch tiles x 4 k-steps
    const float wk[4] = {wv[j].x, wv[j].y, wv[j].z, wv[j].w};
    if (dgrad) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (16 * t >= M) break;
        const float4 d4 = *reinterpret_cast<const float4*>(sdy + min(16 * t + i, M - 1) * SN + n0 + 4 * q);
        const float ak[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) dacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(ak[k], i < nf ? wk[k] : 0.f, dacc[t], 0, 0, 0);
      }
    }
    // weight gradient: A = dY[4s + q][n0 + i] (LDS), two accumulators
    du_f32x4 g0 = du_f32x4{0.f, 0.f, 0.f, 0.f}, g1 = g0;
    const float* col = sdy + n0 + i;
#pragma unroll
    for (int s = 0; s < DU_KS; s += 2) {
      if (4 * s >= M) break;                               // uniform
      const float a0 = col[min(4 * s + q, M - 1) * SN];
      const float a1 = col[min(4 * s + 4 + q, M - 1) * SN];
      g0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, xb[s], g0, 0, 0, 0);
      g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, xb[s + 1], g1, 0, 0, 0);
    }
    // optimizer update of the lane's 4 weights (D lane (i, q) = dW[f0 + i][n0 + 4q + r]);
    // written back after the fold: a store in flight would hold the fold's barrier (the
    // compiler drains vmcnt before it) for the whole 16 MB write-back
    float w[4] = {wv[j].x, wv[j].y, wv[j].z, wv[j].w};
    float s0[4] = {s0v[j].x, s0v[j].y, s0v[j].z, s0v[j].w};
    float s1[4] = {s1v[j].x, s1v[j].y, s1v[j].z, s1v[j].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) opt_update(a.opt, lr, w[r], (g0[r] + g1[r]) * a.scale, s0[r], s1[r]);
    wv[j] = make_float4(w[0], w[1], w[2], w[3]);
    s0v[j] = make_float4(s0[0], s0[1], s0[2], s0[3]);
    s1v[j] = make_float4(s1[0], s1[1], s1[2], s1[3]);
  }
  pin(bw); pin(bs0); pin(bs1); pin(xf); pin(tmean); pin(trstd); pin(ta); pin(tb);
  // bias: column sums of dY over the batch, one column per wave (prefetched operands)
  if (bown) {
    for (int u = wave; u < a.bias_per; u += DU_WAVES) {
      const int n = grp * a.bias_per + u;
      if (n >= N) break;
      float v = lane < M ? sdy[lane * SN + n] : 0.f;
      v = wave_sum(v);
      if (lane == 0) {
        if (u != wave) {
          bw = a.bias[n];
          if (nslot >= 1) bs0 = a.s0b[n];
          if (nslot >= 2) bs1 = a.s1b[n];
        }
        opt_update(a.opt, lr, bw, v * a.scale, bs0, bs1);
        if (u != wave) {                                   // the first column is stored late
          a.bias[n] = bw;
          if (nslot >= 1) a.s0b[n] = bs0;
          if (nslot >= 2) a.s1b[n] = bs1;
        }
      }
    }
  }
  DU_STAMP(3);
  if (!dgrad) {                                            // uniform: first layer
    du_store_w<NSLOT>(a, wv, s0v, s1v, wofs, wave, i, nf, N, bown, bn0, bw, bs0, bs1);
    return;
  }

  // ---- fold the 16 waves' partials.  Layout [wave][t][q][i][r]: lane (i, q) of tile t
  // holds rows 16t + 4q + r of feature i, written as one conflict-free float4; a reading
  // wave (4 rows x 16 features) reads 64 consecutive floats
  __syncthreads();                                         // every dY read is done
  float* fold = sdy;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (16 * t >= M) break;
    *reinterpret_cast<du_f32x4*>(fold + ((wave * 4 + t) * 4 + q) * 64 + 4 * i) = dacc[t];
  }
  __syncthreads();
  DU_STAMP(4);
  du_store_w<NSLOT>(a, wv, s0v, s1v, wofs, wave, i, nf, N, bown, bn0, bw, bs0, bs1);
  float g = 0.f;
  {
    const int t = em >> 4, qq = (em >> 2) & 3, r = em & 3;
    const float* src = fold + (t * 4 + qq) * 64 + 4 * ef + r;
#pragma unroll
    for (int w = 0; w < DU_WAVES; ++w) g += em < M ? src[w * 4 * 4 * 64] : 0.f;
  }
  float v1 = 0.f, v2 = 0.f;
  if (eok) {
    if (tf) {
      float mean = tmean, rstd = trstd, sa = ta, sb = tb;
      if (a.bn_on && !tabs) {
        mean = s_bn[ch]; rstd = s_bn[MAXC_DU + ch]; sa = s_bn[2 * MAXC_DU + ch]; sb = s_bn[3 * MAXC_DU + ch];
      }
      const float z = a.bn_on ? xf * sa + sb : xf;
      const float y = act_fwd(z, a.act, a.alpha);
      g = act_bwd(g, z, y, a.act, a.alpha);
      v1 = g;
      v2 = g * (xf - mean) * rstd;
    }
    a.dX[(long)em * K + f0 + ef] = g;
  }
  DU_STAMP(5);
  if (a.bn_on && a.bwd_slab) {
    // BN-backward statistics per feature in fixed order: the wave's 4 rows by shuffles,
    // the 16 waves through LDS (sxw is free), then one atomic per (feature, statistic)
    // into one of DU_SLAB rows (zeroed every step by the optimizer launch)
    v1 += __shfl_xor(v1, 16, 64); v1 += __shfl_xor(v1, 32, 64);
    v2 += __shfl_xor(v2, 16, 64); v2 += __shfl_xor(v2, 32, 64);
    float* sred = sxw;                                     // [16 waves][2][16]
    if (lane < 16) { sred[wave * 32 + lane] = v1; sred[wave * 32 + 16 + lane] = v2; }
    __syncthreads();
    if (tid < 32 && (tid & 15) < nf) {
      float acc = 0.f;
#pragma unroll
      for (int w = 0; w < DU_WAVES; ++w) acc += sred[w * 32 + tid];
      const int st = tid >> 4, c = (f0 + (tid & 15)) % C;
      atomicAdd(a.bwd_slab + (size_t)(grp % DU_SLAB) * 2 * C + st * C + c, acc);
    }
  }
  DU_STAMP(6);
}

}  // namespace csa

using namespace csa;

CSA_API int csa_du_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_du_dbg), &p, sizeof(p));
}

// Shape family of the fused kernel (0 = outside: the caller uses the separate backward
// kernels + the flat optimizer).  Needs M <= 64, N % 16 == 0, N <= 512, dY in LDS.
CSA_API int csa_dense_bwd_update_ok(int M, int K, int N, int bn_C) {
  if (M < 1 || M > DU_MAXM || K < 1 || N < 16 || N % 16 || N > 16 * DU_WAVES * DU_SUB) return 0;
  if (bn_C > MAXC_DU) return 0;
  return du_lds_floats(M, N) * sizeof(float) <= DU_LDS_MAX ? 1 : 0;
}

// BN-backward slab rows the kernel accumulates into (atomically; the caller zeroes them).
CSA_API int csa_dense_bwd_update_slabs(int K) { return (K + DU_FT - 1) / DU_FT < DU_SLAB ? (K + DU_FT - 1) / DU_FT : DU_SLAB; }

CSA_API int csa_dense_bwd_update(const float* dY, float* W, float* bias, float* dX, int M, int K, int N,
                                 const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                 int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                 const float* bn_offset, float* bwd_slab, const float* Xw, int opt, float lr,
                                 const int64_t* step, float* s0w, float* s1w, float* s0b, float* s1b,
                                 float scale, const float* bn_tab, hipStream_t st) {
  if (!csa_dense_bwd_update_ok(M, K, N, bn_slab ? bn_C : 0)) return -1;
  if (!Xw || !W || !dY) return -2;
  DUArgs a{};
  a.M = M; a.K = K; a.N = N; a.dY = dY; a.W = W; a.bias = bias; a.dX = dX; a.x_fwd = x_fwd;
  a.act = act; a.alpha = alpha;
  a.bn = BNRef{bn_slab, bn_nslab, bn_slab ? bn_C : 1, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr; a.bn_tab = bn_slab ? bn_tab : nullptr;
  a.bwd_slab = bwd_slab; a.Xw = Xw;
  a.opt = opt; a.lr = lr; a.step = step; a.s0w = s0w; a.s1w = s1w; a.s0b = s0b; a.s1b = s1b; a.scale = scale;
  const int groups = (K + DU_FT - 1) / DU_FT;
  a.bias_per = (N + groups - 1) / groups;
  const size_t shm = du_lds_floats(M, N) * sizeof(float);
  static const bool attr =
      hipFuncSetAttribute((const void*)dense_bwd_update_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess &&
      hipFuncSetAttribute((const void*)dense_bwd_update_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess &&
      hipFuncSetAttribute((const void*)dense_bwd_update_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  const int ns = opt_nslots(opt);
  if (ns == 0) hipLaunchKernelGGL(dense_bwd_update_kernel<0>, dim3((unsigned)groups), dim3(DU_THREADS), shm, st, a);
  else if (ns == 1) hipLaunchKernelGGL(dense_bwd_update_kernel<1>, dim3((unsigned)groups), dim3(DU_THREADS), shm, st, a);
  else hipLaunchKernelGGL(dense_bwd_update_kernel<2>, dim3((unsigned)groups), dim3(DU_THREADS), shm, st, a);
  return (int)hipGetLastError();
}
