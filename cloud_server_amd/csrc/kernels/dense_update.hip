// Dense-layer backward + optimizer update in ONE launch (gfx950 / CDNA4).
//
// Reference: the train op minimize() of construct_distribute.py:372-373 — gradients of
// the dense layers (:168-182) followed by ApplyAdagrad on the parameter server.  On one
// GPU nothing needs a dense weight gradient except the optimizer, so it is never written
// to memory.  Every workgroup owns FT = 16 rows of W ([K][N], input x output features)
// and walks N in chunks of 64 columns through a two-stage LDS pipeline (the next chunk's
// dY / W / optimizer-slot loads are in flight while the current chunk computes):
//
//   wgrad   dW[f][n] = sum_m Xw[m][f] dY[m][n]     (v_mfma_f32_16x16x4_f32, K = batch);
//   update  W[f][n] and its slots with the shared per-element rule (optim_common.h), from
//           the OLD W in the LDS stage — no other workgroup reads these rows, so updating
//           in place inside the backward is race-free;
//   dgrad   dX[m][f] += sum_{n in chunk} dY[m][n] W[f][n]  (accumulated over the chunks,
//           the 4 waves' K slices folded in LDS at the end), then through the forward
//           input transform's backward (activation, BatchNorm partial statistics) exactly
//           like csa_dense_dgrad.
//
// One extra workgroup forms the bias gradient (column sums of dY) and updates the bias.
// Memory per step for the sample fc1 (3920 x 512): W and the Adagrad accumulator read
// once and written once (32 MB) instead of the separate backward pair + optimizer pass
// (dW written, re-read, W/acc read and written: ~56 MB and two launches).
//
// LDS stage rows have stride SC = 66 (SC/2 odd): the dgrad operand reads — lanes spanning
// 16 rows x 2 columns — hit 32 distinct banks.  ~45 KB of LDS per workgroup.
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15], D[4*(l>>4)+r][l&15].
#include "common.h"
#include "optim_common.h"
#include <cstdlib>

namespace csa {

typedef float du_f32x4 __attribute__((ext_vector_type(4)));

constexpr int DU_FT = 16;          // W rows per workgroup
constexpr int DU_THREADS = 256;
constexpr int DU_NC = 64;          // output-feature columns per pipeline chunk
constexpr int DU_SC = DU_NC + 2;   // LDS row stride of a stage
constexpr int DU_MAXM = 64;        // batch rows (4 m-tiles of 16)
constexpr int DU_MAXKS = DU_MAXM / 4;
constexpr int DU_DYV = DU_MAXM * (DU_NC / 4) / DU_THREADS;   // dY float4 loads per thread per chunk
constexpr int MAXC_DU = 128;       // BatchNorm channels handled in LDS
constexpr int DU_SLAB = 16;        // BN-backward slab rows (atomically folded)
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
  float* bwd_slab;          // [DU_SLAB][2][C]: {sum dz, sum dz*xhat}, atomically folded
  const float* Xw;          // [M][K] weight-gradient operand (transform applied)
  int opt; float lr; const int64_t* step;
  float* s0w; float* s1w;   // optimizer slots of W (same [K][N] layout) ...
  float* s0b; float* s1b;   // ... and of the bias
  float scale;
  int nmain;                // W-row workgroups (the bias workgroup is block nmain)
  int dbg;                  // diagnostics (CSA_DU_DBG bits): 1 no wgrad, 2 no dgrad, 4 no update, 8 no loads
};

__constant__ long long* g_du_dbg = nullptr;   // diagnostics: s_memtime stamps of block 0
#define DU_STAMP(i)                                                                          \
  do {                                                                                       \
    if (g_du_dbg && threadIdx.x == 0 && blockIdx.x == 0) g_du_dbg[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

__host__ __device__ inline size_t du_stage_floats(int) { return (size_t)(DU_MAXM + DU_FT) * DU_SC; }
constexpr int DU_NSTAGE = 3;       // LDS stages (load / compute / update of 3 chunks in flight)
constexpr int DU_DWF = DU_FT * DU_NC; // one chunk's weight gradient, [16 f][64 n]
__host__ __device__ inline size_t du_lds_floats(int M) {
  const size_t st = DU_NSTAGE * du_stage_floats(M) + 2 * DU_DWF;
  const size_t fold = 4 * 4 * 256;
  return (st > fold ? st : fold) + 6 * MAXC_DU;
}

// Chunk loads of one thread: dY rows (DU_DYV float4, masked) + one float4 of the W rows.
struct DUChunk {
  float4 dy[DU_DYV];
  float4 w;
};

__device__ __forceinline__ void du_load(const DUArgs& a, int c, int f0, int nf, int tid, DUChunk& r) {
  const int M = a.M, N = a.N, n0 = c * DU_NC;
  const int tot = M * (DU_NC / 4);
#pragma unroll
  for (int u = 0; u < DU_DYV; ++u) {
    const int e = min(u * DU_THREADS + tid, tot - 1);
    r.dy[u] = *reinterpret_cast<const float4*>(a.dY + (long)(e >> 4) * N + n0 + 4 * (e & 15));
  }
  const int row = min(tid >> 4, nf - 1);
  r.w = *reinterpret_cast<const float4*>(a.W + (long)(f0 + row) * N + n0 + 4 * (tid & 15));
}

__device__ __forceinline__ void du_store(const DUChunk& r, float* st, int M, int nf, int tid) {
  const int tot = M * (DU_NC / 4);
  float* sdy = st;
  float* sw = st + DU_MAXM * DU_SC;
#pragma unroll
  for (int u = 0; u < DU_DYV; ++u) {
    const int e = u * DU_THREADS + tid;
    if (e < tot) {
      float* d = sdy + (e >> 4) * DU_SC + 4 * (e & 15);
      reinterpret_cast<float2*>(d)[0] = make_float2(r.dy[u].x, r.dy[u].y);
      reinterpret_cast<float2*>(d)[1] = make_float2(r.dy[u].z, r.dy[u].w);
    }
  }
  const int row = tid >> 4;
  const float4 w = row < nf ? r.w : make_float4(0.f, 0.f, 0.f, 0.f);
  float* d = sw + row * DU_SC + 4 * (tid & 15);
  reinterpret_cast<float2*>(d)[0] = make_float2(w.x, w.y);
  reinterpret_cast<float2*>(d)[1] = make_float2(w.z, w.w);
}

__device__ __forceinline__ void du_pin(DUChunk& r) {
#pragma unroll
  for (int u = 0; u < DU_DYV; ++u) pin(r.dy[u]);
  pin(r.w);
}

// The bias workgroup: db[n] = sum_m dY[m][n], then the update (batched, pinned loads).
__device__ __forceinline__ void du_bias(const DUArgs& a) {
  const int tid = threadIdx.x, M = a.M, N = a.N;
  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  const int nslot = opt_nslots(a.opt);
  for (int n = tid; n < N; n += DU_THREADS) {
    float g = 0.f;
    for (int m0 = 0; m0 < M; m0 += 16) {
      float v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = a.dY[(long)min(m0 + u, M - 1) * N + n];
#pragma unroll
      for (int u = 0; u < 16; ++u) pin(v[u]);
#pragma unroll
      for (int u = 0; u < 16; ++u) g += (m0 + u < M) ? v[u] : 0.f;
    }
    float w = a.bias[n];
    float s0 = nslot >= 1 ? a.s0b[n] : 0.f, s1 = nslot >= 2 ? a.s1b[n] : 0.f;
    opt_update(a.opt, lr, w, g * a.scale, s0, s1);
    a.bias[n] = w;
    if (nslot >= 1) a.s0b[n] = s0;
    if (nslot >= 2) a.s1b[n] = s1;
  }
}

__global__ __launch_bounds__(DU_THREADS) void dense_bwd_update_kernel(DUArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if ((int)blockIdx.x >= a.nmain) {
    if (a.bias) du_bias(a);
    return;
  }
  const int M = a.M, K = a.K, N = a.N;
  const size_t stf = du_stage_floats(M);
  float* s_st0 = smem;
  float* s_bn = smem + du_lds_floats(M) - 6 * MAXC_DU;   // [mean | rstd | a | b] x MAXC_DU
  float* s_st = s_bn + 4 * MAXC_DU;                      // [2][MAXC_DU] BN-backward sums
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, q = lane >> 4;
  const int f0 = blockIdx.x * DU_FT;
  const int nf = min(DU_FT, K - f0);
  const int nch = N / DU_NC;
  const bool dgrad = a.dX != nullptr;
  DU_STAMP(0);

  // ---- per-lane constants: weight-gradient B operand (Xw[m][f], m = 4s + q), chunks 0, 1
  DUChunk ca, cb;
  du_load(a, 0, f0, nf, tid, ca);
  if (nch > 1) du_load(a, 1, f0, nf, tid, cb);
  float xb[DU_MAXKS];
#pragma unroll
  for (int s = 0; s < DU_MAXKS; ++s) {
    const int m = 4 * s + q;
    const bool ok = m < M && i16 < nf;
    xb[s] = a.Xw[ok ? (long)m * K + f0 + i16 : 0];
  }
  // dgrad epilogue operand (forward input of the transform), prefetched: thread -> feature
  // tid & 15, batch rows 16u + tid/16
  float xv[4];
  {
    const bool tf0 = dgrad && (a.act != ACT_NONE || a.bn_on) && a.x_fwd;
    const float* xsrc = tf0 ? a.x_fwd : a.dY;              // address select, plain loads
    const int jj = tid & 15;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + DU_THREADS * u;
      const int m = 16 * (e >> 8) + ((e & 255) >> 4);
      const bool ok = tf0 && m < M && jj < nf;
      xv[u] = xsrc[ok ? (long)m * K + f0 + jj : 0];
    }
  }
  const int nslot = opt_nslots(a.opt);
  // this lane's optimizer slots of chunk c: row f0 + i16, columns c*64 + 16*wave + 4q .. +3
  const float* b0 = nslot >= 1 ? a.s0w : a.W;        // address select: loads stay unconditional
  const float* b1 = nslot >= 2 ? a.s1w : a.W;
  // update layout: wave w owns W rows 4w .. 4w+3 of the block, lane -> row 4w + (lane >> 4),
  // columns 4 * (lane & 15) .. +3 of the chunk: each store instruction covers 4 rows x 256
  // contiguous bytes (the MFMA layout would scatter 16 rows x 64 B)
  const int ur = 4 * wave + (lane >> 4), uc = 4 * (lane & 15);
  const long lrow = (long)(f0 + min(ur, nf - 1)) * N + uc;
  float4 p0a = *reinterpret_cast<const float4*>(b0 + lrow);
  float4 p1a = *reinterpret_cast<const float4*>(b1 + lrow);
  const long c1off = nch > 1 ? DU_NC : 0;
  float4 p0b = *reinterpret_cast<const float4*>(b0 + lrow + c1off);
  float4 p1b = *reinterpret_cast<const float4*>(b1 + lrow + c1off);
#pragma unroll
  for (int s = 0; s < DU_MAXKS; ++s) pin(xb[s]);
#pragma unroll
  for (int s = 0; s < DU_MAXKS; ++s) {
    const int m = 4 * s + q;
    xb[s] = (m < M && i16 < nf) ? xb[s] : 0.f;
  }
  // batch rows M..63 of both stages are zero for the whole launch: the MFMA loops below
  // run all 16 k-steps / 4 row tiles without masks
  for (int e = M * DU_SC + tid; e < DU_MAXM * DU_SC; e += DU_THREADS) {
    smem[e] = 0.f;
    smem[stf + e] = 0.f;
  }
  if (dgrad && a.bn_on) bn_reduce_to_lds(a.bn, s_bn, s_bn + MAXC_DU, s_bn + 2 * MAXC_DU, s_bn + 3 * MAXC_DU, s_st);
  du_pin(ca);
  du_store(ca, s_st0, M, nf, tid);
  float* s_dw = s_st0 + DU_NSTAGE * stf;           // [2][16 f][64 n] weight-gradient exchange
  __syncthreads();
  DU_STAMP(1);

  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  du_f32x4 dacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dacc[t] = du_f32x4{0.f, 0.f, 0.f, 0.f};

  for (int c = 0; c < nch; ++c) {
    const float* sdy = s_st0 + (c % DU_NSTAGE) * stf;
    const float* sw = sdy + DU_MAXM * DU_SC;
    float* dwb = s_dw + (c & 1) * DU_DWF;
    // chunk c + 1 (loaded one iteration ago) goes to the other stage FIRST: its wait then
    // covers only old loads — waiting after this iteration's loads were issued would wait
    // for those too (vmcnt is in order), one full round trip per chunk
    float4 ua0 = p0a, ua1 = p1a;
    pin(ua0);
    pin(ua1);
    if (c + 1 < nch) {
      du_pin(cb);
      du_store(cb, s_st0 + ((c + 1) % DU_NSTAGE) * stf, M, nf, tid);
    }
    // chunk c + 2's loads fly under this chunk's MFMAs
    DUChunk cc;
    float4 p0c = p0b, p1c = p1b;
    const bool ahead = c + 2 < nch;
    if (ahead && !(a.dbg & 8)) {
      du_load(a, c + 2, f0, nf, tid, cc);
      p0c = *reinterpret_cast<const float4*>(b0 + lrow + (c + 2) * DU_NC);
      p1c = *reinterpret_cast<const float4*>(b1 + lrow + (c + 2) * DU_NC);
    }
    // -- weight gradient of this wave's 16 columns: rows = n, cols = f, K = batch (64)
    du_f32x4 wacc0 = du_f32x4{0.f, 0.f, 0.f, 0.f}, wacc1 = wacc0;
    if (!(a.dbg & 1)) {
      const float* col = sdy + 16 * wave + i16 + q * DU_SC;
      float av[DU_MAXKS];
#pragma unroll
      for (int s = 0; s < DU_MAXKS; ++s) av[s] = col[4 * s * DU_SC];
#pragma unroll
      for (int s = 0; s < DU_MAXKS; s += 2) {     // two accumulators: no dependent MFMA chain
        wacc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], xb[s], wacc0, 0, 0, 0);
        wacc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s + 1], xb[s + 1], wacc1, 0, 0, 0);
      }
    }
    // D: lane (i16 = f, q) holds n = 16 * wave + 4q + r -> the exchange tile [f][n]
#pragma unroll
    for (int r = 0; r < 4; ++r) dwb[i16 * DU_NC + 16 * wave + 4 * q + r] = wacc0[r] + wacc1[r];
    // -- input gradient partial: K = this wave's 16 columns of the chunk, 4 batch tiles
    if (dgrad && !(a.dbg & 2)) {
      const float* wrow = sw + i16 * DU_SC + 16 * wave + q;
      const float* drow = sdy + i16 * DU_SC + 16 * wave + q;
      float bv[4], av[4][4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        bv[k] = wrow[4 * k];
#pragma unroll
        for (int t = 0; t < 4; ++t) av[k][t] = drow[16 * t * DU_SC + 4 * k];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int t = 0; t < 4; ++t) dacc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[k][t], bv[k], dacc[t], 0, 0, 0);
    }
    __syncthreads();      // chunk c + 1's stage and this chunk's weight gradient are visible
    // -- optimizer update of this lane's 4 weights (old W from the stage, dW exchanged)
    if (!(a.dbg & 4)) {
      const float* wl = sw + ur * DU_SC + uc;
      const float2 w01 = *reinterpret_cast<const float2*>(wl);
      const float2 w23 = *reinterpret_cast<const float2*>(wl + 2);
      const float4 g4 = *reinterpret_cast<const float4*>(dwb + ur * DU_NC + uc);
      float w[4] = {w01.x, w01.y, w23.x, w23.y};
      const float gg[4] = {g4.x, g4.y, g4.z, g4.w};
      float s0[4] = {ua0.x, ua0.y, ua0.z, ua0.w};
      float s1[4] = {ua1.x, ua1.y, ua1.z, ua1.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) opt_update(a.opt, lr, w[r], gg[r] * a.scale, s0[r], s1[r]);
      if (ur < nf) {
        const long gi = lrow + c * DU_NC;
        *reinterpret_cast<float4*>(a.W + gi) = make_float4(w[0], w[1], w[2], w[3]);
        if (nslot >= 1) *reinterpret_cast<float4*>(a.s0w + gi) = make_float4(s0[0], s0[1], s0[2], s0[3]);
        if (nslot >= 2) *reinterpret_cast<float4*>(a.s1w + gi) = make_float4(s1[0], s1[1], s1[2], s1[3]);
      }
    }
    cb = cc;
    p0a = p0b; p1a = p1b;
    p0b = p0c; p1b = p1c;
  }
  DU_STAMP(2);

  // ---- input gradient: fold the 4 waves' K slices, then the transform's backward
  if (dgrad) {
    __syncthreads();                       // last chunk's update reads done: stages are free
    float* s_part = smem;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_part[(wave * 4 + t) * 256 + (4 * q + r) * 16 + i16] = dacc[t][r];
    for (int c = tid; c < 2 * MAXC_DU && a.bn_on; c += DU_THREADS) s_st[c] = 0.f;
    // epilogue: thread -> feature j = tid & 15 (fixed), 4 batch rows
    const int j = tid & 15;
    const int f = f0 + j;
    const int C = a.bn.C > 0 ? a.bn.C : 1;
    const int ch = f % C;
    const bool tf = a.act != ACT_NONE || a.bn_on;
    __syncthreads();
    float sd = 0.f, sdx = 0.f;
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
      // fold into one of DU_SLAB rows (atomics; zeroed every step by the optimizer launch),
      // so the consumer reduces 16 rows instead of one per workgroup
      float* row = a.bwd_slab + (size_t)(blockIdx.x % DU_SLAB) * 2 * C;
      for (int c = tid; c < 2 * C; c += DU_THREADS) atomicAdd(&row[c], c < C ? s_st[c] : s_st[MAXC_DU + c - C]);
    }
  }
  DU_STAMP(3);
}

}  // namespace csa

using namespace csa;

CSA_API int csa_du_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_du_dbg), &p, sizeof(p));
}


// Shape family of the fused kernel (0 = outside: the caller uses the separate backward
// kernels + the flat optimizer).  Needs M <= 64, N % 64 == 0.
CSA_API int csa_dense_bwd_update_ok(int M, int K, int N, int bn_C) {
  if (M < 1 || M > DU_MAXM || K < 1 || N < DU_NC || N % DU_NC) return 0;
  if (bn_C > MAXC_DU) return 0;
  return du_lds_floats(M) * sizeof(float) <= DU_LDS_MAX ? 1 : 0;
}

// BN-backward slab rows the kernel accumulates into (atomically; the caller zeroes them).
CSA_API int csa_dense_bwd_update_slabs(int K) { return (K + DU_FT - 1) / DU_FT < DU_SLAB ? (K + DU_FT - 1) / DU_FT : DU_SLAB; }

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
  a.nmain = (K + DU_FT - 1) / DU_FT;
  static const int dbg = [] { const char* e = getenv("CSA_DU_DBG"); return e ? atoi(e) : 0; }();
  a.dbg = dbg;
  const size_t shm = du_lds_floats(M) * sizeof(float);
  static const bool attr = hipFuncSetAttribute((const void*)dense_bwd_update_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  hipLaunchKernelGGL(dense_bwd_update_kernel, dim3((unsigned)(a.nmain + (bias ? 1 : 0))), dim3(DU_THREADS), shm,
                     st, a);
  return (int)hipGetLastError();
}
