// A first-layer conv PAIR fused forward and backward (gfx950 / CDNA4).
//
// Reference: the DSL's leading `conv, [active], conv, [active], [pool]` layers
// (construct_distribute.py:91-130, 222-240) — in the sample config (API.md:306-332)
// conv[2,2,10] -> conv[2,2,20] -> pool, on 28x28x1 digits.  The per-layer path runs
// conv1, conv2(+pool) forward and route, conv2 dgrad/wgrad, conv1 wgrad backward as five
// launches that pass 1.6-3.1 MB intermediates (c1, dc2, dc1) through HBM.  Here:
//
//   forward  ONE launch: per (image, band of pooled rows) the band's input rows are
//            gathered (uint8, /255) into LDS, conv A is evaluated into an LDS tile
//            (with conv B's zero padding materialised), conv B + act + 2x2 max-pool run
//            on it, the pooled output, argmax and the following BatchNorm's partial
//            statistics are written.  c1 never leaves the CU.
//   backward ONE launch: per band, BatchNorm backward + act backward + pool routing of
//            the band's (and one halo row's) output gradient into an LDS dc2 tile, c1
//            recomputed from the input rows (40 MACs per value: cheaper than storing
//            it), conv B's weight gradient, conv B's input gradient dc1 (through act A),
//            conv A's weight gradient — all from LDS; the weight gradients leave the
//            launch as one atomic add per (workgroup, weight) into S stripes that the
//            optimizer folds.  No dc2 / dc1 / c1 tensor is ever written.
//
// Family: stride-1 convs, kernels <= 5x5 (SAME / VALID), C0 <= 4, C1 <= 32 (even),
// C2 <= 64 (multiple of 4), optional 2x2 stride-2 unpadded pool, H, W <= 64, first layer
// (uint8 dataset rows gathered through the batch index stream).  Everything else uses the
// per-layer kernels (conv.hip).
#include "common.h"
#include "dense_update.h"
#include <vector>
#include <cstdlib>
#include <algorithm>

namespace csa {

constexpr int CP_THREADS = 256;
constexpr int CP_MAXC2 = 64;
constexpr int CP_MAXC1 = 32;
constexpr size_t CP_LDS_MAX = 150 * 1024;

__constant__ long long* g_cp_dbg = nullptr;   // diagnostics: s_memtime stamps of one block
__constant__ int g_cp_dbg_blk = 0;            //   (block 0 unless csa_cp_debug_block chose another)
#define CP_STAMP(i)                                                                           \
  do {                                                                                        \
    if (g_cp_dbg && threadIdx.x == 0 && (int)blockIdx.x == g_cp_dbg_blk) g_cp_dbg[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

struct CPGeom {
  int B, H, W, C0;                 // input
  int KAh, KAw, PTA, PLA, C1;      // conv A (stride 1)
  int H1, W1;                      // conv A output
  int KBh, KBw, PTB, PLB, C2;      // conv B (stride 1)
  int H2, W2;                      // conv B output
  int pool;                        // 2x2 / stride 2 max-pool after conv B (+ act B)
  int PH, PW;                      // unit output (pooled) size
  int PR, nbands;                  // pooled rows per band
};

struct CPFwdArgs {
  CPGeom g;
  const uint8_t* img; const int64_t* idx; const int64_t* cursor;
  const float* wA; const float* bA; int actA; float alphaA;
  const float* wB; const float* bB; int actB; float alphaB;
  float* y; uint8_t* argmax; float* stat; int nslab;
};

// Accumulators of LATER launches of the step zeroed by the pair forward's threads (the
// split-K outputs of the dense forwards, read until the end of the previous step's pair
// backward): one float4 per thread, no launch of their own (round 5: the fused program's
// flat optimizer launch is gone, csa_conv_pair_tail_set).
constexpr int CP_MAXZ = 4;
struct CPZero { float4* p[CP_MAXZ]; long n4[CP_MAXZ]; int n; };

__device__ __forceinline__ void cp_zero_early(const CPZero& z, int nblk) {
  const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long)nblk * blockDim.x;
  for (int k = 0; k < z.n; ++k)
    for (long i = gid; i < z.n4[k]; i += nth) z.p[k][i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Deferred dense-parameter update (round 5, data-parallel programs).  Under data
// parallelism the dense weight gradients exist whole in the flat gradient and are exchanged
// after the backward, so the flat optimizer launch that follows the exchange was a serial
// 11.5 us stream over every parameter (profiles/r5_dp_trace.md).  The dense layers'
// parameters are only read again by the NEXT step's dense forwards, which come after this
// launch: their update rides as extra workgroups of the next step's pair forward (1 % of
// HBM busy), gated by a device flag that the (now small) optimizer launch raises once the
// exchanged gradient is in place.  A host flush (csa_opt_carry_flush) applies a pending
// update at every point that reads the parameters between steps.
constexpr int CP_MAXCS = 4;
struct CPOptCarry {
  int blocks;                          // extra workgroups (0: no carry)
  int opt; float lr; const int64_t* step;
  float* w; const float* g; float* s0; float* s1;
  unsigned* pending;                   // 1: the exchanged gradient awaits its update (cleared
                                       // by the launch after the carrying forward: bn_act_apply)
  int count; long lo4[CP_MAXCS]; long start4[CP_MAXCS + 1];   // flat spans, float4 units
};

// Workgroup k of nblk: a grid-stride streaming update, one float4 of each operand per
// thread and iteration (the carrying forward keeps its occupancy; ~1 000 workgroups keep
// 12 MB in flight).  Segment lookup by unrolled selects (no per-lane index into the
// argument struct).
__device__ __forceinline__ void cp_opt_carry_apply(const CPOptCarry& c, int k, int nblk);

// The flag is cleared right after the carrying forward by the NEXT launch of the step
// (bn_act_apply's block 0: csa_ew_clear_next), so a host flush anywhere after the carry never
// applies the update twice.  (A retire ticket taken by every carrying workgroup
// did the same inside this launch, but ~1 000 same-address atomics made the data-parallel
// step 0.0852 -> 0.1005 ms — measured round 6, profiles/r6_notes.md.)
__device__ __forceinline__ void cp_opt_carry(const CPOptCarry& c, int k, int nblk) {
  __shared__ unsigned s_pend;
  if (threadIdx.x == 0) s_pend = __hip_atomic_load(c.pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (s_pend) cp_opt_carry_apply(c, k, nblk);
}

__device__ __forceinline__ void cp_opt_carry_apply(const CPOptCarry& c, int k, int nblk) {
  const int nslot = opt_nslots(c.opt);
  const float lr = opt_step_lr(c.opt, c.lr, c.step);
  const long m4 = c.start4[c.count];
  const long nth = (long)nblk * blockDim.x;
  float4* w4 = reinterpret_cast<float4*>(c.w);
  const float4* g4 = reinterpret_cast<const float4*>(c.g);
  float4* s04 = reinterpret_cast<float4*>(c.s0);
  float4* s14 = reinterpret_cast<float4*>(c.s1);
  for (long t = (long)k * blockDim.x + threadIdx.x; t < m4; t += nth) {
    long lo = c.lo4[0], st = 0;
#pragma unroll
    for (int q = 1; q < CP_MAXCS; ++q)
      if (q < c.count && t >= c.start4[q]) { lo = c.lo4[q]; st = c.start4[q]; }
    const long i = lo + (t - st);
    float4 w = w4[i];
    const float4 g = g4[i];
    float4 z0 = nslot >= 1 ? s04[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 z1 = nslot >= 2 ? s14[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    opt_update(c.opt, lr, w.x, g.x, z0.x, z1.x);
    opt_update(c.opt, lr, w.y, g.y, z0.y, z1.y);
    opt_update(c.opt, lr, w.z, g.z, z0.z, z1.z);
    opt_update(c.opt, lr, w.w, g.w, z0.w, z1.w);
    w4[i] = w;
    if (nslot >= 1) s04[i] = z0;
    if (nslot >= 2) s14[i] = z1;
  }
}

__global__ __launch_bounds__(256) void cp_opt_carry_kernel(CPOptCarry c) {
  cp_opt_carry(c, (int)blockIdx.x, (int)gridDim.x);
}

// Band tile extents (rows in conv-B-output coordinates and the derived c1 / x rows).
struct CPBand {
  int r2a, r2b;     // conv B output rows computed
  int c1y0, T1H;    // c1 tile: rows c1y0 .. c1y0 + T1H (may extend outside [0, H1): zeros)
  int T1W;          // c1 tile columns: c1 x = tx - PLB
  int TXH, TXW;     // x tile: rows c1y0 - PTA + ty, cols tx - PLB - PLA
};

__host__ __device__ inline CPBand cp_band(const CPGeom& g, int r2a, int r2b) {
  CPBand t;
  t.r2a = r2a; t.r2b = r2b;
  t.c1y0 = r2a - g.PTB;
  t.T1H = (r2b - r2a) + g.KBh - 1;
  t.T1W = g.W2 + g.KBw - 1;
  t.TXH = t.T1H + g.KAh - 1;
  t.TXW = t.T1W + g.KAw - 1;
  return t;
}

__device__ __forceinline__ const uint8_t* cp_image(const uint8_t* img, const int64_t* idx, const int64_t* cursor,
                                                   int b, int B, long imsz) {
  if (!idx) return img + (long)b * imsz;        // staged batch: image b at a fixed address
  const int64_t* id = cursor ? idx + cursor[0] * B : idx;
  return img + id[b] * imsz;
}

// x tile (uint8 -> /255, zero outside the image) into LDS [TXH][TXW][C0].
__device__ __forceinline__ void cp_stage_x(const CPGeom& g, const CPBand& t, const uint8_t* src, float* s_x) {
  const int n = t.TXH * t.TXW * g.C0;
  const int y0 = t.c1y0 - g.PTA, x0 = -g.PLB - g.PLA;
  const FastDiv dw(t.TXW * g.C0), dc(g.C0);
  constexpr int U = 4;
  for (int base = 0; base < n; base += CP_THREADS * U) {
    int ok[U];
    uint8_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + threadIdx.x;
      int r, rem, xx, c;
      dw.divmod(e < n ? e : 0, r, rem);
      dc.divmod(rem, xx, c);
      const int y = y0 + r, x = x0 + xx;
      ok[u] = e < n && y >= 0 && y < g.H && x >= 0 && x < g.W;
      v[u] = src[ok[u] ? ((long)y * g.W + x) * g.C0 + c : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + threadIdx.x;
      if (e < n) s_x[e] = ok[u] ? (float)v[u] * (1.0f / 255.0f) : 0.f;
    }
  }
}

// Weights as a zero-padded [kpad][npad] LDS panel (the MFMA B operand), k = flattened
// (i, j, cin) of the HWIO tensor.
// Batches of 8 loads per thread from clamped addresses, pinned, then the stores: a load
// inside the conditional that consumes it is sunk into it by hipcc and waited for there —
// one serial memory round trip per loop iteration.
__device__ __forceinline__ void cp_stage_panel(float* dst, const float* w, int K, int N, int kpad, int npad) {
  const FastDiv dn(npad);
  const int total = kpad * npad;
  constexpr int U = 8;
  for (int base = 0; base < total; base += CP_THREADS * U) {
    float v[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + (int)threadIdx.x;
      int k, n;
      dn.divmod(e < total ? e : 0, k, n);
      ok[u] = e < total && k < K && n < N;
      v[u] = w[ok[u] ? k * N + n : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) pin(v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + (int)threadIdx.x;
      if (e < total) dst[e] = ok[u] ? v[u] : 0.f;
    }
  }
}

// Forward-kernel inputs in ONE batch of loads: panel A, panel B (the weights) and the x
// tile.  The weight loads are issued first and stay in flight across the cursor -> row
// index -> image chain (scalar loads), so the three round trips of separate staging
// loops collapse into that chain alone.  Falls back to the loops when a thread would
// hold more than the register batch.
__device__ __forceinline__ void cp_stage_fwd_inputs(const CPGeom& g, const CPBand& t, const uint8_t* img,
                                                    const int64_t* idx, const int64_t* cursor, int b,
                                                    float* s_pA, const float* wA, int KA, int kpadA,
                                                    float* s_pB, const float* wB, int KB, int kpadB, int pst,
                                                    float* s_x);

// dst[i] = i < n ? src[i] : 0 for i < total, same batching.
__device__ __forceinline__ void cp_stage_flat(float* dst, const float* src, int n, int total) {
  constexpr int U = 8;
  for (int base = 0; base < total; base += CP_THREADS * U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + (int)threadIdx.x;
      v[u] = src[e < n ? e : 0];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) pin(v[u]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = base + u * CP_THREADS + (int)threadIdx.x;
      if (e < total) dst[e] = e < n ? v[u] : 0.f;
    }
  }
}

__device__ __forceinline__ void cp_stage_fwd_inputs(const CPGeom& g, const CPBand& t, const uint8_t* img,
                                                    const int64_t* idx, const int64_t* cursor, int b,
                                                    float* s_pA, const float* wA, int KA, int kpadA,
                                                    float* s_pB, const float* wB, int KB, int kpadB, int pst,
                                                    float* s_x) {
  constexpr int UP = 8, UX = 2;
  const int nA = kpadA * 16, nB = kpadB * pst, nP = nA + nB;
  const int nX = t.TXH * t.TXW * g.C0;
  if (nP > UP * CP_THREADS || nX > UX * CP_THREADS) {
    cp_stage_x(g, t, cp_image(img, idx, cursor, b, g.B, (long)g.H * g.W * g.C0), s_x);
    cp_stage_panel(s_pA, wA, KA, g.C1, kpadA, 16);
    cp_stage_panel(s_pB, wB, KB, g.C2, kpadB, pst);
    return;
  }
  const FastDiv d16(16), dpst(pst);
  float pv[UP];
  bool pok[UP];
#pragma unroll
  for (int u = 0; u < UP; ++u) {                 // weights: concatenated [panel A | panel B]
    const int e = u * CP_THREADS + (int)threadIdx.x;
    const bool inA = e < nA;
    int k, n;
    if (inA) d16.divmod(e, k, n); else dpst.divmod(e < nP ? e - nA : 0, k, n);
    const bool ok = e < nP && (inA ? (k < KA && n < g.C1) : (k < KB && n < g.C2));
    pok[u] = ok;
    pv[u] = ok ? (inA ? wA[k * g.C1 + n] : wB[k * g.C2 + n]) : 0.f;
  }
  // x tile: the row index chain (scalar loads) runs while the weights are in flight
  const uint8_t* src = cp_image(img, idx, cursor, b, g.B, (long)g.H * g.W * g.C0);
  const int y0 = t.c1y0 - g.PTA, x0 = -g.PLB - g.PLA;
  const FastDiv dw(t.TXW * g.C0), dc(g.C0);
  uint8_t xv[UX];
  bool xok[UX];
#pragma unroll
  for (int u = 0; u < UX; ++u) {
    const int e = u * CP_THREADS + (int)threadIdx.x;
    int r, rem, xx, c;
    dw.divmod(e < nX ? e : 0, r, rem);
    dc.divmod(rem, xx, c);
    const int y = y0 + r, x = x0 + xx;
    xok[u] = e < nX && y >= 0 && y < g.H && x >= 0 && x < g.W;
    xv[u] = src[xok[u] ? ((long)y * g.W + x) * g.C0 + c : 0];
  }
#pragma unroll
  for (int u = 0; u < UP; ++u) pin(pv[u]);
#pragma unroll
  for (int u = 0; u < UP; ++u) {
    const int e = u * CP_THREADS + (int)threadIdx.x;
    if (e < nA) s_pA[e] = pok[u] ? pv[u] : 0.f;
    else if (e < nP) s_pB[e - nA] = pok[u] ? pv[u] : 0.f;
  }
#pragma unroll
  for (int u = 0; u < UX; ++u) {
    const int e = u * CP_THREADS + (int)threadIdx.x;
    if (e < nX) s_x[e] = xok[u] ? (float)xv[u] * (1.0f / 255.0f) : 0.f;
  }
}

// ---------------------------------------------------------------------------------------
// In-LDS GEMM on v_mfma_f32_16x16x4_f32: D[m][n] = sum_k A(m, k) B(k, n) where both operands
// are LDS gathers  A(m, k) = s[abase(m) + aoff[k]],  B(k, n) = s[bbase(n) + boff[k]]
// (aoff / boff: per-k offset tables in LDS).  (m-tile, n-tile) pairs are dealt to the 4
// waves; two accumulators per pair break the dependent-MFMA chain.  epi(tm, tn, acc) gets
// the lane's D fragment: rows tm*16 + 4q + r, column tn*16 + (lane & 15).
// Padding rows / columns read any valid address and are dropped by the epilogue; padded
// k must make one operand zero (a zero panel row or an offset onto a zero cell).
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15], D[4*(l>>4)+r][l&15].
typedef float cp_f32x4 __attribute__((ext_vector_type(4)));

template <class FA, class FB, class FE>
__device__ __forceinline__ void cp_gemm(const float* s, int mt, int nt, int ksteps, const int* aoff, const int* boff,
                                        FA abase, FB bbase, FE epi) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, q = lane >> 4;
  for (int pr = wave; pr < mt * nt; pr += CP_THREADS / 64) {
    const int tm = pr / nt, tn = pr - tm * nt;
    const float* pa = s + abase(tm * 16 + i16);
    const float* pb = s + bbase(tn * 16 + i16);
    cp_f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
    int ks = 0;
    for (; ks + 4 <= ksteps; ks += 4) {
      float av[4], bv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = 4 * (ks + u) + q;
        av[u] = pa[aoff[k]];
        bv[u] = pb[boff[k]];
      }
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[0], bv[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[1], bv[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[2], bv[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[3], bv[3], acc1, 0, 0, 0);
    }
    for (; ks < ksteps; ++ks) {
      const int k = 4 * ks + q;
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[aoff[k]], pb[boff[k]], acc0, 0, 0, 0);
    }
    epi(tm, tn, acc0 + acc1, 0);
  }
}

// c1 tile (post act A; zero outside [0, H1) x [0, W1)) into LDS [T1H][T1W][C1]:
// a [tile pixels] x [C1] GEMM with K = taps of conv A (x tile gather x weight panel).
__device__ __forceinline__ void cp_conv_a(const CPGeom& g, const CPBand& t, float* s, const float* s_x,
                                          const float* s_pA, int kpadA, const int* offA, const int* offPA,
                                          const float* bA, int actA, float alphaA, float* s_c1) {
  const int npix = t.T1H * t.T1W;
  const FastDiv dw(t.T1W);
  cp_gemm(s, (npix + 15) >> 4, 1, kpadA >> 2, offA, offPA,
          [&](int m) {
            int ty, tx;
            dw.divmod(m < npix ? m : 0, ty, tx);
            return (int)(s_x - s) + (ty * t.TXW + tx) * g.C0;
          },
          [&](int n) { return (int)(s_pA - s) + n; },
          [&](int tm, int, cp_f32x4 acc, int) {
            const int lane = threadIdx.x & 63, c = lane & 15, q = lane >> 4;
            if (c >= g.C1) return;
            const float bias = bA ? bA[c] : 0.f;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int m = tm * 16 + 4 * q + r;
              if (m >= npix) continue;
              int ty, tx;
              dw.divmod(m, ty, tx);
              const int y = t.c1y0 + ty, x = tx - g.PLB;
              const bool in = y >= 0 && y < g.H1 && x >= 0 && x < g.W1;
              s_c1[m * g.C1 + c] = in ? act_fwd(acc[r] + bias, actA, alphaA) : 0.f;
            }
          });
}

// per-k offset tables of conv A: x tile offset of tap k = (i, j, c0) and its panel row
__device__ __forceinline__ void cp_tables_a(const CPGeom& g, const CPBand& t, int kpadA, int* offA, int* offPA) {
  const int KA = g.KAh * g.KAw * g.C0;
  for (int k = threadIdx.x; k < kpadA; k += CP_THREADS) {
    int o = 0;
    if (k < KA) {
      const int c0 = k % g.C0, ij = k / g.C0, i = ij / g.KAw, j = ij - i * g.KAw;
      o = (i * t.TXW + j) * g.C0 + c0;
    }
    offA[k] = o;
    offPA[k] = k * 16;
  }
}

__global__ __launch_bounds__(CP_THREADS) void conv_pair_fwd_kernel(CPFwdArgs a, CPZero z) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cp_zero_early(z, (int)gridDim.x);
  __shared__ float s_stat[2 * CP_MAXC2];
  __shared__ int s_offA[32], s_offPA[32];
  const CPGeom& g = a.g;
  const int b = blockIdx.x / g.nbands, band = blockIdx.x % g.nbands;
  const int pr0 = band * g.PR, pr1 = min(g.PH, pr0 + g.PR);
  const int r2a = g.pool ? 2 * pr0 : pr0, r2b = g.pool ? min(g.H2, 2 * pr1) : pr1;
  const CPBand t = cp_band(g, r2a, r2b);
  const int KA = g.KAh * g.KAw * g.C0, kpadA = (KA + 3) & ~3;
  const int KB = g.KBh * g.KBw * g.C1, kpadB = (KB + 3) & ~3, c16 = (g.C2 + 15) & ~15;
  const int pst = (c16 & 31) ? c16 : c16 + 16;          // panel row stride == 16 (mod 32)
  float* s_pA = smem;                                   // [kpadA][16]
  float* s_pB = s_pA + kpadA * 16;                      // [kpadB][pst]
  int* s_offB = reinterpret_cast<int*>(s_pB + kpadB * pst);   // [kpadB] c1 tile offset of tap k
  int* s_offPB = s_offB + kpadB;                               // [kpadB] panel row k * pst
  float* s_x = reinterpret_cast<float*>(s_offPB + kpadB);
  float* s_c1 = s_x + ((t.TXH * t.TXW * g.C0 + 3) & ~3);
  CP_STAMP(0);
  cp_stage_fwd_inputs(g, t, a.img, a.idx, a.cursor, b, s_pA, a.wA, KA, kpadA, s_pB, a.wB, KB, kpadB, pst, s_x);
  CP_STAMP(5);
  CP_STAMP(6);
  cp_tables_a(g, t, kpadA, s_offA, s_offPA);
  for (int k = threadIdx.x; k < kpadB; k += CP_THREADS) {     // c1 tile offset of tap (i, j, c1)
    int o = 0;
    if (k < KB) {
      const int c1 = k % g.C1, ij = k / g.C1, i = ij / g.KBw, j = ij - i * g.KBw;
      o = (i * t.T1W + j) * g.C1 + c1;
    }
    s_offB[k] = o;
    s_offPB[k] = k * pst;
  }
  for (int i = threadIdx.x; i < 2 * g.C2; i += CP_THREADS) s_stat[i] = 0.f;
  __syncthreads();
  CP_STAMP(1);
  cp_conv_a(g, t, smem, s_x, s_pA, kpadA, s_offA, s_offPA, a.bA, a.actA, a.alphaA, s_c1);
  __syncthreads();
  CP_STAMP(2);

  // conv B (+ act, + 2x2 max-pool): rows = (unit pixel, window position) when pooled —
  // a lane's 4 D rows are one pooled pixel's 4 positions, so the pool is in registers
  const int ow = g.pool ? g.PW : g.W2;
  const int nunit = (g.pool ? (pr1 - pr0) : (r2b - r2a)) * ow;
  const int nrows = g.pool ? 4 * nunit : nunit;
  const FastDiv dow(ow);
  cp_gemm(smem, (nrows + 15) >> 4, c16 >> 4, kpadB >> 2, s_offB, s_offPB,
          [&](int m) {                                           // c1 tile offset of row m
            const int mc = m < nrows ? m : 0;
            int y2, x2;
            if (g.pool) {
              int py, px;
              dow.divmod(mc >> 2, py, px);
              y2 = 2 * (pr0 + py) + ((mc & 3) >> 1);
              x2 = 2 * px + (mc & 1);
              if (y2 >= g.H2 || x2 >= g.W2) { y2 = r2a; x2 = 0; }  // outside: dropped below
            } else {
              int py, px;
              dow.divmod(mc, py, px);
              y2 = r2a + py;
              x2 = px;
            }
            return (int)(s_c1 - smem) + ((y2 - r2a) * t.T1W + x2) * g.C1;
          },
          [&](int n) { return (int)(s_pB - smem) + n; },
          [&](int tm, int tn, cp_f32x4 acc, int) {
            const int lane = threadIdx.x & 63, i16 = lane & 15, q = lane >> 4;
            const int c = tn * 16 + i16;
            const float bias = (a.bB && c < g.C2) ? a.bB[c] : 0.f;
            float best = -INFINITY;
            int am = 0;
            float s1 = 0.f, s2 = 0.f;
            if (g.pool) {
              const int u = tm * 4 + q;                          // unit pixel of this lane
              if (u < nunit && c < g.C2) {
                int py, px;
                dow.divmod(u, py, px);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                  const int y2 = 2 * (pr0 + py) + (r >> 1), x2 = 2 * px + (r & 1);
                  if (y2 >= g.H2 || x2 >= g.W2) continue;
                  const float v = act_fwd(acc[r] + bias, a.actB, a.alphaB);
                  if (v > best) { best = v; am = r; }
                }
                const long o = (((long)b * g.PH + pr0 + py) * g.PW + px) * g.C2 + c;
                a.y[o] = best;
                if (a.argmax) a.argmax[o] = (uint8_t)am;
                s1 = best;
                s2 = best * best;
              }
            } else {
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int u = tm * 16 + 4 * q + r;
                if (u >= nunit || c >= g.C2) continue;
                int py, px;
                dow.divmod(u, py, px);
                const float v = act_fwd(acc[r] + bias, a.actB, a.alphaB);
                a.y[(((long)b * g.H2 + r2a + py) * g.W2 + px) * g.C2 + c] = v;
                s1 += v;
                s2 += v * v;
              }
            }
            if (a.stat) {                                        // fold the 4 lane quads
              s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
              s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
              if (q == 0 && c < g.C2) { atomicAdd(&s_stat[c], s1); atomicAdd(&s_stat[g.C2 + c], s2); }
            }
          });
  CP_STAMP(3);
  if (a.stat) {
    __syncthreads();
    float* row = a.stat + (size_t)(blockIdx.x % a.nslab) * 2 * g.C2;
    for (int i = threadIdx.x; i < 2 * g.C2; i += CP_THREADS) atomicAdd(&row[i], s_stat[i]);
  }
  CP_STAMP(4);
}

// --------------------------------------------------------------------------------------
// Backward.
struct CPBwdArgs {
  CPGeom g;
  const uint8_t* img; const int64_t* idx; const int64_t* cursor;
  const float* wA; const float* bA; int actA; float alphaA;
  const float* wB; int actB; float alphaB; int hasBiasB;
  const float* dz;                  // grad wrt the BN output (or the unit output)
  const float* y;                   // unit output (post act, post pool) = BN input
  const uint8_t* argmax;
  BNRef bn; int bn_on; const float* bwd_slab; int bwd_nslab;
  float* dscale; float* doffset; float* run_mean; float* run_var; float momentum;
  float* dwA; float* dbA; float* dwB; float* dbB; int stripes;
  const int* tabs; int tab_stride;  // per-band index tables (csa_conv_pair_bwd_tables) or null
  unsigned* img_tk;                 // tail: +1 per workgroup once its image tile is in LDS (or null)
  const float* bn_tab;              // [mean | rstd | a | b][C2] the step's bn_act_apply wrote, or null
};

// LDS carve of the backward (float offsets), shared by the kernel and the host size check.
struct CPBwdLayout {
  int o2a, o2b, o1a, o1b;           // owned conv-B-output rows / owned c1 rows
  int d2y0, D2H, D2W;               // zero-padded dc2 tile: rows d2y0 .., cols PLB-KBw+1 ..
  int KA, kpadA, KB, kpadB, KD, kpadD, c16, n16a, n16b;
  int npix2, kp2, npix1, kp1;       // owned pixels (conv B out / c1), padded to 4
  int wA, pA, pB, x, c1, dc2, dc1, red, offs, end;
  int rA;                           // dwA's per-wave partials: inside the dc2 tile when it is
                                    // large enough (dead by then), else after the bias sums
};

__host__ __device__ inline CPBwdLayout cp_bwd_layout(const CPGeom& g, int band, int TXH, int TXW, int T1H, int T1W) {
  CPBwdLayout L;
  const int pr0 = band * g.PR, pr1 = min(g.PH, pr0 + g.PR);
  const bool last = band == g.nbands - 1;
  L.o2a = g.pool ? 2 * pr0 : pr0;
  L.o2b = g.pool ? (last ? g.H2 : 2 * pr1) : pr1;
  L.o1a = L.o2a;
  L.o1b = last ? g.H1 : L.o2b;
  L.d2y0 = L.o1a + g.PTB - g.KBh + 1;
  L.D2H = (L.o1b - L.o1a) + g.KBh - 1 + 1;            // + one zero row (padded pixels)
  L.D2W = g.W1 + g.KBw - 1;
  L.KA = g.KAh * g.KAw * g.C0; L.kpadA = (L.KA + 3) & ~3;
  L.KB = g.KBh * g.KBw * g.C1; L.kpadB = (L.KB + 3) & ~3;
  L.KD = g.KBh * g.KBw * g.C2; L.kpadD = (L.KD + 3) & ~3;
  L.c16 = (g.C2 + 15) & ~15; L.n16a = (L.KA + 15) & ~15; L.n16b = (L.KB + 15) & ~15;
  L.npix2 = (L.o2b - L.o2a) * g.W2; L.kp2 = (L.npix2 + 3) & ~3;
  L.npix1 = (L.o1b - L.o1a) * g.W1; L.kp1 = (L.npix1 + 3) & ~3;
  int o = 0;
  L.pA = o; o += L.kpadA * 16;                        // conv A weight panel [kpadA][16]
  L.pB = o; o += L.kpadB * L.c16;                     // conv B weights (HWIO, dense) + pad
  L.x = o; o += (TXH * TXW * g.C0 + 3) & ~3;
  L.c1 = o; o += (T1H * T1W * g.C1 + 3) & ~3;
  L.dc2 = o; o += (L.D2H * L.D2W * g.C2 + 3) & ~3;
  L.dc1 = o; o += ((L.npix1 + 1) * g.C1 + 3) & ~3;    // + one zero pixel row
  // reduction region (round 6: 5 workgroups per CU in the carrying launch need <= ~31 KB):
  //   [n16b x c16] dwB tile | [C2 + C1] bias sums | ([4][16][16] dwA partials, only when the
  //   dc2 tile cannot hold them)
  // and, earlier in the workgroup's life, the BatchNorm scratch: [2 MAXC2] slab sums |
  // [4 MAXC2] tables | [2 MAXC2] backward sums (dead before the dwB tile is written)
  const int dc2n = L.D2H * L.D2W * g.C2;
  const int rmain = L.n16b * L.c16 + g.C2 + g.C1;
  const bool rA_in_dc2 = dc2n >= 4 * 16 * 16;
  const int rsz = rmain + (rA_in_dc2 ? 0 : 4 * 16 * 16);
  L.red = o; o += ((rsz > 8 * CP_MAXC2 ? rsz : 8 * CP_MAXC2) + 3) & ~3;
  L.rA = rA_in_dc2 ? L.dc2 : L.red + rmain;
  L.offs = o; o += 2 * L.kpadA + L.kp2 * 2 + L.kpadD * 2 + L.kp1 * 2 + L.n16b + 16;
  L.end = o;
  (void)L.wA;
  return L;
}

// The backward's per-band index tables (they depend on the band only): into the int region
// at s_offA (layout: see cp_bwd_body).  Computed once per geometry into global memory by
// cp_bwd_tables_kernel, or by every workgroup when no table buffer was given.
__device__ __forceinline__ void cp_bwd_tables(const CPGeom& g, const CPBand& t, const CPBwdLayout& L, int* s_offA) {
  int* s_offPA = s_offA + L.kpadA;
  int* s_pix2 = s_offPA + L.kpadA;
  int* s_pixd = s_pix2 + L.kp2;
  int* s_offD = s_pixd + L.kp2;
  int* s_offW = s_offD + L.kpadD;
  int* s_pix1x = s_offW + L.kpadD;
  int* s_pix1d = s_pix1x + L.kp1;
  int* s_tapB = s_pix1d + L.kp1;
  cp_tables_a(g, t, L.kpadA, s_offA, s_offPA);
  {
    const FastDiv dw2(g.W2), dw1(g.W1);
    const int zrow2 = ((L.D2H - 1) * L.D2W) * g.C2;           // the dc2 tile's zero row
    for (int p = threadIdx.x; p < L.kp2; p += CP_THREADS) {
      int yy, xx;
      dw2.divmod(p < L.npix2 ? p : 0, yy, xx);
      s_pix2[p] = (yy * t.T1W + xx) * g.C1;                   // y2 - o2a = yy
      s_pixd[p] = p < L.npix2 ? ((L.o2a + yy - L.d2y0) * L.D2W + xx + g.KBw - 1 - g.PLB) * g.C2 : zrow2;
    }
    for (int k = threadIdx.x; k < L.kpadD; k += CP_THREADS) {
      int od = 0, ow = 0;
      if (k < L.KD) {
        const int c2 = k % g.C2, ij = k / g.C2, i = ij / g.KBw, j = ij - i * g.KBw;
        od = -(i * L.D2W + j) * g.C2 + c2;
        ow = ij * g.C1 * g.C2 + c2;
      } else {
        ow = L.kpadB * L.c16 - 1 - (g.C1 - 1) * g.C2;   // -> zero pad of the weight area
        if (ow < 0) ow = 0;
      }
      s_offD[k] = od;
      s_offW[k] = ow;
    }
    for (int p = threadIdx.x; p < L.kp1; p += CP_THREADS) {
      int yy, xx;
      dw1.divmod(p < L.npix1 ? p : 0, yy, xx);
      s_pix1x[p] = ((L.o1a + yy - t.c1y0) * t.TXW + xx + g.PLB) * g.C0;
      s_pix1d[p] = (p < L.npix1 ? p : L.npix1) * g.C1;      // padded pixels -> the zero row
    }
    for (int k = threadIdx.x; k < L.n16b; k += CP_THREADS) {
      int o = 0;
      if (k < L.KB) {
        const int c1 = k % g.C1, ij = k / g.C1, i = ij / g.KBw, j = ij - i * g.KBw;
        o = (i * t.T1W + j) * g.C1 + c1;
      }
      s_tapB[k] = o;
    }
  }
}

// Ints of one band's table region (the int area of the LDS carve).
__host__ __device__ inline int cp_bwd_tab_ints(const CPBwdLayout& L) { return L.end - L.offs; }

// Prologue register batch of the backward (ONE = true): weights (panel A + dense wB),
// x tile and BN slab rows per thread.  The host picks ONE when every band fits.
constexpr int CPB_UP = 8, CPB_UX = 2, CPB_US = 8, CPB_UT = 4;

// The route's extent for workgroup (image b, band of L): unit rows [ua, ub) of the pair's
// output (pooled or not) whose gradients land in the band's zero-padded dc2 tile.
constexpr int CP_RU = 4;                   // route operands per thread and chunk
struct CPRoute { int n2a, n2b, ua, n; long base; };
__device__ __forceinline__ CPRoute cp_route(const CPGeom& g, const CPBwdLayout& L, int b) {
  CPRoute r;
  r.n2a = max(0, L.d2y0);
  r.n2b = min(g.H2, L.d2y0 + L.D2H - 1);
  const int ow = g.pool ? g.PW : g.W2;
  r.ua = g.pool ? r.n2a / 2 : r.n2a;
  const int ub = g.pool ? min(g.PH, (r.n2b + 1) / 2) : r.n2b;
  r.n = max(0, ub - r.ua) * ow * g.C2;
  r.base = ((long)b * (g.pool ? g.PH : g.H2) + r.ua) * ow * g.C2;
  return r;
}

template <bool ONE>
__device__ __forceinline__ void cp_bwd_body(const CPBwdArgs& a, const int bid, float* smem) {
  const CPGeom& g = a.g;
  const int b = bid / g.nbands, band = bid % g.nbands;
  const int pr0 = band * g.PR;
  const CPBand t0 = cp_band(g, 0, 0);
  (void)t0;
  const int o2a_ = g.pool ? 2 * pr0 : pr0;
  const bool last_ = band == g.nbands - 1;
  const int o2b_ = g.pool ? (last_ ? g.H2 : 2 * min(g.PH, pr0 + g.PR)) : min(g.PH, pr0 + g.PR);
  const CPBand t = cp_band(g, o2a_, o2b_);            // c1 tile rows o2a - PTB ..
  const CPBwdLayout L = cp_bwd_layout(g, band, t.TXH, t.TXW, t.T1H, t.T1W);
  float* s_pA = smem + L.pA;
  float* s_wB = smem + L.pB;
  float* s_x = smem + L.x;
  float* s_c1 = smem + L.c1;
  float* s_dc2 = smem + L.dc2;
  float* s_dc1 = smem + L.dc1;
  float* s_red = smem + L.red;
  // BatchNorm tables / backward sums: dynamic LDS inside the reduction region (its dwB tile
  // is written only after the route, their last reader) — no static LDS in this launch
  float* s_bn = s_red + 2 * CP_MAXC2;                        // [4][MAXC2] mean | rstd | a | b
  float* s_ss = s_bn + 4 * CP_MAXC2;                         // [2][C2] backward sums
  int* s_offA = reinterpret_cast<int*>(smem + L.offs);      // conv A (recompute): x offsets
  int* s_offPA = s_offA + L.kpadA;                           //                    panel rows
  int* s_pix2 = s_offPA + L.kpadA;                           // dwB: pixel -> c1 tile offset
  int* s_pixd = s_pix2 + L.kp2;                              //      pixel -> dc2 tile offset
  int* s_offD = s_pixd + L.kp2;                              // dc1: k=(i,j,c2) -> dc2 offset
  int* s_offW = s_offD + L.kpadD;                            //      k -> weight offset
  int* s_pix1x = s_offW + L.kpadD;                           // dwA: pixel -> x tile offset
  int* s_pix1d = s_pix1x + L.kp1;                            //      pixel -> dc1 offset
  int* s_tapB = s_pix1d + L.kp1;                             // dwB: tap -> c1 tile offset
  CP_STAMP(8);
  // Prologue.  ONE: every global load of the prologue — the two weight blocks, the x tile,
  // both BN slabs and the BN affine vectors — is issued first, the index tables below are
  // computed while they travel (VALU work that otherwise sat between dependent round
  // trips), then the LDS stores and the slab reduction.
  const int nA = L.kpadA * 16, nWB = L.KB * g.C2, nP = nA + L.kpadB * L.c16;
  const int nX = t.TXH * t.TXW * g.C0;
  const int C2x2 = 2 * g.C2, sper = CP_THREADS / C2x2;
  const int scol = (int)threadIdx.x % C2x2, srow = (int)threadIdx.x / C2x2;
  const bool sact = srow < sper;
  float pv[CPB_UP], vf[CPB_US], vb[CPB_US], sc = 0.f, of = 0.f;
  const CPRoute rt = cp_route(g, L, b);
  float rgz[CP_RU], ryv[CP_RU];
  int ram[CP_RU];
  bool pok[CPB_UP], xok[CPB_UX];
  uint8_t xv[CPB_UX];
  // precomputed index tables: issued first (the host checks that a band's region fits
  // CPB_UT ints per thread)
  const int ntab = cp_bwd_tab_ints(L);
  int tv[CPB_UT];
  if (a.tabs) {
    const int* tsrc = a.tabs + (long)band * a.tab_stride;
#pragma unroll
    for (int u = 0; u < CPB_UT; ++u) {              // (batches past the table: not issued)
      const int e = u * CP_THREADS + (int)threadIdx.x;
      tv[u] = 0;
      if (u * CP_THREADS < ntab) tv[u] = tsrc[e < ntab ? e : 0];
    }
  }
  if (ONE) {
    if (a.bn_on) for (int i = threadIdx.x; i < C2x2; i += CP_THREADS) { s_red[i] = 0.f; s_ss[i] = 0.f; }
#pragma unroll
    for (int u = 0; u < CPB_UP; ++u) {             // [panel A (padded to 16 cols) | wB dense]
      const int e = u * CP_THREADS + (int)threadIdx.x;
      const bool inA = e < nA;
      const int k = e >> 4, n = e & 15, f = e - nA;
      const bool ok = inA ? (k < L.KA && n < g.C1) : (e < nP && f < nWB);
      pok[u] = ok;
      pv[u] = 0.f;
      const float* p = !ok ? a.wA : (inA ? a.wA + k * g.C1 + n : a.wB + f);
      if (u * CP_THREADS < nP) pv[u] = *p;         // (whole batches past the panels: none)
    }
    if (a.bn_on && a.bn_tab) {
      // the forward tables come folded (one value per thread); of the backward slab only
      // the row batches that exist are loaded (a uniform branch per batch)
      sc = a.bn_tab[min((int)threadIdx.x, 4 * g.C2 - 1)];
#pragma unroll
      for (int u = 0; u < CPB_US; ++u) {
        const int r = srow + u * sper;
        vb[u] = 0.f;
        if (u * sper < a.bwd_nslab) vb[u] = a.bwd_slab[(size_t)(sact && r < a.bwd_nslab ? r : 0) * C2x2 + scol];
      }
    } else if (a.bn_on) {
      const int cc = (int)threadIdx.x < g.C2 ? (int)threadIdx.x : g.C2 - 1;
#pragma unroll
      for (int u = 0; u < CPB_US; ++u) {
        const int r = srow + u * sper;
        vf[u] = a.bn.slab[(size_t)(sact && r < a.bn.nslab ? r : 0) * C2x2 + scol];
        vb[u] = a.bwd_slab[(size_t)(sact && r < a.bwd_nslab ? r : 0) * C2x2 + scol];
      }
      sc = a.bn.scale[cc];
      of = a.bn.offset[cc];
    }
    const uint8_t* src = cp_image(a.img, a.idx, a.cursor, b, g.B, (long)g.H * g.W * g.C0);
    const int y0 = t.c1y0 - g.PTA, x0 = -g.PLB - g.PLA;
    const FastDiv dw(t.TXW * g.C0), dc(g.C0);
#pragma unroll
    for (int u = 0; u < CPB_UX; ++u) {
      const int e = u * CP_THREADS + (int)threadIdx.x;
      int r, rem, xx, c;
      dw.divmod(e < nX ? e : 0, r, rem);
      dc.divmod(rem, xx, c);
      const int y = y0 + r, x = x0 + xx;
      xok[u] = e < nX && y >= 0 && y < g.H && x >= 0 && x < g.W;
      xv[u] = 0;
      if (u * CP_THREADS < nX) xv[u] = src[xok[u] ? ((long)y * g.W + x) * g.C0 + c : 0];
    }
    // the route's first chunk (dz, y, argmax of the band's unit rows: written by earlier
    // launches) — in flight under the tables and the BatchNorm fold instead of a round
    // trip of its own after them
    if (rt.n > 0) {
#pragma unroll
      for (int u = 0; u < CP_RU; ++u) {
        const int i = min(u * CP_THREADS + (int)threadIdx.x, rt.n - 1);
        rgz[u] = ryv[u] = 0.f;
        ram[u] = 0;
        if (u * CP_THREADS < rt.n) {               // (batches past the band's rows: none)
          rgz[u] = a.dz[rt.base + i];
          ryv[u] = a.y[rt.base + i];
          ram[u] = g.pool ? (int)a.argmax[rt.base + i] : 0;
        }
      }
    }
  } else {
    const uint8_t* src = cp_image(a.img, a.idx, a.cursor, b, g.B, (long)g.H * g.W * g.C0);
    cp_stage_x(g, t, src, s_x);
    cp_stage_panel(s_pA, a.wA, L.KA, g.C1, L.kpadA, 16);
    cp_stage_flat(s_wB, a.wB, L.KB * g.C2, L.kpadB * L.c16);
  }
  CP_STAMP(16);
  for (int i = threadIdx.x; i < L.D2H * L.D2W * g.C2; i += CP_THREADS) s_dc2[i] = 0.f;
  for (int i = threadIdx.x; i < g.C1; i += CP_THREADS) s_dc1[L.npix1 * g.C1 + i] = 0.f;
  if (!a.tabs) cp_bwd_tables(g, t, L, s_offA);
  CP_STAMP(17);
  if (a.tabs) {
#pragma unroll
    for (int u = 0; u < CPB_UT; ++u) pin(tv[u]);
#pragma unroll
    for (int u = 0; u < CPB_UT; ++u) {
      const int e = u * CP_THREADS + (int)threadIdx.x;
      if (e < ntab) s_offA[e] = tv[u];
    }
  }
  if (ONE) {
#pragma unroll
    for (int u = 0; u < CPB_UP; ++u) pin(pv[u]);
#pragma unroll
    for (int u = 0; u < CPB_UP; ++u) {
      const int e = u * CP_THREADS + (int)threadIdx.x;
      if (e < nA) s_pA[e] = pok[u] ? pv[u] : 0.f;
      else if (e < nP) s_wB[e - nA] = pok[u] ? pv[u] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < CPB_UX; ++u) {
      const int e = u * CP_THREADS + (int)threadIdx.x;
      if (e < nX) s_x[e] = xok[u] ? (float)xv[u] * (1.0f / 255.0f) : 0.f;
    }
  }
  CP_STAMP(18);
  // BatchNorm tables of the unit output and the backward sums (every block reduces the
  // small slabs; block 0 writes the BN parameter gradients and running statistics)
  CP_STAMP(19);
  if (a.bn_on) {
    if (ONE && a.bn_tab) {
      pin(sc);
      float ab = 0.f;
#pragma unroll
      for (int u = 0; u < CPB_US; ++u) {
        pin(vb[u]);
        ab += srow + u * sper < a.bwd_nslab ? vb[u] : 0.f;
      }
      if ((int)threadIdx.x < 4 * g.C2) {
        const int k = (int)threadIdx.x / g.C2;
        s_bn[k * CP_MAXC2 + (int)threadIdx.x - k * g.C2] = sc;
      }
      __syncthreads();                             // the zeroing of s_ss
      if (sact) atomicAdd(&s_ss[scol], ab);
      __syncthreads();
    } else if (ONE) {
#pragma unroll
      for (int u = 0; u < CPB_US; ++u) { pin(vf[u]); pin(vb[u]); }
      float af = 0.f, ab = 0.f;
#pragma unroll
      for (int u = 0; u < CPB_US; ++u) {
        const int r = srow + u * sper;
        af += r < a.bn.nslab ? vf[u] : 0.f;
        ab += r < a.bwd_nslab ? vb[u] : 0.f;
      }
      __syncthreads();                             // the zeroing of s_red / s_ss
      if (sact) {
        atomicAdd(&s_red[scol], af);
        atomicAdd(&s_ss[scol], ab);
      }
      __syncthreads();
      if ((int)threadIdx.x < g.C2) {
        const int c = threadIdx.x;
        const float mean = s_red[c] / a.bn.count;
        const float var = fmaxf(s_red[g.C2 + c] / a.bn.count - mean * mean, 0.f);
        const float rstd = rsqrtf(var + a.bn.eps);
        const float aa = sc * rstd;
        s_bn[c] = mean;
        s_bn[CP_MAXC2 + c] = rstd;
        s_bn[2 * CP_MAXC2 + c] = aa;
        s_bn[3 * CP_MAXC2 + c] = of - mean * aa;
      }
      __syncthreads();
    } else {
      bn_reduce_to_lds(a.bn, s_bn, s_bn + CP_MAXC2, s_bn + 2 * CP_MAXC2, s_bn + 3 * CP_MAXC2, s_ss);
      __syncthreads();
      slab_sum_to_lds(a.bwd_slab, a.bwd_nslab, 2 * g.C2, s_ss);
    }
    if (bid == 0)
      for (int c = threadIdx.x; c < g.C2; c += CP_THREADS) {
        a.doffset[c] = s_ss[c];
        a.dscale[c] = s_ss[g.C2 + c];
        if (a.run_mean) {
          const float mean = s_bn[c];
          const float var = 1.0f / (s_bn[CP_MAXC2 + c] * s_bn[CP_MAXC2 + c]) - a.bn.eps;
          a.run_mean[c] = (1.f - a.momentum) * a.run_mean[c] + a.momentum * mean;
          a.run_var[c] = (1.f - a.momentum) * a.run_var[c] + a.momentum * var;
        }
      }
  }
  __syncthreads();
  // (every thread's image values are in LDS: this workgroup no longer reads the staged
  // batch, which the tail's staging workgroups overwrite with the next one)
  if (a.img_tk && threadIdx.x == 0)
    __hip_atomic_fetch_add(a.img_tk + (bid % 16) * 16, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  CP_STAMP(9);
  // ---- route: dc2 (zero-padded tile) for conv-B-output rows [d2y0, d2y0 + D2H - 1)
  {
    const int n2a = rt.n2a, n2b = rt.n2b;
    const int ow = g.pool ? g.PW : g.W2;
    const int ua = rt.ua;
    const int n = rt.n;
    const float inv_n = a.bn_on ? 1.0f / a.bn.count : 0.f;
    const long base = rt.base;
    const FastDiv dC(g.C2), dow(ow);
    constexpr int U = CP_RU;
    for (int i0 = 0; i0 < n; i0 += CP_THREADS * U) {
      float gz[U], yv[U];
      int am[U];
      if (ONE && i0 == 0) {                        // prefetched with the prologue
#pragma unroll
        for (int u = 0; u < U; ++u) { pin(rgz[u]); pin(ryv[u]); gz[u] = rgz[u]; yv[u] = ryv[u]; am[u] = ram[u]; }
      } else {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = min(i0 + u * CP_THREADS + (int)threadIdx.x, n - 1);
          gz[u] = a.dz[base + i];
          yv[u] = a.y[base + i];
          am[u] = g.pool ? (int)a.argmax[base + i] : 0;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * CP_THREADS + (int)threadIdx.x;
        if (i >= n) break;
        int pix, c, ry, px;
        dC.divmod(i, pix, c);
        dow.divmod(pix, ry, px);
        float gv = gz[u];
        if (a.bn_on) {
          const float xhat = (yv[u] - s_bn[c]) * s_bn[CP_MAXC2 + c];
          gv = s_bn[2 * CP_MAXC2 + c] * (gv - s_ss[c] * inv_n - xhat * s_ss[g.C2 + c] * inv_n);
        }
        gv = act_bwd(gv, yv[u], yv[u], a.actB, a.alphaB);
        const int y2 = g.pool ? 2 * (ua + ry) + (am[u] >> 1) : ua + ry;
        const int x2 = g.pool ? 2 * px + (am[u] & 1) : px;
        if (y2 >= n2a && y2 < n2b && x2 < g.W2)
          s_dc2[((y2 - L.d2y0) * L.D2W + x2 + g.KBw - 1 - g.PLB) * g.C2 + c] = gv;
      }
    }
  }
  CP_STAMP(10);
  // ---- c1 tile (rows o2a - PTB ..) recomputed from the input rows
  cp_conv_a(g, t, smem, s_x, s_pA, L.kpadA, s_offA, s_offPA, a.bA, a.actA, a.alphaA, s_c1);
  __syncthreads();
  CP_STAMP(11);
  // ---- weight gradient B: [taps (i, j, c1)] x [C2], K = owned conv-B-output pixels
  float* s_rB = s_red;                                        // [n16b][c16]
  float* s_bias = s_red + L.n16b * L.c16;                     // [C2] + [C1]
  float* s_rA = smem + L.rA;                                  // [4 waves][16][16] partials
  const bool rA_alias = L.rA == L.dc2;                        // (uniform)
  cp_gemm(smem, L.n16b >> 4, L.c16 >> 4, L.kp2 >> 2, s_pix2, s_pixd,
          [&](int m) { return L.c1 + s_tapB[m]; },
          [&](int n) { return L.dc2 + n; },
          [&](int tm, int tn, cp_f32x4 acc, int) {
            const int lane = threadIdx.x & 63, i16 = lane & 15, q = lane >> 4;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              s_rB[(tm * 16 + 4 * q + r) * L.c16 + tn * 16 + i16] = acc[r];
            }
          });
  // bias B: column sums of the owned dc2 pixels (4 threads per channel + LDS atomics)
  for (int i = threadIdx.x; i < g.C2 + g.C1; i += CP_THREADS) s_bias[i] = 0.f;
  CP_STAMP(12);
  // ---- dc1 of the owned c1 pixels: [pixels] x [C1], K = (i, j, c2), then act A backward
  {
    const FastDiv dw1(g.W1);
    cp_gemm(smem, (L.npix1 + 15) >> 4, 1, L.kpadD >> 2, s_offD, s_offW,
            [&](int m) {
              int yy, xx;
              dw1.divmod(m < L.npix1 ? m : 0, yy, xx);
              return L.dc2 + ((L.o1a + yy + g.PTB - L.d2y0) * L.D2W + xx + g.PLB + g.KBw - 1 - g.PLB) * g.C2;
            },
            [&](int n) { return L.pB + (n < g.C1 ? n : 0) * g.C2; },
            [&](int tm, int, cp_f32x4 acc, int) {
              const int lane = threadIdx.x & 63, c1 = lane & 15, q = lane >> 4;
              if (c1 >= g.C1) return;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int m = tm * 16 + 4 * q + r;
                if (m >= L.npix1) continue;
                int yy, xx;
                dw1.divmod(m, yy, xx);
                float d = acc[r];
                if (a.actA) {                                  // post-activation c1 decides act'
                  const int ty = L.o1a + yy - t.c1y0;
                  const float v = (ty >= 0 && ty < t.T1H) ? s_c1[(ty * t.T1W + xx + g.PLB) * g.C1 + c1] : 0.f;
                  d = act_bwd(d, v, v, a.actA, a.alphaA);
                }
                s_dc1[m * g.C1 + c1] = d;
              }
            });
  }
  __syncthreads();
  CP_STAMP(13);
  // bias sums (dc2 over the owned conv-B pixels, dc1 over the owned c1 pixels)
  {
    const int per = CP_THREADS / (g.C2 + g.C1);
    const int col = threadIdx.x % (g.C2 + g.C1), part = threadIdx.x / (g.C2 + g.C1);
    if (per > 0 && part < per) {
      float acc = 0.f;
      if (col < g.C2) {
        for (int p = part; p < L.npix2; p += per) acc += s_dc2[s_pixd[p] + col];
      } else {
        for (int p = part; p < L.npix1; p += per) acc += s_dc1[p * g.C1 + col - g.C2];
      }
      atomicAdd(&s_bias[col], acc);
    }
  }
  // ---- weight gradient A: [taps (i, j, c0)] x [C1], K = owned c1 pixels split over the
  // 4 waves (partials in LDS)
  {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, q = lane >> 4;
    const int kst = L.kp1 >> 2, per = (kst + 3) / 4, k0 = wave * per, k1 = min(kst, k0 + per);
    const float* pa = s_x + s_offA[i16 < L.kpadA ? i16 : 0];
    const float* pb = s_dc1 + (i16 < g.C1 ? i16 : 0);
    cp_f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int ks = k0; ks < k1; ++ks) {
      const int p = 4 * ks + q;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[s_pix1x[p]], pb[s_pix1d[p]], acc, 0, 0, 0);
    }
    // the partials overwrite the dc2 tile: every wave's bias sums (its last reader) first
    if (rA_alias) __syncthreads();
#pragma unroll
    for (int r = 0; r < 4; ++r) s_rA[wave * 256 + (4 * q + r) * 16 + i16] = acc[r];
  }
  __syncthreads();
  CP_STAMP(14);
  // ---- one atomic per (workgroup, weight) into stripe blockIdx % S, in memory order
  {
    const int sidx = bid % a.stripes;
    const int nB = L.KB * g.C2;
    for (int o = threadIdx.x; o < nB; o += CP_THREADS) {
      const int tap = o / g.C2, c2 = o - tap * g.C2;
      atomicAdd(&a.dwB[(long)sidx * nB + o], s_rB[tap * L.c16 + c2]);
    }
    if (a.hasBiasB)
      for (int o = threadIdx.x; o < g.C2; o += CP_THREADS) atomicAdd(&a.dbB[(long)sidx * g.C2 + o], s_bias[o]);
    const int nA = L.KA * g.C1;
    for (int o = threadIdx.x; o < nA; o += CP_THREADS) {
      const int tap = o / g.C1, c1 = o - tap * g.C1;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += s_rA[w * 256 + tap * 16 + c1];
      atomicAdd(&a.dwA[(long)sidx * nA + o], v);
    }
    if (a.bA)
      for (int o = threadIdx.x; o < g.C1; o += CP_THREADS) atomicAdd(&a.dbA[(long)sidx * g.C1 + o], s_bias[g.C2 + o]);
  }
  CP_STAMP(15);
}

template <bool ONE>
__global__ __launch_bounds__(CP_THREADS) void conv_pair_bwd_kernel(CPBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cp_bwd_body<ONE>(a, (int)blockIdx.x, smem);
}

// Horizontal fusion (round 4): the pair backward's workgroups [0, B * nbands) followed by
// the deferred dense weight-gradient + update segments (csa_dense_update_defer; 128-column
// 256-thread workgroups of du_body, dX = null).  The pair backward is a latency chain that
// leaves most CU cycles and memory bandwidth idle (3 % HBM, 8 % MFMA: profiles/
// r3_roofline.md); the dense updates only have to finish before the next step's forward
// of their layer, so they run inside this launch instead of as serial links of the chain.
// The pair's workgroups come first: the dispatcher deals blocks in index order, so the
// critical pair blocks all start before any update block takes a slot.
//
// Tail (round 5): the rest of the fused program's optimizer launch, as workgroups of this
// launch.  What that launch still did after horizontal fusion — fold the conv weight-
// gradient stripes and update the conv and BatchNorm parameters, zero the BN statistic
// slabs for the next step, stage the next step's batch — depends only on THIS launch's
// pair workgroups, which finish well before its dense update workgroups (pair chain
// ~21 us, launch ~28 us: profiles/r4_notes.md).  So, after the update segments:
//   tail 0            waits until every pair workgroup is done (ticket 0), then folds /
//                     updates the striped and direct-gradient parameters and zeroes;
//   tail 1 .. NS      wait until every pair workgroup has its image tile in LDS (ticket
//                     1), then copy the next batch (rows[cursor]) into the staging buffers.
// Tail workgroups take slots only after every pair / update workgroup was dispatched, so
// their (bounded) waits are on workgroups that already run; the last tail workgroup to
// finish resets the tickets for the next launch.  The head's parameters are updated in
// the last dense segment's head epilogue and the metric ring is written there too, so the
// fused program's step has no optimizer launch at all.
constexpr int CPT_MAXSEG = 8;
// Tickets: 700 workgroups adding into ONE word serialise at the memory side, and a wave's
// next vmcnt wait includes its own atomic — so each count is spread over CPT_SPREAD words
// on separate 64-byte lines (workgroup b adds into word b % CPT_SPREAD; waiters sum them).
constexpr int CPT_SPREAD = 16, CPT_LINE = 16;         // words, words per line
constexpr int CPT_TK_WORDS = (2 * CPT_SPREAD + 1) * CPT_LINE;   // (the last line: unused)
static_assert(CPT_SPREAD == 16 && CPT_LINE == 16, "cp_bwd_body spreads the image ticket the same way");
__host__ __device__ __forceinline__ unsigned* cpt_word(unsigned* tk, int count, int b) {
  return tk + (count * CPT_SPREAD + (b % CPT_SPREAD)) * CPT_LINE;
}
// One parameter workgroup of the tail: elements [base, base + 256) of one parameter tensor
// (w updated with g = sum_s src[s * ld + i]).  A device table built once at plan time
// (csa_conv_pair_tail_plan): each workgroup reads its own entry with a uniform address (a
// scalar load) — per-lane selection among argument arrays made the compiler copy the whole
// argument struct to scratch in EVERY workgroup of the launch.
struct CPTailSeg {
  float* w; float* s0; float* s1; float* src;
  int S, ld, n, zero, base, store, pad1, pad2;   // store: w[i] = the sum (a gradient fold,
};                                               // data parallel: exchanged before the update)
struct CPTail {
  int on, param_blocks, stage_blocks;
  unsigned* tk;                     // [CPT_TK_WORDS]: pair workgroups done | image tiles
                                    // consumed (CPT_SPREAD words each) | tails done
  int* err;                         // [1]: a tail wait timed out (nothing of that tail ran)
  int* force;                       // [1] or null: debug — while nonzero every tail's wait
                                    // asks for one ticket more than exists (forced timeout);
                                    // the closing tail clears it (one-shot, host-armed)
  int opt; float lr; const int64_t* step;
  const CPTailSeg* segs;            // [param_blocks]
  int nz; float* zp[CP_MAXZ]; int zn[CP_MAXZ];
  // next batch: out_img[b][..] = img[rows[cursor * B + b]][..] (32-bit words), out_lbl
  const uint32_t* img; const int64_t* labels; const int64_t* rows; const int64_t* cursor;
  int B, words; uint32_t* out_img; int64_t* out_lbl;
};

__device__ __forceinline__ bool cp_tail_wait(const CPTail& t, int k, unsigned want, bool acquire = true) {
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    int ok = 1;
    // relaxed polls (an acquire per poll invalidates this XCD's L2 every iteration — under
    // every other workgroup of the launch), ONE acquire once the count is reached
    for (;;) {
      unsigned have = 0;
#pragma unroll
      for (int j = 0; j < CPT_SPREAD; ++j)
        have += __hip_atomic_load(cpt_word(t.tk, k, j), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (have >= want) break;
      if (wall_clock64() - t0 > 100000000ull) {           // 1 s: never a hung launch
        __hip_atomic_store(t.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(8);
    }
    if (acquire) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    s_ok = ok;
  }
  __syncthreads();
  return s_ok != 0;
}

// Tail workgroup k < param_blocks: its table entry's 256 elements.  The entry and the
// parameter / slot values (which no pair workgroup writes) are loaded BEFORE the wait, so
// after the last pair workgroup only the stripe loads — one round trip — remain.
struct CPTailPre { CPTailSeg d; float wv, z0, z1; };
__device__ __forceinline__ CPTailPre cp_tail_prefetch(const CPTail& t, int k) {
  CPTailPre p;
  p.d = t.segs[k];                                     // uniform address: scalar loads
  const int i = max(min(p.d.base + (int)threadIdx.x, p.d.n - 1), 0);
  const int nslot = opt_nslots(t.opt);
  p.wv = p.d.w[i];
  p.z0 = nslot >= 1 ? p.d.s0[i] : 0.f;
  p.z1 = nslot >= 2 ? p.d.s1[i] : 0.f;
  return p;
}

__device__ __forceinline__ void cp_tail_params(const CPTail& t, int k, CPTailPre& p) {
  const CPTailSeg& d = p.d;
  const int i = d.base + (int)threadIdx.x;
  if (i < d.n) {
    const int nslot = opt_nslots(t.opt);
    float v[16];
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) v[s2] = d.src[(s2 < d.S ? s2 : 0) * d.ld + i];   // all in flight
    float wv = p.wv, z0 = p.z0, z1 = p.z1;
    float gsum = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < 16; ++s2) gsum += s2 < d.S ? v[s2] : 0.f;
    if (d.store) {
      d.w[i] = gsum;
    } else {
      opt_update(t.opt, opt_step_lr(t.opt, t.lr, t.step), wv, gsum, z0, z1);
      d.w[i] = wv;
      if (nslot >= 1) d.s0[i] = z0;
      if (nslot >= 2) d.s1[i] = z1;
    }
    if (d.zero)
#pragma unroll
      for (int s2 = 0; s2 < 16; ++s2)
        if (s2 < d.S) d.src[s2 * d.ld + i] = 0.f;
  }
  // the statistic slabs, spread over the parameter workgroups
#pragma unroll
  for (int z = 0; z < CP_MAXZ; ++z) {
    if (z >= t.nz) break;
    for (int j = k * CP_THREADS + (int)threadIdx.x; j < t.zn[z]; j += t.param_blocks * CP_THREADS) t.zp[z][j] = 0.f;
  }
}

__device__ __forceinline__ void cp_tail_stage(const CPTail& t, int blk) {
  const long i = (long)blk * CP_THREADS + threadIdx.x;
  const long total = (long)t.B * t.words;
  const int64_t c = *t.cursor;
  if (i < t.B) t.out_lbl[i] = t.labels[t.rows[c * t.B + i]];
  if (i >= total) return;
  const long b = i / t.words, off = i - b * t.words;
  t.out_img[i] = t.img[t.rows[c * t.B + b] * t.words + off];
}

__device__ __forceinline__ void cp_tail_body(const CPTail& t, int npair, int k) {
  // (debug) a host-armed forced timeout: the wait asks for a ticket no workgroup adds
  const unsigned want = (unsigned)npair +
      ((t.force && __hip_atomic_load(t.force, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 1u : 0u);
  if (k < t.param_blocks) {
    CPTailPre p = cp_tail_prefetch(t, k);
    if (cp_tail_wait(t, 0, want)) cp_tail_params(t, k, p);
  } else {
    // (the staging copy reads nothing the pairs write — it only must not overwrite an
    // image before every pair has it in LDS — so no acquire: that would invalidate this
    // XCD's L2 under the update workgroups)
    if (cp_tail_wait(t, 1, want, false)) cp_tail_stage(t, k - t.param_blocks);
  }
  // The tickets are NOT reset here: the next step's pair forward zeroes them (its zero
  // list, hip_program._plan_tail), after this launch ended.  A closing "last tail resets"
  // counter made every tail's exit wait for an RMW round trip — on the launch's critical
  // path, after the last pair.  (A forced timeout is disarmed by the tails that saw it: they
  // all read the flag at their start, a second before any of them times out.)
  if (want != (unsigned)npair && threadIdx.x == 0)
    __hip_atomic_store(t.force, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool ONE, int NSLOT>
__device__ __forceinline__ void cp_bwd_upd_body(const CPBwdArgs& a, const DUSegs& u, const CPTail& t, float* smem) {
  const int npair = a.g.B * a.g.nbands;
  const int bid = (int)blockIdx.x;
  if (bid < npair) {
    cp_bwd_body<ONE>(a, bid, smem);
    if (t.on) {
      // the barrier drains every wave's stripe atomics (device-scope: visible once done);
      // block 0's plain stores (BN parameter gradients, running statistics) get ONE
      // release — not 700 L2 write-backs
      //
      // Why the ticket add below may be RELAXED (memory-ordering argument):
      //  * what the tail reads from the pairs are the weight-gradient stripes, written
      //    ONLY by device-scope atomic adds (agent scope: performed at the L2 that owns the
      //    line, never cached dirty in this CU's L1 / another XCD's L2 — there is no copy
      //    to publish);
      //  * __syncthreads() compiles to s_waitcnt vmcnt(0) + s_barrier: every wave of this
      //    workgroup has had its atomics RETURN (performed, globally visible at agent scope)
      //    before thread 0 passes the barrier, so the ticket add is issued strictly after
      //    them; a relaxed atomic cannot be hoisted above the barrier;
      //  * the tail's poll sees the ticket count reach `want` only after every pair's add
      //    issued, hence after all of that pair's stripe atomics were performed; its single
      //    agent-scope ACQUIRE after the poll invalidates its own L1 / non-coherent lines
      //    so its stripe loads read the L2 value;
      //  * block 0's plain (non-atomic) stores — BN parameter gradients, running
      //    statistics — are the only non-atomic data the tail reads, hence block 0's one
      //    agent-scope RELEASE before its ticket add (write-back of its dirty lines).
      // The staging tails read nothing any pair writes (they wait only so an image is not
      // overwritten before every pair loaded it into LDS), so they skip the acquire.
      // Pinned by tests/test_gpu_dp_overlap.py (tail error word stays 0 over many steps,
      // results equal the deterministic program's) and test_hip_step's per-step gradients.
      __syncthreads();
      if (threadIdx.x == 0) {
        if (bid == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(cpt_word(t.tk, 0, bid), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  const int nupd = u.start[u.nseg];
  if (bid < npair + nupd) {
    du_segs_body<NSLOT, true>(u, bid - npair, smem);
    return;
  }
  cp_tail_body(t, npair, bid - npair - nupd);
}

// diagnostics: [block][2] start / end (s_memrealtime, 100 MHz, one clock for every XCD) of
// each workgroup of the carrying launch (scripts/microbench.py MB_HF)
__constant__ long long* g_cp_life = nullptr;
// the same for the VALU pair forward (csa_cpv_life_debug)
__constant__ long long* g_cpv_life = nullptr;

template <bool ONE, int NSLOT>
__device__ __forceinline__ void cp_bwd_upd_entry(const CPBwdArgs& a, const DUSegs& u, const CPTail& t) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if (g_cp_life && threadIdx.x == 0) g_cp_life[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  cp_bwd_upd_body<ONE, NSLOT>(a, u, t, smem);
  if (g_cp_life) {
    __syncthreads();
    if (threadIdx.x == 0) g_cp_life[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  }
}

// Residency (round 6): 5 workgroups per CU.  The registers: the update-only body stages dY
// through LDS-DMA (no staging VGPRs), 95-96 VGPRs at 5 waves per SIMD without spills for
// 0 / 1 optimizer slots; the LDS: <= 31.2 KB per workgroup (the pair's BatchNorm scratch and
// dwA partials alias dead regions, the head epilogue reuses the Xw slice, no static LDS).
// Two slots (Adam) would spill at 5 waves: that form keeps the compiler's choice (4).
template <bool ONE, int NSLOT>
__global__ __launch_bounds__(CP_THREADS) __attribute__((amdgpu_waves_per_eu(5)))
void conv_pair_bwd_upd_kernel(CPBwdArgs a, DUSegs u, CPTail t) {
  cp_bwd_upd_entry<ONE, NSLOT>(a, u, t);
}
template <bool ONE>
__global__ __launch_bounds__(CP_THREADS) void conv_pair_bwd_upd2_kernel(CPBwdArgs a, DUSegs u, CPTail t) {
  cp_bwd_upd_entry<ONE, 2>(a, u, t);
}

// ---------------------------------------------------------------------------------------
// Small-pair VALU forward (round 3).  For the DSL's typical first pair — the sample's
// conv[2,2,10] -> conv[2,2,20] -> pool is 40 MACs per conv-B output — the MFMA forward
// above spent its time in dependent LDS phases (offset tables, 16x16x4 tiles for K = 4,
// per-tile epilogues: stamps convA 2.2 us, convB+pool 3.4 us of a 12.9 us launch).  Here
// every phase is one pass of plain FMAs over LDS with the whole workgroup busy:
//   loads   weights of both convs, biases and the band's uint8 input rows in ONE batch
//   conv A  one thread per c1 value of the band's tile (+ act A, zero outside the image)
//   conv B  one thread per (unit pixel, output channel): the pool window's positions
//           (+ bias, act B, max + argmax) with every weight read once per position
//   stats   per-channel {sum, sum^2} of the band folded in fixed order, one row per band
//           workgroup or an atomic fold into nslab rows
// Family (cpv_ok): C0 <= 4, C1 <= 16, C2 <= 32, kernels <= 3x3, and the weights / input
// tile fit one register batch of the workgroup.
constexpr int CPV_T = 256;
constexpr int CPV_MAXC1 = 16, CPV_MAXC2 = 32, CPV_MAXTAPS = 9;
constexpr int CPV_UW = 8, CPV_UX = 2;                  // per-thread load batch (weights, x)
constexpr int CPV_MAXKA = 16;                          // conv-A taps x C0 held in registers

struct CPVFwdArgs {
  CPGeom g;
  const uint8_t* img; const int64_t* idx; const int64_t* cursor;
  const float* wA; const float* bA; int actA; float alphaA;
  const float* wB; const float* bB; int actB; float alphaB;
  float* y; uint8_t* argmax; float* stat; int nslab;
};

__host__ __device__ inline int cpv_txw(const CPGeom& g) { return g.W2 + g.KBw - 1 + g.KAw - 1; }

template <int KBH, int KBW, bool CARRY>
__global__ __launch_bounds__(CPV_T) void cpv_fwd_kernel(CPVFwdArgs a, CPZero z, CPOptCarry oc) {
  const CPGeom& g = a.g;
  // CARRY: the deferred dense update's workgroups follow the pair's (its own instantiation:
  // the update's registers stay out of the plain forward)
  const int npair = CARRY ? (int)gridDim.x - oc.blocks : (int)gridDim.x;
  if (CARRY && (int)blockIdx.x >= npair) {
    cp_opt_carry(oc, (int)blockIdx.x - npair, oc.blocks);
    return;
  }
  __shared__ float s_w[CPV_UW * CPV_T];                 // [wA (KA x C1) | wB (KB x C2)]
  __shared__ int s_koffA[CPV_MAXKA];                    // x-tile offset of conv-A tap k
  __shared__ float s_b[CPV_MAXC1 + CPV_MAXC2];
  __shared__ float s_x[CPV_UX * CPV_T];
  extern __shared__ __attribute__((aligned(16))) float smem[];   // c1 tile | unit outputs
  const int b = blockIdx.x / g.nbands, band = blockIdx.x % g.nbands;
  const int pr0 = band * g.PR, pr1 = min(g.PH, pr0 + g.PR);
  const int r2a = g.pool ? 2 * pr0 : pr0, r2b = g.pool ? min(g.H2, 2 * pr1) : pr1;
  const CPBand t = cp_band(g, r2a, r2b);
  const int KA = g.KAh * g.KAw * g.C0, KB = g.KBh * g.KBw * g.C1;
  const int nwA = KA * g.C1, nwA4 = (nwA + 3) & ~3, nw = nwA4 + KB * g.C2, nb = g.C1 + g.C2;
  const int nX = t.TXH * t.TXW * g.C0;
  const int tid = threadIdx.x;
  CP_STAMP(0);
  if (g_cpv_life && tid == 0) g_cpv_life[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  // ---- one batch of loads: weights + biases first, then the image rows (the staged
  // image is at a fixed address; otherwise its row index chain runs under the weights).
  // LDS weights: [wA | pad to 4 | wB] (wB read as float2 / float4 rows)
  float wv[CPV_UW];
#pragma unroll
  for (int u = 0; u < CPV_UW; ++u) {                     // (batches wholly past the weights:
    const int e = u * CPV_T + tid;                          //  not issued)
    const float* p = e < nwA ? a.wA + e : (e >= nwA4 && e < nw ? a.wB + (e - nwA4) : a.wA);
    wv[u] = 0.f;
    if (u * CPV_T < nw) wv[u] = *p;
  }
  float bv = 0.f;
  if (tid < nb) bv = tid < g.C1 ? (a.bA ? a.bA[tid] : 0.f) : (a.bB ? a.bB[tid - g.C1] : 0.f);
  const uint8_t* src = cp_image(a.img, a.idx, a.cursor, b, g.B, (long)g.H * g.W * g.C0);
  const int y0 = t.c1y0 - g.PTA, x0 = -g.PLB - g.PLA;
  uint8_t xv[CPV_UX];
  bool xok[CPV_UX];
#pragma unroll
  for (int u = 0; u < CPV_UX; ++u) {
    const int e = u * CPV_T + tid;
    const int c = e % g.C0, rem = e / g.C0, xx = rem % t.TXW, r = rem / t.TXW;
    const int yy = y0 + r, xg = x0 + xx;
    xok[u] = e < nX && yy >= 0 && yy < g.H && xg >= 0 && xg < g.W;
    xv[u] = 0;
    if (u * CPV_T < nX) xv[u] = src[xok[u] ? ((long)yy * g.W + xg) * g.C0 + c : 0];
  }
#pragma unroll
  for (int u = 0; u < CPV_UW; ++u) pin(wv[u]);
#pragma unroll
  for (int u = 0; u < CPV_UW; ++u) {
    const int e = u * CPV_T + tid;
    if (e < nw) s_w[e] = wv[u];
  }
  if (tid < nb) s_b[tid] = bv;
#pragma unroll
  for (int u = 0; u < CPV_UX; ++u) {
    const int e = u * CPV_T + tid;
    if (e < nX) s_x[e] = xok[u] ? (float)xv[u] * (1.0f / 255.0f) : 0.f;
  }
  if (tid < KA) {
    const int c0 = tid % g.C0, ij = tid / g.C0, i = ij / g.KAw, j = ij - i * g.KAw;
    s_koffA[tid] = (i * t.TXW + j) * g.C0 + c0;
  }
  __syncthreads();
  CP_STAMP(1);
  // ---- conv A: the c1 tile [T1H][T1W][C1] (zero outside [0, H1) x [0, W1)): one thread
  // per (tile pixel, channel pair) — all 256 threads busy (one thread per pixel left 2/3 of
  // them idle behind a C1/2-long chain) — tap offsets held in registers
  float* s_c1 = smem;
  const int npx1 = t.T1H * t.T1W;
  {
    int koff[CPV_MAXKA];
#pragma unroll
    for (int k = 0; k < CPV_MAXKA; ++k) koff[k] = k < KA ? s_koffA[k] : 0;
    const int nc1p = g.C1 >> 1;
    for (int it = tid; it < npx1 * nc1p; it += CPV_T) {
      const int cp = it % nc1p, pix = it / nc1p, c1 = 2 * cp;
      const int tx = pix % t.T1W, ty = pix / t.T1W;
      const int yy = t.c1y0 + ty, xx = tx - g.PLB;
      const bool in = yy >= 0 && yy < g.H1 && xx >= 0 && xx < g.W1;
      const float* xb = s_x + (ty * t.TXW + tx) * g.C0;
      float a0 = s_b[c1], a1 = s_b[c1 + 1];
#pragma unroll
      for (int k = 0; k < CPV_MAXKA; ++k) {
        if (k >= KA) break;                                 // uniform
        const float xv = xb[koff[k]];
        const float2 w = *reinterpret_cast<const float2*>(s_w + k * g.C1 + c1);
        a0 = fmaf(xv, w.x, a0);
        a1 = fmaf(xv, w.y, a1);
      }
      *reinterpret_cast<float2*>(s_c1 + pix * g.C1 + c1) =
          in ? make_float2(act_fwd(a0, a.actA, a.alphaA), act_fwd(a1, a.actA, a.alphaA)) : make_float2(0.f, 0.f);
    }
  }
  __syncthreads();
  CP_STAMP(2);
  // ---- conv B (+ act B, + 2x2 max-pool): one thread per (unit pixel, channel pair).  Per
  // input channel the pool window's c1 values (WR x WC) and the pair's KBH x KBW weights
  // are loaded once and feed every (position, tap) FMA: 4 x taps x 2 FMAs per ~WR WC + taps loads
  const int ow = g.pool ? g.PW : g.W2;
  const int nunit = (g.pool ? (pr1 - pr0) : (r2b - r2a)) * ow;
  const int nout = nunit * g.C2;
  float* s_out = s_c1 + ((npx1 * g.C1 + 3) & ~3);          // [nunit][C2] outputs for the stats
  const float* wB = s_w + nwA4;
  constexpr int WR = KBH + 1, WC = KBW + 1;                // pool window footprint in c1
  const int ncp = g.C2 >> 1, npos = g.pool ? 4 : 1;
  for (int o = tid; o < nunit * ncp; o += CPV_T) {
    const int cp = o % ncp, u = o / ncp, py = u / ow, px = u - py * ow, c2 = 2 * cp;
    const int y2b = g.pool ? 2 * (pr0 + py) : r2a + py, x2b = g.pool ? 2 * px : px;
    float acc[4][2];
    const float b0 = s_b[g.C1 + c2], b1 = s_b[g.C1 + c2 + 1];
#pragma unroll
    for (int q = 0; q < 4; ++q) { acc[q][0] = b0; acc[q][1] = b1; }
    const float* cb = s_c1 + ((y2b - r2a) * t.T1W + x2b) * g.C1;
    const bool wide = g.pool != 0;                           // window rows/cols beyond KBH x KBW
#pragma unroll 2
    for (int c1 = 0; c1 < g.C1; ++c1) {
      float cv[WR][WC];
#pragma unroll
      for (int r = 0; r < WR; ++r)
#pragma unroll
        for (int c = 0; c < WC; ++c)
          cv[r][c] = (wide || (r < KBH && c < KBW)) ? cb[(r * t.T1W + c) * g.C1 + c1] : 0.f;
      float2 wv[KBH * KBW];
#pragma unroll
      for (int k = 0; k < KBH * KBW; ++k)
        wv[k] = *reinterpret_cast<const float2*>(wB + (k * g.C1 + c1) * g.C2 + c2);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int dy = q >> 1, dx = q & 1;
#pragma unroll
        for (int i = 0; i < KBH; ++i)
#pragma unroll
          for (int j = 0; j < KBW; ++j) {
            acc[q][0] = fmaf(cv[dy + i][dx + j], wv[i * KBW + j].x, acc[q][0]);
            acc[q][1] = fmaf(cv[dy + i][dx + j], wv[i * KBW + j].y, acc[q][1]);
          }
      }
    }
    float best0 = -INFINITY, best1 = -INFINITY;
    int am0 = 0, am1 = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (q >= npos) break;
      const int y2 = y2b + (q >> 1), x2 = x2b + (q & 1);
      if (y2 >= g.H2 || x2 >= g.W2) continue;
      const float v0 = act_fwd(acc[q][0], a.actB, a.alphaB), v1 = act_fwd(acc[q][1], a.actB, a.alphaB);
      if (v0 > best0) { best0 = v0; am0 = q; }
      if (v1 > best1) { best1 = v1; am1 = q; }
    }
    const int oo = u * g.C2 + c2;
    const long off = g.pool ? (((long)b * g.PH + pr0) * g.PW) * g.C2 + oo
                            : (((long)b * g.H2 + r2a) * g.W2) * g.C2 + oo;
    out_store2(a.y + off, best0, best1);
    if (g.pool && a.argmax) {
      a.argmax[off] = (uint8_t)am0;
      a.argmax[off + 1] = (uint8_t)am1;
    }
    *reinterpret_cast<float2*>(s_out + oo) = make_float2(best0, best1);
  }
  (void)nout;
  CP_STAMP(3);
  if (a.stat) {                                           // per-channel sums, fixed order
    // (column, unit slice) per thread, slices combined in order
    __shared__ float s_sp[CPV_T];
    __syncthreads();
    const int cols = 2 * g.C2, nsl = max(1, CPV_T / cols), per = (nunit + nsl - 1) / nsl;
    if (tid < cols * nsl) {
      const int col = tid % cols, sl = tid / cols, c = col % g.C2, sq = col / g.C2;
      float acc = 0.f;
      for (int u = sl * per; u < min(nunit, (sl + 1) * per); ++u) {
        const float v = s_out[u * g.C2 + c];
        acc += sq ? v * v : v;
      }
      s_sp[tid] = acc;
    }
    __syncthreads();
    if (tid < cols) {
      float acc = 0.f;
      for (int sl = 0; sl < nsl; ++sl) acc += s_sp[sl * cols + tid];
      float* row = a.stat + (size_t)(blockIdx.x % a.nslab) * 2 * g.C2;
      if (a.nslab >= npair) row[tid] = acc;                    // one row per workgroup
      else atomicAdd(&row[tid], acc);
    }
  }
  cp_zero_early(z, npair);            // (at the end: stores in front would delay the loads)
  CP_STAMP(4);
  if (g_cpv_life && tid == 0) g_cpv_life[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
}

// Small-pair VALU backward (round 3).  One workgroup per (image, band) as the MFMA
// backward, but every phase is one FMA pass over LDS with all 256 threads:
//   loads   both weight blocks, the band's input rows, the route operands (dz, y, argmax
//           of the unit rows the band's dc2 tile touches) and both BatchNorm slabs — one
//           batch, every load in flight before the first use
//   P1      BN tables (fwd slab -> mean / rstd / a, bwd slab -> S1 / S2, rows summed in
//           fixed order) and the c1 tile recomputed from the input rows
//   P2      route: dc2 tile = act_B'(BN'(dz)) placed at the argmax position of each unit
//   P3      conv-B weight gradient (owned conv-B pixels) | dc1 of the owned c1 pixels
//           through act A | conv-B bias gradient
//   P4      conv-A weight / bias gradients; weight gradients leave as one atomic per
//           (workgroup, weight) into stripe blockIdx % S, folded by the optimizer
constexpr int CPV_UR = 4;                                // route operand batch per thread
constexpr int CPV_US = 8;                                // slab values per thread (fwd + bwd)

struct CPVBwdTile {
  int o2a, o2b, o1a, o1b;        // owned conv-B output rows / owned c1 rows
  int d2a, d2b;                  // dc2 tile rows (owned conv-B rows + halo for dc1)
  int c1a, c1b, T1W;             // c1 tile rows; columns tx <-> c1 x = tx - PLB
  int xa, TXH, TXW;              // x tile: rows xa .., cols tx <-> x = tx - PLB - PLA
  int ua, ub;                    // unit rows of the route operands
};

__host__ __device__ inline CPVBwdTile cpv_bwd_tile(const CPGeom& g, int band) {
  CPVBwdTile t;
  const int pr0 = band * g.PR, pr1 = min(g.PH, pr0 + g.PR);
  const bool last = band == g.nbands - 1;
  t.o2a = g.pool ? 2 * pr0 : pr0;
  t.o2b = g.pool ? (last ? g.H2 : 2 * pr1) : pr1;
  t.o1a = t.o2a;
  t.o1b = last ? g.H1 : t.o2b;
  t.d2a = max(0, min(t.o2a, t.o1a + g.PTB - g.KBh + 1));
  t.d2b = min(g.H2, max(t.o2b, t.o1b + g.PTB));
  t.c1a = min(t.o2a - g.PTB, t.o1a);
  t.c1b = max(t.o2b - g.PTB + g.KBh - 1, t.o1b);
  t.T1W = g.W2 + g.KBw - 1;
  t.xa = t.c1a - g.PTA;
  t.TXH = (t.c1b - t.c1a) + g.KAh - 1;
  t.TXW = t.T1W + g.KAw - 1;
  t.ua = g.pool ? t.d2a / 2 : t.d2a;
  t.ub = g.pool ? min(g.PH, (t.d2b + 1) / 2) : t.d2b;
  return t;
}

struct CPVBwdLds { int x, c1, dc2, dc1, red, end; };

__host__ __device__ inline CPVBwdLds cpv_bwd_lds(const CPGeom& g, const CPVBwdTile& t) {
  CPVBwdLds L;
  int o = 0;
  L.x = o; o += (t.TXH * t.TXW * g.C0 + 3) & ~3;
  L.c1 = o; o += ((t.c1b - t.c1a) * t.T1W * g.C1 + 3) & ~3;
  L.dc2 = o; o += ((t.d2b - t.d2a) * g.W2 * g.C2 + 3) & ~3;
  L.dc1 = o; o += ((t.o1b - t.o1a) * g.W1 * g.C1 + 3) & ~3;
  // slab rows (fwd | bwd) staged for the fold, later the weight-gradient slice partials
  const int KB = g.KBh * g.KBw * g.C1, combos = g.C1 * (g.C2 / 2), nsl = combos > 0 ? (CPV_T / combos > 0 ? CPV_T / combos : 1) : 1;
  const int partB = nsl * (KB * g.C2 + g.C2), partA = CPV_T * 2;
  int red = (32 + 16) * 2 * CPV_MAXC2 + 4 * 4 * CPV_MAXC2;
  red = red > partB ? red : partB;
  red = red > partA ? red : partA;
  L.red = o; o += red;
  L.end = o;
  return L;
}

template <int KBH, int KBW>
__global__ __launch_bounds__(CPV_T) void cpv_bwd_kernel(CPBwdArgs a) {
  const CPGeom& g = a.g;
  __shared__ float s_w[CPV_UW * CPV_T];                 // [wA (KA x C1) | wB (KB x C2)]
  __shared__ float s_bA[CPV_MAXC1];
  __shared__ float s_bn[6 * CPV_MAXC2];                 // mean | rstd | a | S1 | S2 | -
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int b = blockIdx.x / g.nbands, band = blockIdx.x % g.nbands;
  const CPVBwdTile t = cpv_bwd_tile(g, band);
  const CPVBwdLds L = cpv_bwd_lds(g, t);
  float* s_x = smem + L.x;
  float* s_c1 = smem + L.c1;
  float* s_dc2 = smem + L.dc2;
  float* s_dc1 = smem + L.dc1;
  float* s_red = smem + L.red;
  const int tid = threadIdx.x;
  const int KA = g.KAh * g.KAw * g.C0, KB = g.KBh * g.KBw * g.C1;
  const int nwA = KA * g.C1, nwA4 = (nwA + 3) & ~3, nw = nwA4 + KB * g.C2;
  const int C2x2 = 2 * g.C2;
  const int ow = g.pool ? g.PW : g.W2;
  const int nroute = (t.ub - t.ua) * ow * g.C2;
  const long rbase = ((long)b * (g.pool ? g.PH : g.H2) + t.ua) * ow * g.C2;
  const int nX = t.TXH * t.TXW * g.C0;
  const int nsf = a.bn_on ? a.bn.nslab * C2x2 : 0, nsb = a.bn_on ? a.bwd_nslab * C2x2 : 0;
  CP_STAMP(8);
  // ---- one batch of loads
  float wv[CPV_UW];
#pragma unroll
  for (int u = 0; u < CPV_UW; ++u) {
    const int e = u * CPV_T + tid;
    wv[u] = *(e < nwA ? a.wA + e : (e >= nwA4 && e < nw ? a.wB + (e - nwA4) : a.wA));
  }
  const float bav = (a.bA && tid < g.C1) ? a.bA[tid] : 0.f;
  float rz[CPV_UR], ry[CPV_UR];
  int ram[CPV_UR];
#pragma unroll
  for (int u = 0; u < CPV_UR; ++u) {
    const int e = min(u * CPV_T + tid, max(nroute - 1, 0));
    rz[u] = a.dz[rbase + e];
    ry[u] = a.y[rbase + e];
    ram[u] = g.pool ? (int)a.argmax[rbase + e] : 0;
  }
  float sv[CPV_US];
#pragma unroll
  for (int u = 0; u < CPV_US; ++u) {
    const int e = u * CPV_T + tid;
    const float* p = e < nsf ? a.bn.slab + e : (e < nsf + nsb ? a.bwd_slab + (e - nsf) : a.wA);
    sv[u] = *p;
  }
  float sc = 0.f, of = 0.f;
  if (a.bn_on && tid < g.C2) { sc = a.bn.scale[tid]; of = a.bn.offset[tid]; }
  const uint8_t* src = cp_image(a.img, a.idx, a.cursor, b, g.B, (long)g.H * g.W * g.C0);
  uint8_t xv[CPV_UX];
  bool xok[CPV_UX];
#pragma unroll
  for (int u = 0; u < CPV_UX; ++u) {
    const int e = u * CPV_T + tid;
    const int c = e % g.C0, rem = e / g.C0, xx = rem % t.TXW, r = rem / t.TXW;
    const int yy = t.xa + r, xg = xx - g.PLB - g.PLA;
    xok[u] = e < nX && yy >= 0 && yy < g.H && xg >= 0 && xg < g.W;
    xv[u] = src[xok[u] ? ((long)yy * g.W + xg) * g.C0 + c : 0];
  }
  // ---- LDS stores
#pragma unroll
  for (int u = 0; u < CPV_UW; ++u) {
    pin(wv[u]);
    const int e = u * CPV_T + tid;
    if (e < nw) s_w[e] = wv[u];
  }
  if (tid < g.C1) s_bA[tid] = bav;
#pragma unroll
  for (int u = 0; u < CPV_US; ++u) {
    pin(sv[u]);
    const int e = u * CPV_T + tid;
    if (e < nsf + nsb) s_red[e] = sv[u];
  }
#pragma unroll
  for (int u = 0; u < CPV_UX; ++u) {
    const int e = u * CPV_T + tid;
    if (e < nX) s_x[e] = xok[u] ? (float)xv[u] * (1.0f / 255.0f) : 0.f;
  }
  const int n2 = (t.d2b - t.d2a) * g.W2 * g.C2;
  for (int e = tid; e < n2; e += CPV_T) s_dc2[e] = 0.f;
  __syncthreads();
  CP_STAMP(9);
  // ---- P1: BN tables (rows summed in fixed order) | c1 tile
  if (a.bn_on) {
    // fixed-order two-level fold of both slabs: column x row-slice partials, then slices
    // in order (a one-thread-per-column chain of 48 dependent LDS reads took ~2 us)
    constexpr int NSL = 4;
    float* s_sl = s_red + nsf + nsb;                         // [NSL][4 C2]
    const int cols = 2 * C2x2;                               // fwd S1 | fwd S2 | bwd S1 | bwd S2
    for (int e = tid; e < NSL * cols; e += CPV_T) {
      const int col = e % cols, sl = e / cols;
      const bool fw = col < C2x2;
      const int nr = fw ? a.bn.nslab : a.bwd_nslab, c = fw ? col : col - C2x2;
      const float* base = s_red + (fw ? 0 : nsf);
      const int rper = (nr + NSL - 1) / NSL;
      float acc = 0.f;
      for (int r = sl * rper; r < min(nr, (sl + 1) * rper); ++r) acc += base[r * C2x2 + c];
      s_sl[sl * cols + col] = acc;
    }
    __syncthreads();
    if (tid < g.C2) {
      const int c = tid;
      float s1 = 0.f, s2 = 0.f, b1 = 0.f, b2 = 0.f;
#pragma unroll
      for (int sl = 0; sl < NSL; ++sl) {
        s1 += s_sl[sl * cols + c];
        s2 += s_sl[sl * cols + g.C2 + c];
        b1 += s_sl[sl * cols + C2x2 + c];
        b2 += s_sl[sl * cols + C2x2 + g.C2 + c];
      }
      const float mean = s1 / a.bn.count;
      const float var = fmaxf(s2 / a.bn.count - mean * mean, 0.f);
      const float rstd = rsqrtf(var + a.bn.eps);
      s_bn[c] = mean;
      s_bn[CPV_MAXC2 + c] = rstd;
      s_bn[2 * CPV_MAXC2 + c] = sc * rstd;
      s_bn[3 * CPV_MAXC2 + c] = b1;
      s_bn[4 * CPV_MAXC2 + c] = b2;
      if (blockIdx.x == 0) {
        a.doffset[c] = b1;
        a.dscale[c] = b2;
        if (a.run_mean) {
          a.run_mean[c] = (1.f - a.momentum) * a.run_mean[c] + a.momentum * mean;
          a.run_var[c] = (1.f - a.momentum) * a.run_var[c] + a.momentum * var;
        }
      }
    }
  }
  (void)of;
  const int n1 = (t.c1b - t.c1a) * t.T1W * g.C1;
  for (int e = tid; e < n1; e += CPV_T) {
    const int c1 = e % g.C1, pix = e / g.C1, tx = pix % t.T1W, ty = pix / t.T1W;
    const int yy = t.c1a + ty, xx = tx - g.PLB;
    float v = 0.f;
    if (yy >= 0 && yy < g.H1 && xx >= 0 && xx < g.W1) {
      float acc = s_bA[c1];
      for (int i = 0; i < g.KAh; ++i)
        for (int j = 0; j < g.KAw; ++j) {
          const float* xr = s_x + ((ty + i) * t.TXW + tx + j) * g.C0;
          const float* wr = s_w + ((i * g.KAw + j) * g.C0) * g.C1 + c1;
          for (int c0 = 0; c0 < g.C0; ++c0) acc = fmaf(xr[c0], wr[c0 * g.C1], acc);
        }
      v = act_fwd(acc, a.actA, a.alphaA);
    }
    s_c1[e] = v;
  }
  __syncthreads();
  CP_STAMP(10);
  // ---- P2: route into the dc2 tile (registers hold the operands since the prologue)
  {
    const float inv_n = a.bn_on ? 1.0f / a.bn.count : 0.f;
#pragma unroll
    for (int u = 0; u < CPV_UR; ++u) {
      const int e = u * CPV_T + tid;
      if (e >= nroute) break;
      const int c = e % g.C2, pix = e / g.C2, px = pix % ow, uy = pix / ow;
      float gv = rz[u];
      if (a.bn_on) {
        const float xhat = (ry[u] - s_bn[c]) * s_bn[CPV_MAXC2 + c];
        gv = s_bn[2 * CPV_MAXC2 + c] * (gv - s_bn[3 * CPV_MAXC2 + c] * inv_n - xhat * s_bn[4 * CPV_MAXC2 + c] * inv_n);
      }
      gv = act_bwd(gv, ry[u], ry[u], a.actB, a.alphaB);
      const int y2 = g.pool ? 2 * (t.ua + uy) + (ram[u] >> 1) : t.ua + uy;
      const int x2 = g.pool ? 2 * px + (ram[u] & 1) : px;
      if (y2 >= t.d2a && y2 < t.d2b && x2 < g.W2) s_dc2[((y2 - t.d2a) * g.W2 + x2) * g.C2 + c] = gv;
    }
  }
  __syncthreads();
  CP_STAMP(11);
  const int sidx = blockIdx.x % a.stripes;
  float* s_part = s_red;                                   // slab staging is dead now: partials
  // ---- P3a: conv-B weight (+ bias) gradient over the owned conv-B pixels.  Thread =
  // (c1, channel pair, pixel slice): per pixel the c1 values of the KBH x KBW taps and the
  // pair's dc2 (float2) feed taps x 2 FMAs; slices folded through LDS in fixed order.
  {
    const int ncp = g.C2 >> 1, combos = g.C1 * ncp, nsl = max(1, CPV_T / combos);
    const int npx2 = (t.o2b - t.o2a) * g.W2;
    const int nBw = KB * g.C2;
    const int bias_off = nsl * nBw;                        // [nsl][C2] bias partials after the weights
    if (tid < combos * nsl) {
      const int cp = tid % ncp, c1 = (tid / ncp) % g.C1, sl = tid / combos, c2 = 2 * cp;
      float acc[KBH * KBW][2], ab[2] = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < KBH * KBW; ++k) { acc[k][0] = 0.f; acc[k][1] = 0.f; }
#pragma unroll 4
      for (int p = sl; p < npx2; p += nsl) {
        const int y2 = t.o2a + p / g.W2, x2 = p % g.W2;
        const float2 d = *reinterpret_cast<const float2*>(s_dc2 + ((y2 - t.d2a) * g.W2 + x2) * g.C2 + c2);
        const float* cr = s_c1 + ((y2 - g.PTB - t.c1a) * t.T1W + x2) * g.C1 + c1;
        float cv[KBH * KBW];
#pragma unroll
        for (int i = 0; i < KBH; ++i)
#pragma unroll
          for (int j = 0; j < KBW; ++j) cv[i * KBW + j] = cr[(i * t.T1W + j) * g.C1];
#pragma unroll
        for (int k = 0; k < KBH * KBW; ++k) {
          acc[k][0] = fmaf(cv[k], d.x, acc[k][0]);
          acc[k][1] = fmaf(cv[k], d.y, acc[k][1]);
        }
        ab[0] += d.x;
        ab[1] += d.y;
      }
#pragma unroll
      for (int k = 0; k < KBH * KBW; ++k)
        *reinterpret_cast<float2*>(s_part + sl * nBw + (k * g.C1 + c1) * g.C2 + c2) = make_float2(acc[k][0], acc[k][1]);
      if (c1 == 0) *reinterpret_cast<float2*>(s_part + bias_off + sl * g.C2 + c2) = make_float2(ab[0], ab[1]);
    }
    __syncthreads();
    for (int o = tid; o < nBw + g.C2; o += CPV_T) {
      float v = 0.f;
      if (o < nBw) {
        for (int q = 0; q < nsl; ++q) v += s_part[q * nBw + o];
        atomicAdd(&a.dwB[(long)sidx * nBw + o], v);
      } else if (a.hasBiasB) {
        for (int q = 0; q < nsl; ++q) v += s_part[bias_off + q * g.C2 + o - nBw];
        atomicAdd(&a.dbB[(long)sidx * g.C2 + o - nBw], v);
      }
    }
  }
  // ---- P3b: dc1 of the owned c1 pixels (through act A).  Thread = (pixel, c1 pair): per
  // valid tap one float4 of dc2 and two float4 weight rows feed 8 FMAs.
  {
    const float* wB = s_w + nwA4;
    const int npx1 = (t.o1b - t.o1a) * g.W1, nc1p = g.C1 >> 1;
    for (int e = tid; e < npx1 * nc1p; e += CPV_T) {
      const int c1 = 2 * (e % nc1p), pix = e / nc1p, x1 = pix % g.W1, y1 = t.o1a + pix / g.W1;
      float a0 = 0.f, a1 = 0.f;
#pragma unroll
      for (int i = 0; i < KBH; ++i) {
        const int y2 = y1 + g.PTB - i;
        if (y2 < t.d2a || y2 >= t.d2b) continue;
#pragma unroll
        for (int j = 0; j < KBW; ++j) {
          const int x2 = x1 + g.PLB - j;
          if (x2 < 0 || x2 >= g.W2) continue;
          const float* dr = s_dc2 + ((y2 - t.d2a) * g.W2 + x2) * g.C2;
          const float* w0 = wB + ((i * KBW + j) * g.C1 + c1) * g.C2;
          const float* w1 = w0 + g.C2;
#pragma unroll
          for (int c2 = 0; c2 < CPV_MAXC2; c2 += 4) {
            if (c2 >= g.C2) break;                           // uniform
            const float4 d = *reinterpret_cast<const float4*>(dr + c2);
            const float4 u0 = *reinterpret_cast<const float4*>(w0 + c2);
            const float4 u1 = *reinterpret_cast<const float4*>(w1 + c2);
            a0 = fmaf(d.x, u0.x, a0); a0 = fmaf(d.y, u0.y, a0); a0 = fmaf(d.z, u0.z, a0); a0 = fmaf(d.w, u0.w, a0);
            a1 = fmaf(d.x, u1.x, a1); a1 = fmaf(d.y, u1.y, a1); a1 = fmaf(d.z, u1.z, a1); a1 = fmaf(d.w, u1.w, a1);
          }
        }
      }
      if (a.actA) {                                        // post-activation c1 decides act'
        const float* cv = s_c1 + ((y1 - t.c1a) * t.T1W + x1 + g.PLB) * g.C1 + c1;
        a0 = act_bwd(a0, cv[0], cv[0], a.actA, a.alphaA);
        a1 = act_bwd(a1, cv[1], cv[1], a.actA, a.alphaA);
      }
      *reinterpret_cast<float2*>(s_dc1 + pix * g.C1 + c1) = make_float2(a0, a1);
    }
  }
  __syncthreads();
  CP_STAMP(12);
  // ---- P4: conv-A weight / bias gradients over the owned c1 pixels.  Thread = (tap or the
  // bias row, c1 pair, pixel slice); slices folded through LDS in fixed order.
  {
    const int npx = (t.o1b - t.o1a) * g.W1, nc1p = g.C1 >> 1;
    const int rows = KA + (a.bA ? 1 : 0), combos = rows * nc1p, nsl = max(1, CPV_T / combos);
    if (tid < combos * nsl) {
      const int cp = tid % nc1p, k = (tid / nc1p) % rows, sl = tid / combos, c1 = 2 * cp;
      int koff = 0;
      if (k < KA) {
        const int c0 = k % g.C0, ij = k / g.C0, i = ij / g.KAw, j = ij - i * g.KAw;
        koff = (i * t.TXW + j) * g.C0 + c0;
      }
      float a0 = 0.f, a1 = 0.f;
#pragma unroll 4
      for (int p = sl; p < npx; p += nsl) {
        const int y1 = t.o1a + p / g.W1, x1 = p % g.W1;
        const float xv2 = k < KA ? s_x[((y1 - g.PTA - t.xa) * t.TXW + x1 + g.PLB) * g.C0 + koff] : 1.f;
        const float2 d = *reinterpret_cast<const float2*>(s_dc1 + p * g.C1 + c1);
        a0 = fmaf(xv2, d.x, a0);
        a1 = fmaf(xv2, d.y, a1);
      }
      *reinterpret_cast<float2*>(s_part + (sl * rows + k) * g.C1 + c1) = make_float2(a0, a1);
    }
    __syncthreads();
    for (int o = tid; o < rows * g.C1; o += CPV_T) {
      float v = 0.f;
      for (int q = 0; q < nsl; ++q) v += s_part[q * rows * g.C1 + o];
      if (o < KA * g.C1) atomicAdd(&a.dwA[(long)sidx * KA * g.C1 + o], v);
      else atomicAdd(&a.dbA[(long)sidx * g.C1 + o - KA * g.C1], v);
    }
  }
  CP_STAMP(13);
}

static bool cpv_ok(const CPGeom& g) {
  if (g.C0 > 4 || g.C1 > CPV_MAXC1 || g.C2 > CPV_MAXC2) return false;
  if (g.KAh * g.KAw * g.C0 > CPV_MAXKA || g.C1 % 2 || g.C2 % 2) return false;
  if (!((g.KBh == 2 && g.KBw == 2) || (g.KBh == 3 && g.KBw == 3))) return false;   // instantiated
  if (g.pool && (g.PH * 2 > g.H2 + 1 || g.PW * 2 > g.W2 + 1)) return false;
  const int KA = g.KAh * g.KAw * g.C0, KB = g.KBh * g.KBw * g.C1;
  if (((KA * g.C1 + 3) & ~3) + KB * g.C2 > CPV_UW * CPV_T) return false;
  const int rows = g.pool ? 2 * g.PR : g.PR;
  const int TXH = rows + g.KBh - 1 + g.KAh - 1;
  if (TXH * cpv_txw(g) * g.C0 > CPV_UX * CPV_T) return false;
  return true;
}

static size_t cp_lds(const CPGeom& g, bool bwd);
static bool cp_lds_ok_bwd(const CPGeom& g) { return cp_lds(g, true) <= CP_LDS_MAX; }

static bool cpv_bwd_ok(const CPBwdArgs& a) {
  const CPGeom& g = a.g;
  if (!cpv_ok(g)) return false;
  if (a.bn_on && (a.bn.nslab > 32 || a.bwd_nslab > 16 ||
                  (a.bn.nslab + a.bwd_nslab) * 2 * g.C2 > CPV_US * CPV_T)) return false;
  for (int band = 0; band < g.nbands; ++band) {
    const CPVBwdTile t = cpv_bwd_tile(g, band);
    const int ow = g.pool ? g.PW : g.W2;
    if ((t.ub - t.ua) * ow * g.C2 > CPV_UR * CPV_T) return false;
    if (t.TXH * t.TXW * g.C0 > CPV_UX * CPV_T) return false;
    if (cpv_bwd_lds(g, t).end * sizeof(float) > CP_LDS_MAX) return false;
  }
  return true;
}

static size_t cpv_bwd_lds_max(const CPGeom& g) {
  size_t mx = 0;
  for (int band = 0; band < g.nbands; ++band) mx = std::max(mx, (size_t)cpv_bwd_lds(g, cpv_bwd_tile(g, band)).end);
  return mx * sizeof(float);
}

static size_t cpv_fwd_lds(const CPGeom& g) {
  const int rows = g.pool ? 2 * g.PR : g.PR;
  const int T1H = rows + g.KBh - 1, T1W = g.W2 + g.KBw - 1;
  const int units = (g.pool ? g.PR * g.PW : g.PR * g.W2);
  return (size_t)(((T1H * T1W * g.C1 + 3) & ~3) + units * g.C2) * sizeof(float);
}

static bool cp_geom(const int* v, CPGeom& g) {
  g = CPGeom{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12], v[13], v[14], v[15],
             v[16], v[17], v[18], v[19], v[20], 0, 0};
  if (g.C0 < 1 || g.C0 > 4 || g.C1 < 2 || g.C1 > CP_MAXC1 || g.C1 % 2 || g.C2 < 4 || g.C2 > CP_MAXC2 || g.C2 % 4) return false;
  if (g.KAh > 5 || g.KAw > 5 || g.KBh > 5 || g.KBw > 5 || g.H > 64 || g.W > 64) return false;
  if (g.W1 < 1 || g.H2 < 1 || g.W2 < 1) return false;
  // conv A is ONE 16-column MFMA tile in this family: its forward (cp_conv_a) writes
  // c1 channels < 16 and its weight gradient covers taps (i, j, c0) < 16 — a wider conv A
  // lowers to separate conv units (tests/test_hip_step.py "wide_conv_a", "wide_c1")
  if (g.KAh * g.KAw * g.C0 > 16 || g.C1 > 16) return false;
  const int rows = g.pool ? g.PH : g.H2;
  // packed profile: two pooled rows per workgroup (350 instead of 700 for B = 50) — less
  // per-band staging CU-time: K = 8 jobs 995.4k vs 930.5k samples/s (profiles/r2_multitenant.md)
  const int pr_env = g_csa_packed ? 2 : 0;
  // unit rows per workgroup: PR = 1 (pooled) measured 120.0 vs 124.8 (PR 2) vs 130.5 us (PR 3)
  // per graph step — more workgroups (700 for B = 50) beat the per-band staging overhead
  g.PR = pr_env > 0 ? pr_env : (g.pool ? 1 : 2);
  g.nbands = (rows + g.PR - 1) / g.PR;
  return true;
}

// Does every band's backward prologue fit the one-batch register budget?
static bool cp_bwd_one_batch(const CPBwdArgs& a) {
  const CPGeom& g = a.g;
  const int C2x2 = 2 * g.C2, per = CP_THREADS / C2x2;
  if (a.bn_on && (per == 0 || a.bn.nslab > CPB_US * per || a.bwd_nslab > CPB_US * per)) return false;
  for (int band = 0; band < g.nbands; ++band) {
    const int pr0 = band * g.PR, pr1 = std::min(g.PH, pr0 + g.PR);
    const bool last = band == g.nbands - 1;
    const int r2a = g.pool ? 2 * pr0 : pr0, r2b = g.pool ? (last ? g.H2 : 2 * pr1) : pr1;
    const int T1H = (r2b - r2a) + g.KBh - 1, T1W = g.W2 + g.KBw - 1;
    const int TXH = T1H + g.KAh - 1, TXW = T1W + g.KAw - 1;
    const CPBwdLayout L = cp_bwd_layout(g, band, TXH, TXW, T1H, T1W);
    if (L.kpadA * 16 + L.kpadB * L.c16 > CPB_UP * CP_THREADS || TXH * TXW * g.C0 > CPB_UX * CP_THREADS ||
        g.C1 > 16)
      return false;
  }
  return true;
}

static size_t cp_lds(const CPGeom& g, bool bwd) {
  size_t mx = 0;
  for (int band = 0; band < g.nbands; ++band) {
    const int pr0 = band * g.PR, pr1 = std::min(g.PH, pr0 + g.PR);
    const bool last = band == g.nbands - 1;
    const int r2a = g.pool ? 2 * pr0 : pr0;
    const int r2b = bwd ? (g.pool ? (last ? g.H2 : 2 * pr1) : pr1) : (g.pool ? std::min(g.H2, 2 * pr1) : pr1);
    const int T1H = (r2b - r2a) + g.KBh - 1, T1W = g.W2 + g.KBw - 1;
    const int TXH = T1H + g.KAh - 1, TXW = T1W + g.KAw - 1;
    size_t f;
    if (bwd) {
      f = cp_bwd_layout(g, band, TXH, TXW, T1H, T1W).end;
    } else {
      const int KA = g.KAh * g.KAw * g.C0, KB = g.KBh * g.KBw * g.C1;
      const int kpadA = (KA + 3) & ~3, kpadB = (KB + 3) & ~3, c16 = (g.C2 + 15) & ~15;
      const int pst = (c16 & 31) ? c16 : c16 + 16;
      f = kpadA * 16 + kpadB * pst + 2 * kpadB + ((TXH * TXW * g.C0 + 3) & ~3) + ((T1H * T1W * g.C1 + 3) & ~3);
      if (kpadA > 32) return (size_t)-1;             // offset tables are static [32]
    }
    mx = std::max(mx, f);
  }
  return mx * sizeof(float);
}

}  // namespace csa

using namespace csa;

CSA_API int csa_cp_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_cp_dbg), &p, sizeof(p));
}

// this code object's copy of the dense-update stamps (dense_update.h, [block][8]) for the
// update workgroups carried by the pair backward (segment-local block numbers)
CSA_API int csa_cp_du_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_du_dbg), &p, sizeof(p));
}

CSA_NT_SETTER(csa_nt_out_cp)

CSA_API int csa_cpv_life_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_cpv_life), &p, sizeof(p));
}

CSA_API int csa_cp_life_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_cp_life), &p, sizeof(p));
}

CSA_API int csa_cp_debug_block(int b) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_cp_dbg_blk), &b, sizeof(b));
}

// geom = {B, H, W, C0, KAh, KAw, PTA, PLA, C1, H1, W1, KBh, KBw, PTB, PLB, C2, H2, W2, pool, PH, PW}
// Returns 1 when the pair is inside the fused family (the launchers below accept it).
CSA_API int csa_conv_pair_ok(const int* geom) {
  CPGeom g;
  if (!cp_geom(geom, g)) return 0;
  return cp_lds(g, true) <= CP_LDS_MAX ? 1 : 0;
}

// Workgroups of the pair launches (one per (image, band)): deterministic mode gives every
// workgroup its own statistic row and weight-gradient stripe.
CSA_API int csa_conv_pair_grid(const int* geom) {
  CPGeom g;
  return cp_geom(geom, g) ? g.B * g.nbands : 0;
}

// Is the VALU pair family (cpv kernels: fixed-order in-workgroup reductions) in use for geom?
CSA_API int csa_conv_pair_valu_ok(const int* geom) {
  CPGeom g;
  return cp_geom(geom, g) && cpv_ok(g) ? 1 : 0;
}

// The deferred dense update (CPOptCarry) the NEXT csa_conv_pair_fwd on this thread carries
// (host state, like the tail of the carrying backward); csa_opt_carry_flush applies the same
// update standalone.  Spans [lo, hi) of the flat buffer, float4-aligned.
static thread_local CPOptCarry g_cp_carry{};

static int cp_carry_make(CPOptCarry& c, int opt, float lr, const int64_t* step, float* w, const float* g, float* s0,
                         float* s1, unsigned* pending, int nseg, const long* seg_lo, const long* seg_hi,
                         int blocks) {
  c = CPOptCarry{};
  if (nseg < 1 || nseg > CP_MAXCS || !w || !g || !pending || blocks < 1) return -1;
  if (opt_nslots(opt) >= 1 && !s0) return -1;
  if (opt_nslots(opt) >= 2 && !s1) return -1;
  c.opt = opt; c.lr = lr; c.step = step; c.w = w; c.g = g; c.s0 = s0; c.s1 = s1; c.pending = pending;
  c.count = nseg;
  c.start4[0] = 0;
  for (int i = 0; i < nseg; ++i) {
    if (seg_lo[i] % 4 || seg_hi[i] % 4 || seg_hi[i] <= seg_lo[i]) return -1;
    c.lo4[i] = seg_lo[i] / 4;
    c.start4[i + 1] = c.start4[i] + (seg_hi[i] - seg_lo[i]) / 4;
  }
  c.blocks = blocks;
  return 0;
}

CSA_API int csa_conv_pair_fwd_carry(int opt, float lr, const int64_t* step, float* w, const float* g, float* s0,
                                    float* s1, unsigned* pending, int nseg, const long* seg_lo,
                                    const long* seg_hi, int blocks) {
  return cp_carry_make(g_cp_carry, opt, lr, step, w, g, s0, s1, pending, nseg, seg_lo, seg_hi, blocks);
}

// Apply a pending deferred update now (a no-op on the device when none is pending), then
// clear the flag: every host read of the parameters between steps goes through this.
CSA_API int csa_opt_carry_flush(int opt, float lr, const int64_t* step, float* w, const float* g, float* s0,
                                float* s1, unsigned* pending, int nseg, const long* seg_lo, const long* seg_hi,
                                int blocks, hipStream_t st) {
  CPOptCarry c;
  const int rc = cp_carry_make(c, opt, lr, step, w, g, s0, s1, pending, nseg, seg_lo, seg_hi, blocks);
  if (rc) return rc;
  hipLaunchKernelGGL(cp_opt_carry_kernel, dim3((unsigned)blocks), dim3(256), 0, st, c);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return (int)e;
  return (int)hipMemsetAsync(pending, 0, sizeof(unsigned), st);
}

CSA_API int csa_conv_pair_fwd(const int* geom, const uint8_t* img, const int64_t* idx, const int64_t* cursor,
                              const float* wA, const float* bA, int actA, float alphaA, const float* wB,
                              const float* bB, int actB, float alphaB, float* y, uint8_t* argmax, float* stat,
                              int nslab, float* const* zero_ptrs, const long* zero_n, int nzero, hipStream_t st) {
  CPZero z{};
  if (nzero < 0 || nzero > CP_MAXZ) return -2;
  for (int k = 0; k < nzero; ++k) {
    if (((uintptr_t)zero_ptrs[k] & 15) || (zero_n[k] & 3)) return -2;
    z.p[k] = reinterpret_cast<float4*>(zero_ptrs[k]);
    z.n4[k] = zero_n[k] / 4;
  }
  z.n = nzero;
  const CPOptCarry oc = g_cp_carry;
  g_cp_carry = CPOptCarry{};
  CPFwdArgs a{};
  if (!cp_geom(geom, a.g) || cp_lds(a.g, false) > CP_LDS_MAX) return -1;
  a.img = img; a.idx = idx; a.cursor = cursor; a.wA = wA; a.bA = bA; a.actA = actA; a.alphaA = alphaA;
  a.wB = wB; a.bB = bB; a.actB = actB; a.alphaB = alphaB; a.y = y; a.argmax = argmax; a.stat = stat;
  a.nslab = nslab < 1 ? 1 : nslab;
  if (cpv_ok(a.g)) {
    CPVFwdArgs v{a.g, img, idx, cursor, wA, bA, actA, alphaA, wB, bB, actB, alphaB, y, argmax, stat, a.nslab};
    const unsigned grid = (unsigned)(a.g.B * a.g.nbands + oc.blocks);
    if (oc.blocks) {
      if (a.g.KBh == 2) hipLaunchKernelGGL((cpv_fwd_kernel<2, 2, true>), dim3(grid), dim3(CPV_T), cpv_fwd_lds(a.g), st, v, z, oc);
      else hipLaunchKernelGGL((cpv_fwd_kernel<3, 3, true>), dim3(grid), dim3(CPV_T), cpv_fwd_lds(a.g), st, v, z, oc);
    } else {
      if (a.g.KBh == 2) hipLaunchKernelGGL((cpv_fwd_kernel<2, 2, false>), dim3(grid), dim3(CPV_T), cpv_fwd_lds(a.g), st, v, z, oc);
      else hipLaunchKernelGGL((cpv_fwd_kernel<3, 3, false>), dim3(grid), dim3(CPV_T), cpv_fwd_lds(a.g), st, v, z, oc);
    }
    return (int)hipGetLastError();
  }
  if (oc.blocks) return -7;                        // only the VALU forward carries the update
  static bool attr = hipFuncSetAttribute((const void*)conv_pair_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                         (int)CP_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  hipLaunchKernelGGL(conv_pair_fwd_kernel, dim3((unsigned)(a.g.B * a.g.nbands)), dim3(CP_THREADS),
                     cp_lds(a.g, false), st, a, z);
  return (int)hipGetLastError();
}

// The tail of the next carrying launch on this thread (csa_conv_pair_tail_set), like the
// deferred dense segments: host state consumed by that launch.
static thread_local CPTail g_cp_tail{};

template <bool ONE, int NSLOT>
static int cp_launch_bwd_upd_t(const CPBwdArgs& a, const DUSegs& u, const CPTail& t, size_t lds, hipStream_t st) {
  const void* fn = NSLOT == 2 ? (const void*)conv_pair_bwd_upd2_kernel<ONE>
                              : (const void*)conv_pair_bwd_upd_kernel<ONE, NSLOT < 2 ? NSLOT : 0>;
  static const bool attr = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)CP_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  const unsigned blocks = (unsigned)(a.g.B * a.g.nbands + u.start[u.nseg] + (t.on ? t.param_blocks + t.stage_blocks : 0));
  if constexpr (NSLOT == 2)
    hipLaunchKernelGGL((conv_pair_bwd_upd2_kernel<ONE>), dim3(blocks), dim3(CP_THREADS), lds, st, a, u, t);
  else
    hipLaunchKernelGGL((conv_pair_bwd_upd_kernel<ONE, NSLOT>), dim3(blocks), dim3(CP_THREADS), lds, st, a, u, t);
  return (int)hipGetLastError();
}

// The MFMA pair backward carrying the deferred dense update segments taken for it (and the
// tail, when one was set for this launch).
static int cp_launch_bwd_upd(CPBwdArgs a, const DUSegs& u, hipStream_t st) {
  const CPTail t = g_cp_tail;
  g_cp_tail = CPTail{};
  if (t.on) a.img_tk = cpt_word(t.tk, 1, 0);
  size_t lds = cp_lds(a.g, true);
  const size_t dl = du_upo_lds_floats(u.seg[0].M) * sizeof(float);     // the update-only body
  for (int s = 1; s < u.nseg; ++s)
    if (du_upo_lds_floats(u.seg[s].M) * sizeof(float) > dl) return -5;
  if (dl > lds) lds = dl;
  const int ns = opt_nslots(u.seg[0].opt);
  const bool one = cp_bwd_one_batch(a);
  if (ns == 0) return one ? cp_launch_bwd_upd_t<true, 0>(a, u, t, lds, st) : cp_launch_bwd_upd_t<false, 0>(a, u, t, lds, st);
  if (ns == 1) return one ? cp_launch_bwd_upd_t<true, 1>(a, u, t, lds, st) : cp_launch_bwd_upd_t<false, 1>(a, u, t, lds, st);
  return one ? cp_launch_bwd_upd_t<true, 2>(a, u, t, lds, st) : cp_launch_bwd_upd_t<false, 2>(a, u, t, lds, st);
}

// Tail plan: the parameter table of the tail's parameter workgroups, written to the device
// buffer `table` (at least csa_conv_pair_tail_table_bytes(n, nseg)).  Parameter k < nseg:
// w[k][i] updated with sum_s src[k][s * ld[k] + i] (S[k] <= 16 rows; zero[k]: the rows are
// re-zeroed, their only reader is this fold).  Returns the parameter workgroup count.
CSA_API long csa_conv_pair_tail_table_bytes(const int* n, int nseg) {
  long blocks = 0;
  for (int k = 0; k < nseg; ++k) blocks += (n[k] + CP_THREADS - 1) / CP_THREADS;
  return blocks * (long)sizeof(CPTailSeg);
}

CSA_API int csa_conv_pair_tail_plan(void* table, int opt, int nseg, float* const* w, float* const* s0,
                                    float* const* s1, float* const* src, const int* S, const int* ld, const int* n,
                                    const int* zero, int store) {
  if (!table || nseg < 1 || nseg > CPT_MAXSEG) return -1;
  const int ns = store ? 0 : opt_nslots(opt);
  std::vector<CPTailSeg> segs;
  for (int k = 0; k < nseg; ++k) {
    if (!w[k] || !src[k] || S[k] < 1 || S[k] > 16 || n[k] < 1 || ld[k] < n[k]) return -2;
    if ((ns >= 1 && !s0[k]) || (ns >= 2 && !s1[k])) return -2;
    for (int base = 0; base < n[k]; base += CP_THREADS)
      segs.push_back(CPTailSeg{w[k], s0[k], s1[k], src[k], S[k], ld[k], n[k], zero[k], base, store ? 1 : 0, 0, 0});
  }
  if (hipMemcpy(table, segs.data(), segs.size() * sizeof(CPTailSeg), hipMemcpyHostToDevice) != hipSuccess) return -3;
  return (int)segs.size();
}

// Tail of the NEXT pair backward launched by this thread (it must carry deferred dense
// segments: the MFMA carrier): `param_blocks` workgroups over the planned table, nz <= 4
// float regions zeroed, the next batch staged when out_img != null (imsz % 4 == 0).
// tk: 3 zeroed uints, err: 1 int (device).
// (debug) the forced-timeout word of the tail set NEXT by this thread (null: none)
static thread_local int* g_cp_tail_force = nullptr;
CSA_API void csa_conv_pair_tail_force(int* force) { g_cp_tail_force = force; }

CSA_API int csa_conv_pair_tail_set(unsigned* tk, int* err, int opt, float lr, const int64_t* step,
                                   const void* table, int param_blocks, int nz, float* const* zp, const long* zn,
                                   const uint8_t* img, const int64_t* labels, const int64_t* rows,
                                   const int64_t* cursor, int B, long imsz, uint8_t* out_img, int64_t* out_lbl) {
  if (!tk || !err || !step || !table || param_blocks < 1 || nz < 0 || nz > CP_MAXZ) return -1;
  CPTail t{};
  t.on = 1; t.tk = tk; t.err = err; t.force = g_cp_tail_force; t.opt = opt; t.lr = lr; t.step = step;
  t.segs = static_cast<const CPTailSeg*>(table); t.param_blocks = param_blocks;
  t.nz = nz;
  for (int k = 0; k < nz; ++k) { t.zp[k] = zp[k]; t.zn[k] = (int)zn[k]; }
  if (out_img) {
    if (imsz % 4 || B < 1 || !img || !labels || !rows || !cursor || !out_lbl) return -3;
    t.img = reinterpret_cast<const uint32_t*>(img); t.labels = labels; t.rows = rows; t.cursor = cursor;
    t.B = B; t.words = (int)(imsz / 4);
    t.out_img = reinterpret_cast<uint32_t*>(out_img); t.out_lbl = out_lbl;
    const long total = (long)B * t.words > B ? (long)B * t.words : B;
    t.stage_blocks = (int)((total + CP_THREADS - 1) / CP_THREADS);
  }
  g_cp_tail = t;
  return 0;
}

CSA_API int csa_conv_pair_tail_pending() { return g_cp_tail.on; }
CSA_API int csa_conv_pair_tail_ticket_words() { return CPT_TK_WORDS; }

__global__ __launch_bounds__(CP_THREADS) void cp_bwd_tables_kernel(CPGeom g, int* out, int stride) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int band = blockIdx.x, pr0 = band * g.PR;
  const bool last = band == g.nbands - 1;
  const int o2a = g.pool ? 2 * pr0 : pr0;
  const int o2b = g.pool ? (last ? g.H2 : 2 * min(g.PH, pr0 + g.PR)) : min(g.PH, pr0 + g.PR);
  const CPBand t = cp_band(g, o2a, o2b);
  const CPBwdLayout L = cp_bwd_layout(g, band, t.TXH, t.TXW, t.T1H, t.T1W);
  int* s = reinterpret_cast<int*>(smem);
  cp_bwd_tables(g, t, L, s);
  __syncthreads();
  for (int i = threadIdx.x; i < cp_bwd_tab_ints(L); i += CP_THREADS) out[(long)band * stride + i] = s[i];
}

static int cp_bwd_tab_stride(const CPGeom& g) {
  int m = 0;
  for (int band = 0; band < g.nbands; ++band) {
    const int pr0 = band * g.PR;
    const bool last = band == g.nbands - 1;
    const int o2a = g.pool ? 2 * pr0 : pr0;
    const int o2b = g.pool ? (last ? g.H2 : 2 * std::min(g.PH, pr0 + g.PR)) : std::min(g.PH, pr0 + g.PR);
    const CPBand t = cp_band(g, o2a, o2b);
    m = std::max(m, cp_bwd_tab_ints(cp_bwd_layout(g, band, t.TXH, t.TXW, t.T1H, t.T1W)));
  }
  return (m + 3) & ~3;
}

// Ints of the backward's per-band index-table buffer (0: the pair keeps computing them per
// workgroup — a band's region exceeds the prologue's register batch).
CSA_API long csa_conv_pair_bwd_tables_size(const int* geom) {
  CPGeom g;
  if (!cp_geom(geom, g)) return -1;
  const int stride = cp_bwd_tab_stride(g);
  if (stride > CPB_UT * CP_THREADS) return 0;
  return (long)stride * g.nbands;
}

// Fill the table buffer (once per geometry, at plan time).  The ~440 ints of the sample
// pair's band were recomputed by all 700 workgroups every step: ~4.6k cycles of integer
// VALU work at three waves per SIMD in front of the first route store
// (profiles/r4_roofline.md).
CSA_API int csa_conv_pair_bwd_tables(const int* geom, int* out, hipStream_t st) {
  CPGeom g;
  if (!cp_geom(geom, g) || !out) return -1;
  const int stride = cp_bwd_tab_stride(g);
  hipLaunchKernelGGL(cp_bwd_tables_kernel, dim3((unsigned)g.nbands), dim3(CP_THREADS), (size_t)stride * sizeof(int),
                     st, g, out, stride);
  return (int)hipGetLastError();
}

// The forward BatchNorm tables of the NEXT csa_conv_pair_bwd call (bn_act_apply's [4][C2]
// output for this step), so its workgroups load them instead of folding the statistic slab.
static thread_local const float* g_cp_bn_tab = nullptr;
CSA_API void csa_conv_pair_bn_tab(const float* tab) { g_cp_bn_tab = tab; }

CSA_API int csa_conv_pair_bwd(const int* geom, const uint8_t* img, const int64_t* idx, const int64_t* cursor,
                              const float* wA, const float* bA, int actA, float alphaA, const float* wB, int hasBiasB,
                              int actB, float alphaB, const float* dz, const float* y, const uint8_t* argmax,
                              const float* bn_slab, int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                              const float* bn_offset, const float* bwd_slab, int bwd_nslab, float* dscale,
                              float* doffset, float* run_mean, float* run_var, float momentum, float* dwA, float* dbA,
                              float* dwB, float* dbB, int stripes, const int* tabs, hipStream_t st) {
  CPBwdArgs a{};
  const float* bn_tab = g_cp_bn_tab;                 // consumed by this call, whatever it returns
  g_cp_bn_tab = nullptr;
  if (!cp_geom(geom, a.g) || cp_lds(a.g, true) > CP_LDS_MAX) return -1;
  a.tabs = tabs;
  a.tab_stride = tabs ? cp_bwd_tab_stride(a.g) : 0;
  if (tabs && a.tab_stride > CPB_UT * CP_THREADS) return -6;
  a.img = img; a.idx = idx; a.cursor = cursor; a.wA = wA; a.bA = bA; a.actA = actA; a.alphaA = alphaA;
  a.wB = wB; a.actB = actB; a.alphaB = alphaB; a.hasBiasB = hasBiasB; a.dz = dz; a.y = y; a.argmax = argmax;
  a.bn = BNRef{bn_slab, bn_nslab, a.g.C2, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr; a.bwd_slab = bwd_slab; a.bwd_nslab = bwd_nslab;
  a.bn_tab = a.bn_on ? bn_tab : nullptr;
  a.dscale = dscale; a.doffset = doffset; a.run_mean = run_mean; a.run_var = run_var; a.momentum = momentum;
  a.dwA = dwA; a.dbA = dbA; a.dwB = dwB; a.dbB = dbB; a.stripes = stripes < 1 ? 1 : stripes;
  static bool attr = hipFuncSetAttribute((const void*)conv_pair_bwd_kernel<true>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)CP_LDS_MAX) == hipSuccess &&
                     hipFuncSetAttribute((const void*)conv_pair_bwd_kernel<false>,
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)CP_LDS_MAX) == hipSuccess;
  if (!attr) return -3;
  const dim3 grid((unsigned)(a.g.B * a.g.nbands));
  // VALU backward only in deterministic mode (its in-workgroup reductions are fixed-order);
  // otherwise the MFMA backward: 20.9 vs 24.5 us per launch for the sample pair
  // (profiles/r3_notes.md), while the VALU forward stays the faster forward
  if (cpv_bwd_ok(a) && (g_csa_det || !cp_lds_ok_bwd(a.g))) {
    static bool vattr = hipFuncSetAttribute((const void*)cpv_bwd_kernel<2, 2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)CP_LDS_MAX) == hipSuccess &&
                        hipFuncSetAttribute((const void*)cpv_bwd_kernel<3, 3>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                            (int)CP_LDS_MAX) == hipSuccess;
    if (!vattr) return -3;
    if (a.g.KBh == 2) hipLaunchKernelGGL((cpv_bwd_kernel<2, 2>), grid, dim3(CPV_T), cpv_bwd_lds_max(a.g), st, a);
    else hipLaunchKernelGGL((cpv_bwd_kernel<3, 3>), grid, dim3(CPV_T), cpv_bwd_lds_max(a.g), st, a);
    if (g_cp_tail.on) return -7;                                // a tail needs the MFMA carrier
    DUSegs u;                                                   // deferred updates on their own
    if (du_take(u) > 0) return du_flush_segs(u, st);
    return (int)hipGetLastError();
  }
  DUSegs u;
  if (du_take(u) > 0) return cp_launch_bwd_upd(a, u, st);
  if (g_cp_tail.on) return -7;
  if (cp_bwd_one_batch(a))
    hipLaunchKernelGGL(conv_pair_bwd_kernel<true>, grid, dim3(CP_THREADS), cp_lds(a.g, true), st, a);
  else
    hipLaunchKernelGGL(conv_pair_bwd_kernel<false>, grid, dim3(CP_THREADS), cp_lds(a.g, true), st, a);
  return (int)hipGetLastError();
}
