// Direct NHWC convolution kernels for the DSL's small convs (gfx950 / CDNA4).
//
// Reference ops: tf.nn.conv2d (construct_distribute.py:91-118) with TF 'SAME'/'VALID'
// padding, tf.nn.max_pool (:121-130), activation (:133-152) and BatchNorm (:155-165).
// The reference's convs are tiny (2x2 kernels, 1->10->20 channels): VALU work, not MFMA
// work.  Layout of the forward / input-gradient kernels:
//   * one workgroup per (image, row band, channel block): the band's input rows are
//     staged ONCE into LDS with coalesced loads — with the input transform (uint8
//     gather + /255, or BN-apply + activation) applied during staging, so it costs one
//     evaluation per element instead of one per use;
//   * one lane per output pixel with a register block of output channels; the weight
//     addresses are wave-uniform (channel block from blockIdx.y), so they become scalar
//     loads and the inner loop is v_fma_f32 with an SGPR operand;
//   * fused epilogues: bias, activation, max-pool (argmax kept as uint8 for backward)
//     and the BatchNorm partial statistics of the output (per-workgroup slab).
// Weight gradients: a direct LDS-staged reduction kernel (conv_wgrad_kernel).
#include "common.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace csa {

constexpr int CONV_THREADS = 256;

__constant__ long long* g_conv_dbg = nullptr;   // diagnostics: s_memtime stamps of WG 0
#define CONV_STAMP(i)                                                                       \
  do {                                                                                      \
    if (g_conv_dbg && threadIdx.x == 0 && blockIdx.x == 0)                                  \
      g_conv_dbg[i] = (long long)__builtin_amdgcn_s_memtime();                               \
  } while (0)

struct ConvGeom {
  int B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH, OW, Cout;
};

struct PoolGeom {
  int on;                      // pool fused after conv (+act)
  int KH, KW, SH, SW, PT, PL, OH, OW;
};

struct ConvFwdArgs {
  ConvGeom g;
  PoolGeom pool;
  int nbands, band_rows;       // output rows (pooled rows if pool) per band
  int band_rows_in;            // max staged input rows per band (LDS carve)
  int nslab;                   // BN slab rows (workgroups fold into blockIdx % nslab)
  int det;                     // deterministic mode: row blockIdx (nslab = #workgroups)
  const float* x;              // fp32 NHWC input (or null)
  const uint8_t* img;          // uint8 dataset [N][H*W*Cin] (first layer) ...
  const int64_t* idx;          // ... gathered through idx[b] (rows of the index stream)
  const int64_t* cursor;       // if set: this step's row = idx + cursor[0] * B
  BNRef in_bn; int in_bn_on; int in_act; float in_alpha;   // input transform
  const float* w; const float* bias; int out_act; float out_alpha;
  float* y;                    // [B, OH|POH, OW|POW, Cout] post-act (post-pool) output
  uint8_t* argmax;             // [B, POH, POW, Cout] window index (pool only)
  float* stat_slab;            // [B*nbands][2][Cout] partial {sum y, sum y^2} or null
};

template <int CB, bool U8>
__global__ __launch_bounds__(CONV_THREADS) void conv_fwd_kernel(ConvFwdArgs a) {
  // dynamic LDS: [input rows of the band][W][Cin] then weights [(i,j,ci)][Cout]
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_bn[4 * 128 + 2 * 128];
  __shared__ float s_stat[2 * 128];
  const ConvGeom& g = a.g;
  const int b = blockIdx.x / a.nbands, band = blockIdx.x % a.nbands;
  const int G = (g.Cout + CB - 1) / CB;            // channel groups (one per lane of a pixel)
  const int OHo = a.pool.on ? a.pool.OH : g.OH;
  const int OWo = a.pool.on ? a.pool.OW : g.OW;
  const int r0 = band * a.band_rows, r1 = min(OHo, r0 + a.band_rows);
  int c0 = r0, c1 = r1;                             // conv-output rows of the band
  if (a.pool.on) {
    c0 = max(0, r0 * a.pool.SH - a.pool.PT);
    c1 = min(g.OH, (r1 - 1) * a.pool.SH - a.pool.PT + a.pool.KH);
  }
  const int y0 = max(0, c0 * g.SH - g.PT);
  const int y1 = min(g.H, (c1 - 1) * g.SH - g.PT + g.KH);
  const int rowlen = g.W * g.Cin;
  const int nin = max(0, y1 - y0) * rowlen;
  const int nw = g.KH * g.KW * g.Cin * g.Cout;
  float* s_in = smem;
  float* s_w = smem + ((a.band_rows_in * rowlen + 3) & ~3);

  if (a.in_bn_on) bn_reduce_to_lds(a.in_bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_bn + 512);
  for (int i = threadIdx.x; i < 2 * g.Cout; i += blockDim.x) s_stat[i] = 0.f;
  stage_to_lds<4>(s_w, a.w, nw, [](float v, int) { return v; });
  if (U8) {
    const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * g.B : a.idx;
    const uint8_t* src = a.img + idx[b] * (long)(g.H * rowlen) + (long)y0 * rowlen;
    stage_to_lds<8>(s_in, src, nin, [](uint8_t v, int) { return (float)v * (1.0f / 255.0f); });
  } else {
    __syncthreads();   // BN tables ready
    const float* src = a.x + ((long)b * g.H + y0) * rowlen;
    const float* ta = s_bn + 256;
    const float* tb = s_bn + 384;
    const FastDiv dc(g.Cin);
    const int bn_on = a.in_bn_on, act = a.in_act;
    const float alpha = a.in_alpha;
    stage_to_lds<8>(s_in, src, nin, [&](float v, int i) {
      if (bn_on) { int q, ci; dc.divmod(i, q, ci); v = v * ta[ci] + tb[ci]; }
      return act_fwd(v, act, alpha);
    });
  }
  __syncthreads();

  const int npix = (r1 - r0) * OWo;
  const int npos = a.pool.on ? a.pool.KH * a.pool.KW : 1;
  const int cg = threadIdx.x % G;
  const int co0 = cg * CB;
  const int nco = min(CB, g.Cout - co0);
  float bsum[CB], bsq[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) { bsum[c] = 0.f; bsq[c] = 0.f; }
  const int ppp = blockDim.x / G;                   // pixels per pass
  for (int q = threadIdx.x / G; q < npix && threadIdx.x < ppp * G; q += ppp) {
    const int oy = r0 + q / OWo, ox = q % OWo;
    float out[CB];
    int amax[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) { out[c] = -INFINITY; amax[c] = 0; }
    for (int pos = 0; pos < npos; ++pos) {
      int cy = oy, cx = ox;
      if (a.pool.on) {
        cy = oy * a.pool.SH - a.pool.PT + pos / a.pool.KW;
        cx = ox * a.pool.SW - a.pool.PL + pos % a.pool.KW;
        if (cy < 0 || cy >= g.OH || cx < 0 || cx >= g.OW) continue;   // -inf padding
      }
      float acc[CB];
#pragma unroll
      for (int c = 0; c < CB; ++c) acc[c] = (a.bias && c < nco) ? a.bias[co0 + c] : 0.f;
      for (int i = 0; i < g.KH; ++i) {
        const int yy = cy * g.SH - g.PT + i;
        if (yy < 0 || yy >= g.H) continue;
        for (int j = 0; j < g.KW; ++j) {
          const int xx = cx * g.SW - g.PL + j;
          if (xx < 0 || xx >= g.W) continue;
          const float* in = s_in + (yy - y0) * rowlen + xx * g.Cin;
          const float* wr = s_w + (i * g.KW + j) * g.Cin * g.Cout + co0;
          // 4 input channels per step: all 4 + 4*CB LDS reads issue before the FMAs
          // (a runtime-bound loop otherwise waits on every ds_read).
          int ci = 0;
          for (; ci + 4 <= g.Cin; ci += 4) {
            float v[4], w[4][CB];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              v[u] = in[ci + u];
#pragma unroll
              for (int c = 0; c < CB; ++c) w[u][c] = wr[(ci + u) * g.Cout + c];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int c = 0; c < CB; ++c) acc[c] = fmaf(v[u], w[u][c], acc[c]);
          }
          for (; ci < g.Cin; ++ci) {
            const float v = in[ci];
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[c] = fmaf(v, wr[ci * g.Cout + c], acc[c]);
          }
        }
      }
#pragma unroll
      for (int c = 0; c < CB; ++c) {
        const float v = act_fwd(acc[c], a.out_act, a.out_alpha);
        if (v > out[c]) { out[c] = v; amax[c] = pos; }
      }
    }
    const long p = ((long)b * OHo + oy) * OWo + ox;
    float* yrow = a.y + p * g.Cout + co0;
#pragma unroll
    for (int c = 0; c < CB; ++c)
      if (c < nco) { yrow[c] = out[c]; bsum[c] += out[c]; bsq[c] += out[c] * out[c]; }
    if (a.pool.on && a.argmax) {
      uint8_t* arow = a.argmax + p * g.Cout + co0;
#pragma unroll
      for (int c = 0; c < CB; ++c)
        if (c < nco) arow[c] = (uint8_t)amax[c];
    }
  }
  if (a.stat_slab && a.det) {
    // deterministic mode: fixed-order fold (s_bn is dead after staging), then this
    // workgroup's EXCLUSIVE slab row (nslab = #workgroups) with plain stores
    det_fold_groups<CB>(bsum, bsq, G, g.Cout, s_bn, s_stat);
    float* row = a.stat_slab + (size_t)blockIdx.x * 2 * g.Cout;
    for (int i = threadIdx.x; i < 2 * g.Cout; i += blockDim.x) row[i] = s_stat[i];
  } else if (a.stat_slab) {
#pragma unroll
    for (int c = 0; c < CB; ++c)
      if (c < nco) { atomicAdd(&s_stat[co0 + c], bsum[c]); atomicAdd(&s_stat[g.Cout + co0 + c], bsq[c]); }
    __syncthreads();
    // fold into one of a.nslab rows (atomics, zeroed each step by the optimizer launch)
    float* row = a.stat_slab + (size_t)(blockIdx.x % a.nslab) * 2 * g.Cout;
    for (int i = threadIdx.x; i < 2 * g.Cout; i += blockDim.x) atomicAdd(&row[i], s_stat[i]);
  }
}

// -----------------------------------------------------------------------------------
// Backward of a conv unit's OUTPUT side: BatchNorm backward (if the unit output fed a
// norm), activation backward and max-pool routing.  One lane per unit-output element.
//   dz   : grad wrt the BN output (or wrt the unit output if no BN)       [B,h,w,C]
//   y    : unit output (post act, post pool) = BN input                  [B,h,w,C]
//   dc   : grad wrt the conv pre-activation output                        [B,OH,OW,C]
// BN backward: dx = a*(dz - S1/N - xhat*S2/N), a = scale*rstd, S1 = sum dz, S2 = sum dz*xhat.
// Block 0 also writes dscale = S2, doffset = S1 into the gradient buffer.
// -----------------------------------------------------------------------------------
struct RouteArgs {
  const float* dz; const float* y; const uint8_t* argmax; float* dc;
  int B, h, w, C;             // unit-output geometry
  int OH, OW;                 // conv output geometry (pre-pool)
  int pool_on, PKW, PSH, PSW, PPT, PPL, overlap;
  int out_act; float out_alpha;
  BNRef bn; int bn_on; const float* bwd_slab; int bwd_nslab;
  float* dscale; float* doffset;
  float* run_mean; float* run_var; float momentum;   // BN running statistics (block 0)
};

__global__ __launch_bounds__(256) void route_bwd_kernel(RouteArgs a) {
  __shared__ float s_bn[4 * 128];
  __shared__ float s_s[2 * 128];
  // this lane's element loads go out first: their round trip overlaps the BN-slab
  // reductions below (clamped index, so the loads are unconditional)
  const long n = (long)a.B * a.h * a.w * a.C;
  const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long ec = e < n ? e : 0;
  float g = a.dz[ec];
  const float yv = a.y[ec];
  const int am = a.pool_on ? (int)a.argmax[ec] : 0;
  if (a.bn_on) {
    bn_reduce_to_lds(a.bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_s);
    __syncthreads();
    slab_sum_to_lds(a.bwd_slab, a.bwd_nslab, 2 * a.C, s_s);
    if (blockIdx.x == 0)
      for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
        a.doffset[c] = s_s[c];
        a.dscale[c] = s_s[a.C + c];
        if (a.run_mean) {   // running stats from this step's batch statistics
          const float mean = s_bn[c];
          const float var = 1.0f / (s_bn[128 + c] * s_bn[128 + c]) - a.bn.eps;
          a.run_mean[c] = (1.f - a.momentum) * a.run_mean[c] + a.momentum * mean;
          a.run_var[c] = (1.f - a.momentum) * a.run_var[c] + a.momentum * var;
        }
      }
  }
  __syncthreads();
  if (e >= n) return;
  const int c = (int)(e % a.C);
  if (a.bn_on) {
    const float inv_n = 1.0f / a.bn.count;
    const float xhat = (yv - s_bn[c]) * s_bn[128 + c];
    g = s_bn[256 + c] * (g - s_s[c] * inv_n - xhat * s_s[a.C + c] * inv_n);
  }
  // activation backward (y is the post-activation value; pooling keeps the max's value)
  g = act_bwd(g, yv, yv, a.out_act, a.out_alpha);
  if (!a.pool_on) { a.dc[e] = g; return; }
  const long pix = e / a.C;
  const int px = (int)(pix % a.w), py = (int)((pix / a.w) % a.h), b = (int)(pix / ((long)a.w * a.h));
  // non-overlapping windows (kernel == stride): this lane owns its whole window and
  // writes it with plain stores (zeros included); otherwise atomics into a zeroed dc.
  const int ky = am / a.PKW, kx = am % a.PKW;
  const int cy = py * a.PSH - a.PPT + ky, cx = px * a.PSW - a.PPL + kx;
  if (a.overlap) {
    atomicAdd(&a.dc[(((long)b * a.OH + cy) * a.OW + cx) * a.C + c], g);
  } else {
    for (int wy = 0; wy < a.PSH; ++wy)
      for (int wx = 0; wx < a.PSW; ++wx) {
        const int yy = py * a.PSH - a.PPT + wy, xx = px * a.PSW - a.PPL + wx;
        if (yy < 0 || yy >= a.OH || xx < 0 || xx >= a.OW) continue;
        a.dc[(((long)b * a.OH + yy) * a.OW + xx) * a.C + c] = (yy == cy && xx == cx) ? g : 0.f;
      }
  }
}

// Route backward fused into its consumer (the conv unit's input-gradient / weight-gradient
// pair): the pair's workgroups build the BN tables of the route once each (two tiny slab
// reductions) and then compute the route value of exactly the conv-output rows they
// stage, instead of reading a dc tensor a separate route launch wrote.  Non-overlapping
// pools (kernel == stride, no padding) or no pool.
struct RouteTables { float* bn; float* ss; };   // bn: [mean|rstd|a|b] x 128, ss: [S1|S2] x 128

__device__ __forceinline__ void route_prologue(const RouteArgs& a, const RouteTables& t, int bid) {
  if (a.bn_on) {
    bn_reduce_to_lds(a.bn, t.bn, t.bn + 128, t.bn + 256, t.bn + 384, t.ss);
    __syncthreads();
    slab_sum_to_lds(a.bwd_slab, a.bwd_nslab, 2 * a.C, t.ss);
    if (bid == 0)
      for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
        a.doffset[c] = t.ss[c];
        a.dscale[c] = t.ss[a.C + c];
        if (a.run_mean) {
          const float mean = t.bn[c];
          const float var = 1.0f / (t.bn[128 + c] * t.bn[128 + c]) - a.bn.eps;
          a.run_mean[c] = (1.f - a.momentum) * a.run_mean[c] + a.momentum * mean;
          a.run_var[c] = (1.f - a.momentum) * a.run_var[c] + a.momentum * var;
        }
      }
  }
  __syncthreads();
}

// dst(oy - oa, ox, c) = dc[b, oy, ox, c] for conv-output rows [oa, ob) of image b.  The
// caller has zero-filled the destination (positions a pool window did not select).
template <class DST>
__device__ __forceinline__ void route_stage(const RouteArgs& a, const RouteTables& t, int b, int oa, int ob,
                                            DST dst) {
  const int PSH = a.pool_on ? a.PSH : 1, PSW = a.pool_on ? a.PSW : 1;
  const int py0 = oa / PSH, py1 = min(a.h, (ob - 1) / PSH + 1);
  const int wc = a.w * a.C;
  const int n = max(0, py1 - py0) * wc;
  const FastDiv dwc(wc), dC(a.C);
  const float inv_n = a.bn_on ? 1.0f / a.bn.count : 0.f;
  const long base = ((long)b * a.h + py0) * wc;
  if (n <= 0) return;
  constexpr int U = 4;
  for (int i0 = 0; i0 < n; i0 += CONV_THREADS * U) {
    float gz[U], yv[U];
    int am[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = min(i0 + u * CONV_THREADS + (int)threadIdx.x, n - 1);
      gz[u] = a.dz[base + i];
      yv[u] = a.y[base + i];
      am[u] = a.pool_on ? (int)a.argmax[base + i] : 0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * CONV_THREADS + (int)threadIdx.x;
      if (i >= n) break;
      int pr, rem, px, c;
      dwc.divmod(i, pr, rem);
      dC.divmod(rem, px, c);
      float g = gz[u];
      if (a.bn_on) {
        const float xhat = (yv[u] - t.bn[c]) * t.bn[128 + c];
        g = t.bn[256 + c] * (g - t.ss[c] * inv_n - xhat * t.ss[a.C + c] * inv_n);
      }
      g = act_bwd(g, yv[u], yv[u], a.out_act, a.out_alpha);
      const int oy = (py0 + pr) * PSH + (a.pool_on ? am[u] / a.PKW : 0);
      const int ox = px * PSW + (a.pool_on ? am[u] % a.PKW : 0);
      if (oy >= oa && oy < ob && ox < a.OW) dst(oy - oa, ox, c, g);
    }
  }
}

// -----------------------------------------------------------------------------------
// Conv input gradient:  dx[b,y,x,ci] = sum_{i,j,co} dc[b,oy,ox,co] * W[i,j,ci,co]
// (one workgroup per image x row band x input-channel block, dc rows staged in LDS),
// then through the input transform of the forward (act, BN) like the dense dgrad
// epilogue: stores dz and emits the BN-backward slab {sum dz, sum dz*xhat}.
// -----------------------------------------------------------------------------------
struct ConvDgradArgs {
  ConvGeom g;
  int nbands, band_rows;       // input rows per band
  int band_rows_in;            // max staged dc rows per band
  int nslab;
  int det;                     // deterministic mode: exclusive bwd_slab row per workgroup
  const float* dc; const float* w; float* dx;
  const float* x_fwd; int in_act; float in_alpha; BNRef in_bn; int in_bn_on;
  float* bwd_slab;   // [B*nbands][2][Cin]
};

template <int CB>
__device__ __forceinline__ void conv_dgrad_body(const ConvDgradArgs& a, int bid, float* smem,
                                                float* s_bn, float* s_stat,
                                                const RouteArgs* rt = nullptr, RouteTables rtt = {}) {
  // smem (dynamic): dc rows of the band [rows][OW][Cout] then weights [(i,j,ci)][Cout]
  const ConvGeom& g = a.g;
  const int b = bid / a.nbands, band = bid % a.nbands;
  const int G = (g.Cin + CB - 1) / CB;
  const int y0 = band * a.band_rows, y1 = min(g.H, y0 + a.band_rows);
  // dc rows that touch input rows [y0, y1): oy*SH - PT + i in [y0, y1)
  const int o0 = max(0, (y0 + g.PT - g.KH + 1 + g.SH - 1) / g.SH);
  const int o1 = min(g.OH, (y1 - 1 + g.PT) / g.SH + 1);
  const int rowlen = g.OW * g.Cout;
  const int nw = g.KH * g.KW * g.Cin * g.Cout;
  float* s_dc = smem;
  float* s_w = smem + ((a.band_rows_in * rowlen + 3) & ~3);
  if (a.in_bn_on) bn_reduce_to_lds(a.in_bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_bn + 512);
  for (int i = threadIdx.x; i < 2 * g.Cin; i += blockDim.x) s_stat[i] = 0.f;
  stage_to_lds<4>(s_w, a.w, nw, [](float v, int) { return v; });
  const int nd = max(0, o1 - o0) * rowlen;
  if (rt) {             // dc rows computed here from the unit output (route fused)
    for (int e = threadIdx.x; e < nd; e += CONV_THREADS) s_dc[e] = 0.f;
    __syncthreads();
    route_stage(*rt, rtt, b, o0, o1, [&](int r, int ox, int c, float v) { s_dc[r * rowlen + ox * g.Cout + c] = v; });
  } else {
    const float* src = a.dc + ((long)b * g.OH + o0) * rowlen;
    stage_to_lds<8>(s_dc, src, nd, [](float v, int) { return v; });
  }
  __syncthreads();

  const int npix = (y1 - y0) * g.W;
  const int cg = threadIdx.x % G;
  const int ci0 = cg * CB;
  const int nci = min(CB, g.Cin - ci0);
  float dsum[CB], dxs[CB];
#pragma unroll
  for (int c = 0; c < CB; ++c) { dsum[c] = 0.f; dxs[c] = 0.f; }
  const int ppp = blockDim.x / G;
  for (int q = threadIdx.x / G; q < npix && threadIdx.x < ppp * G; q += ppp) {
    const int y = y0 + q / g.W, x = q % g.W;
    float acc[CB];
#pragma unroll
    for (int c = 0; c < CB; ++c) acc[c] = 0.f;
    for (int i = 0; i < g.KH; ++i) {
      const int ty = y + g.PT - i;
      if (ty < 0 || ty % g.SH) continue;
      const int oy = ty / g.SH;
      if (oy >= g.OH) continue;
      for (int j = 0; j < g.KW; ++j) {
        const int tx = x + g.PL - j;
        if (tx < 0 || tx % g.SW) continue;
        const int ox = tx / g.SW;
        if (ox >= g.OW) continue;
        const float* drow = s_dc + (oy - o0) * rowlen + ox * g.Cout;
        const float* wbase = s_w + ((i * g.KW + j) * g.Cin + ci0) * g.Cout;
        int co = 0;
        for (; co + 4 <= g.Cout; co += 4) {
          float gv[4], w[CB][4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            gv[u] = drow[co + u];
#pragma unroll
            for (int c = 0; c < CB; ++c) w[c][u] = wbase[c * g.Cout + co + u];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < CB; ++c) acc[c] = fmaf(gv[u], w[c][u], acc[c]);
        }
        for (; co < g.Cout; ++co) {
          const float gv = drow[co];
#pragma unroll
          for (int c = 0; c < CB; ++c) acc[c] = fmaf(gv, wbase[c * g.Cout + co], acc[c]);
        }
      }
    }
    const long p = ((long)b * g.H + y) * g.W + x;
    const float* xrow = a.x_fwd ? a.x_fwd + p * g.Cin + ci0 : nullptr;
    float* dxrow = a.dx + p * g.Cin + ci0;
#pragma unroll
    for (int c = 0; c < CB; ++c) {
      if (c >= nci) break;
      float gv = acc[c];
      if (xrow && (a.in_act || a.in_bn_on)) {
        const float xv = xrow[c];
        const int ch = ci0 + c;
        const float z = a.in_bn_on ? xv * s_bn[256 + ch] + s_bn[384 + ch] : xv;
        const float yv = act_fwd(z, a.in_act, a.in_alpha);
        gv = act_bwd(gv, z, yv, a.in_act, a.in_alpha);
        if (a.in_bn_on) {
          const float xh = (xv - s_bn[ch]) * s_bn[128 + ch];
          dsum[c] += gv;
          dxs[c] += gv * xh;
        }
      }
      dxrow[c] = gv;
    }
  }
  if (a.in_bn_on && a.bwd_slab && a.det) {
    // deterministic mode: fixed-order fold through s_bn, exclusive row bid — once every
    // thread is past the loop, which reads the BN tables in s_bn
    __syncthreads();
    det_fold_groups<CB>(dsum, dxs, G, g.Cin, s_bn, s_stat);
    float* row = a.bwd_slab + (size_t)bid * 2 * g.Cin;
    for (int i = threadIdx.x; i < 2 * g.Cin; i += blockDim.x) row[i] = s_stat[i];
  } else if (a.in_bn_on && a.bwd_slab) {
#pragma unroll
    for (int c = 0; c < CB; ++c)
      if (c < nci) { atomicAdd(&s_stat[ci0 + c], dsum[c]); atomicAdd(&s_stat[g.Cin + ci0 + c], dxs[c]); }
    __syncthreads();
    float* row = a.bwd_slab + (size_t)(bid % a.nslab) * 2 * g.Cin;
    for (int i = threadIdx.x; i < 2 * g.Cin; i += blockDim.x) atomicAdd(&row[i], s_stat[i]);
  }
}

template <int CB>
__global__ __launch_bounds__(CONV_THREADS) void conv_dgrad_kernel(ConvDgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_bn[4 * 128 + 2 * 128];
  __shared__ float s_stat[2 * 128];
  conv_dgrad_body<CB>(a, blockIdx.x, smem, s_bn, s_stat);
}


// -----------------------------------------------------------------------------------
// Conv forward as an implicit GEMM on v_mfma_f32_16x16x4_f32 (the VALU kernel above is
// the fallback).  Rows = output pixels, K = taps (i, j, ci), columns = Cout.  The band's
// input tile is staged ZERO-PADDED in LDS (with the input transform applied once per
// element), the weights as a [K][Cout16] panel and a per-tap offset table, so an A
// operand is ONE ds_read at (pixel base + tap offset) and the inner loop is branch-free.
// With the fused 2x2 / stride-2 max-pool, the 16 rows of a tile are 4 pooled pixels x
// their 4 window positions in the order that the MFMA D layout hands to one lane
// (lane l holds rows 4*(l>>4)..+3 of column l&15): max + argmax stay in registers.
// Bias, activation, pooled store, argmax and the BN partial statistics are fused.
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15], D[4*(l>>4)+r][l&15].
// -----------------------------------------------------------------------------------
typedef float cf32x4 __attribute__((ext_vector_type(4)));

struct ConvMfmaArgs {
  ConvGeom g;
  int pool_on;                  // 2x2 / stride 2 / no padding pool fused
  int OHo, OWo;                 // unit-output geometry (pooled if pool_on)
  int nbands, band_rows;        // unit-output rows per band
  int tile_rows, tile_w;        // staged zero-padded input tile: rows x (Wp * Cin) floats
  int kpad, c16;                // K rounded up to 4, Cout rounded up to 16
  const float* x; const uint8_t* img; const int64_t* idx; const int64_t* cursor;
  BNRef in_bn; int in_bn_on; int in_act; float in_alpha;
  const float* w; const float* bias; int out_act; float out_alpha;
  float* y; uint8_t* argmax; float* stat_slab; int nslab;
  int det;                      // deterministic mode: exclusive slab row per workgroup
};

template <bool U8, bool POOL>
__global__ __launch_bounds__(CONV_THREADS) void conv_fwd_mfma_kernel(ConvMfmaArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_bn[4 * 128 + 2 * 128];
  __shared__ float s_stat[2 * 128];
  const ConvGeom& g = a.g;
  const int b = blockIdx.x / a.nbands, band = blockIdx.x % a.nbands;
  const int OWo = a.OWo;
  const int r0 = band * a.band_rows, r1 = min(a.OHo, r0 + a.band_rows);
  const int c0 = POOL ? 2 * r0 : r0;                // first conv-output row of the band
  const int ty0 = c0 * g.SH - g.PT;                 // image row of tile row 0
  const int tw = a.tile_w, ntile = a.tile_rows * tw;
  float* s_x = smem;
  float* s_w = smem + ((ntile + 3) & ~3);
  int* s_koff = reinterpret_cast<int*>(s_w + a.kpad * a.c16);
  const int K = g.KH * g.KW * g.Cin;
  const int tid = threadIdx.x;

  // ---- staging.  The band's input rows are ONE contiguous global range: the first
  // batch of their loads is issued before anything else, so its round trip overlaps the
  // LDS zero-fill, the weight panel / tap table and the BN table reduction.
  const int iy0 = max(0, ty0), iy1 = min(g.H, ty0 + a.tile_rows);
  const int irow = g.W * g.Cin;
  const int nx = max(0, iy1 - iy0) * irow;
  constexpr int U = 8;
  using T = typename std::conditional<U8, uint8_t, float>::type;
  const T* src;
  if (U8) {
    const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * g.B : a.idx;
    src = reinterpret_cast<const T*>(a.img + idx[b] * (long)(g.H * irow) + (long)iy0 * irow);
  } else {
    src = reinterpret_cast<const T*>(a.x + ((long)b * g.H + iy0) * irow);
  }
  CONV_STAMP(0);
  T v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { const int e = u * CONV_THREADS + tid; v[u] = src[e < nx ? e : 0]; }
  CONV_STAMP(1);

  for (int e = tid; e < ntile; e += CONV_THREADS) s_x[e] = 0.f;
  const FastDiv dc16(a.c16);
  for (int e = tid; e < a.kpad * a.c16; e += CONV_THREADS) {
    int k, co;
    dc16.divmod(e, k, co);
    s_w[e] = (k < K && co < g.Cout) ? a.w[k * g.Cout + co] : 0.f;
  }
  for (int k = tid; k < a.kpad; k += CONV_THREADS) {
    int off = 0;
    if (k < K) {
      const int ci = k % g.Cin, ij = k / g.Cin, i = ij / g.KW, j = ij - i * g.KW;
      off = i * tw + j * g.Cin + ci;
    }
    s_koff[k] = off;
  }
  for (int i = tid; i < 2 * g.Cout; i += CONV_THREADS) s_stat[i] = 0.f;
  if (!U8 && a.in_bn_on) bn_reduce_to_lds(a.in_bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_bn + 512);
  CONV_STAMP(2);
  __syncthreads();
  CONV_STAMP(3);
  {  // scatter into the zero-padded rows (transform applied once per element)
    float* dst0 = s_x + (iy0 - ty0) * tw + g.PL * g.Cin;
    const int cmax = min(irow, tw - g.PL * g.Cin);   // VALID: columns past the last tap unused
    const FastDiv drow(irow), dcin(g.Cin);
    const int bn_on = a.in_bn_on, act = a.in_act;
    const float alpha = a.in_alpha;
    for (int base = 0; base < nx; base += CONV_THREADS * U) {
      if (base > 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) { const int e = base + u * CONV_THREADS + tid; v[u] = src[e < nx ? e : 0]; }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * CONV_THREADS + tid;
        if (e >= nx) continue;
        int r, c;
        drow.divmod(e, r, c);
        if (c >= cmax) continue;
        float t;
        if (U8) {
          t = (float)v[u] * (1.0f / 255.0f);
        } else {
          t = (float)v[u];
          if (bn_on) { int q, ci; dcin.divmod(c, q, ci); t = t * s_bn[256 + ci] + s_bn[384 + ci]; }
          t = act_fwd(t, act, alpha);
        }
        dst0[r * tw + c] = t;
      }
    }
  }
  __syncthreads();
  CONV_STAMP(4);

  // ---- MFMA over (row tiles) x (Cout tiles), K = taps ----
  const int lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int ntn = a.c16 >> 4;
  const int nunit = (r1 - r0) * OWo;                // unit-output pixels of the band
  const int nmt = POOL ? (nunit + 3) >> 2 : (nunit + 15) >> 4;
  const int ksteps = a.kpad >> 2;
  float bias[8], bsum[8], bsq[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) {
    const int co = nt * 16 + lr;
    bias[nt] = (nt < ntn && a.bias && co < g.Cout) ? a.bias[co] : 0.f;
    bsum[nt] = 0.f;
    bsq[nt] = 0.f;
  }
  for (int mt = wave; mt < nmt; mt += 4) {
    // this lane's A row (pixel lr of the tile)
    int cy, cx;
    bool okr;
    if (POOL) {
      const int pp = mt * 4 + (lr >> 2), pos = lr & 3;
      okr = pp < nunit;
      const int ppc = okr ? pp : 0;
      cy = 2 * (r0 + ppc / OWo) + (pos >> 1);
      cx = 2 * (ppc % OWo) + (pos & 1);
      okr = okr && cy < g.OH && cx < g.OW;
    } else {
      const int p = mt * 16 + lr;
      okr = p < nunit;
      const int pc = okr ? p : 0;
      cy = r0 + pc / OWo;
      cx = pc % OWo;
    }
    const int pixbase = okr ? (cy - c0) * g.SH * tw + cx * g.SW * g.Cin : 0;
    cf32x4 acc[8];
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) acc[nt] = cf32x4{0.f, 0.f, 0.f, 0.f};
    for (int s2 = 0; s2 < ksteps; ++s2) {
      const int k = 4 * s2 + lk;
      const float av = s_x[pixbase + s_koff[k]];
      const float* wrow = s_w + k * a.c16 + lr;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt)
        if (nt < ntn) acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wrow[nt * 16], acc[nt], 0, 0, 0);
    }
    if (mt == 0) CONV_STAMP(5);
    // ---- epilogue: lane holds rows 4*lk .. 4*lk+3 of column lr ----
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      if (nt >= ntn) break;
      const int co = nt * 16 + lr;
      if (co >= g.Cout) continue;
      if (POOL) {
        const int pp = mt * 4 + lk;
        if (pp >= nunit) continue;
        const int py = r0 + pp / OWo, px = pp % OWo;
        float out = -INFINITY;
        int am = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int cyy = 2 * py + (r >> 1), cxx = 2 * px + (r & 1);
          if (cyy >= g.OH || cxx >= g.OW) continue;
          const float v = act_fwd(acc[nt][r] + bias[nt], a.out_act, a.out_alpha);
          if (v > out) { out = v; am = r; }
        }
        const long o = (((long)b * a.OHo + py) * OWo + px) * g.Cout + co;
        a.y[o] = out;
        if (a.argmax) a.argmax[o] = (uint8_t)am;
        bsum[nt] += out;
        bsq[nt] += out * out;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = mt * 16 + 4 * lk + r;
          if (p >= nunit) continue;
          const float v = act_fwd(acc[nt][r] + bias[nt], a.out_act, a.out_alpha);
          const int oy = r0 + p / OWo, ox = p % OWo;
          a.y[(((long)b * a.OHo + oy) * OWo + ox) * g.Cout + co] = v;
          bsum[nt] += v;
          bsq[nt] += v * v;
        }
      }
    }
  }
  if (a.stat_slab && a.det) {
    // deterministic mode: the 4 waves' column sums folded in wave order through s_bn
    // (dead after staging), one statistic per pass, then the EXCLUSIVE row blockIdx
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) {
        if (nt >= ntn) break;
        float s = pass ? bsq[nt] : bsum[nt];
        s += __shfl_xor(s, 16, 64); s += __shfl_xor(s, 32, 64);
        const int co = nt * 16 + lr;
        if (lk == 0 && co < g.Cout) s_bn[wave * 128 + co] = s;
      }
      __syncthreads();
      for (int co = tid; co < g.Cout; co += CONV_THREADS)
        s_stat[pass * g.Cout + co] = ((s_bn[co] + s_bn[128 + co]) + s_bn[256 + co]) + s_bn[384 + co];
      __syncthreads();
    }
    float* row = a.stat_slab + (size_t)blockIdx.x * 2 * g.Cout;
    for (int i = tid; i < 2 * g.Cout; i += CONV_THREADS) row[i] = s_stat[i];
  } else if (a.stat_slab) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) {
      if (nt >= ntn) break;
      float s1 = bsum[nt], s2 = bsq[nt];
      s1 += __shfl_xor(s1, 16, 64); s1 += __shfl_xor(s1, 32, 64);
      s2 += __shfl_xor(s2, 16, 64); s2 += __shfl_xor(s2, 32, 64);
      const int co = nt * 16 + lr;
      if (lk == 0 && co < g.Cout) { atomicAdd(&s_stat[co], s1); atomicAdd(&s_stat[g.Cout + co], s2); }
    }
    CONV_STAMP(6);
    __syncthreads();
    float* row = a.stat_slab + (size_t)(blockIdx.x % a.nslab) * 2 * g.Cout;
    for (int i = tid; i < 2 * g.Cout; i += CONV_THREADS) atomicAdd(&row[i], s_stat[i]);
  }
  CONV_STAMP(7);
}

constexpr int CB_T = 4;                  // channels per lane
constexpr int STAGE_FLOATS = 12288;      // 48 KiB of staged rows per workgroup
constexpr int SLAB_ROWS = 32;            // BN partial-slab rows (atomically folded)

static int groups(int c) { return (c + CB_T - 1) / CB_T; }

// Rows per band: one pass of the 256 lanes over (pixel, channel-group) pairs, and the
// staged input rows within STAGE_FLOATS.
// -----------------------------------------------------------------------------------
// Conv weight gradient:  dW[i,j,ci,co] = sum_{b,oy,ox} xin[b, oy*SH-PT+i, ox*SW-PL+j, ci]
// * dc[b,oy,ox,co],  db[co] = sum dc[b,oy,ox,co]  — a GEMM with a huge reduction
// dimension (pixels: 39,200 for the sample) and a tiny output (taps x Cout: 40 x 20).
// One workgroup per (image, band of output rows):
//   * stages the band's input tile ZERO-PADDED (SAME padding materialised, so no bounds
//     checks in the inner loop) with the forward input transform (uint8 /255 for the
//     first layer, BN-apply + activation otherwise) and the band's dc rows
//     (channel-padded to a multiple of 16) in LDS — one batched round trip;
//   * runs v_mfma_f32_16x16x4_f32 over (tap-row tiles of 16) x (Cout tiles of 16) with
//     the band's pixels as K, split across the 4 waves; A (im2col of the LDS tile) and
//     B (dc) are read straight from LDS with per-lane precomputed offsets;
//   * folds the 4 waves' partial tiles in LDS and issues one atomicAdd per output into
//     stripe (workgroup % S) of dW/db ([S][taps*Cout], [S][Cout]; zeroed by the
//     optimizer, which sums the stripes when it applies the update).  Atomics to one
//     128-B line serialise at ~1 ns each: 350 workgroups x 800 outputs on the sample
//     conv2 cost 14 us unstriped.  S = 1 (data parallel: the all-reduce needs the plain
//     gradient) accumulates straight into the flat gradient.
// The tap row == KH*KW*Cin is the ones row (bias gradient).
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15], D[4*(l>>4)+r][l&15].
// -----------------------------------------------------------------------------------
typedef float wg_f32x4 __attribute__((ext_vector_type(4)));

struct ConvWgradArgs {
  ConvGeom g;
  int nbands, band_rows;
  int tile_rows, tile_w;        // zero-padded input tile: rows x (Wp * Cin) floats
  int c16;                      // dc channel stride in LDS (Cout rounded up to 16)
  int mtiles, ntiles, ntaps;    // ntaps = KH*KW*Cin (+1 if bias); 16x16 output tiles
  const float* x; const uint8_t* img; const int64_t* idx; const int64_t* cursor;
  BNRef in_bn; int in_bn_on; int in_act; float in_alpha;
  const float* dc; float* dw; float* db; int stripes;
};

template <bool U8>
__device__ __forceinline__ void conv_wgrad_body(const ConvWgradArgs& a, int bid, float* smem,
                                                float* s_bn, const RouteArgs* rt = nullptr,
                                                RouteTables rtt = {}) {
  const ConvGeom& g = a.g;
  const int b = bid / a.nbands, band = bid % a.nbands;
  const int r0 = band * a.band_rows, r1 = min(g.OH, r0 + a.band_rows);
  const int nrows = r1 - r0;
  const int ty0 = r0 * g.SH - g.PT;                 // image row of tile row 0
  const int tw = a.tile_w;                          // floats per tile row (Wp * Cin)
  const int ntile = a.tile_rows * tw;
  float* s_x = smem;
  float* s_dc = smem + ((ntile + 3) & ~3);
  const int npix = nrows * g.OW;
  const int kpad = (npix + 15) & ~15;               // pixels padded: 4 waves x k-steps of 4
  float* s_part = s_dc + kpad * a.c16;              // [4 waves][8 tiles][16][16]

  // ---- staging: the band's dc rows and the in-image rows of the input tile are each
  // ONE contiguous global range; both are loaded as float4 (uint8x4 for the first layer)
  // in a single batch — every load of a thread in flight before the first LDS store —
  // and scattered into the padded LDS layouts, whose padding is zero-filled separately.
  const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * g.B : a.idx;
  const int iy0 = max(0, ty0), iy1 = min(g.H, ty0 + a.tile_rows);
  const int irow = g.W * g.Cin;                     // floats per image row
  const int nx = max(0, iy1 - iy0) * irow;          // input elements to load
  const int nd = npix * g.Cout;                     // dc elements to load
  const long xoff = ((long)b * g.H + iy0) * irow;
  const long doff = ((long)b * g.OH + r0) * g.OW * g.Cout;
  // zero-fill: whole tile + whole dc area (cheap LDS stores; overwritten below)
  for (int e = threadIdx.x; e < ntile; e += CONV_THREADS) s_x[e] = 0.f;
  for (int e = threadIdx.x; e < kpad * a.c16; e += CONV_THREADS) s_dc[e] = 0.f;
  if (!U8 && a.in_bn_on) bn_reduce_to_lds(a.in_bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_bn + 512);
  __syncthreads();
  {
    const long ioff = U8 ? idx[b] * (long)(g.H * irow) + (long)iy0 * irow : xoff;
    const bool v4 = ((ioff | nx | (rt ? 0 : doff | nd)) & 3) == 0;
    const int sx = v4 ? 4 : 1;
    const int nxv = (nx + sx - 1) / sx, ndv = rt ? 0 : (nd + sx - 1) / sx, nmax = max(nxv, ndv);
    const uint8_t* isrc = U8 ? a.img + ioff : nullptr;
    const float* xsrc = U8 ? nullptr : a.x + xoff;
    // with the route fused the dc rows come from route_stage below: the dc loads then read
    // one valid element (unconditional, branch-free) and are discarded
    const float* dsrc = rt ? rt->dz : a.dc + doff;
    const FastDiv dirow(irow), dcout(g.Cout), dcin(g.Cin);
    const int xcol0 = g.PL * g.Cin, trow0 = iy0 - ty0;
    constexpr int U = 4;
    // Input and dc loads go to two separate register arrays with clamped indices: a
    // per-element "input or dc" select between two loads made hipcc branch around every
    // load and wait for it before issuing the next (8 serial round trips per thread).
    for (int base = 0; base < nmax; base += CONV_THREADS * U) {
      float4 vx[U], vd[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * CONV_THREADS + threadIdx.x;
        const int jx = min(i, max(nxv - 1, 0)), jd = rt ? 0 : min(i, max(ndv - 1, 0));
        if (v4) {
          if (U8) {
            const uchar4 q = reinterpret_cast<const uchar4*>(isrc)[jx];
            vx[u] = make_float4(q.x, q.y, q.z, q.w);
          } else {
            vx[u] = reinterpret_cast<const float4*>(xsrc)[jx];
          }
          vd[u] = reinterpret_cast<const float4*>(dsrc)[jd];
        } else {
          vx[u] = make_float4(U8 ? (float)isrc[jx] : xsrc[jx], 0.f, 0.f, 0.f);
          vd[u] = make_float4(dsrc[jd], 0.f, 0.f, 0.f);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = base + u * CONV_THREADS + threadIdx.x;
        const float xs[4] = {vx[u].x, vx[u].y, vx[u].z, vx[u].w};
        const float ds[4] = {vd[u].x, vd[u].y, vd[u].z, vd[u].w};
        if (i < nxv) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = i * sx + q;
            if (q >= sx || e >= nx) break;
            int r, c;
            dirow.divmod(e, r, c);
            float t = xs[q];
            if (U8) {
              t *= (1.0f / 255.0f);
            } else {
              if (a.in_bn_on) {
                int xq, ci;
                dcin.divmod(c, xq, ci);
                t = t * s_bn[256 + ci] + s_bn[384 + ci];
              }
              t = act_fwd(t, a.in_act, a.in_alpha);
            }
            if (c < tw - xcol0) s_x[(trow0 + r) * tw + xcol0 + c] = t;   // VALID: unused tail
          }
        }
        if (i < ndv) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = i * sx + q;
            if (q >= sx || e >= nd) break;
            int pix, c;
            dcout.divmod(e, pix, c);
            s_dc[pix * a.c16 + c] = ds[q];
          }
        }
      }
    }
  }
  if (rt)               // dc rows computed here from the unit output (route fused)
    route_stage(*rt, rtt, b, r0, r1, [&](int r, int ox, int c, float v) { s_dc[(r * g.OW + ox) * a.c16 + c] = v; });
  __syncthreads();

  // ---- MFMA: rows = taps (i, j, ci | bias), cols = Cout, K = band pixels (wave-split).
  // Output tiles (16 taps x 16 channels) are processed in blocks of up to 8.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int ntiles = a.mtiles * a.ntiles;
  const int ncombo = g.KH * g.KW * g.Cin;
  const int kq = kpad / 4;                          // pixels per wave (multiple of 4)
  for (int t0 = 0; t0 < ntiles; t0 += 8) {
    const int nt_blk = min(8, ntiles - t0);
    // per-lane A row offset of each tile's tap: >= 0 tile offset, -1 zero row, -2 bias row
    int tapoff[8], bcol[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int tt = t0 + t;
      const int mt = tt / a.ntiles, nt = tt - mt * a.ntiles;
      const int tap = mt * 16 + lr;
      int off = -1;
      if (t < nt_blk && tap < a.ntaps) {
        if (tap >= ncombo) off = -2;
        else {
          const int ci = tap % g.Cin, ij = tap / g.Cin;
          const int i = ij / g.KW, j = ij - i * g.KW;
          off = i * tw + j * g.Cin + ci;
        }
      }
      tapoff[t] = off;
      bcol[t] = nt * 16 + lr;
    }
    wg_f32x4 acc[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = wg_f32x4{0.f, 0.f, 0.f, 0.f};
    // this lane's pixel walks k = wave*kq + lk, +4 per step: (oy, ox) advanced
    // incrementally (no division in the loop); two k-steps per iteration so the next
    // step's LDS operand reads are in flight under this step's MFMAs
    int p = wave * kq + lk;
    int oyl = p / g.OW, ox = p - (p / g.OW) * g.OW;
    const int pend = (wave + 1) * kq;
    const int xstep = 4 * g.SW * g.Cin, ystep = g.SH * tw - g.OW * g.SW * g.Cin;
    int pixoff = oyl * g.SH * tw + ox * g.SW * g.Cin;
#pragma unroll 2
    for (; p < pend; p += 4) {
      const bool okp = p < npix;
      const float* drow = s_dc + p * a.c16;         // zero beyond npix / Cout
      float av[8], bv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (t >= nt_blk) break;
        const int to = tapoff[t];
        const float x = s_x[okp ? pixoff + (to > 0 ? to : 0) : 0];
        av[t] = (to >= 0 && okp) ? x : ((to == -2 && okp) ? 1.f : 0.f);
        bv[t] = drow[bcol[t]];
      }
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        if (t >= nt_blk) break;
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv[t], acc[t], 0, 0, 0);
      }
      ox += 4;
      pixoff += xstep;
      while (ox >= g.OW) { ox -= g.OW; pixoff += ystep; }
    }
    // fold the 4 waves' tiles in LDS, one atomic per output
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (t < nt_blk) {
#pragma unroll
        for (int r = 0; r < 4; ++r) s_part[(wave * 8 + t) * 256 + (4 * lk + r) * 16 + lr] = acc[t][r];
      }
    }
    __syncthreads();
    if (ntiles <= 8) {
      // every output in this block: walk them in memory order so each atomic
      // wave-instruction covers 256 contiguous bytes of dW (row = tap, Cout wide)
      const int nout = a.ntaps * g.Cout;
      const int sidx = bid % a.stripes;
      for (int o = threadIdx.x; o < nout; o += CONV_THREADS) {
        const int tap = o / g.Cout, co = o - tap * g.Cout;
        const int t = (tap >> 4) * a.ntiles + (co >> 4);
        const int el = (tap & 15) * 16 + (co & 15);
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) v += s_part[(w * 8 + t) * 256 + el];
        if (tap >= ncombo) atomicAdd(&a.db[sidx * g.Cout + co], v);
        else atomicAdd(&a.dw[(long)sidx * ncombo * g.Cout + o], v);
      }
      break;                                        // single block: done
    }
    for (int e = threadIdx.x; e < nt_blk * 256; e += CONV_THREADS) {
      const int t = e >> 8, rr = (e >> 4) & 15, cc = e & 15;
      const int tt = t0 + t;
      const int mt = tt / a.ntiles, nt = tt - mt * a.ntiles;
      const int tap = mt * 16 + rr, co = nt * 16 + cc;
      if (tap >= a.ntaps || co >= g.Cout) continue;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) v += s_part[(w * 8 + t) * 256 + (e & 255)];
      const int sidx = bid % a.stripes;
      if (tap >= ncombo) atomicAdd(&a.db[sidx * g.Cout + co], v);
      else atomicAdd(&a.dw[(long)sidx * ncombo * g.Cout + tap * g.Cout + co], v);
    }
    __syncthreads();                                // s_part reused by the next block
  }
}

template <bool U8>
__global__ __launch_bounds__(CONV_THREADS) void conv_wgrad_kernel(ConvWgradArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_bn[4 * 128 + 2 * 128];
  conv_wgrad_body<U8>(a, blockIdx.x, smem, s_bn);
}

// A conv unit's input gradient and weight gradient (independent: both read dc) in ONE
// launch — blocks [0, nd) run the dgrad body, the rest the wgrad body (see
// gemm_pair_kernel in gemm.hip for why this beats a forked graph branch).
__global__ __launch_bounds__(CONV_THREADS) void conv_bwd_pair_kernel(ConvDgradArgs d, ConvWgradArgs w,
                                                                     int nd) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_bn[4 * 128 + 2 * 128];
  __shared__ float s_stat[2 * 128];
  if ((int)blockIdx.x < nd) conv_dgrad_body<CB_T>(d, blockIdx.x, smem, s_bn, s_stat);
  else conv_wgrad_body<false>(w, blockIdx.x - nd, smem, s_bn);
}


static void fwd_bands(const ConvGeom& g, const PoolGeom& p, int& nbands, int& rows, int& rows_in) {
  const int out_rows = p.on ? p.OH : g.OH, out_w = p.on ? p.OW : g.OW;
  const int ppp = CONV_THREADS / groups(g.Cout);
  rows = std::max(1, std::min(out_rows, ppp / std::max(1, out_w)));
  auto in_rows = [&](int r) {
    int crow = p.on ? (r - 1) * p.SH + p.KH : r;
    return std::min(g.H, (crow - 1) * g.SH + g.KH);
  };
  while (rows > 1 && in_rows(rows) * g.W * g.Cin > STAGE_FLOATS) --rows;
  nbands = (out_rows + rows - 1) / rows;
  rows_in = in_rows(rows);
}

static void dgrad_bands(const ConvGeom& g, int& nbands, int& rows, int& rows_in) {
  const int ppp = CONV_THREADS / groups(g.Cin);
  rows = std::max(1, std::min(g.H, ppp / std::max(1, g.W)));
  auto in_rows = [&](int r) { return std::min(g.OH, (r + g.KH - 1) / g.SH + 1); };
  while (rows > 1 && in_rows(rows) * g.OW * g.Cout > STAGE_FLOATS) --rows;
  nbands = (g.H + rows - 1) / rows;
  rows_in = in_rows(rows);
}

static ConvGeom geom_from(const int* v) {
  return ConvGeom{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12]};
}

static bool set_lds_attr(const void* fn) {
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024) == hipSuccess;
}


// Launch the MFMA conv forward when the shape is inside its family; false = use the VALU
// kernel.  Bands: ~700 workgroups over the batch.
// Geometry of the MFMA forward (false: shape outside its family).
static bool conv_fwd_mfma_plan(const ConvGeom& g, const PoolGeom& p, ConvMfmaArgs& a, size_t& shm) {
  constexpr int target = 700;
  const bool pool = p.on != 0;
  if (pool && !(p.KH == 2 && p.KW == 2 && p.SH == 2 && p.SW == 2 && p.PT == 0 && p.PL == 0)) return false;
  if (g.Cout > 128) return false;
  a = ConvMfmaArgs{};
  a.g = g; a.pool_on = pool;
  a.OHo = pool ? p.OH : g.OH; a.OWo = pool ? p.OW : g.OW;
  const int K = g.KH * g.KW * g.Cin;
  a.kpad = (K + 3) & ~3;
  a.c16 = (g.Cout + 15) & ~15;
  a.tile_w = ((g.OW - 1) * g.SW + g.KW) * g.Cin;
  const int per_img = std::max(1, (target + g.B - 1) / g.B);
  int rows = std::max(1, (a.OHo + per_img - 1) / per_img);
  auto tile_rows = [&](int r) { return ((pool ? 2 * r : r) - 1) * g.SH + g.KH; };
  auto lds = [&](int r) {
    return ((((size_t)tile_rows(r) * a.tile_w + 3) & ~(size_t)3) + (size_t)a.kpad * a.c16 + a.kpad) * sizeof(float);
  };
  while (rows > 1 && lds(rows) > 150 * 1024) --rows;
  if (lds(rows) > 150 * 1024) return false;
  a.band_rows = rows;
  a.tile_rows = tile_rows(rows);
  a.nbands = (a.OHo + rows - 1) / rows;
  shm = lds(rows);
  return true;
}

static bool conv_fwd_mfma(const ConvFwdArgs& f, hipStream_t st) {
  ConvMfmaArgs a;
  size_t shm;
  if (!conv_fwd_mfma_plan(f.g, f.pool, a, shm)) return false;
  const ConvGeom& g = f.g;
  const bool pool = a.pool_on != 0;
  a.x = f.x; a.img = f.img; a.idx = f.idx; a.cursor = f.cursor;
  a.in_bn = f.in_bn; a.in_bn_on = f.in_bn_on; a.in_act = f.in_act; a.in_alpha = f.in_alpha;
  a.w = f.w; a.bias = f.bias; a.out_act = f.out_act; a.out_alpha = f.out_alpha;
  a.y = f.y; a.argmax = f.argmax; a.stat_slab = f.stat_slab; a.nslab = f.nslab; a.det = f.det;
  static bool attr = set_lds_attr((const void*)conv_fwd_mfma_kernel<true, true>) &&
                     set_lds_attr((const void*)conv_fwd_mfma_kernel<true, false>) &&
                     set_lds_attr((const void*)conv_fwd_mfma_kernel<false, true>) &&
                     set_lds_attr((const void*)conv_fwd_mfma_kernel<false, false>);
  (void)attr;
  dim3 grid((unsigned)(g.B * a.nbands));
  if (f.img) {
    if (pool) hipLaunchKernelGGL((conv_fwd_mfma_kernel<true, true>), grid, dim3(CONV_THREADS), shm, st, a);
    else hipLaunchKernelGGL((conv_fwd_mfma_kernel<true, false>), grid, dim3(CONV_THREADS), shm, st, a);
  } else {
    if (pool) hipLaunchKernelGGL((conv_fwd_mfma_kernel<false, true>), grid, dim3(CONV_THREADS), shm, st, a);
    else hipLaunchKernelGGL((conv_fwd_mfma_kernel<false, false>), grid, dim3(CONV_THREADS), shm, st, a);
  }
  return true;
}

}  // namespace csa

using namespace csa;

CSA_API int csa_conv_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_conv_dbg), &p, sizeof(p));
}

// Number of BN partial-slab rows a csa_conv_fwd launch writes (the slab must be zeroed
// before every launch: rows are accumulated with atomics).
static PoolGeom pool_from(const int* v) {
  return PoolGeom{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8]};
}

// Workgroups of a csa_conv_fwd launch (the MFMA kernel when the shape is in its family).
static int conv_fwd_blocks(const ConvGeom& g, const PoolGeom& p) {
  ConvMfmaArgs m;
  size_t shm;
  if (conv_fwd_mfma_plan(g, p, m, shm)) return g.B * m.nbands;
  int nb, rows, rows_in;
  fwd_bands(g, p, nb, rows, rows_in);
  return g.B * nb;
}

// Deterministic mode: every workgroup writes its own row (rows = workgroups), folded in
// row order by the consumer (csa_rows_fold) instead of atomics into SLAB_ROWS rows.
CSA_API int csa_conv_fwd_nslab(const int* geom, const int* pool) {
  if (g_csa_det && geom && pool) return conv_fwd_blocks(geom_from(geom), pool_from(pool));
  return SLAB_ROWS;
}

// Forward conv unit: y = pool(act(conv(T(x)) + bias)), T = optional bn+act on the input.
CSA_API int csa_conv_fwd(const float* x, const uint8_t* img, const int64_t* idx, const float* w,
                         const float* bias, float* y, uint8_t* argmax, float* stat_slab,
                         const int* geom /*13*/, const int* pool /*9*/, const float* in_bn_slab,
                         int in_bn_nslab, float in_bn_count, float in_bn_eps,
                         const float* in_bn_scale, const float* in_bn_offset, int in_act,
                         float in_alpha, int out_act, float out_alpha, const int64_t* cursor,
                         hipStream_t st) {
  ConvFwdArgs a{};
  a.cursor = cursor;
  a.g = geom_from(geom);
  a.pool = pool_from(pool);
  if (a.g.Cin > 128 || a.g.Cout > 128) return -1;
  a.x = x; a.img = img; a.idx = idx;
  a.in_bn = BNRef{in_bn_slab, in_bn_nslab, a.g.Cin, in_bn_count, in_bn_eps, in_bn_scale, in_bn_offset};
  a.in_bn_on = in_bn_slab != nullptr;
  a.in_act = in_act; a.in_alpha = in_alpha;
  a.w = w; a.bias = bias; a.out_act = out_act; a.out_alpha = out_alpha;
  a.y = y; a.argmax = argmax; a.stat_slab = stat_slab;
  a.det = g_csa_det;
  a.nslab = a.det ? conv_fwd_blocks(a.g, a.pool) : SLAB_ROWS;
  if (conv_fwd_mfma(a, st)) return (int)hipGetLastError();
  fwd_bands(a.g, a.pool, a.nbands, a.band_rows, a.band_rows_in);
  const size_t nin = ((size_t)a.band_rows_in * a.g.W * a.g.Cin + 3) & ~(size_t)3;
  const size_t shm = (nin + (size_t)a.g.KH * a.g.KW * a.g.Cin * a.g.Cout) * sizeof(float);
  if (shm > 150 * 1024) return -2;
  static bool attr = set_lds_attr((const void*)conv_fwd_kernel<CB_T, true>) &&
                     set_lds_attr((const void*)conv_fwd_kernel<CB_T, false>);
  (void)attr;
  dim3 grid((unsigned)(a.g.B * a.nbands));
  if (img) hipLaunchKernelGGL((conv_fwd_kernel<CB_T, true>), grid, dim3(CONV_THREADS), shm, st, a);
  else hipLaunchKernelGGL((conv_fwd_kernel<CB_T, false>), grid, dim3(CONV_THREADS), shm, st, a);
  return (int)hipGetLastError();
}

// g = {B, h, w, C, OH, OW, pool_on, PKH, PKW, PSH, PSW, PPT, PPL}.  When the pool windows
// are not a tiling (kernel != stride) dc must be zeroed by the caller (atomics).
CSA_API int csa_route_bwd(const float* dz, const float* y, const uint8_t* argmax, float* dc,
                          const int* g /*13*/, int out_act, float out_alpha, const float* bn_slab,
                          int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                          const float* bn_offset, const float* bwd_slab, int bwd_nslab,
                          float* dscale, float* doffset, float* run_mean, float* run_var,
                          float momentum, hipStream_t st) {
  RouteArgs a{};
  a.run_mean = run_mean; a.run_var = run_var; a.momentum = momentum;
  a.dz = dz; a.y = y; a.argmax = argmax; a.dc = dc;
  a.B = g[0]; a.h = g[1]; a.w = g[2]; a.C = g[3]; a.OH = g[4]; a.OW = g[5];
  a.pool_on = g[6]; a.PKW = g[8]; a.PSH = g[9]; a.PSW = g[10]; a.PPT = g[11]; a.PPL = g[12];
  if (a.C > 128) return -1;
  a.overlap = a.pool_on && (g[7] != g[9] || g[8] != g[10]);
  a.out_act = out_act; a.out_alpha = out_alpha;
  a.bn = BNRef{bn_slab, bn_nslab, a.C, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr;
  a.bwd_slab = bwd_slab; a.bwd_nslab = bwd_nslab; a.dscale = dscale; a.doffset = doffset;
  long n = (long)a.B * a.h * a.w * a.C;
  hipLaunchKernelGGL(route_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

CSA_API int csa_conv_dgrad_nslab(const int* geom) {
  if (!g_csa_det || !geom) return SLAB_ROWS;
  int nb, rows, rows_in;             // deterministic mode: one row per dgrad workgroup
  const ConvGeom g = geom_from(geom);
  dgrad_bands(g, nb, rows, rows_in);
  return g.B * nb;
}

static int dgrad_args(const float* dc, const float* w, float* dx, const int* geom, const float* x_fwd,
                      int in_act, float in_alpha, const float* bn_slab, int bn_nslab, float bn_count,
                      float bn_eps, const float* bn_scale, const float* bn_offset, float* bwd_slab,
                      ConvDgradArgs& a, size_t& shm) {
  a = ConvDgradArgs{};
  a.g = geom_from(geom);
  if (a.g.Cin > 128 || a.g.Cout > 128) return -1;
  a.dc = dc; a.w = w; a.dx = dx; a.x_fwd = x_fwd; a.in_act = in_act; a.in_alpha = in_alpha;
  a.in_bn = BNRef{bn_slab, bn_nslab, a.g.Cin, bn_count, bn_eps, bn_scale, bn_offset};
  a.in_bn_on = bn_slab != nullptr;
  a.bwd_slab = bwd_slab; a.nslab = SLAB_ROWS; a.det = g_csa_det;
  dgrad_bands(a.g, a.nbands, a.band_rows, a.band_rows_in);
  const size_t nd = ((size_t)a.band_rows_in * a.g.OW * a.g.Cout + 3) & ~(size_t)3;
  shm = (nd + (size_t)a.g.KH * a.g.KW * a.g.Cin * a.g.Cout) * sizeof(float);
  return shm > 150 * 1024 ? -2 : 0;
}

CSA_API int csa_conv_dgrad(const float* dc, const float* w, float* dx, const int* geom,
                           const float* x_fwd, int in_act, float in_alpha, const float* bn_slab,
                           int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                           const float* bn_offset, float* bwd_slab, hipStream_t st) {
  ConvDgradArgs a;
  size_t shm;
  const int rc = dgrad_args(dc, w, dx, geom, x_fwd, in_act, in_alpha, bn_slab, bn_nslab, bn_count, bn_eps,
                            bn_scale, bn_offset, bwd_slab, a, shm);
  if (rc) return rc;
  static bool attr = set_lds_attr((const void*)conv_dgrad_kernel<CB_T>);
  (void)attr;
  dim3 grid((unsigned)(a.g.B * a.nbands));
  hipLaunchKernelGGL((conv_dgrad_kernel<CB_T>), grid, dim3(CONV_THREADS), shm, st, a);
  return (int)hipGetLastError();
}

static int wgrad_args(const float* x, const uint8_t* img, const int64_t* idx, const float* dOut,
                      float* dW, float* db, int stripes, int B, int H, int W, int Cin, int KH, int KW,
                      int SH, int SW, int PT, int PL, int OH, int OW, int Cout, const float* bn_slab,
                      int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                      const float* bn_offset, int in_act, float in_alpha, const int64_t* cursor,
                      ConvWgradArgs& a, size_t& shm) {
  a = ConvWgradArgs{};
  a.g = ConvGeom{B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH, OW, Cout};
  a.ntaps = KH * KW * Cin + (db ? 1 : 0);
  a.mtiles = (a.ntaps + 15) / 16;
  a.ntiles = (Cout + 15) / 16;
  if (Cin > 128 || (!x && !img)) return -1;
  a.x = x; a.img = img; a.idx = idx; a.cursor = cursor; a.dc = dOut; a.dw = dW; a.db = db;
  a.stripes = stripes < 1 ? 1 : stripes;
  a.in_bn = BNRef{bn_slab, bn_nslab, Cin, bn_count, bn_eps, bn_scale, bn_offset};
  a.in_bn_on = bn_slab != nullptr && !img;
  a.in_act = img ? 0 : in_act; a.in_alpha = in_alpha;
  a.c16 = a.ntiles * 16;
  a.tile_w = ((OW - 1) * SW + KW) * Cin;
  auto tile_rows = [&](int r) { return (r - 1) * SH + KH; };
  auto lds = [&](int r) {
    const size_t kpad = ((size_t)r * OW + 15) & ~(size_t)15;
    return (((size_t)tile_rows(r) * a.tile_w + 3) / 4 * 4 + kpad * a.c16 +
            4 * 8 * 256) * sizeof(float);
  };
  // Bands: the batch is cut into ~`target` workgroups.  Each ends in one atomicAdd per
  // output and atomics to one 128-B line serialise, so fewer, larger bands win until
  // the per-wave pixel loop dominates (swept: profiles/r1_conv_wgrad_iterations.md).
  constexpr int target = 700;
  const int per_img = std::max(1, (target + B - 1) / B);
  int rows = std::max(1, (OH + per_img - 1) / per_img);
  while (rows > 1 && lds(rows) > 150 * 1024) --rows;
  if (lds(rows) > 150 * 1024) return -2;
  a.band_rows = rows;
  a.tile_rows = tile_rows(rows);
  a.nbands = (OH + rows - 1) / rows;
  shm = lds(rows);
  return 0;
}

// Workgroups of a conv weight-gradient launch (csa_conv_wgrad, or the wgrad half of
// csa_conv_bwd): with that many stripes every workgroup owns one stripe and adds each of
// its outputs ONCE into a zeroed row — the deterministic-mode layout, folded in stripe
// order by csa_rows_fold.  geom = {B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH, OW, Cout}.
CSA_API int csa_conv_wgrad_blocks(const int* geom, int bias) {
  static const float probe = 0.f;    // wgrad_args needs an input; the plan never reads it
  float dummy_db = 0.f;
  const ConvGeom g = geom_from(geom);
  ConvWgradArgs a;
  size_t shm;
  if (wgrad_args(&probe, nullptr, nullptr, nullptr, nullptr, bias ? &dummy_db : nullptr, 1, g.B, g.H, g.W,
                 g.Cin, g.KH, g.KW, g.SH, g.SW, g.PT, g.PL, g.OH, g.OW, g.Cout, nullptr, 0, 0.f, 0.f, nullptr,
                 nullptr, 0, 0.f, nullptr, a, shm))
    return -1;
  return g.B * a.nbands;
}

// dW/db (+)= conv weight gradient, accumulated with atomics into `stripes` copies
// (dW: [stripes][KH*KW*Cin*Cout], db: [stripes][Cout]); the caller zeroes them.
// Input = x (fp32 NHWC, forward input transform BN/act applied on the fly) or the
// uint8 dataset rows img[idx[b] (+ cursor * B)] / 255 for the first layer.
CSA_API int csa_conv_wgrad(const float* x, const uint8_t* img, const int64_t* idx, const float* dOut,
                           float* dW, float* db, int stripes, int B, int H, int W, int Cin, int KH, int KW, int SH,
                           int SW, int PT, int PL, int OH, int OW, int Cout, const float* bn_slab,
                           int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                           const float* bn_offset, int in_act, float in_alpha, const int64_t* cursor,
                           hipStream_t st) {
  ConvWgradArgs a;
  size_t shm;
  const int rc = wgrad_args(x, img, idx, dOut, dW, db, stripes, B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH,
                            OW, Cout, bn_slab, bn_nslab, bn_count, bn_eps, bn_scale, bn_offset, in_act,
                            in_alpha, cursor, a, shm);
  if (rc) return rc;
  static bool attr = set_lds_attr((const void*)conv_wgrad_kernel<true>) &&
                     set_lds_attr((const void*)conv_wgrad_kernel<false>);
  (void)attr;
  dim3 grid((unsigned)(B * a.nbands));
  if (img) hipLaunchKernelGGL((conv_wgrad_kernel<true>), grid, dim3(CONV_THREADS), shm, st, a);
  else hipLaunchKernelGGL((conv_wgrad_kernel<false>), grid, dim3(CONV_THREADS), shm, st, a);
  return (int)hipGetLastError();
}

static RouteArgs route_args(const float* dz, const float* y, const uint8_t* argmax, float* dc, const int* g,
                            int out_act, float out_alpha, const float* bn_slab, int bn_nslab, float bn_count,
                            float bn_eps, const float* bn_scale, const float* bn_offset, const float* bwd_slab,
                            int bwd_nslab, float* dscale, float* doffset, float* run_mean, float* run_var,
                            float momentum) {
  RouteArgs a{};
  a.run_mean = run_mean; a.run_var = run_var; a.momentum = momentum;
  a.dz = dz; a.y = y; a.argmax = argmax; a.dc = dc;
  a.B = g[0]; a.h = g[1]; a.w = g[2]; a.C = g[3]; a.OH = g[4]; a.OW = g[5];
  a.pool_on = g[6]; a.PKW = g[8]; a.PSH = g[9]; a.PSW = g[10]; a.PPT = g[11]; a.PPL = g[12];
  a.overlap = a.pool_on && (g[7] != g[9] || g[8] != g[10]);
  a.out_act = out_act; a.out_alpha = out_alpha;
  a.bn = BNRef{bn_slab, bn_nslab, a.C, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr;
  a.bwd_slab = bwd_slab; a.bwd_nslab = bwd_nslab; a.dscale = dscale; a.doffset = doffset;
  return a;
}

// Conv unit backward in ONE launch: input gradient (as csa_conv_dgrad) + weight gradient
// of a non-first layer (as csa_conv_wgrad with x, never the uint8 images).
CSA_API int csa_conv_bwd(const float* dc, const float* w, float* dx, const int* geom, const float* x_fwd,
                         int in_act, float in_alpha, const float* bn_slab, int bn_nslab, float bn_count,
                         float bn_eps, const float* bn_scale, const float* bn_offset, float* bwd_slab,
                         float* dW, float* db, int stripes, hipStream_t st) {
  ConvDgradArgs d;
  ConvWgradArgs wg;
  size_t shm_d, shm_w;
  int rc = dgrad_args(dc, w, dx, geom, x_fwd, in_act, in_alpha, bn_slab, bn_nslab, bn_count, bn_eps,
                      bn_scale, bn_offset, bwd_slab, d, shm_d);
  if (rc) return rc;
  const ConvGeom& g = d.g;
  rc = wgrad_args(x_fwd, nullptr, nullptr, dc, dW, db, stripes, g.B, g.H, g.W, g.Cin, g.KH, g.KW, g.SH, g.SW,
                  g.PT, g.PL, g.OH, g.OW, g.Cout, bn_slab, bn_nslab, bn_count, bn_eps, bn_scale, bn_offset,
                  in_act, in_alpha, nullptr, wg, shm_w);
  if (rc) return rc;
  static bool attr = set_lds_attr((const void*)conv_bwd_pair_kernel);
  (void)attr;
  const int nd = g.B * d.nbands;
  dim3 grid((unsigned)(nd + g.B * wg.nbands));
  hipLaunchKernelGGL(conv_bwd_pair_kernel, grid, dim3(CONV_THREADS), std::max(shm_d, shm_w), st, d, wg, nd);
  return (int)hipGetLastError();
}
