// Head + the last dense layer's input gradient (head_dgrad): the device body, shared by its
// own launch (head.hip) and by the fused forward chain (dense_direct.hip: fc1 forward ->
// fc2 forward -> head_dgrad as one launch with ticket hand-offs).
#pragma once
#include "common.h"

namespace csa {

#ifndef CSA_NCLS_DEFINED
#define CSA_NCLS_DEFINED
constexpr int NCLS = 10;
#endif

// ---------------------------------------------------------------------------------
// Head + the LAST dense layer's input gradient in ONE launch (round 4, horizontal-fusion
// program).  The head's outputs per batch row (dlogits, loss, #correct, the head input
// gradient dh) need nothing but that row, and the last dense layer's input gradient
//   dX[m][f] = act'( sum_n dh[m][n] W[f][n] )           (W = [K1][Kh], this layer)
// needs nothing but row m's dh — so a workgroup owning R rows x FS input features
// recomputes the (tiny) head for its R rows and finishes dX for its features, with no
// batch-wide reduction anywhere.  The dense layer's weight gradient + update and the head's
// batch reductions (dWh, dbh, the metric ring entry) are deferred into the pair backward
// launch (dense_update.h, csa_dense_update_defer).  Replaces head_row_kernel + the fused
// dense backward of that layer on the critical path (5.0 + 13.5 us in the round-3 trace).
//
// Per workgroup: ONE batch of loads (R rows of h, all of Wh, the FS x Kh slice of W as
// float4s, the epilogue's forward inputs), R x 10 wave reductions for the logits, one wave
// per row for the softmax, dh into LDS, then 16 lanes per feature dot their W float4s with
// dh and reduce by DPP inside their 16-lane row.  Workgroups that share a W slice are
// dealt to one XCD (blocks b and b + 8 share an XCD under round-robin dispatch: speed only).
// ---------------------------------------------------------------------------------
constexpr int HD_T = 256;
constexpr int HD_R = 4;                  // batch rows per workgroup (one wave each for the softmax)
constexpr int HD_FS = HD_T / 16;         // input features per workgroup (16 lanes each)

struct HeadDgradArgs {
  const float* h; int M, Kh; int in_act; float in_alpha;     // head input + its transform
  const float* w; const float* b;                             // head [Kh][10], [10]
  const int64_t* labels; const int64_t* idx; const int64_t* cursor;
  int loss; float grad_scale;
  float* dh; float* dl; float* rloss; int* rcorr;             // written by feature slice 0
  int64_t* step; int64_t* adv_cursor; long wrap;
  const float* W; int K1;                                     // last dense layer [K1][Kh]
  const float* x_fwd; int act; float alpha;                   // its pre-transform input [M][K1]
  float* dX;                                                  // [M][K1]
};

__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, false)));
  return v;
}

__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  return v;
}

// KPT = head-input values per thread (Kh <= 256 KPT), KQ = W float4s per thread (Kh = 64 KQ)
// diagnostics (csa_head_debug, scripts/microbench.py MB_HD): per workgroup b, six
// s_memrealtime stamps (100 MHz, one clock for every XCD) at [8 + 8 b]: start | head input
// landed (act applied) | logits done | softmax + dh done | dX dot done | dX stored
static __constant__ long long* g_hd_dbg = nullptr;   // (per code object: csa_head_debug,
                                                      //  csa_chain_head_debug)
#define HD_STAMP(k)                                                                           \
  do {                                                                                        \
    if (g_hd_dbg && threadIdx.x == 0) g_hd_dbg[8 + 8 * (long)bid + (k)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)

template <int KPT, int KQ>
__device__ __forceinline__ void head_dgrad_body(const HeadDgradArgs& a, const int bid) {
  __shared__ float s_part[HD_T / 64][HD_R][NCLS];
  __shared__ float s_dl[HD_R][NCLS];
  __shared__ __attribute__((aligned(16))) float s_dh[HD_R][64 * KQ];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.M, Kh = a.Kh, K1 = a.K1;
  const int nrt = (M + HD_R - 1) / HD_R, nfs = (K1 + HD_FS - 1) / HD_FS;
  int rt, fs;
  if (nfs % 8 == 0) {                    // slices {x, x+8, ..} on XCD x
    const int xcd = bid & 7, idx = bid >> 3;
    fs = xcd + 8 * (idx / nrt);
    rt = idx % nrt;
  } else {
    fs = bid / nrt;
    rt = bid % nrt;
  }
  const int m0 = rt * HD_R, f0 = fs * HD_FS;
  const int nr = min(HD_R, M - m0);
  HD_STAMP(0);
  if (bid == 0 && tid == 0) {
    *a.step += 1;
    if (a.adv_cursor) {
      const int64_t c = *a.adv_cursor + 1;
      *a.adv_cursor = (a.wrap > 0 && c >= a.wrap) ? 0 : c;
    }
  }
  // ---- every load first
  const int f = tid >> 4, c = tid & 15;
  const int frow = min(f0 + f, K1 - 1);
  float4 wq[KQ];
#pragma unroll
  for (int u = 0; u < KQ; ++u)
    wq[u] = reinterpret_cast<const float4*>(a.W + (long)frow * Kh)[u * 16 + c];
  float hv[HD_R][KPT], wv[KPT][NCLS];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int k = min(u * HD_T + tid, Kh - 1);
#pragma unroll
    for (int r = 0; r < HD_R; ++r) hv[r][u] = a.h[(long)min(m0 + r, M - 1) * Kh + k];
#pragma unroll
    for (int j = 0; j < NCLS; j += 2) {
      const float2 t = *reinterpret_cast<const float2*>(a.w + (long)k * NCLS + j);
      wv[u][j] = t.x; wv[u][j + 1] = t.y;
    }
  }
  const float bias = lane < NCLS ? a.b[lane] : 0.f;
  int label = 0;
  if (wave < nr) {
    const int m = m0 + wave;
    if (!a.idx) label = (int)a.labels[m];
    else label = (int)a.labels[(a.cursor ? a.idx + a.cursor[0] * a.M : a.idx)[m]];
  }
  // epilogue operand: lane c < R of feature f stores row m0 + c
  const float xe = (a.x_fwd && c < HD_R) ? a.x_fwd[(long)min(m0 + c, M - 1) * K1 + frow] : 0.f;
  // ---- logits
  float hx[HD_R][KPT];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const bool ok = u * HD_T + tid < Kh;
#pragma unroll
    for (int r = 0; r < HD_R; ++r) hx[r][u] = ok ? act_fwd(hv[r][u], a.in_act, a.in_alpha) : 0.f;
  }
  if (g_hd_dbg) {                                          // (diagnostics: after hx exists)
    float z = 0.f;
#pragma unroll
    for (int r = 0; r < HD_R; ++r) z += hx[r][0];
    if (threadIdx.x == 0) g_hd_dbg[8 + 8 * (long)bid + 1] = (long long)__builtin_amdgcn_s_memrealtime() + (z == 12345.f);
  }
  // the R x 10 logit partials of this thread's k values, then their sums over the 256
  // threads.  Round 6: a transposed reduction instead of 40 wave reductions (each 4 DPP +
  // 2 cross-row shuffles, serialised: 4.7 us of the launch's 9 us workgroup life,
  // scripts/mb/graph_life.py): two DPP exchange rounds inside each quad halve the values
  // per lane twice (40 -> 20 -> 10, a lane keeps one half and adds its partner's copy of
  // it), the quads' 40 sums go to LDS output-major, 160 threads sum 16 quads each, in fixed
  // order (bitwise-repeatable).
  {
    float v[HD_R * NCLS];
#pragma unroll
    for (int r = 0; r < HD_R; ++r)
#pragma unroll
      for (int j = 0; j < NCLS; ++j) {
        float acc = 0.f;
#pragma unroll
        for (int u = 0; u < KPT; ++u) acc = fmaf(hx[r][u], wv[u][j], acc);
        v[r * NCLS + j] = acc;
      }
    constexpr int NO = HD_R * NCLS, H1 = NO / 2, H2 = NO / 4;
    const bool b0 = lane & 1, b1 = lane & 2;
    float w1[H1];
#pragma unroll
    for (int m = 0; m < H1; ++m) {                         // partner lane ^ 1
      const float send = b0 ? v[m] : v[m + H1], keep = b0 ? v[m + H1] : v[m];
      w1[m] = keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0xb1, 0xf, 0xf, false));
    }
    // [NO][68]: 64 quads of the workgroup per output, +4 so the 4 lanes of a quad (4
    // different outputs) hit different banks
    __shared__ __attribute__((aligned(16))) float s_red[HD_R * NCLS * 68];
    const int gq = wave * 16 + (lane >> 2), base = (b0 ? H1 : 0) + (b1 ? H2 : 0);
#pragma unroll
    for (int m = 0; m < H2; ++m) {                         // partner lane ^ 2
      const float send = b1 ? w1[m] : w1[m + H2], keep = b1 ? w1[m + H2] : w1[m];
      const float w2 = keep + __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(send), 0x4e, 0xf, 0xf, false));
      s_red[(base + m) * 68 + gq] = w2;
    }
    __syncthreads();
    if (tid < NO * 4) {                                    // output o, wave w: its 16 quads
      const int o = tid >> 2, w = tid & 3;
      const float4* p4 = reinterpret_cast<const float4*>(s_red + o * 68 + w * 16);
      const float4 x0 = p4[0], x1 = p4[1], x2 = p4[2], x3 = p4[3];
      float acc = ((x0.x + x0.y) + (x0.z + x0.w)) + ((x1.x + x1.y) + (x1.z + x1.w));
      acc += ((x2.x + x2.y) + (x2.z + x2.w)) + ((x3.x + x3.y) + (x3.z + x3.w));
      s_part[w][o / NCLS][o % NCLS] = acc;
    }
  }
  __syncthreads();
  HD_STAMP(2);
  if (wave < nr) {
    // wave r: row m0 + r; lane j < 10: logit j (waves folded in fixed order)
    const int r = wave, m = m0 + r;
    float z = -INFINITY;
    if (lane < NCLS) z = s_part[0][r][lane] + s_part[1][r][lane] + s_part[2][r][lane] + s_part[3][r][lane] + bias;
    // the 10 classes live in lanes 0..9 (row 0 of the wave): 16-lane DPP reductions, no
    // cross-row shuffles (lanes >= 16 reduce their own rows, unused)
    const float mx = row16_max(z);
    const unsigned long long hit = __ballot(lane < NCLS && z == mx);
    const int am = __builtin_ctzll(hit);       // lowest index attaining the max (tf.argmax)
    float d = 0.f, lterm = 0.f;
    if (a.loss == 0) {
      const float e = lane < NCLS ? __expf(z - mx) : 0.f;
      const float se = row16_sum(e);
      const float lse = mx + __logf(se);
      if (lane < NCLS) {
        d = (__expf(z - lse) - (lane == label ? 1.f : 0.f)) * (a.grad_scale / (float)M);
        lterm = lane == label ? lse - z : 0.f;
      }
    } else if (lane < NCLS) {
      const float t = z - (lane == label ? 1.f : 0.f);
      lterm = t * t;
      d = t * (2.f * a.grad_scale / (float)(M * NCLS));
    }
    const float ls = row16_sum(lterm);
    if (lane < NCLS) s_dl[r][lane] = d;
    if (fs == 0) {
      if (lane < NCLS) a.dl[(long)m * NCLS + lane] = d;
      if (lane == 0) {
        a.rloss[m] = ls;
        a.rcorr[m] = am == label ? 1 : 0;
      }
    }
  }
  __syncthreads();
  // ---- dh = act'(dl . Wh^T) for the R rows -> LDS (slice 0 also stores it: the deferred
  // weight gradient of the dense layer reads it as its dY)
#pragma unroll
  for (int r = 0; r < HD_R; ++r) {
    float dl[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) dl[j] = s_dl[r][j];
#pragma unroll
    for (int u = 0; u < KPT; ++u) {
      const int k = u * HD_T + tid;
      if (k >= Kh) break;
      float g = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) g = fmaf(dl[j], wv[u][j], g);
      if (a.in_act) g = act_bwd(g, hv[r][u], hx[r][u], a.in_act, a.in_alpha);   // x-based: any alpha
      g = r < nr ? g : 0.f;
      s_dh[r][k] = g;
      if (fs == 0 && r < nr) out_store(a.dh + (long)(m0 + r) * Kh + k, g);
    }
  }
  __syncthreads();
  HD_STAMP(3);
  // ---- dX[m0 + r][f0 + f] = sum_k dh[r][k] W[f][k]: 16 lanes per feature, DPP row sums
  float p[HD_R];
#pragma unroll
  for (int r = 0; r < HD_R; ++r) p[r] = 0.f;
#pragma unroll
  for (int u = 0; u < KQ; ++u) {
    const int k4 = u * 16 + c;
#pragma unroll
    for (int r = 0; r < HD_R; ++r) {
      const float4 d4 = reinterpret_cast<const float4*>(&s_dh[r][0])[k4];
      p[r] = fmaf(d4.x, wq[u].x, fmaf(d4.y, wq[u].y, fmaf(d4.z, wq[u].z, fmaf(d4.w, wq[u].w, p[r]))));
    }
  }
  float mine = 0.f;
#pragma unroll
  for (int r = 0; r < HD_R; ++r) {
    const float t = row16_sum(p[r]);
    mine = c == r ? t : mine;
  }
  if (g_hd_dbg && threadIdx.x == 0) g_hd_dbg[8 + 8 * (long)bid + 4] = (long long)__builtin_amdgcn_s_memrealtime() + (mine == 12345.f);
  if (c < nr && f0 + f < K1) {
    float g = mine;
    if (a.act) g = act_bwd(g, xe, act_fwd(xe, a.act, a.alpha), a.act, a.alpha);
    out_store(a.dX + (long)(m0 + c) * K1 + f0 + f, g);
  }
  HD_STAMP(5);
}

// Recorder for the fused forward chain (dense_direct.hip): while on, csa_head_dgrad stores
// its arguments here instead of launching.
struct HDRecord { int on, has, kq; HeadDgradArgs a; };
extern thread_local HDRecord g_hd_rec;

}  // namespace csa
