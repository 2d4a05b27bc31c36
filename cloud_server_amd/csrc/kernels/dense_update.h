// Device code of the fused dense backward (+ optimizer update) — shared by its own launch
// (dense_update.hip) and by launches that carry its workgroups beside other work
// (conv_pair.hip: the pair backward with the dense weight-gradient + update workgroups).
// See dense_update.hip for the design.
#pragma once
#include "common.h"
#include "optim_common.h"

namespace csa {

typedef float du_f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int du_u32x4 __attribute__((ext_vector_type(4)));

constexpr int DU_FT = 16;            // W rows per row group
constexpr int DU_SUB = 2;            // 16-column sub-tiles per wave (= the two column halves)
constexpr int DU_MAXM = 64;          // batch rows (4 tiles of 16)
constexpr int DU_KS = DU_MAXM / 4;   // wgrad MFMA k-steps (4 batch rows each)
constexpr int MAXC_DU = 128;         // BatchNorm channels handled in LDS
constexpr int DU_SLAB = 16;          // BN-backward slab rows (atomically folded)
constexpr int DU_PART = DU_MAXM * DU_FT;   // floats of one block's input-gradient partial
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
  int det;                  // deterministic mode: bwd_slab has one EXCLUSIVE row per row
                            // group (plain stores, folded in fixed order by csa_rows_fold)
  const float* Xw;          // [M][K] weight-gradient operand (transform applied)
  int opt; float lr; const int64_t* step;
  float* s0w; float* s1w;   // optimizer slots of W (same [K][N] layout) ...
  float* s0b; float* s1b;   // ... and of the bias
  float scale;
  // gradient mode (gW != null, data parallel): the weight / bias GRADIENTS are stored whole
  // into gW / gb (the flat gradient, all-reduced before the optimizer) instead of updating
  float* gW; float* gb;
  int cs;                   // column blocks per row group (> 1: partial hand-off)
  float* part;              // [groups * cs][DU_PART] input-gradient partials (write-through)
  unsigned* cnt;            // [groups] arrival tickets (zero between launches)
  // head epilogue (the LAST dense layer of the fused program; head_row_kernel ran before):
  // this layer's OUTPUT is the head input hy [M][N]; the block reduces the head's weight
  // gradient for its share of the N features, one block the bias gradient and metrics
  const float* hy;          // [M][N] (null: no head epilogue)
  const float* hdl;         // [M][10] dlogits (scaled)
  float* hgw; float* hgb;   // dWh [N][10], dbh [10] (plain stores into the flat gradient)
  const float* hrl; const int* hrc;   // [M] per-row loss / correct
  float* ring_loss; int* ring_correct; int ring; float ldiv;
  int hact; float halpha;   // the head's input transform: the head reads act(hy)
  // head parameters updated IN PLACE by the epilogue (round 5, the pair-backward tail
  // program: no flat optimizer launch) instead of storing dWh / dbh into hgw / hgb
  float* hw; float* hb; float* hs0w; float* hs1w; float* hs0b; float* hs1b;
};

constexpr int DU_HNC = 10;           // head classes

// Weight-gradient + update segments recorded by csa_dense_update_defer (host state of the
// calling thread, like the deterministic flag) until a carrying launch consumes them.
constexpr int DU_MAXDEF = 4;
struct DUDeferred {
  DUArgs seg[DU_MAXDEF];
  int blocks[DU_MAXDEF];    // workgroups of each segment (128-column, 256-thread)
  int n = 0;
  int head = -1;            // segment carrying the head epilogue (-1: none)
};
extern thread_local DUDeferred g_du_def;

// The segments one carrying launch runs: segment s = extra blocks [start[s], start[s + 1]).
struct DUSegs {
  DUArgs seg[DU_MAXDEF];
  int start[DU_MAXDEF + 1];
  int nseg, head;
};
// Host: move the deferred segments into `out` (order kept); returns their count.
int du_take(DUSegs& out);
// Host: the segments as standalone update-only launches.
int du_flush_segs(const DUSegs& u, hipStream_t st);
}  // namespace csa
extern "C" int csa_dense_update_flush(hipStream_t st);
namespace csa {


// diagnostics: s_memrealtime stamps (100 MHz, one clock for all XCDs) of EVERY block,
// [block][16] = start, dY staged, W landed, MFMA + update done, fold done, dX stored, end
// (update-only bodies: 4 / 5 / 7 / 8 stamp the column halves)
// (scripts/microbench.py MB_DU)
static __constant__ long long* g_du_dbg = nullptr;   // (per code object)
#define DU_STAMP(i)                                                                          \
  do {                                                                                       \
    if (g_du_dbg && threadIdx.x == 0) g_du_dbg[bid * 16 + (i)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)

__host__ __device__ constexpr int du_nb(int waves) { return 32 * waves; }      // columns per block
// The input-gradient fold in LDS: [wave][t][q] blocks of DU_FT features x 4 rows, each
// feature's 4 rows at stride DU_FOLD_FS = 5 (not 4): the item threads' reads (feature
// quads 16 floats apart, q blocks 64 apart with stride 4) hit 8 banks 4-8 times over;
// with the odd stride both the writes and the reads are conflict-free (32 or 64 banks)
constexpr int DU_FOLD_FS = 5, DU_FOLD_BLK = DU_FT * DU_FOLD_FS;
// Update-only (carried) body, 4 waves: the two 64-column dY halves land in LDS straight from
// global memory (global_load_lds_dwordx4: no staging registers), each as [M4][64] with the
// column quads of row r rotated by r (the bank spread the +4 row padding gave the register
// path: a wave's LDS-DMA writes 1 KB contiguous, 4 rows); then the Xw slice [64][16], whose
// space the head epilogue reuses ([64][DU_HMAXR] | [64][10]).  M = 50: 31.2 KB, so the
// carrying launch fits 5 workgroups per CU (round 6).
__host__ __device__ constexpr int du_upo_hw_floats() { return 64 * (8 + 10); }
__host__ __device__ inline size_t du_upo_lds_floats(int M) {
  const size_t m4 = (size_t)((M + 3) & ~3);
  const size_t tail = 1024 > du_upo_hw_floats() ? 1024 : du_upo_hw_floats();
  return 2 * m4 * 64 + tail;
}
__host__ __device__ inline size_t du_lds_floats(int M, int waves) {
  const size_t a = (size_t)M * (du_nb(waves) + 4), b = (size_t)waves * 4 * 4 * DU_FOLD_BLK;   // dY | the fold
  return (a > b ? a : b) + DU_MAXM * DU_FT + 6 * MAXC_DU + 4;
}

__device__ __forceinline__ du_u32x4 du_bits(float4 v) { du_u32x4 u; __builtin_memcpy(&u, &v, 16); return u; }
__device__ __forceinline__ float4 du_f4(du_u32x4 u) { float4 v; __builtin_memcpy(&v, &u, 16); return v; }

// Write back the updated W / slot float4s of a lane's sub-tiles (rows < nf, columns < N)
// and the wave's first bias column.
template <int NSLOT>
__device__ __forceinline__ void du_store_w(const DUArgs& a, const float4 (&wv)[DU_SUB], const float4 (&s0v)[DU_SUB],
                                           const float4 (&s1v)[DU_SUB], const long (&wofs)[DU_SUB],
                                           const bool (&sok)[DU_SUB], int i, int nf, bool bown, int bn0, float bw,
                                           float bs0, float bs1) {
  if (bown && (threadIdx.x & 63) == 0) {
    (a.gW ? a.gb : a.bias)[bn0] = bw;
    if (NSLOT >= 1) a.s0b[bn0] = bs0;
    if (NSLOT >= 2) a.s1b[bn0] = bs1;
  }
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    if (!sok[j] || i >= nf) continue;
    *reinterpret_cast<float4*>((a.gW ? a.gW : a.W) + wofs[j]) = wv[j];
    if (NSLOT >= 1) *reinterpret_cast<float4*>(a.s0w + wofs[j]) = s0v[j];
    if (NSLOT >= 2) *reinterpret_cast<float4*>(a.s1w + wofs[j]) = s1v[j];
  }
}

// NSLOT = optimizer slots (0 SGD, 1 Adagrad, 2 Adam / Adadelta): unused slot registers
// are not allocated.  WAVES = 16 (one block per row group, all N <= 512 columns) or 4
// (128 columns per block, cs blocks per row group: narrow layers use more CUs).
// Head epilogue.  Block (row group grp, column block cblk) owns the dWh rows
// n in [hn0, hn0 + nh) of its column block (nh = ceil(nb / groups)).  Its operands are tiny
// — hy[:, hn0 .. hn0 + nh) (M x nh, contiguous per row) and all of dl (M x 10) — and are
// requested right after the layer's own loads (vmcnt retires in order), staged to LDS at
// the end, then one thread per (n, j) output sums the batch in fixed order.
constexpr int DU_HMAXR = 8;          // staged dWh rows per block (more: direct global loop)

struct DUHead {
  int hn0, nh;
  float hy[2];             // staged hy elements e = t + u THREADS: m = e / 8, r = e % 8 (e < 8 M)
  float dl[3];             // dl elements t + u THREADS (M * 10 <= 640 <= 3 * 256)
};

template <int THREADS>
__device__ __forceinline__ void du_head_prefetch(const DUArgs& a, int grp, int groups, int cb, int nb, DUHead& h) {
  const int hper = (nb + groups - 1) / groups;
  h.hn0 = cb + grp * hper;
  h.nh = max(0, min(hper, cb + nb - h.hn0));
  const int t = threadIdx.x;
#pragma unroll
  for (int u = 0; u < 2; ++u) {                 // 8 M <= 512 <= 2 THREADS
    const int e = t + u * THREADS, m = e / DU_HMAXR, r = e % DU_HMAXR;
    h.hy[u] = a.hy[(long)min(m, a.M - 1) * a.N + min(h.hn0 + min(r, max(h.nh - 1, 0)), a.N - 1)];
  }
  const int n10 = a.M * DU_HNC;
#pragma unroll
  for (int u = 0; u < 3; ++u) h.dl[u] = a.hdl[min(t + u * THREADS, n10 - 1)];
}

template <int THREADS>
__device__ __forceinline__ void du_head_finish(const DUArgs& a, DUHead& h, float* s_hw, bool last_block) {
  // s_hw: [64][DU_HMAXR] act(hy) | [64][10] dl
  const int t = threadIdx.x, M = a.M;
  float* s_y = s_hw;
  float* s_d = s_hw + 64 * DU_HMAXR;
  pin(h.hy[0]); pin(h.hy[1]); pin(h.dl[0]); pin(h.dl[1]); pin(h.dl[2]);
  if (t < M * DU_HMAXR) s_y[t] = act_fwd(h.hy[0], a.hact, a.halpha);
  if (t + THREADS < M * DU_HMAXR) s_y[t + THREADS] = act_fwd(h.hy[1], a.hact, a.halpha);
#pragma unroll
  for (int u = 0; u < 3; ++u)
    if (t + u * THREADS < M * DU_HNC) s_d[t + u * THREADS] = h.dl[u];
  __syncthreads();
  const int outs = h.nh * DU_HNC;
  for (int o = t; o < outs; o += THREADS) {
    const int rr = o / DU_HNC, j = o - rr * DU_HNC, n = h.hn0 + rr;
    float v = 0.f;
    if (h.nh <= DU_HMAXR) {
      for (int m = 0; m < M; ++m) v = fmaf(s_y[m * DU_HMAXR + rr], s_d[m * DU_HNC + j], v);
    } else {
      for (int m = 0; m < M; ++m) v = fmaf(act_fwd(a.hy[(long)m * a.N + n], a.hact, a.halpha), s_d[m * DU_HNC + j], v);
    }
    if (a.hw) {                                            // in-place update (shared rule)
      const long k = (long)n * DU_HNC + j;
      float w = a.hw[k], z0 = a.hs0w ? a.hs0w[k] : 0.f, z1 = a.hs1w ? a.hs1w[k] : 0.f;
      opt_update(a.opt, opt_step_lr(a.opt, a.lr, a.step), w, v, z0, z1);
      a.hw[k] = w;
      if (a.hs0w) a.hs0w[k] = z0;
      if (a.hs1w) a.hs1w[k] = z1;
    } else {
      a.hgw[(long)n * DU_HNC + j] = v;
    }
  }
  if (last_block) {                                        // dbh and the step's metrics
    const int lane = t & 63, w = t >> 6;
    if (w == 0) {
      if (lane < DU_HNC) {
        float v = 0.f;
        for (int m = 0; m < M; ++m) v += s_d[m * DU_HNC + lane];
        if (a.hb) {
          float wb = a.hb[lane], z0 = a.hs0b ? a.hs0b[lane] : 0.f, z1 = a.hs1b ? a.hs1b[lane] : 0.f;
          opt_update(a.opt, opt_step_lr(a.opt, a.lr, a.step), wb, v, z0, z1);
          a.hb[lane] = wb;
          if (a.hs0b) a.hs0b[lane] = z0;
          if (a.hs1b) a.hs1b[lane] = z1;
        } else {
          a.hgb[lane] = v;
        }
      }
    } else if (w == 1) {
      float l = lane < M ? a.hrl[lane] : 0.f;
      float c = lane < M ? (float)a.hrc[lane] : 0.f;
      l = wave_sum(l);
      c = wave_sum(c);
      if (lane == 0) {
        const int pos = (int)((*a.step - 1) % a.ring);    // the head advanced the counter
        a.ring_loss[pos] = l / a.ldiv;
        a.ring_correct[pos] = (int)(c + 0.5f);
      }
    }
  }
}

// One workgroup's work: ``bid`` in [0, nblk) is its index in this layer's grid (a launch
// that carries the layer beside other work passes its own offset-free numbering).
// DGO (dgrad only): the input gradient + transform backward + BN statistics alone — no
// weight gradient, no update, no parameter stores (the update runs later in a launch that
// carries du_body<.., false> workgroups with dX = null beside other work).
// UPO (update only, dX must be null): the carried form — no input-gradient code at all, so
// the registers of the carrying launch stay low.
template <int NSLOT, int WAVES, bool HEAD, bool DGO = false, bool UPO = false>
__device__ __forceinline__ void du_body(const DUArgs& a, const int bid, const int nblk, float* smem) {
  constexpr int THREADS = 64 * WAVES, NB = du_nb(WAVES), SN = NB + 4, HW = 16 * WAVES;
  const int M = a.M, K = a.K, N = a.N, cs = a.cs;
  static_assert(!UPO || WAVES == 4, "the update-only body is the 4-wave carried form");
  float* sdy = smem;                                       // [M][SN] dY columns of the block, later the fold
  float* s_bn = smem + du_lds_floats(M, WAVES) - 6 * MAXC_DU - 4;   // [mean | rstd | a | b] x MAXC_DU
  const int M4 = (M + 3) & ~3;                             // UPO: rows of one DMA'd dY half
  // [64 m][16 f] Xw slice, later BN partials (UPO: after the two dY halves, later s_hw)
  float* sxw = UPO ? smem + 2 * M4 * 64 : s_bn - DU_MAXM * DU_FT;
  float* s_st = s_bn + 4 * MAXC_DU;                        // [2][MAXC_DU] slab-reduction scratch
  int* s_flag = reinterpret_cast<int*>(s_st + 2 * MAXC_DU);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 15, q = lane >> 4;
  const int grp = bid / cs, cblk = bid - grp * cs;
  const int f0 = grp * DU_FT, nf = min(DU_FT, K - f0);
  const int cb = cblk * NB, nb = min(NB, N - cb);          // the block's columns [cb, cb + nb)
  const int groups = nblk / cs;
  const bool dgrad = !UPO && a.dX != nullptr;
  const bool tf = dgrad && (a.act != ACT_NONE || a.bn_on);
  const bool tabs = a.bn_on && a.bn_tab;
  const int C = a.bn.C > 0 ? a.bn.C : 1;
  constexpr int nslot = NSLOT;
  DU_STAMP(0);
  float* s_hw;
  if constexpr (UPO) {
    s_hw = sxw;                                            // dead after the j = 1 barrier
  } else {
    __shared__ float s_hw_st[HEAD ? 64 * (DU_HMAXR + DU_HNC) : 1];
    s_hw = s_hw_st;
  }
  DUHead hd;

  // ---- every load, issued in the order it is consumed (vmcnt retires in order).  Two
  // column halves: half j = block columns [HW j, HW (j + 1)) = every wave's sub-tile j, so
  // the MFMAs of half 0 run while half 1's dY and W are still in flight.
  // (0) the weight-gradient operand slice Xw[m][f0 .. f0+15], 16 m-rows per 256 threads
  float xw1[1024 / THREADS];
#pragma unroll
  for (int u = 0; u < 1024 / THREADS; ++u) {
    const int e = u * THREADS + tid;
    if (!DGO) xw1[u] = a.Xw[(long)min(e >> 4, M - 1) * K + f0 + min(e & 15, nf - 1)];
  }
  // (0b) BN tables -> LDS (4C <= 512 values)
  const float* tsrc = tabs ? a.bn_tab : a.Xw;               // address select: unconditional loads
  float tv[512 / THREADS > 0 ? 512 / THREADS : 1];
  constexpr int NTV = UPO ? 0 : (512 / THREADS > 0 ? 512 / THREADS : 1);   // (UPO: no BN)
#pragma unroll
  for (int u = 0; u < NTV; ++u) {
    const int e = u * THREADS + tid;
    tv[u] = tsrc[tabs && e < 4 * C ? e : 0];
  }
  const int n4 = N >> 2;
  int h4[DU_SUB];
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) h4[j] = max(min(nb - HW * j, HW), 0) >> 2;
  const float* b0 = nslot >= 1 ? a.s0w : a.W;
  const float* b1 = nslot >= 2 ? a.s1w : a.W;
  const int frow = f0 + min(i, nf - 1);
  float4 dyv[DU_SUB][4], wv[DU_SUB], s0v[DU_SUB], s1v[DU_SUB];
  long wofs[DU_SUB];
  bool sok[DU_SUB];
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    if constexpr (UPO) {
      // (1') dY half j straight into LDS: chunk c = 4 rows x 16 quads (one wave instruction);
      // lane l writes LDS quad p = l & 15 of row r = 4c + l / 16, which holds column quad
      // (p - r) & 15.  Chunks wave + 4u; a wave past the last chunk re-loads the last one
      // (identical bytes to identical addresses).  Rows >= M: clamped, never read as data.
      const int nch = M4 >> 2;
#pragma unroll
      for (int u = 0; u < DU_MAXM / 16; ++u) {
        const int c = min(wave + 4 * u, nch - 1);
        const int r = 4 * c + (lane >> 4), cq = ((lane & 15) - r) & 15;
        const float* src = a.dY + (long)min(r, M - 1) * N + cb + HW * j + 4 * cq;
        __builtin_amdgcn_global_load_lds(src, sdy + (j * M4 + 4 * c) * 64, 16, 0, 0);
      }
    } else {
    // (1) dY half j: float4 e = u * THREADS + tid -> row e / h4, block column HW j + 4 (e % h4)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * THREADS + tid;
      int row = 0, c4 = 0;
      if (h4[j] == HW / 4) { row = e / (HW / 4); c4 = e % (HW / 4); }
      else if (h4[j] > 0) { row = e / h4[j]; c4 = e - row * h4[j]; }
      dyv[j][u] = reinterpret_cast<const float4*>(a.dY)[min(row, M - 1) * n4 + (h4[j] > 0 ? (cb + HW * j) / 4 + c4 : 0)];
    }
    }
    // (2) W and slot float4s of sub-tile j
    const int lc = 16 * (wave + WAVES * j);                 // block-local first column
    sok[j] = lc < nb;
    wofs[j] = (long)frow * N + cb + min(lc, nb - 16) + 4 * q;
    wv[j] = *reinterpret_cast<const float4*>(a.W + wofs[j]);
    s0v[j] = s1v[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (nslot >= 1) s0v[j] = *reinterpret_cast<const float4*>(b0 + wofs[j]);
    if (nslot >= 2) s1v[j] = *reinterpret_cast<const float4*>(b1 + wofs[j]);
  }
  // (3) bias: the block's columns are spread over the row groups, one per wave (+WAVES r);
  //     the first column's operands prefetched (unconditional loads from selected
  //     addresses: a load inside a branch is waited for right there, and vmcnt is in order)
  const int bper = (nb + groups - 1) / groups;
  const int bn0 = cb + grp * bper + wave;
  const bool bown = !DGO && (a.bias || a.gW) && wave < bper && grp * bper + wave < nb;
  const int bnc = bown ? bn0 : 0;
  float bw = (a.bias ? a.bias : a.dY)[bnc];
  float bs0 = (nslot >= 1 && a.bias ? a.s0b : a.dY)[bnc];
  float bs1 = (nslot >= 2 && a.bias ? a.s1b : a.dY)[bnc];
  // (4) epilogue operands: item it = tid < 256 -> batch row em = it / 4, features 4 (it % 4) ..
  const int em = tid >> 2, fq = 4 * (tid & 3);
  const bool eitem = tid < 256;
  const float* xsrc = tf && a.x_fwd ? a.x_fwd : a.Xw;      // address select (same [M][K] shape)
  float4 xf = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!UPO) xf = *reinterpret_cast<const float4*>(xsrc + (long)min(em, M - 1) * K + f0 + min(fq, nf - 4));
  // (5) head epilogue operands (last dense layer only)
  if (HEAD) du_head_prefetch<THREADS>(a, grp, groups, cb, nb, hd);

  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  du_f32x4 dacc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dacc[t] = du_f32x4{0.f, 0.f, 0.f, 0.f};
  float xb[DU_KS];                                         // weight-gradient B: Xw[4s + q][f0 + i]
#pragma unroll
  for (int j = 0; j < DU_SUB; ++j) {
    if (j == 0) {
#pragma unroll
      for (int u = 0; u < 1024 / THREADS; ++u) {
        if (DGO) break;
        const int e = u * THREADS + tid;
        pin(xw1[u]);
        sxw[e] = ((e >> 4) < M && (e & 15) < nf) ? xw1[u] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < NTV; ++u) {
        const int e = u * THREADS + tid;
        pin(tv[u]);
        if (tabs && e < 4 * C) s_bn[(e / C) * MAXC_DU + e % C] = tv[u];
      }
    }
    // stage dY half j (rows < M only: dgrad rows >= M are clamped reads whose outputs are
    // dropped, wgrad rows >= M meet Xw = 0); its columns are disjoint from half 0's, which
    // other waves may still be reading.  (UPO: already in LDS; the compiler waits for the
    // LDS-DMA before the barrier below.)
    if constexpr (!UPO) {
#pragma unroll
    for (int u = 0; u < 4; ++u) pin(dyv[j][u]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = u * THREADS + tid;
      if (h4[j] > 0 && e < M * h4[j]) {
        const int row = h4[j] == HW / 4 ? e / (HW / 4) : e / h4[j];
        const int c4 = e - row * h4[j];
        *reinterpret_cast<float4*>(sdy + row * SN + HW * j + 4 * c4) = dyv[j][u];
      }
    }
    }
    if (j == 0 && a.bn_on && dgrad && !tabs)              // no precomputed tables: reduce here
      bn_reduce_to_lds(a.bn, s_bn, s_bn + MAXC_DU, s_bn + 2 * MAXC_DU, s_bn + 3 * MAXC_DU, s_st);
    __syncthreads();
    if (UPO && j == 1) DU_STAMP(4);                        // (update-only: stamps 4 / 5 are free)
    if (j == 0) {
      DU_STAMP(1);
#pragma unroll
      for (int s = 0; s < DU_KS; ++s) xb[s] = DGO ? 0.f : sxw[(4 * s + q) * DU_FT + i];
    }
    pin(wv[j]); pin(s0v[j]); pin(s1v[j]);
    if (j == 0) DU_STAMP(2);
    if (UPO && j == 1) DU_STAMP(5);
    if (!sok[j]) continue;                                 // wave-uniform
    const int n0 = 16 * (wave + WAVES * j);                // block-local
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
    if (DGO) continue;
    // weight gradient: A = dY[4s + q][n0 + i] (LDS), two accumulators
    // every k-step's A operand is read before the first MFMA (one LDS round trip instead of
    // one per step: an early exit at M would keep the reads behind it).  Steps past the
    // batch read a clamped row and meet Xw = 0 (the slice is zero-filled), adding nothing.
    du_f32x4 g0 = du_f32x4{0.f, 0.f, 0.f, 0.f}, g1 = g0;
    const float* col = sdy + n0 + i;
    float av[DU_KS];
    if constexpr (UPO) {
      // rotated half: column lc = 16 wave + i of half j, row r at quad ((lc >> 2) + r) & 15
      const float* hb = sdy + j * M4 * 64;
      const int lc = 16 * wave + i;
#pragma unroll
      for (int s = 0; s < DU_KS; ++s) {
        const int r = min(4 * s + q, M - 1);
        av[s] = hb[r * 64 + ((((lc >> 2) + r) & 15) << 2) + (lc & 3)];
      }
    } else {
#pragma unroll
      for (int s = 0; s < DU_KS; ++s) av[s] = col[min(4 * s + q, M - 1) * SN];
    }
#pragma unroll
    for (int s = 0; s < DU_KS; s += 2) {
      g0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], xb[s], g0, 0, 0, 0);
      g1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s + 1], xb[s + 1], g1, 0, 0, 0);
    }
    // optimizer update of the lane's 4 weights (D lane (i, q) = dW[f0 + i][n0 + 4q + r]);
    // written back late: a store in flight would hold the next barrier (the compiler drains
    // vmcnt before it) for the whole write-back
    float w[4] = {wv[j].x, wv[j].y, wv[j].z, wv[j].w};
    float s0[4] = {s0v[j].x, s0v[j].y, s0v[j].z, s0v[j].w};
    float s1[4] = {s1v[j].x, s1v[j].y, s1v[j].z, s1v[j].w};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (a.gW) w[r] = (g0[r] + g1[r]) * a.scale;          // gradient mode: the store below writes dW
      else opt_update(a.opt, lr, w[r], (g0[r] + g1[r]) * a.scale, s0[r], s1[r]);
    }
    wv[j] = make_float4(w[0], w[1], w[2], w[3]);
    s0v[j] = make_float4(s0[0], s0[1], s0[2], s0[3]);
    s1v[j] = make_float4(s1[0], s1[1], s1[2], s1[3]);
    if (UPO && j == 0) DU_STAMP(7);
    if (UPO && j == 1) DU_STAMP(8);
  }
  pin(bw); pin(bs0); pin(bs1); pin(xf);
  // bias: column sums of dY over the batch, one column per wave (prefetched operands)
  if (bown) {
    for (int u = wave; u < bper; u += WAVES) {
      const int lcol = grp * bper + u;
      if (lcol >= nb) break;
      const int n = cb + lcol;
      float v;
      if constexpr (UPO) {
        const int lh = lcol & 63;
        v = lane < M ? sdy[((lcol >> 6) * M4 + lane) * 64 + ((((lh >> 2) + lane) & 15) << 2) + (lh & 3)] : 0.f;
      } else {
        v = lane < M ? sdy[lane * SN + lcol] : 0.f;
      }
      v = wave_sum(v);
      if (lane == 0) {
        if (u == wave) {                                   // the prefetched first column,
          if (a.gW) bw = v * a.scale;                      // stored late (du_store_w)
          else opt_update(a.opt, lr, bw, v * a.scale, bs0, bs1);
        } else {                                           // further columns (bper > WAVES):
          float cw = 0.f, c0 = 0.f, c1 = 0.f;              // their own registers — the first
          if (!a.gW) {                                     // column's values must survive
            cw = a.bias[n];
            if (nslot >= 1) c0 = a.s0b[n];
            if (nslot >= 2) c1 = a.s1b[n];
          }
          if (a.gW) cw = v * a.scale;
          else opt_update(a.opt, lr, cw, v * a.scale, c0, c1);
          (a.gW ? a.gb : a.bias)[n] = cw;
          if (nslot >= 1) a.s0b[n] = c0;
          if (nslot >= 2) a.s1b[n] = c1;
        }
      }
    }
  }
  DU_STAMP(3);
  if (HEAD) du_head_finish<THREADS>(a, hd, s_hw, bid == nblk - 1);
  if (!dgrad) {                                            // uniform: first layer
    if (!DGO) du_store_w<NSLOT>(a, wv, s0v, s1v, wofs, sok, i, nf, bown, bn0, bw, bs0, bs1);
    DU_STAMP(6);
    return;
  }

  // ---- fold the waves' partials.  Layout [wave][t][q][i][r] (feature stride DU_FOLD_FS):
  // lane (i, q) of tile t holds rows 16t + 4q + r of feature i
  __syncthreads();                                         // every dY read is done
  float* fold = sdy;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    if (16 * t >= M) break;
    float* dst = fold + ((wave * 4 + t) * 4 + q) * DU_FOLD_BLK + DU_FOLD_FS * i;
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[r] = dacc[t][r];
  }
  __syncthreads();
  DU_STAMP(4);
  // item (em, fq): the block's partial of dX[em][f0 + fq .. +3], waves summed in order
  float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f);
  if (eitem && em < M) {
    const int t = em >> 4, qq = (em >> 2) & 3, r = em & 3;
    const float* src = fold + (t * 4 + qq) * DU_FOLD_BLK + DU_FOLD_FS * fq + r;
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
      const float* p = src + w * 4 * 4 * DU_FOLD_BLK;
      g4.x += p[0]; g4.y += p[DU_FOLD_FS]; g4.z += p[2 * DU_FOLD_FS]; g4.w += p[3 * DU_FOLD_FS];
    }
  }
  if (cs > 1) {
    // publish write-through (sc1), drain, one agent-scope ticket per block; the row
    // group's last arriving block sums the cs partials in column-block order
    const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
        a.part, 0, (int)((size_t)nblk * DU_PART * sizeof(float)), 0x00020000);
    if (eitem && em < M)
      __builtin_amdgcn_raw_buffer_store_b128(du_bits(g4), prs, (int)(((size_t)bid * DU_PART + em * DU_FT + fq) * 4), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // every storing wave drains
    __syncthreads();
    if (tid == 0) {
      const unsigned old = __hip_atomic_fetch_add(a.cnt + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(cs - 1);
      if (last) __hip_atomic_store(a.cnt + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // next launch
      *s_flag = last;
    }
    __syncthreads();
    if (!DGO) du_store_w<NSLOT>(a, wv, s0v, s1v, wofs, sok, i, nf, bown, bn0, bw, bs0, bs1);
    if (!*s_flag) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler-only: loads stay below
    g4 = make_float4(0.f, 0.f, 0.f, 0.f);
    if (eitem && em < M) {
      float4 v[8];
      for (int c0 = 0; c0 < cs; c0 += 8) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = du_f4(__builtin_amdgcn_raw_buffer_load_b128(
              prs, (int)((((size_t)grp * cs + min(c0 + u, cs - 1)) * DU_PART + em * DU_FT + fq) * 4), 0, 16));
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (c0 + u < cs) { g4.x += v[u].x; g4.y += v[u].y; g4.z += v[u].z; g4.w += v[u].w; }
      }
    }
  } else {
    if (!DGO) du_store_w<NSLOT>(a, wv, s0v, s1v, wofs, sok, i, nf, bown, bn0, bw, bs0, bs1);
  }
  // ---- transform backward (activation; BN statistics), dX
  float v1[4] = {0.f, 0.f, 0.f, 0.f}, v2[4] = {0.f, 0.f, 0.f, 0.f};
  if (eitem && em < M && fq < nf) {
    float g[4] = {g4.x, g4.y, g4.z, g4.w};
    const float x[4] = {xf.x, xf.y, xf.z, xf.w};
    if (tf) {
      int ch = (f0 + fq) % C;                             // one division, then wrap
#pragma unroll
      for (int r = 0; r < 4; ++r, ch = (ch + 1 == C) ? 0 : ch + 1) {
        const float z = a.bn_on ? x[r] * s_bn[2 * MAXC_DU + ch] + s_bn[3 * MAXC_DU + ch] : x[r];
        const float y = act_fwd(z, a.act, a.alpha);
        g[r] = act_bwd(g[r], z, y, a.act, a.alpha);
        v1[r] = g[r];
        v2[r] = a.bn_on ? g[r] * (x[r] - s_bn[ch]) * s_bn[MAXC_DU + ch] : 0.f;
      }
    }
    out_store4(a.dX + (long)em * K + f0 + fq, make_float4(g[0], g[1], g[2], g[3]));
  }
  DU_STAMP(5);
  if (a.bn_on && a.bwd_slab) {
    // BN-backward statistics per feature in fixed order: the wave's 16 rows by shuffles
    // (lanes l, l ^ 4, .. share a feature quad), the 4 item waves through LDS, then one
    // atomic per (feature, statistic) into one of DU_SLAB rows (zeroed every step by the
    // optimizer launch)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) {
        v1[r] += __shfl_xor(v1[r], o, 64);
        v2[r] += __shfl_xor(v2[r], o, 64);
      }
    }
    float* sred = sxw;                                     // [4 item waves][2][16]
    if (eitem && lane < 4) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        sred[wave * 32 + 4 * lane + r] = v1[r];
        sred[wave * 32 + 16 + 4 * lane + r] = v2[r];
      }
    }
    __syncthreads();
    if (a.det) {
      // the group's whole row [2][C], features of one channel summed in feature order
      if (tid < 2 * C) {
        const int st = tid / C, c = tid - st * C;
        float acc = 0.f;
        for (int ff = 0; ff < nf; ++ff)
          if ((f0 + ff) % C == c) {
            const int e = 16 * st + ff;
            acc += sred[e] + sred[32 + e] + sred[64 + e] + sred[96 + e];
          }
        a.bwd_slab[(size_t)grp * 2 * C + tid] = acc;
      }
    } else if (tid < 32 && (tid & 15) < nf) {
      const float acc = sred[tid] + sred[32 + tid] + sred[64 + tid] + sred[96 + tid];
      const int st = tid >> 4, c = (f0 + (tid & 15)) % C;
      atomicAdd(a.bwd_slab + (size_t)(grp % DU_SLAB) * 2 * C + st * C + c, acc);
    }
  }
  DU_STAMP(6);
}

// Extra block e of a carrying launch: the update-only body of its deferred segment
// (HEADOK = false: the carrier never holds the head segment, its code is not compiled in).
// (Measured round 4: fc1's segment riding in the optimizer launch instead ran 0.0906-0.0911
// ms/step against 0.0885-0.0887 in the pair backward — profiles/r4_notes.md.)
template <int NSLOT, bool HEADOK>
__device__ __forceinline__ void du_segs_body(const DUSegs& u, int e, float* smem) {
  int s = 0;
#pragma unroll
  for (int k = 1; k < DU_MAXDEF; ++k) s += (k < u.nseg && e >= u.start[k]) ? 1 : 0;
  const DUArgs& d = u.seg[s];
  const int lb = e - u.start[s], nb = u.start[s + 1] - u.start[s];
  if (HEADOK && s == u.head) du_body<NSLOT, 4, true, false, true>(d, lb, nb, smem);
  else du_body<NSLOT, 4, false, false, true>(d, lb, nb, smem);
}

}  // namespace csa
