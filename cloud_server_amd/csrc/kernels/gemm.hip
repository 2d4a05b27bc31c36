// f32 MFMA GEMM family for the digit-CNN training step (gfx950 / CDNA4).
//
// The dense layers of the reference model (construct_distribute.py:168-182, 252-264) are
// skinny: M = per-GPU batch (50), N and K in the hundreds/thousands.  A square-tile library
// GEMM leaves most of the chip idle on such shapes (hipBLASLt took 7-17 µs per call in
// profiles/r1_torch_baseline.md).  This kernel instead:
//   * uses the exact-f32 MFMA v_mfma_f32_32x32x2_f32 (one 32x32 accumulator per wave),
//   * splits K across the 4 waves of a workgroup (WK) and across workgroups (split-K),
//     so every shape launches ~1000 waves (one per SIMD) even at M = 50,
//   * builds operands through loader functors: row-major, transposed and a fused
//     BatchNorm-apply + activation prologue (conv weight gradients moved to a direct
//     reduction kernel in conv.hip),
//   * ends in epilogue functors: store, split-K atomic add, bias, and the fused
//     activation-backward + BatchNorm-backward partial statistics.
//
// MFMA 32x32x2 f32 operand map (cdna_hip_programming.md §3):
//   A: lane l holds A[i = l&31][k = l>>5];  B: lane l holds B[k = l>>5][j = l&31]
//   D: reg r of lane l is D[row = (r&3) + 8*(r>>2) + 4*(l>>5)][col = l&31]
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace csa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KC = 64;        // K chunk staged per iteration (32 MFMAs); most waves need 1-2
constexpr int LDS_PAD = 33;   // row stride of the 32-wide staging tiles (conflict-free)
constexpr int MAXC = 128;     // max BatchNorm channels handled in LDS
constexpr int BN_SLAB_ROWS = 16;   // BN-backward slab rows (atomically folded)

// LDS tables shared by loaders/epilogues: [mean | rstd | a | b] x MAXC
struct BNTables { const float *mean, *rstd, *a, *b; };

// ----------------------------------------------------------------------------------
// Loaders: element (r, c) with r the "outer" index (m for A, n for B), c the K index.
// Split in two so the staging loop stays branch-free around memory:
//   raw(r, c)      -> issues ONE load from a clamped address (no branch around it),
//   post(v, r, c)  -> validity select + transform (BN-apply, activation, /255) applied
//                     when the chunk is committed to LDS, i.e. after the loads of the
//                     whole chunk are in flight (hipcc otherwise waits vmcnt(0) per load).
// KCONTIG says whether consecutive K are contiguous in memory (picks the lane mapping).
// ----------------------------------------------------------------------------------
template <bool V4 = false>
struct LoadRowMajor {          // elem(r, c) = p[r * ld + c]
  const float* p; long ld; int rows, cols;
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC4 = V4;   // ld % 4 == 0 && cols % 4 == 0 (launcher checks)
  __device__ float4 raw4(int r, int c) const {   // (r, c..c+3), c % 4 == 0
    const int rr = r < rows ? r : 0;
    const int cc = min(c, cols - 4);
    return *reinterpret_cast<const float4*>(p + (long)rr * ld + cc);
  }
  __device__ void bind(const BNTables&) {}
  __device__ float raw(int r, int c) const {
    const bool ok = r < rows && c < cols;
    return p[ok ? (long)r * ld + c : 0];
  }
  __device__ float post(float v, int r, int c) const { return (r < rows && c < cols) ? v : 0.f; }
};

// ONES: row r == rows reads as 1 (c < cols) — the bias-gradient row of a weight gradient.
template <bool V4 = false, bool ONES = false>
struct LoadColMajor {          // elem(r, c) = p[c * ld + r]
  const float* p; long ld; int rows, cols;
  static constexpr bool KCONTIG = false;
  static constexpr bool VEC4 = V4;   // ld % 4 == 0 && rows % 4 == 0
  __device__ float4 raw4(int r, int c) const {   // (r..r+3, c), r % 4 == 0
    const int rr = min(r, rows - 4);
    const int cc = c < cols ? c : 0;
    return *reinterpret_cast<const float4*>(p + (long)cc * ld + rr);
  }
  __device__ void bind(const BNTables&) {}
  __device__ float raw(int r, int c) const {
    const bool ok = r < rows && c < cols;
    return p[ok ? (long)c * ld + r : 0];
  }
  __device__ float post(float v, int r, int c) const {
    if (ONES && r == rows) return c < cols ? 1.f : 0.f;
    return (r < rows && c < cols) ? v : 0.f;
  }
};

// Activation tensor X[m][f] read through an optional BN-apply (channel = f % C) and act.
// ROWS_ARE_BATCH: elem(r=m, c=f) (dense fwd A);  else elem(r=f, c=m) (dense wgrad A).
// ones_row: for wgrad, row f == feat returns 1 (m < batch) -> bias gradient row.
template <bool ROWS_ARE_BATCH, bool V4 = false>
struct LoadBNAct {
  const float* x; long ld; int batch, feat; FastDiv C; int act; float alpha; int has_bn, ones_row;
  const float* ta; const float* tb;
  static constexpr bool KCONTIG = ROWS_ARE_BATCH;
  static constexpr bool VEC4 = V4;   // ld % 4 == 0 && feat % 4 == 0
  __device__ float4 raw4(int r, int c) const {   // 4 consecutive features of one row m
    int m = ROWS_ARE_BATCH ? r : c, f = ROWS_ARE_BATCH ? c : r;
    m = m < batch ? m : 0;
    f = min(f, feat - 4);
    return *reinterpret_cast<const float4*>(x + (long)m * ld + f);
  }
  __device__ void bind(const BNTables& t) { ta = t.a; tb = t.b; }
  __device__ float raw(int r, int c) const {
    const int m = ROWS_ARE_BATCH ? r : c, f = ROWS_ARE_BATCH ? c : r;
    const bool ok = m < batch && f < feat;
    return x[ok ? (long)m * ld + f : 0];
  }
  __device__ float post(float v, int r, int c) const {
    const int m = ROWS_ARE_BATCH ? r : c, f = ROWS_ARE_BATCH ? c : r;
    if (m >= batch) return 0.f;
    if (f >= feat) return (ones_row && f == feat) ? 1.f : 0.f;
    if (has_bn) { int q, ch; C.divmod(f, q, ch); v = v * ta[ch] + tb[ch]; }
    return act_fwd(v, act, alpha);
  }
};

// ----------------------------------------------------------------------------------
// Epilogues: called once per output element with the fully (intra-WG) reduced value.
// ----------------------------------------------------------------------------------
struct EpiStore {              // C[m][n] (+)= v (+ bias[n] once); row m == M -> extra row
  float* c; long ldc; int M, N; const float* bias; int atomic; float* extra; float scale;
  static constexpr bool NEEDS_LDS = false;
  __device__ void bind(const BNTables&) {}
  // Global operands of the epilogue are fetched for all 16 elements of a lane BEFORE any
  // store/atomic is issued: vmcnt counts loads, stores and atomics in issue order, so a
  // load placed after an atomic waits for that atomic (measured: 16 serial round trips,
  // ~15k cycles per workgroup, when the bias was read inside the store loop).
  __device__ float prefetch(int, int n, bool first_split) const {
    return (bias && first_split) ? bias[n < N ? n : 0] : 0.f;
  }
  __device__ void flush(int, float*) {}
  __device__ void operator()(int m, int n, float v, bool first_split, float*, float aux) const {
    if (n >= N) return;
    float* p;
    if (m < M) p = c + (long)m * ldc + n;
    else if (extra && m == M) p = extra + n;
    else return;
    v *= scale;
    if (bias && first_split && m < M) v += aux;
    if (atomic) atomicAdd(p, v); else *p = v;
  }
};

// Dense/conv dgrad epilogue through the activation (and optional BatchNorm) that formed
// the GEMM's A operand in the forward pass: g = dL/dh with h = act(bn(x)):
//   dz = act'(g); store dz; per-channel {sum dz, sum dz*xhat} into LDS for BN backward.
struct EpiActBNBwd {
  float* dz; long ld; int M, F; FastDiv C; const float* x; int act; float alpha; int has_bn;
  BNTables t;
  static constexpr bool NEEDS_LDS = true;
  __device__ void bind(const BNTables& tt) { t = tt; }
  __device__ float prefetch(int m, int f, bool) const {   // branch-free clamped load
    const bool ok = m < M && f < F;
    return x[ok ? (long)m * ld + f : 0];
  }
  // A lane's 16 elements share one column f (the MFMA D layout varies only the row), so
  // the BN-backward sums are kept in registers and flushed with ONE pair of LDS atomics
  // per lane (per-element LDS float atomics on 20 channels serialised: ~8k cycles).
  float sd = 0.f, sdx = 0.f;
  __device__ void operator()(int m, int f, float g, bool, float*, float xv) {
    if (m >= M || f >= F) return;
    int q, ch;
    C.divmod(f, q, ch);
    float z = has_bn ? xv * t.a[ch] + t.b[ch] : xv;
    float y = act_fwd(z, act, alpha);
    float d = act_bwd(g, z, y, act, alpha);
    dz[(long)m * ld + f] = d;
    if (has_bn) {
      sd += d;
      sdx += d * (xv - t.mean[ch]) * t.rstd[ch];
    }
  }
  __device__ void flush(int f, float* lds_acc) {
    if (!has_bn || f >= F) return;
    int q, ch;
    C.divmod(f, q, ch);
    atomicAdd(&lds_acc[ch], sd);
    atomicAdd(&lds_acc[MAXC + ch], sdx);
  }
};

// ----------------------------------------------------------------------------------
// Per-wave staging of one operand tile (32 outer rows x KC) into LDS [kk][r] (pad 33).
// Scalar path: PER branch-free loads per lane.  VEC4 path: 2 float4 loads per lane
// along the operand's contiguous dimension.  fetch() only issues loads; commit()
// applies validity + transform and writes LDS (after the loads had a chunk to land).
// ----------------------------------------------------------------------------------
template <class L>
struct Stage {
  static constexpr int PER = (32 * KC) / 64;          // elements per lane per chunk
  static constexpr int NV = L::VEC4 ? PER / 4 : PER;  // loads per lane per chunk
  float v[PER];
  int lane;
  // lane/e -> (outer row, k) of load e (compile-time e: pure shifts, no index arrays)
  __device__ __forceinline__ void map(int e, int& ro, int& ko) const {
    const int idx = lane + 64 * e;
    if (L::VEC4) {
      if (L::KCONTIG) { ro = idx / (KC / 4); ko = (idx % (KC / 4)) * 4; }
      else { ko = idx >> 3; ro = (idx & 7) * 4; }
    } else {
      if (L::KCONTIG) { ro = idx / KC; ko = idx % KC; }
      else { ko = idx >> 5; ro = idx & 31; }
    }
  }
  __device__ void init(int l) { lane = l; }
  __device__ void fetch(const L& l, int r0, int k, int ke) {
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      int ro, ko;
      map(e, ro, ko);
      if (L::VEC4) {
        const int kk = L::KCONTIG ? min(k + ko, ke - 4) : min(k + ko, ke - 1);
        const float4 q = l.raw4(r0 + ro, kk);
        v[4 * e] = q.x; v[4 * e + 1] = q.y; v[4 * e + 2] = q.z; v[4 * e + 3] = q.w;
      } else {
        v[e] = l.raw(r0 + ro, min(k + ko, ke - 1));
      }
    }
  }
  __device__ void commit(const L& l, float* dst, int r0, int k, int ke) const {
#pragma unroll
    for (int e = 0; e < NV; ++e) {
      int ro, ko;
      map(e, ro, ko);
      if (L::VEC4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r = L::KCONTIG ? ro : ro + u;
          const int kk = L::KCONTIG ? ko + u : ko;
          dst[kk * LDS_PAD + r] = (k + kk < ke) ? l.post(v[4 * e + u], r0 + r, k + kk) : 0.f;
        }
      } else {
        dst[ko * LDS_PAD + ro] = (k + ko < ke) ? l.post(v[e], r0 + ro, k + ko) : 0.f;
      }
    }
  }
};

// ----------------------------------------------------------------------------------
// The kernel.  Grid: x = N tiles, y = M tiles, z = split-K slices.
// WG tile = (32*WM) x (32*WN); its K slice is split WK ways across the waves.
// ----------------------------------------------------------------------------------
__constant__ long long* g_gemm_dbg = nullptr;   // diagnostics: s_memtime stamps of WG 0
#define GEMM_STAMP(i)                                                                       \
  do {                                                                                      \
    if (g_gemm_dbg && threadIdx.x == 0 && tid.x == 0 && tid.y == 0 && tid.z == 0)              \
      g_gemm_dbg[i] = (long long)__builtin_amdgcn_s_memtime();                               \
  } while (0)

// XCD-aware tile order.  Workgroups are dealt round-robin over the 8 XCDs (block b and
// b + 8 share one L2; MI355X_MICROARCH.md "Workgroup dispatch"), so with the natural order
// the 16 N-tiles that re-read one split-K slice of the activations, and the 2 M-tiles that
// re-read one weight tile, land on 8 different XCDs and every re-read goes to HBM/MALL.
// The 1-D grid is instead mapped so that XCD x owns a contiguous range of tasks ordered
// (split, N tile, M tile) fastest-last: re-reads hit that XCD's L2.  Speed only — any
// placement is correct.  The grid is padded to a multiple of 8 (padding blocks exit).
struct TileId { int x, y, z; bool valid; };
__device__ __forceinline__ TileId gemm_tile(int X, int Y, int Z, int L, int G) {   // G % 8 == 0
  const int t = (L & 7) * (G >> 3) + (L >> 3);
  TileId id;
  id.valid = t < X * Y * Z;
  id.y = t % Y;
  id.x = (t / Y) % X;
  id.z = t / (X * Y);
  return id;
}

// LDS arena of one GEMM workgroup: per-wave staging tiles (reused for the WK reduction),
// BN tables, epilogue accumulators.  One static array per kernel, passed to the body, so
// a kernel that hosts two GEMM bodies (gemm_pair_kernel) still allocates it once.
constexpr int GEMM_LDS_FLOATS = 4 * 2 * KC * LDS_PAD + 4 * MAXC + 2 * MAXC;

template <int WM, int WN, int WK, class LA, class LB, class EPI>
__device__ __forceinline__ void gemm_body(LA la, LB lb, EPI epi, int M, int N, int K,
                                          int k_per_split, const BNRef& bn, int bn_on,
                                          float* bn_slab_out, int slab_C, int GX, int GY, int GZ,
                                          int bid, int nblk, float* lds, int det = 0) {
  static_assert(WM * WN * WK == 4, "4 waves per workgroup");
  const TileId tid = gemm_tile(GX, GY, GZ, bid, nblk);
  if (!tid.valid) return;                 // whole workgroup: grid padding
  typedef float StageT[2][KC * LDS_PAD];
  StageT* s_stage = reinterpret_cast<StageT*>(lds);
  float* s_bn = lds + 4 * 2 * KC * LDS_PAD;
  float* s_acc = s_bn + 4 * MAXC;

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int wk = wave / (WM * WN), wmn = wave % (WM * WN);
  const int wm = wmn / WN, wn = wmn % WN;
  const int m0 = tid.y * 32 * WM + wm * 32;
  const int n0 = tid.x * 32 * WN + wn * 32;
  GEMM_STAMP(0);
  const BNTables tabs{s_bn, s_bn + MAXC, s_bn + 2 * MAXC, s_bn + 3 * MAXC};
  la.bind(tabs);
  lb.bind(tabs);
  epi.bind(tabs);
  // K range of this wave (multiples of KC keep every wave's chunks aligned)
  const int ks0 = tid.z * k_per_split;
  const int ks1 = min(K, ks0 + k_per_split);
  const int klen = max(0, ks1 - ks0);
  const int kw_len = ((klen + WK - 1) / WK + 3) / 4 * 4;
  const int kb = ks0 + wk * kw_len;
  const int ke = min(ks1, kb + kw_len);

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  float* sa = s_stage[wave][0];
  float* sb = s_stage[wave][1];
  Stage<LA> stA;
  Stage<LB> stB;
  stA.init(lane);
  stB.init(lane);
  GEMM_STAMP(1);
  // first chunk's operand loads go out BEFORE the BN-slab reduction, so the two
  // memory round trips overlap
  if (kb < ke) { stA.fetch(la, m0, kb, ke); stB.fetch(lb, n0, kb, ke); }
  if (bn_on) bn_reduce_to_lds(bn, s_bn, s_bn + MAXC, s_bn + 2 * MAXC, s_bn + 3 * MAXC, s_acc);
  if (EPI::NEEDS_LDS) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * MAXC; i += blockDim.x) s_acc[i] = 0.f;
  }
  __syncthreads();
  int it = 0;
  for (int k = kb; k < ke; k += KC) {
    if (it < 4) GEMM_STAMP(2 + it);
    ++it;
    stA.commit(la, sa, m0, k, ke);
    if (it == 1) GEMM_STAMP(10);
    stB.commit(lb, sb, n0, k, ke);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (it == 1) GEMM_STAMP(11);
    if (k + KC < ke) {   // next chunk's global loads fly under the MFMAs
      stA.fetch(la, m0, k + KC, ke);
      stB.fetch(lb, n0, k + KC, ke);
    }
    // all of the chunk's operand reads are issued before the MFMA chain (read -> MFMA
    // pairs left each MFMA waiting on its own ds_read: ~120 cycles per 64-cycle MFMA)
    float av[KC / 2], bv[KC / 2];
#pragma unroll
    for (int kk = 0; kk < KC; kk += 2) {
      av[kk / 2] = sa[(kk + (lane >> 5)) * LDS_PAD + (lane & 31)];
      bv[kk / 2] = sb[(kk + (lane >> 5)) * LDS_PAD + (lane & 31)];
    }
#pragma unroll
    for (int kk = 0; kk < KC / 2; ++kk) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[kk], bv[kk], acc, 0, 0, 0);
    if (it == 1) GEMM_STAMP(12);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }

  GEMM_STAMP(6);
  // epilogue operands (bias / forward activations) in flight under the WK reduction
  const bool first = tid.z == 0;
  float aux[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
    aux[i] = wk == 0 ? epi.prefetch(m0 + row, n0 + (lane & 31), first) : 0.f;
  }
  GEMM_STAMP(8);
  if (WK > 1) {  // intra-workgroup split-K reduction through LDS (each wave's own stage area)
    float* mine = s_stage[wave][0];
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int i = 0; i < 16; ++i) mine[i * 64 + lane] = acc[i];
    __syncthreads();
    if (wk == 0) {
      for (int s2 = 1; s2 < WK; ++s2) {
        const float* src = s_stage[s2 * (WM * WN) + wmn][0];
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] += src[i * 64 + lane];
      }
    }
  }
  GEMM_STAMP(9);
  if (wk == 0) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      int row = (i & 3) + 8 * (i >> 2) + 4 * (lane >> 5);
      epi(m0 + row, n0 + (lane & 31), acc[i], first, s_acc, aux[i]);
    }
    if (!det) epi.flush(n0 + (lane & 31), s_acc);
  }
  GEMM_STAMP(7);
  if (EPI::NEEDS_LDS && bn_slab_out) {
    if (det) {
      // deterministic mode: no float atomics.  Every lane's {sum dz, sum dz*xhat} goes to
      // LDS (the stage area: every operand / split-K read is behind the barrier), one
      // thread per statistic folds them in (wave, lane) order, and the workgroup writes
      // its OWN slab row (csa_dense_dgrad_slabs: one per workgroup; folded in row order)
      float* s_det = lds;
      __syncthreads();
      if (wk == 0) {
        if constexpr (EPI::NEEDS_LDS) {
          s_det[wmn * 128 + 2 * lane] = epi.sd;
          s_det[wmn * 128 + 2 * lane + 1] = epi.sdx;
        }
      }
      __syncthreads();
      const int slab_row = (tid.z * GY + tid.y) * GX + tid.x;
      for (int i = threadIdx.x; i < 2 * slab_C; i += blockDim.x) {
        const int ch = i < slab_C ? i : i - slab_C, which = i < slab_C ? 0 : 1;
        float v = 0.f;
        for (int w = 0; w < WM * WN; ++w) {
          const int nw = tid.x * 32 * WN + (w % WN) * 32;
          for (int l = 0; l < 64; ++l) {
            const int f = nw + (l & 31);
            if (f < N && f % slab_C == ch) v += s_det[w * 128 + 2 * l + which];
          }
        }
        bn_slab_out[(size_t)slab_row * 2 * slab_C + i] = v;
      }
      return;
    }
    // fold into one of BN_SLAB_ROWS rows (atomics; the caller zeroes the slab every step),
    // so a consumer reduces 16 rows instead of one per workgroup
    __syncthreads();
    const int slab_row = ((tid.z * GY + tid.y) * GX + tid.x) % BN_SLAB_ROWS;
    for (int i = threadIdx.x; i < 2 * slab_C; i += blockDim.x)
      atomicAdd(&bn_slab_out[(size_t)slab_row * 2 * slab_C + i], s_acc[(i < slab_C) ? i : (MAXC + i - slab_C)]);
  }
}

// A GEMM problem bound to its arguments (what one launch — or one half of a pair — runs).
template <int WM, int WN, int WK, class LA, class LB, class EPI>
struct GemmProblem {
  LA la; LB lb; EPI epi; int M, N, K, kps; BNRef bn; int bn_on; float* slab_out; int slab_C;
  int GX, GY, GZ;
  int det;                             // deterministic mode: exclusive BN slab rows, no atomics
  __host__ __device__ int nblocks() const { return (GX * GY * GZ + 7) / 8 * 8; }
  __device__ __forceinline__ void run(int bid, float* lds) const {
    gemm_body<WM, WN, WK>(la, lb, epi, M, N, K, kps, bn, bn_on, slab_out, slab_C, GX, GY, GZ, bid,
                          nblocks(), lds, det);
  }
};

template <class P>
__global__ __launch_bounds__(256) void gemm_f32_kernel(P p) {
  __shared__ float lds[GEMM_LDS_FLOATS];
  p.run(blockIdx.x, lds);
}

// Horizontal fusion: two independent GEMMs (a dense layer's input gradient and weight
// gradient) in ONE launch — blocks [0, n1) run the first, the rest the second.  HIP-graph
// branches on a second stream measured slower than serial launches on this runtime
// (profiles/r1_ab_wgrad_stream.txt); one grid overlaps the two for free and removes a
// kernel boundary.  n1 is a multiple of 8, so each half keeps its XCD-aware tile order.
template <class P1, class P2>
__global__ __launch_bounds__(256) void gemm_pair_kernel(P1 p1, P2 p2) {
  __shared__ float lds[GEMM_LDS_FLOATS];
  const int n1 = p1.nblocks();
  if ((int)blockIdx.x < n1) p1.run(blockIdx.x, lds);
  else p2.run(blockIdx.x - n1, lds);
}

// Wave layout + split-K so that one launch has ~1024 waves (one per SIMD on 256 CUs).
struct Plan { int wm, wn, wk, splits, kps; };

static Plan plan_gemm(int M, int N, int K, bool allow_split) {
  int tm = (M + 31) / 32, tn = (N + 31) / 32;
  int tiles = tm * tn;
  Plan p;
  if (tiles >= 512) { p.wm = 2; p.wn = 2; p.wk = 1; }
  else if (tiles >= 256) { p.wm = 1; p.wn = 2; p.wk = 2; }
  else { p.wm = 1; p.wn = 1; p.wk = 4; }
  const int wg = ((tm + p.wm - 1) / p.wm) * ((tn + p.wn - 1) / p.wn);
  // split K across workgroups until each wave owns <= one KC chunk (one memory round
  // trip per wave), keeping the launch under ~4096 waves and 512 slices
  constexpr int maxw = 4096;
  int splits = 1;
  if (allow_split && !g_csa_det)           // deterministic mode: no cross-workgroup atomics
    while ((K + splits * p.wk - 1) / (splits * p.wk) > KC && wg * 4 * splits * 2 <= maxw && splits < 512)
      splits *= 2;
  p.splits = splits;
  const int kps = (K + splits - 1) / splits;
  p.kps = (kps + 3) / 4 * 4;
  return p;
}

static int grid_slabs(const Plan& p, int M, int N) {
  const int g = ((N + 32 * p.wn - 1) / (32 * p.wn)) * ((M + 32 * p.wm - 1) / (32 * p.wm)) * p.splits;
  if (g_csa_det) return g;                 // deterministic mode: one exclusive row per workgroup
  return g < BN_SLAB_ROWS ? g : BN_SLAB_ROWS;
}

// Bind a plan's wave layout into a GemmProblem type and hand it to f.
template <class LA, class LB, class EPI, class F>
static int with_problem(const Plan& p, LA la, LB lb, EPI epi, int M, int N, int K, const BNRef& bn,
                        int bn_on, float* slab_out, int slab_C, F f) {
  const int GX = (N + 32 * p.wn - 1) / (32 * p.wn), GY = (M + 32 * p.wm - 1) / (32 * p.wm);
  const int GZ = p.splits;
#define CSA_P(WM, WN, WK) \
  return f(GemmProblem<WM, WN, WK, LA, LB, EPI>{la, lb, epi, M, N, K, p.kps, bn, bn_on, slab_out, slab_C, GX, GY, GZ, \
                                                g_csa_det})
  if (p.wm == 2 && p.wn == 2) CSA_P(2, 2, 1);
  if (p.wm == 1 && p.wn == 2) CSA_P(1, 2, 2);
  CSA_P(1, 1, 4);
#undef CSA_P
}

template <class LA, class LB, class EPI>
static int launch_gemm(const Plan& p, LA la, LB lb, EPI epi, int M, int N, int K, const BNRef& bn,
                       int bn_on, float* slab_out, int slab_C, hipStream_t st) {
  return with_problem(p, la, lb, epi, M, N, K, bn, bn_on, slab_out, slab_C, [&](auto prob) {
    hipLaunchKernelGGL((gemm_f32_kernel<decltype(prob)>), dim3((unsigned)prob.nblocks()), dim3(256), 0,
                       st, prob);
    return (int)hipGetLastError();
  });
}


// Call f(std::integral_constant<bool, a>, std::integral_constant<bool, b>) — picks the
// float4 loader instantiations when the operands' strides allow it.
template <class F>
static int dispatch2(bool a, bool b, F f) {
  using T = std::true_type;
  using Fl = std::false_type;
  if (a && b) return f(T{}, T{});
  if (a) return f(T{}, Fl{});
  if (b) return f(Fl{}, T{});
  return f(Fl{}, Fl{});
}

static BNRef make_bn(const float* slab, int nslab, int C, float count, float eps,
                     const float* scale, const float* offset) {
  return BNRef{slab, nslab, C, count, eps, scale, offset};
}

}  // namespace csa

using namespace csa;

// ===================================================================================
// C ABI (called through ctypes from cloud_server_amd/ops/fused.py)
// ===================================================================================

// Diagnostics: set the device pointer that receives GEMM stamps (null disables).
CSA_API int csa_gemm_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_gemm_dbg), &p, sizeof(p));
}

// How many split-K slices a dense forward of this shape uses (>1 => Y must be zeroed).
CSA_API int csa_dense_fwd_splits(int M, int N, int K) { return plan_gemm(M, N, K, true).splits; }

// Y[M][N] (+)= act(bn(X))[M][K] @ W[K][N] + bias.  Y zeroed by caller when splits > 1.
CSA_API int csa_dense_fwd(const float* X, const float* W, const float* bias, float* Y, int M,
                          int N, int K, const float* bn_slab, int bn_nslab, int bn_C,
                          float bn_count, float bn_eps, const float* bn_scale,
                          const float* bn_offset, int in_act, float in_alpha, hipStream_t st) {
  if (bn_slab && bn_C > MAXC) return -1;
  Plan p = plan_gemm(M, N, K, true);
  BNRef bn = make_bn(bn_slab, bn_nslab, bn_C, bn_count, bn_eps, bn_scale, bn_offset);
  EpiStore epi{Y, (long)N, M, N, bias, p.splits > 1, nullptr, 1.f};
  return dispatch2(K % 4 == 0 && K >= 4, N % 4 == 0 && N >= 4, [&](auto va, auto vb) {
    LoadColMajor<decltype(vb)::value> lb{W, (long)N, N, K};          // B(k, n) = W[k][n]
    if (!bn_slab && in_act == ACT_NONE) {   // plain operand: no per-element transform code
      LoadRowMajor<decltype(va)::value> la{X, (long)K, M, K};
      return launch_gemm(p, la, lb, epi, M, N, K, bn, 0, nullptr, 0, st);
    }
    LoadBNAct<true, decltype(va)::value> la{X, (long)K, M, K, FastDiv(bn_C > 0 ? bn_C : 1), in_act,
                                             in_alpha, bn_slab != nullptr, 0, nullptr, nullptr};
    return launch_gemm(p, la, lb, epi, M, N, K, bn, bn_slab != nullptr, nullptr, 0, st);
  });
}

// dX[M][Kin] = dY[M][Nout] @ W[Kin][Nout]^T, then (optionally) through the forward
// input transform h = act(bn(x)):  stores dz = dL/d(bn input or act input) and emits
// the BN-backward partial slab [nslab][2][C] ({sum dz, sum dz*xhat}).
// Returns the slab row count used (>= 1) or a negative error.
CSA_API int csa_dense_dgrad(const float* dY, const float* W, float* dX, int M, int Kin, int Nout,
                            const float* x_fwd, int act, float alpha, const float* bn_slab,
                            int bn_nslab, int bn_C, float bn_count, float bn_eps,
                            const float* bn_scale, const float* bn_offset, float* bwd_slab,
                            hipStream_t st) {
  if (bn_slab && bn_C > MAXC) return -1;
  const bool transform = (act != ACT_NONE) || (bn_slab != nullptr);
  Plan p = plan_gemm(M, Kin, Nout, !transform);
  BNRef bn = make_bn(bn_slab, bn_nslab, bn_C, bn_count, bn_eps, bn_scale, bn_offset);
  const bool v4 = Nout % 4 == 0 && Nout >= 4;
  int rc = dispatch2(v4, v4, [&](auto va, auto vb) {
    LoadRowMajor<decltype(va)::value> la{dY, (long)Nout, M, Nout};   // A(m, k=n) = dY[m][n]
    LoadRowMajor<decltype(vb)::value> lb{W, (long)Nout, Kin, Nout};  // B(k=n, j) = W[j][n]
    if (transform) {
      EpiActBNBwd epi{dX, (long)Kin, M, Kin, FastDiv(bn_C > 0 ? bn_C : 1), x_fwd, act, alpha,
                      bn_slab != nullptr, BNTables{}};
      return launch_gemm(p, la, lb, epi, M, Kin, Nout, bn, bn_slab != nullptr,
                         bn_slab ? bwd_slab : nullptr, bn_C, st);
    }
    EpiStore epi{dX, (long)Kin, M, Kin, nullptr, p.splits > 1, nullptr, 1.f};
    return launch_gemm(p, la, lb, epi, M, Kin, Nout, bn, 0, nullptr, 0, st);
  });
  if (rc) return -rc;
  return grid_slabs(p, M, Kin);
}

CSA_API int csa_dense_dgrad_splits(int M, int Kin, int Nout, int transform) {
  return plan_gemm(M, Kin, Nout, !transform).splits;
}

CSA_API int csa_dense_dgrad_slabs(int M, int Kin, int Nout) {
  Plan p = plan_gemm(M, Kin, Nout, false);
  return grid_slabs(p, M, Kin);
}

// dW[Kin][Nout] (+)= act(bn(X))^T @ dY * scale, db[Nout] (+)= colsum(dY) * scale.
// Output accumulated with atomics when split (caller zeroes dW/db) — see *_splits.
CSA_API int csa_dense_wgrad_splits(int M, int Kin, int Nout) {
  return plan_gemm(Kin + 1, Nout, M, true).splits;
}

CSA_API int csa_dense_wgrad(const float* X, const float* dY, float* dW, float* db, int M, int Kin,
                            int Nout, const float* bn_slab, int bn_nslab, int bn_C, float bn_count,
                            float bn_eps, const float* bn_scale, const float* bn_offset, int in_act,
                            float in_alpha, float scale, hipStream_t st) {
  if (bn_slab && bn_C > MAXC) return -1;
  const int Mg = Kin + (db ? 1 : 0);
  Plan p = plan_gemm(Mg, Nout, M, true);
  BNRef bn = make_bn(bn_slab, bn_nslab, bn_C, bn_count, bn_eps, bn_scale, bn_offset);
  EpiStore epi{dW, (long)Nout, Kin, Nout, nullptr, p.splits > 1, db, scale};
  return dispatch2(Kin % 4 == 0 && Kin >= 4, Nout % 4 == 0 && Nout >= 4, [&](auto va, auto vb) {
    LoadColMajor<decltype(vb)::value> lb{dY, (long)Nout, Nout, M};   // B(k=m, n) = dY[m][n]
    if (!bn_slab && in_act == ACT_NONE) {   // plain operand (+ ones row for the bias gradient)
      if (db) {
        LoadColMajor<decltype(va)::value, true> la{X, (long)Kin, Kin, M};   // A(f, m) = X[m][f]
        return launch_gemm(p, la, lb, epi, Mg, Nout, M, bn, 0, nullptr, 0, st);
      }
      LoadColMajor<decltype(va)::value> la{X, (long)Kin, Kin, M};
      return launch_gemm(p, la, lb, epi, Mg, Nout, M, bn, 0, nullptr, 0, st);
    }
    LoadBNAct<false, decltype(va)::value> la{X, (long)Kin, M, Kin, FastDiv(bn_C > 0 ? bn_C : 1), in_act,
                                              in_alpha, bn_slab != nullptr, db != nullptr, nullptr, nullptr};
    return launch_gemm(p, la, lb, epi, Mg, Nout, M, bn, bn_slab != nullptr, nullptr, 0, st);
  });
}


// Dense layer backward in ONE launch (gemm_pair_kernel): the input gradient dX (with the
// forward input transform's backward in its epilogue, as csa_dense_dgrad) and the weight
// gradient dW/db of an untransformed / materialised input Xw (as csa_dense_wgrad).
// Returns the dgrad BN-slab row count (>= 1), 0 when the shape is outside the fused family
// (the caller then launches the two GEMMs separately), or a negative error.
CSA_API int csa_dense_bwd(const float* dY, const float* W, float* dX, int M, int Kin, int Nout,
                          const float* x_fwd, int act, float alpha, const float* bn_slab,
                          int bn_nslab, int bn_C, float bn_count, float bn_eps,
                          const float* bn_scale, const float* bn_offset, float* bwd_slab,
                          const float* Xw, float* dW, float* db, float scale, hipStream_t st) {
  if (Nout % 4 || Kin % 4 || Nout < 4 || Kin < 4) return 0;
  if (bn_slab && bn_C > MAXC) return -1;
  const bool transform = (act != ACT_NONE) || (bn_slab != nullptr);
  const Plan pd = plan_gemm(M, Kin, Nout, !transform);
  if (!(pd.wm == 1 && pd.wn == 1 && pd.wk == 4)) return 0;
  const int Mg = Kin + (db ? 1 : 0);
  const Plan pw = plan_gemm(Mg, Nout, M, true);
  const BNRef bn = make_bn(bn_slab, bn_nslab, bn_C, bn_count, bn_eps, bn_scale, bn_offset);
  const LoadRowMajor<true> la{dY, (long)Nout, M, Nout};     // A(m, k=n) = dY[m][n]
  const LoadRowMajor<true> lb{W, (long)Nout, Kin, Nout};    // B(k=n, j) = W[j][n]
  const LoadColMajor<true> lbw{dY, (long)Nout, Nout, M};    // B(k=m, n) = dY[m][n]
  const EpiStore ew{dW, (long)Nout, Kin, Nout, nullptr, pw.splits > 1, db, scale};
  const int GX = (Kin + 31) / 32, GY = (M + 31) / 32;
  auto go = [&](auto ed, int bn_on, float* so, int sc) {
    using ED = decltype(ed);
    const GemmProblem<1, 1, 4, LoadRowMajor<true>, LoadRowMajor<true>, ED> a{
        la, lb, ed, M, Kin, Nout, pd.kps, bn, bn_on, so, sc, GX, GY, pd.splits, g_csa_det};
    auto launch = [&](auto law) {
      return with_problem(pw, law, lbw, ew, Mg, Nout, M, BNRef{}, 0, nullptr, 0, [&](auto b) {
        hipLaunchKernelGGL((gemm_pair_kernel<decltype(a), decltype(b)>),
                           dim3((unsigned)(a.nblocks() + b.nblocks())), dim3(256), 0, st, a, b);
        return (int)hipGetLastError();
      });
    };
    if (db) return launch(LoadColMajor<true, true>{Xw, (long)Kin, Kin, M});   // A(f, m) = Xw[m][f]
    return launch(LoadColMajor<true>{Xw, (long)Kin, Kin, M});
  };
  int rc;
  if (transform) {
    EpiActBNBwd ed{dX, (long)Kin, M, Kin, FastDiv(bn_C > 0 ? bn_C : 1), x_fwd, act, alpha,
                   bn_slab != nullptr, BNTables{}};
    rc = go(ed, bn_slab != nullptr, bn_slab ? bwd_slab : nullptr, bn_C);
  } else {
    EpiStore ed{dX, (long)Kin, M, Kin, nullptr, pd.splits > 1, nullptr, 1.f};
    rc = go(ed, 0, nullptr, 0);
  }
  if (rc) return -rc;
  return grid_slabs(pd, M, Kin);
}

// ===================================================================================
// Wide convolutions as implicit GEMMs on the same f32 MFMA body.
//
// The direct conv kernels (conv.hip, conv_pair.hip) keep a conv's weights and BatchNorm
// tables in LDS, which bounds them to <= 128 channels.  The DSL accepts any
// filter:[kh, kw, cout] (construct_distribute.py:222-233), so a conv with more channels
// runs as three GEMMs whose operands are gathered on the fly by loader functors — no
// im2col buffer is ever materialised:
//   forward  Z[m = (b,oy,ox)][co]   = im2col(X)[m][k = (i,j,ci)] @ W[k][co] (+ bias)
//   wgrad    dW[k][co] (+db)        = im2col(X)^T @ dZ           (ones row -> db)
//   dgrad    dX[p = (b,y,x)][ci]    = dZ~[p][k' = (i,j,co)] @ W~[k'][ci]
// where dZ~ gathers dZ[b][(y+PT-i)/SH][(x+PL-j)/SW][co] (zero unless the division is
// exact and in range) and W~[k'][ci] = W[i][j][ci][co].  HWIO weights make k = (i,j,ci)
// row-major exactly the im2col order.  Activation / pool / BatchNorm around a wide conv
// run as standalone units (norm_pool.hip), so these GEMMs carry no transforms.
// ===================================================================================
namespace csa {

struct GConvGeom { int B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH, OW, Cout; };

// im2col(X)[m][k].  T = false: elem(r = m, c = k) (forward A, K contiguous in ci);
// T = true: elem(r = k, c = m) (weight-gradient A; ONES: row k == Kd reads 1 -> db).
template <bool T, bool ONES = false>
struct LoadIm2col {
  const float* x; GConvGeom g; FastDiv dOW, dOHW, dCin, dKW; int M, Kd;
  static constexpr bool KCONTIG = !T;
  static constexpr bool VEC4 = false;
  __device__ float4 raw4(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void bind(const BNTables&) {}
  __device__ __forceinline__ long addr(int m, int k, bool& ok) const {
    int b, pix, oy, ox, tap, ci, i, j;
    dOHW.divmod(m, b, pix);
    dOW.divmod(pix, oy, ox);
    dCin.divmod(k, tap, ci);
    dKW.divmod(tap, i, j);
    const int yy = oy * g.SH - g.PT + i, xx = ox * g.SW - g.PL + j;
    ok = m < M && k < Kd && yy >= 0 && yy < g.H && xx >= 0 && xx < g.W;
    return ok ? (((long)b * g.H + yy) * g.W + xx) * g.Cin + ci : 0;
  }
  __device__ float raw(int r, int c) const {
    bool ok;
    return x[addr(T ? c : r, T ? r : c, ok)];
  }
  __device__ float post(float v, int r, int c) const {
    const int m = T ? c : r, k = T ? r : c;
    if (ONES && k == Kd) return m < M ? 1.f : 0.f;
    bool ok;
    addr(m, k, ok);
    return ok ? v : 0.f;
  }
};

// dZ~[p][k'] for the input gradient: p = (b, y, x) input pixel, k' = (i, j, co).
struct LoadConvDZ {
  const float* dz; GConvGeom g; FastDiv dW, dHW, dCout, dKW; int P, Kd;
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC4 = false;
  __device__ float4 raw4(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void bind(const BNTables&) {}
  __device__ __forceinline__ long addr(int p, int k, bool& ok) const {
    int b, pix, y, x, tap, co, i, j;
    dHW.divmod(p, b, pix);
    dW.divmod(pix, y, x);
    dCout.divmod(k, tap, co);
    dKW.divmod(tap, i, j);
    const int ty = y + g.PT - i, tx = x + g.PL - j;
    const int oy = ty / g.SH, ox = tx / g.SW;     // only used when ty, tx >= 0 and exact
    ok = p < P && k < Kd && ty >= 0 && tx >= 0 && oy * g.SH == ty && ox * g.SW == tx &&
         oy < g.OH && ox < g.OW;
    return ok ? (((long)b * g.OH + oy) * g.OW + ox) * g.Cout + co : 0;
  }
  __device__ float raw(int r, int c) const {
    bool ok;
    return dz[addr(r, c, ok)];
  }
  __device__ float post(float v, int r, int c) const {
    bool ok;
    addr(r, c, ok);
    return ok ? v : 0.f;
  }
};

// W~[k' = (i,j,co)][ci] = W[i][j][ci][co], read as elem(r = ci, c = k') (K contiguous in co).
struct LoadConvWT {
  const float* w; int Cin, Cout, Kd; FastDiv dCout;
  static constexpr bool KCONTIG = true;
  static constexpr bool VEC4 = false;
  __device__ float4 raw4(int, int) const { return make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ void bind(const BNTables&) {}
  __device__ __forceinline__ long addr(int ci, int k, bool& ok) const {
    int tap, co;
    dCout.divmod(k, tap, co);
    ok = ci < Cin && k < Kd;
    return ok ? ((long)tap * Cin + ci) * Cout + co : 0;
  }
  __device__ float raw(int r, int c) const {
    bool ok;
    return w[addr(r, c, ok)];
  }
  __device__ float post(float v, int r, int c) const { return (r < Cin && c < Kd) ? v : 0.f; }
};

static bool gconv_ok(const GConvGeom& g) {
  const long M = (long)g.B * g.OH * g.OW, P = (long)g.B * g.H * g.W;
  const long K1 = (long)g.KH * g.KW * g.Cin, K2 = (long)g.KH * g.KW * g.Cout;
  // FastDiv is exact below 2^22; the launch grid is one 32-bit dimension
  return g.B > 0 && g.Cin > 0 && g.Cout > 0 && g.KH > 0 && g.KW > 0 && g.SH > 0 && g.SW > 0 &&
         g.OH > 0 && g.OW > 0 && M < (1 << 22) && P < (1 << 22) && K1 < (1 << 22) && K2 < (1 << 22);
}

static GConvGeom gconv_geom(const int* v) {
  return GConvGeom{v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], v[8], v[9], v[10], v[11], v[12]};
}

}  // namespace csa

// geom = [B, H, W, Cin, KH, KW, SH, SW, PT, PL, OH, OW, Cout] (as csa_conv_fwd)
CSA_API int csa_gconv_fwd_splits(const int* geom) {
  const GConvGeom g = gconv_geom(geom);
  return plan_gemm(g.B * g.OH * g.OW, g.Cout, g.KH * g.KW * g.Cin, true).splits;
}

// Z[B][OH][OW][Cout] (+)= conv(X) + bias.  Z zeroed by the caller when splits > 1.
CSA_API int csa_gconv_fwd(const float* X, const float* W, const float* bias, float* Z, const int* geom,
                          hipStream_t st) {
  const GConvGeom g = gconv_geom(geom);
  if (!gconv_ok(g)) return -1;
  const int M = g.B * g.OH * g.OW, N = g.Cout, K = g.KH * g.KW * g.Cin;
  const Plan p = plan_gemm(M, N, K, true);
  const LoadIm2col<false> la{X, g, FastDiv(g.OW), FastDiv(g.OH * g.OW), FastDiv(g.Cin), FastDiv(g.KW), M, K};
  const LoadColMajor<false> lb{W, (long)N, N, K};                 // B(k, n) = W[k][n]
  const EpiStore epi{Z, (long)N, M, N, bias, p.splits > 1, nullptr, 1.f};
  return launch_gemm(p, la, lb, epi, M, N, K, BNRef{}, 0, nullptr, 0, st);
}

CSA_API int csa_gconv_wgrad_splits(const int* geom, int has_bias) {
  const GConvGeom g = gconv_geom(geom);
  return plan_gemm(g.KH * g.KW * g.Cin + (has_bias ? 1 : 0), g.Cout, g.B * g.OH * g.OW, true).splits;
}

// dW[KH*KW*Cin][Cout] (+)= im2col(X)^T @ dZ * scale, db (+)= colsum(dZ) * scale.
// Accumulated with atomics when split (caller zeroes dW / db, see *_splits).
CSA_API int csa_gconv_wgrad(const float* X, const float* dZ, float* dW, float* db, const int* geom,
                            float scale, hipStream_t st) {
  const GConvGeom g = gconv_geom(geom);
  if (!gconv_ok(g)) return -1;
  const int M = g.B * g.OH * g.OW, Kd = g.KH * g.KW * g.Cin, N = g.Cout;
  const int Mg = Kd + (db ? 1 : 0);
  const Plan p = plan_gemm(Mg, N, M, true);
  const LoadColMajor<false> lb{dZ, (long)N, N, M};                // B(k = m, n) = dZ[m][n]
  const EpiStore epi{dW, (long)N, Kd, N, nullptr, p.splits > 1, db, scale};
  const FastDiv a(g.OW), b(g.OH * g.OW), c(g.Cin), d(g.KW);
  if (db) return launch_gemm(p, LoadIm2col<true, true>{X, g, a, b, c, d, M, Kd}, lb, epi, Mg, N, M,
                             BNRef{}, 0, nullptr, 0, st);
  return launch_gemm(p, LoadIm2col<true>{X, g, a, b, c, d, M, Kd}, lb, epi, Mg, N, M, BNRef{}, 0, nullptr,
                     0, st);
}

CSA_API int csa_gconv_dgrad_splits(const int* geom) {
  const GConvGeom g = gconv_geom(geom);
  return plan_gemm(g.B * g.H * g.W, g.Cin, g.KH * g.KW * g.Cout, true).splits;
}

// dX[B][H][W][Cin] (+)= conv-transpose(dZ).  dX zeroed by the caller when splits > 1.
CSA_API int csa_gconv_dgrad(const float* dZ, const float* W, float* dX, const int* geom, hipStream_t st) {
  const GConvGeom g = gconv_geom(geom);
  if (!gconv_ok(g)) return -1;
  const int P = g.B * g.H * g.W, N = g.Cin, K = g.KH * g.KW * g.Cout;
  const Plan p = plan_gemm(P, N, K, true);
  const LoadConvDZ la{dZ, g, FastDiv(g.W), FastDiv(g.H * g.W), FastDiv(g.Cout), FastDiv(g.KW), P, K};
  const LoadConvWT lb{W, g.Cin, g.Cout, K, FastDiv(g.Cout)};
  const EpiStore epi{dX, (long)N, P, N, nullptr, p.splits > 1, nullptr, 1.f};
  return launch_gemm(p, la, lb, epi, P, N, K, BNRef{}, 0, nullptr, 0, st);
}
