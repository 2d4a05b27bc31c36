// Fused classifier head + loss + head backward + step bookkeeping.
//
// Reference: the fixed 10-way head (construct_distribute.py:252-264), the loss
// (softmax-xent 'entropy' or 'mse', :285-298), the accuracy op (:381-382) and the
// global_step increment done by minimize() (:372-373).  At B = 50 the head is ~0.8 MFLOP:
// latency, not math.  The main path (head_rows_kernel) spreads the batch over
// ceil(M/16) workgroups that each do every phase for their rows with 16x16x4 f32 MFMA
// (10 classes pad to 16 columns), accumulate dWh/dbh with atomics and hand the metric
// bookkeeping to the last arriving workgroup:
//   ring_loss[step % R] = loss, ring_correct[step % R] = #correct, step += 1
// so metrics never force a host sync inside the training loop.  A VALU fallback
// (head_generic_kernel) covers K % 4 != 0 or inputs too wide for LDS.
#include "common.h"
#include "head_dgrad.h"

namespace csa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int HT = 1024;
constexpr int NW = HT / 64;
#ifndef CSA_NCLS_DEFINED
#define CSA_NCLS_DEFINED
constexpr int NCLS = 10;
#endif
constexpr size_t HEAD_LDS_MAX = 150 * 1024;

struct HeadArgs {
  const float* h; int M, K; int in_act; float in_alpha;
  const float* w; const float* b;          // [K][10], [10]
  const int64_t* labels;                   // dataset labels ...
  const int64_t* idx;                      // ... gathered through the batch index stream
  const int64_t* cursor;                   // if set: this step's row = idx + cursor[0] * M
  int loss;                                // 0 = softmax xent, 1 = mse
  float grad_scale;
  float* dw; float* db; float* dh;         // grads (dh may be null)
  float* logits_out;                       // optional [M][10]
  int64_t* step; float* ring_loss; int* ring_correct; int ring;
};


__device__ __forceinline__ int drow(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Loss / dlogits / accuracy on LDS logits (one lane per row) + step bookkeeping.
// Callers: s_log holds logits (without bias), s_red/s_cor scratch.  Ends with a barrier.
__device__ __forceinline__ void head_loss(const HeadArgs& a, const int64_t* idx, float* s_log,
                                          float* s_red, int* s_cor, int label0 = -1) {
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int M = a.M;
  float lsum = 0.f;
  for (int m = tid; m < M; m += HT) {
    const int y = (label0 >= 0 && m == tid) ? label0 : (int)a.labels[idx[m]];
    float* row = s_log + m * NCLS;
#pragma unroll
    for (int j = 0; j < NCLS; ++j) row[j] += a.b[j];
    float mx = row[0];
    int am = 0;
#pragma unroll
    for (int j = 1; j < NCLS; ++j)
      if (row[j] > mx) { mx = row[j]; am = j; }
    if (am == y) atomicAdd(s_cor, 1);
    if (a.logits_out) {
#pragma unroll
      for (int j = 0; j < NCLS; ++j) a.logits_out[m * NCLS + j] = row[j];
    }
    if (a.loss == 0) {
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) se += __expf(row[j] - mx);
      const float lse = mx + __logf(se);
      lsum += lse - row[y];
      const float inv = a.grad_scale / (float)M;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) row[j] = (__expf(row[j] - lse) - (j == y ? 1.f : 0.f)) * inv;
    } else {
      const float inv = 2.f * a.grad_scale / (float)(M * NCLS);
#pragma unroll
      for (int j = 0; j < NCLS; ++j) {
        const float d = row[j] - (j == y ? 1.f : 0.f);
        lsum += d * d;
        row[j] = d * inv;
      }
    }
  }
  lsum = wave_sum(lsum);
  if (lane == 0) s_red[wave] = lsum;
  __syncthreads();
  if (tid == 0) {
    float t = 0.f;
    for (int i = 0; i < NW; ++i) t += s_red[i];
    t = (a.loss == 0) ? t / M : t / (M * NCLS);
    const int64_t st = *a.step;
    const int pos = (int)(st % a.ring);
    a.ring_loss[pos] = t;
    a.ring_correct[pos] = *s_cor;
    *a.step = st + 1;
  }
  if (tid < NCLS) {
    float acc = 0.f;
    for (int m = 0; m < M; ++m) acc += s_log[m * NCLS + tid];
    a.db[tid] = acc;
  }
}

// Row-group MFMA path (K % 4 == 0 and 16 rows of T(h) + Wh fit in LDS): one 256-thread
// workgroup per 16 batch rows, so the batch's head runs on ceil(M/16) CUs in parallel
// instead of serialising every phase inside one workgroup (21 µs -> see profiles/).
// Per workgroup: stage T(h) rows + Wh (one batched round trip), logits with
// v_mfma_f32_16x16x4_f32 (4 waves = 4 K quarters, partials folded in LDS), loss /
// dlogits / #correct for its rows, dh rows (plain stores), and its partial dWh / dbh
// (atomicAdd; the optimizer zeroes them every step).  The step bookkeeping is done by
// the LAST workgroup to arrive (agent-scope acq_rel counter, cdna_hip_programming.md
// §6 G16): it reads the batch loss / #correct accumulated with atomics, writes the
// metric ring, advances the step counter and re-zeroes the workspace for the next step.
// 16x16x4 map: A lane l = A[l&15][l>>4], B lane l = B[l>>4][l&15],
// D reg r of lane l = D[4*(l>>4) + r][l&15].
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int RT = 256;           // threads per row-group workgroup
constexpr int RG = 16;            // batch rows per workgroup

__global__ __launch_bounds__(RT) void head_rows_kernel(HeadArgs a, int* ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int M = a.M, K = a.K, KP = K + 1;
  const int g = blockIdx.x, m0 = g * RG, mrows = min(RG, M - m0);
  float* s_log = smem;                     // [16][10] logits, then dlogits (rows >= mrows zero)
  float* s_part = s_log + RG * NCLS;       // [4 waves][16][16]
  float* s_red = s_part + 4 * 256;         // [8]
  float* s_w = s_red + 8;                  // [K][10]
  float* s_h = s_w + K * NCLS;             // [16][K+1]  T(h) rows
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * M : a.idx;
  int my_label = 0;
  if (tid < mrows) my_label = (int)a.labels[idx[m0 + tid]];
  {  // Wh and the 16 rows of T(h): every load of a thread in flight together
    const int act = a.in_act;
    const float alpha = a.in_alpha;
    const int K4 = K >> 2, nw4 = (K * NCLS) >> 2, nh4 = mrows * K4;
    const float4* w4 = reinterpret_cast<const float4*>(a.w);
    const float4* h4 = reinterpret_cast<const float4*>(a.h + (long)m0 * K);
    const FastDiv dk4(K4);
    for (int base = 0; base < nw4 + nh4; base += RT * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * RT + tid;
        // select the ADDRESS, then one unconditional load (a select between two loads
        // made hipcc branch around each and wait for it: 8 serial round trips)
        const float4* p = i < nw4 ? w4 + i : h4 + ((i - nw4 < nh4) ? i - nw4 : 0);
        v[u] = *p;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * RT + tid;
        if (i < nw4) {
          reinterpret_cast<float4*>(s_w)[i] = v[u];
        } else if (i - nw4 < nh4) {
          int m, k4;
          dk4.divmod(i - nw4, m, k4);
          float* d = s_h + m * KP + 4 * k4;
          d[0] = act_fwd(v[u].x, act, alpha);
          d[1] = act_fwd(v[u].y, act, alpha);
          d[2] = act_fwd(v[u].z, act, alpha);
          d[3] = act_fwd(v[u].w, act, alpha);
        }
      }
    }
  }
  __syncthreads();

  const int r = lane & 15, hk = lane >> 4;
  {  // ---- logits partials: wave = K quarter ----
    const int kper = ((K + 3) / 4 + 3) & ~3;
    const int kb = wave * kper, ke = min(K, kb + kper);
    const int m = min(r, mrows - 1);
    const bool okm = r < mrows, okj = r < NCLS;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = kb; k < ke; k += 4) {
      const int kk = k + hk;
      const int kc = min(kk, K - 1);
      const float hv = s_h[m * KP + kc];
      const float wv = s_w[kc * NCLS + (okj ? r : 0)];
      const bool okk = kk < ke;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32((okm && okk) ? hv : 0.f, (okj && okk) ? wv : 0.f,
                                                 acc, 0, 0, 0);
    }
    float* part = s_part + wave * 256;
#pragma unroll
    for (int i = 0; i < 4; ++i) part[(4 * hk + i) * 16 + r] = acc[i];
  }
  __syncthreads();
  if (tid < RG * NCLS) {
    const int row = tid / NCLS, j = tid % NCLS;
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) v += s_part[q * 256 + row * 16 + j];
    s_log[tid] = row < mrows ? v : 0.f;
  }
  __syncthreads();

  // ---- loss / dlogits / #correct for this group's rows (one lane per row) ----
  float lsum = 0.f;
  int cor = 0;
  if (tid < mrows) {
    const int y = my_label;
    float* row = s_log + tid * NCLS;
#pragma unroll
    for (int j = 0; j < NCLS; ++j) row[j] += a.b[j];
    float mx = row[0];
    int am = 0;
#pragma unroll
    for (int j = 1; j < NCLS; ++j)
      if (row[j] > mx) { mx = row[j]; am = j; }
    cor = (am == y);
    if (a.logits_out) {
#pragma unroll
      for (int j = 0; j < NCLS; ++j) a.logits_out[(long)(m0 + tid) * NCLS + j] = row[j];
    }
    if (a.loss == 0) {
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) se += __expf(row[j] - mx);
      const float lse = mx + __logf(se);
      lsum = lse - row[y];
      const float inv = a.grad_scale / (float)M;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) row[j] = (__expf(row[j] - lse) - (j == y ? 1.f : 0.f)) * inv;
    } else {
      const float inv = 2.f * a.grad_scale / (float)(M * NCLS);
#pragma unroll
      for (int j = 0; j < NCLS; ++j) {
        const float d = row[j] - (j == y ? 1.f : 0.f);
        lsum += d * d;
        row[j] = d * inv;
      }
    }
  }
  if (wave == 0) {
    lsum = wave_sum(lsum);
    const unsigned long long ball = __ballot(cor != 0);
    if (lane == 0) {
      atomicAdd(reinterpret_cast<float*>(ws + 1), lsum);
      atomicAdd(ws + 2, __popcll(ball));
    }
  }
  __syncthreads();
  if (tid < NCLS) {   // dbh partial
    float acc = 0.f;
    for (int m = 0; m < mrows; ++m) acc += s_log[m * NCLS + tid];
    atomicAdd(&a.db[tid], acc);
  }

  // ---- dWh partial[k][j] = sum_{rows} T(h)[m][k] dl[m][j]: 16-k tiles over the waves ----
  for (int kt = wave; kt * 16 < K; kt += 4) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int kc = min(kt * 16 + r, K - 1);
#pragma unroll
    for (int m = 0; m < RG; m += 4) {
      const int mm = m + hk;                       // s_log rows >= mrows are zero
      const float hv = s_h[min(mm, mrows - 1) * KP + kc];
      const float lv = s_log[mm * NCLS + (r < NCLS ? r : 0)];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hv, r < NCLS ? lv : 0.f, acc, 0, 0, 0);
    }
    if (r < NCLS) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int kr = kt * 16 + 4 * hk + i;
        if (kr < K) atomicAdd(&a.dw[kr * NCLS + r], acc[i]);
      }
    }
  }

  // ---- dh rows[m][k] = (sum_j dl[m][j] Wh[k][j]) * T'(h): 16-col k tiles over the waves ----
  if (a.dh) {
    for (int kt = wave; kt * 16 < K; kt += 4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int k = kt * 16 + r;
#pragma unroll
      for (int j = 0; j < 12; j += 4) {            // 10 classes -> 3 k-steps of 4
        const int jj = j + hk;
        const bool okj = jj < NCLS;
        const float lv = s_log[r * NCLS + (okj ? jj : 0)];
        const float wv = s_w[min(k, K - 1) * NCLS + (okj ? jj : 0)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(okj ? lv : 0.f, (okj && k < K) ? wv : 0.f, acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mr = 4 * hk + i;
        if (mr < mrows && k < K) {
          float gv = acc[i];
          if (a.in_act) {  // post-activation value decides every supported derivative
            const float y = s_h[mr * KP + k];
            gv = act_bwd(gv, y, y, a.in_act, a.in_alpha);
          }
          a.dh[(long)(m0 + mr) * K + k] = gv;
        }
      }
    }
  }

  // ---- last workgroup: metric ring + step counter, re-arm the workspace ----
  __syncthreads();
  if (tid == 0) {
    const int old = __hip_atomic_fetch_add(ws, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (old == (int)gridDim.x - 1);
  }
  __syncthreads();
  if (s_last && tid == 0) {
    const float tot = __hip_atomic_load(reinterpret_cast<float*>(ws + 1), __ATOMIC_ACQUIRE,
                                        __HIP_MEMORY_SCOPE_AGENT);
    const int ncor = __hip_atomic_load(ws + 2, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t st = *a.step;
    const int pos = (int)(st % a.ring);
    a.ring_loss[pos] = (a.loss == 0) ? tot / M : tot / (M * NCLS);
    a.ring_correct[pos] = ncor;
    *a.step = st + 1;
    __hip_atomic_store(reinterpret_cast<float*>(ws + 1), 0.f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ws + 2, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(ws, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------------------------
// Row-group head with PARTIAL outputs (the fused-update step program): ceil(M / RG)
// workgroups of 4 waves, RG <= 16 batch rows each; the waves split K (hidden features).
// Every output has exactly one writer, so there are no atomics, no arrival counter and
// nothing to zero:
//   * dh rows [RG][K]            — plain stores (consumer: the last dense layer's backward);
//   * dWh/dbh partial row g       — part[g][K*10 + 10] (the optimizer folds the G rows
//                                   while it applies the head's update);
//   * loss sum / #correct of g    — mpart[g], mcorr[g] (the optimizer writes the metric ring).
// Block 0 advances the device step counter first thing, so every parameter update of the
// step (fused dense updates, the optimizer) sees the same 1-based t (optim_common.h).
// The row-group kernel above spent most of its 14.5 µs in ~20k same-line dWh atomics and
// a last-arriver hand-off.
// ---------------------------------------------------------------------------------
// diagnostics: s_memtime stamps of workgroup 0 (null disables; csa_head_debug)
__constant__ long long* g_head_dbg = nullptr;
#define HEAD_STAMP(i)                                                                         \
  do {                                                                                        \
    if (g_head_dbg && threadIdx.x == 0 && blockIdx.x == 0) g_head_dbg[i] = (long long)__builtin_amdgcn_s_memtime(); \
  } while (0)

constexpr int PRG_MAX = 16;        // rows per workgroup
constexpr size_t PHEAD_LDS_MAX = 150 * 1024;

struct HeadPartArgs {
  const float* h; int M, K, RG; int in_act; float in_alpha;
  const float* w; const float* b;
  const int64_t* labels; const int64_t* idx; const int64_t* cursor;
  int loss; float grad_scale;
  float* dh;                 // [M][K] or null
  float* part;               // [G][K*10 + 10, padded to a multiple of 4]
  float* mpart; int* mcorr;  // [G]
  float* logits_out;         // optional [M][10]
  int64_t* step;
  int64_t* adv_cursor;       // batch staging: block 0 advances the stream cursor (mod wrap)
  long wrap;
};

__host__ __device__ inline size_t head_part_lds(int RG, int K) {
  return ((size_t)RG * K + (size_t)K * NCLS + (size_t)PRG_MAX * NCLS * 2) * sizeof(float);
}

// Stages the group's T(h) rows and Wh in LDS (one batched round trip: every load of a
// thread in flight, pinned, then the stores), then everything runs from LDS.
__global__ __launch_bounds__(256) void head_part_kernel(HeadPartArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ float s_loss[PRG_MAX];
  __shared__ int s_cor[PRG_MAX];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int M = a.M, K = a.K, RG = a.RG;
  const int g = blockIdx.x, m0 = g * RG, rows = min(RG, M - m0);
  float* s_h = smem;                       // [RG][K]  T(h)
  float* s_w = s_h + RG * K;               // [K][10]
  float* s_lg = s_w + K * NCLS;            // [PRG_MAX][10] logits
  float* s_dl = s_lg + PRG_MAX * NCLS;     // [PRG_MAX][10] dlogits
  HEAD_STAMP(0);
  float bias[NCLS];                // read first: consumed after the logits
#pragma unroll
  for (int j = 0; j < NCLS; ++j) bias[j] = a.b[j];
  if (g == 0 && tid == 0) {
    *a.step += 1;
    if (a.adv_cursor) {          // the step's batch is staged: its kernels no longer read the cursor
      const int64_t c = *a.adv_cursor + 1;
      *a.adv_cursor = (a.wrap > 0 && c >= a.wrap) ? 0 : c;
    }
  }
  {
    const int K4 = K >> 2, nh4 = rows * K4, nw4 = (K * NCLS) >> 2, tot = nh4 + nw4;
    const float4* h4 = reinterpret_cast<const float4*>(a.h + (long)m0 * K);
    const float4* w4 = reinterpret_cast<const float4*>(a.w);
    constexpr int U = 16;
    for (int base = 0; base < tot; base += 256 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = min(base + u * 256 + tid, tot - 1);
        const float4* src = e < nh4 ? h4 + e : w4 + (e - nh4);
        v[u] = *src;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) pin(v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = base + u * 256 + tid;
        if (e < nh4) {
          float4 t = v[u];
          t.x = act_fwd(t.x, a.in_act, a.in_alpha); t.y = act_fwd(t.y, a.in_act, a.in_alpha);
          t.z = act_fwd(t.z, a.in_act, a.in_alpha); t.w = act_fwd(t.w, a.in_act, a.in_alpha);
          reinterpret_cast<float4*>(s_h)[e] = t;
        } else if (e < tot) {
          reinterpret_cast<float4*>(s_w)[e - nh4] = v[u];
        }
      }
    }
  }
  HEAD_STAMP(1);
  // the label chain (cursor -> row index -> label) is only needed after the logits: it is
  // issued after the staging loads so its two dependent round trips overlap them
  int label = 0;
  if (!a.idx) {                    // staged labels
    if (tid < rows) label = (int)a.labels[m0 + tid];
  } else {
    const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * M : a.idx;
    if (tid < rows) label = (int)a.labels[idx[m0 + tid]];
  }
  __syncthreads();
  HEAD_STAMP(2);
  // logits: wave w takes rows w, w+4, ...; lane l owns k = 4l + 256i (one float4 of h and
  // the 40 contiguous weights of those 4 k as ten float4 LDS reads), then a DPP wave
  // reduction per class
  for (int r = wave; r < rows; r += 4) {
    float acc[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) acc[j] = 0.f;
    for (int k4 = lane * 4; k4 < K; k4 += 256) {
      const float4 hv = *reinterpret_cast<const float4*>(s_h + r * K + k4);
      const float4* wr = reinterpret_cast<const float4*>(s_w + k4 * NCLS);
      float wv[4 * NCLS];
#pragma unroll
      for (int q = 0; q < NCLS; ++q) {
        const float4 t = wr[q];
        wv[4 * q] = t.x; wv[4 * q + 1] = t.y; wv[4 * q + 2] = t.z; wv[4 * q + 3] = t.w;
      }
      const float hs[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2)
#pragma unroll
        for (int j = 0; j < NCLS; ++j) acc[j] = fmaf(hs[s2], wv[s2 * NCLS + j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < NCLS; ++j) {
      const float t = wave_sum_dpp(acc[j]);
      if (lane == 0) s_lg[r * NCLS + j] = t;
    }
  }
  __syncthreads();
  HEAD_STAMP(3);
  // loss / dlogits / correct: one thread per row
  if (tid < rows) {
    float row[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) row[j] = s_lg[tid * NCLS + j] + bias[j];
    float mx = row[0];
    int am = 0;
#pragma unroll
    for (int j = 1; j < NCLS; ++j)
      if (row[j] > mx) { mx = row[j]; am = j; }
    if (a.logits_out) {
#pragma unroll
      for (int j = 0; j < NCLS; ++j) a.logits_out[(long)(m0 + tid) * NCLS + j] = row[j];
    }
    float ls = 0.f;
    if (a.loss == 0) {
      float se = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) se += __expf(row[j] - mx);
      const float lse = mx + __logf(se);
      ls = lse - row[label];
      const float inv = a.grad_scale / (float)M;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) s_dl[tid * NCLS + j] = (__expf(row[j] - lse) - (j == label ? 1.f : 0.f)) * inv;
    } else {
      const float inv = 2.f * a.grad_scale / (float)(M * NCLS);
#pragma unroll
      for (int j = 0; j < NCLS; ++j) {
        const float d = row[j] - (j == label ? 1.f : 0.f);
        ls += d * d;
        s_dl[tid * NCLS + j] = d * inv;
      }
    }
    s_loss[tid] = ls;
    s_cor[tid] = am == label;
  }
  __syncthreads();
  if (tid == 0) {
    float ls = 0.f;
    int nc = 0;
    for (int r = 0; r < rows; ++r) { ls += s_loss[r]; nc += s_cor[r]; }
    a.mpart[g] = ls;
    a.mcorr[g] = nc;
  }
  HEAD_STAMP(4);
  // rows padded to a float4 multiple: the optimizer folds the G rows with float4 loads
  float* prow = a.part + (long)g * ((K * NCLS + NCLS + 3) & ~3);
  if (tid < NCLS) {            // dbh partial
    float acc = 0.f;
    for (int r = 0; r < rows; ++r) acc += s_dl[r * NCLS + tid];
    prow[K * NCLS + tid] = acc;
  }
  // one thread per k: dWh partial[k][:] and dh[:][k]
  for (int k = tid; k < K; k += 256) {
    float dw[NCLS], wk[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) { dw[j] = 0.f; wk[j] = s_w[k * NCLS + j]; }
    for (int r = 0; r < rows; ++r) {
      const float hv = s_h[r * K + k];
      float gv = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) {
        const float d = s_dl[r * NCLS + j];
        dw[j] = fmaf(hv, d, dw[j]);
        gv = fmaf(d, wk[j], gv);
      }
      if (a.dh) {
        if (a.in_act) gv = act_bwd(gv, hv, hv, a.in_act, a.in_alpha);   // post-activation value
        a.dh[(long)(m0 + r) * K + k] = gv;
      }
    }
    float2* p2 = reinterpret_cast<float2*>(prow + k * NCLS);    // part rows: 8 B aligned
#pragma unroll
    for (int j = 0; j < NCLS / 2; ++j) p2[j] = make_float2(dw[2 * j], dw[2 * j + 1]);
  }
  HEAD_STAMP(5);
}

// ---------------------------------------------------------------------------------
// One batch ROW per 256-thread workgroup (the fused one-GPU program, round 3).  The
// head's gradient REDUCTIONS over the batch (dWh, dbh, loss, #correct) are not done
// here: every workgroup writes only its row's outputs, and the last dense layer's fused
// backward (dense_update.hip, "head epilogue") folds them while it runs anyway:
//   dh[m][:]   = act'(dlogits[m] . Wh^T)            (plain stores: that kernel's dY)
//   dl[m][:]   = dlogits[m] (already / M and grad-scaled)
//   rloss[m], rcorr[m]
// The chain is one batched round trip (the row of h and all of Wh, one thread per k),
// 40 FMAs, ten wave reductions folded in fixed order, one lane's softmax, 10 FMAs per k.
// Block 0 advances the device step counter (and the staged batch stream's cursor)
// before any parameter update of the step reads it.
// ---------------------------------------------------------------------------------
constexpr int HR_T = 256;
constexpr int HR_KPT = 4;               // k per thread at most: K <= 1024

struct HeadRowArgs {
  const float* h; int M, K; int in_act; float in_alpha;
  const float* w; const float* b;
  const int64_t* labels; const int64_t* idx; const int64_t* cursor;
  int loss; float grad_scale;
  float* dh; float* dl; float* rloss; int* rcorr;
  int64_t* step; int64_t* adv_cursor; long wrap;
};

// KPT = k per thread, the smallest that covers K (no clamped duplicate loads of Wh rows)
template <int KPT>
__global__ __launch_bounds__(HR_T) void head_row_kernel(HeadRowArgs a) {
  __shared__ float s_part[HR_T / 64][NCLS];
  __shared__ float s_dl[NCLS];
  const int m = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int K = a.K;
  if (m == 0 && tid == 0) {
    *a.step += 1;
    if (a.adv_cursor) {
      const int64_t c = *a.adv_cursor + 1;
      *a.adv_cursor = (a.wrap > 0 && c >= a.wrap) ? 0 : c;
    }
  }
  // every load first: this thread's h values and Wh rows (clamped addresses), the bias
  // and the row's label (the label chain runs under the h / Wh loads)
  float hv[KPT], wv[KPT][NCLS];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int k = min(u * HR_T + tid, K - 1);
    hv[u] = a.h[(long)m * K + k];
#pragma unroll
    for (int j = 0; j < NCLS; j += 2) {
      const float2 t = *reinterpret_cast<const float2*>(a.w + (long)k * NCLS + j);
      wv[u][j] = t.x; wv[u][j + 1] = t.y;
    }
  }
  float bias = lane < NCLS ? a.b[lane] : 0.f;
  int label = 0;
  if (wave == 0) {
    if (!a.idx) label = (int)a.labels[m];
    else label = (int)a.labels[(a.cursor ? a.idx + a.cursor[0] * a.M : a.idx)[m]];
  }
  float acc[NCLS];
#pragma unroll
  for (int j = 0; j < NCLS; ++j) acc[j] = 0.f;
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const bool ok = u * HR_T + tid < K;
    hv[u] = ok ? act_fwd(hv[u], a.in_act, a.in_alpha) : 0.f;     // post-activation value
#pragma unroll
    for (int j = 0; j < NCLS; ++j) acc[j] = fmaf(hv[u], wv[u][j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < NCLS; ++j) {
    const float t = wave_sum_dpp(acc[j]);
    if (lane == 0) s_part[wave][j] = t;
  }
  __syncthreads();
  if (wave == 0) {
    // lane j < 10: logit j (waves folded in fixed order), softmax / mse over the 10 lanes
    float z = -INFINITY;
    if (lane < NCLS) z = s_part[0][lane] + s_part[1][lane] + s_part[2][lane] + s_part[3][lane] + bias;
    const float mx = wave_max(z);
    // argmax: lowest class index attaining the max (the reference's tf.argmax)
    const unsigned long long hit = __ballot(lane < NCLS && z == mx);
    const int am = __builtin_ctzll(hit);
    float d = 0.f, lterm = 0.f;
    if (a.loss == 0) {
      const float e = lane < NCLS ? __expf(z - mx) : 0.f;
      const float se = wave_sum(e);
      const float lse = mx + __logf(se);
      if (lane < NCLS) {
        d = (__expf(z - lse) - (lane == label ? 1.f : 0.f)) * (a.grad_scale / (float)a.M);
        lterm = lane == label ? lse - z : 0.f;
      }
    } else if (lane < NCLS) {
      const float t = z - (lane == label ? 1.f : 0.f);
      lterm = t * t;
      d = t * (2.f * a.grad_scale / (float)(a.M * NCLS));
    }
    const float ls = wave_sum(lterm);
    if (lane < NCLS) {
      s_dl[lane] = d;
      a.dl[(long)m * NCLS + lane] = d;
    }
    if (lane == 0) {
      a.rloss[m] = ls;
      a.rcorr[m] = am == label ? 1 : 0;
    }
  }
  __syncthreads();
  float dl[NCLS];
#pragma unroll
  for (int j = 0; j < NCLS; ++j) dl[j] = s_dl[j];
#pragma unroll
  for (int u = 0; u < KPT; ++u) {
    const int k = u * HR_T + tid;
    if (k >= K) break;
    float g = 0.f;
#pragma unroll
    for (int j = 0; j < NCLS; ++j) g = fmaf(dl[j], wv[u][j], g);
    if (a.in_act) g = act_bwd(g, hv[u], hv[u], a.in_act, a.in_alpha);
    a.dh[(long)m * K + k] = g;
  }
}


template <int KPT, int KQ>
__global__ __launch_bounds__(HD_T) void head_dgrad_kernel(HeadDgradArgs a) {
  head_dgrad_body<KPT, KQ>(a, (int)blockIdx.x);
}

// General fallback (M > 64 or too large for LDS): VALU, operands through L2.
__global__ __launch_bounds__(HT) void head_generic_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_log = smem;
  float* s_red = s_log + a.M * NCLS;
  int* s_cor = (int*)(s_red + 16);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * a.M : a.idx;
  if (tid == 0) *s_cor = 0;
  for (int m = wave; m < a.M; m += NW) {
    float acc[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) acc[j] = 0.f;
    for (int k = lane; k < a.K; k += 64) {
      const float v = act_fwd(a.h[(long)m * a.K + k], a.in_act, a.in_alpha);
#pragma unroll
      for (int j = 0; j < NCLS; ++j) acc[j] = fmaf(v, a.w[(long)k * NCLS + j], acc[j]);
    }
#pragma unroll
    for (int j = 0; j < NCLS; ++j) {
      const float s = wave_sum(acc[j]);
      if (lane == j) s_log[m * NCLS + j] = s;
    }
  }
  __syncthreads();
  head_loss(a, idx, s_log, s_red, s_cor);
  __syncthreads();
  for (int e = tid; e < a.K * NCLS; e += HT) {
    const int k = e / NCLS, j = e % NCLS;
    float acc = 0.f;
    for (int m = 0; m < a.M; ++m)
      acc = fmaf(act_fwd(a.h[(long)m * a.K + k], a.in_act, a.in_alpha), s_log[m * NCLS + j], acc);
    a.dw[e] = acc;
  }
  if (a.dh) {
    for (long e = tid; e < (long)a.M * a.K; e += HT) {
      const int m = (int)(e / a.K), k = (int)(e % a.K);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) acc = fmaf(s_log[m * NCLS + j], a.w[(long)k * NCLS + j], acc);
      if (a.in_act) {
        const float x = a.h[e];
        acc = act_bwd(acc, x, act_fwd(x, a.in_act, a.in_alpha), a.in_act, a.in_alpha);
      }
      a.dh[e] = acc;
    }
  }
}

}  // namespace csa

using namespace csa;

// Rows per workgroup of the partial-output head (0: shape outside its family: more than
// 16 groups of <= 16 rows, K % 4, or the LDS budget).
CSA_NT_SETTER(csa_nt_out_head)

CSA_API int csa_head_debug(long long* p) {
  const int rc = (int)hipMemcpyToSymbol(HIP_SYMBOL(g_hd_dbg), &p, sizeof(p));
  return rc ? rc : (int)hipMemcpyToSymbol(HIP_SYMBOL(g_head_dbg), &p, sizeof(p));
}

CSA_API int csa_head_part_rows(int M, int K) {
  if (M < 1 || K < 4 || K % 4) return 0;
  int rg = 4;
  while ((M + rg - 1) / rg > 16 && rg < PRG_MAX) rg *= 2;
  if ((M + rg - 1) / rg > 16 || head_part_lds(rg, K) > PHEAD_LDS_MAX) return 0;
  return rg;
}

CSA_API int csa_head_part2(const float* h, int M, int K, int in_act, float in_alpha, const float* w,
                           const float* b, const int64_t* labels, const int64_t* idx, const int64_t* cursor,
                           int loss, float grad_scale, float* dh, float* part, float* mpart, int* mcorr,
                           float* logits_out, int64_t* step, int64_t* adv_cursor, long wrap, hipStream_t st);

// Row-per-workgroup head (see head_row_kernel): 0 when K is outside its family.
CSA_API int csa_head_row_ok(int M, int K) { return M >= 1 && K >= 1 && K <= HR_KPT * HR_T && K % 2 == 0 ? 1 : 0; }

CSA_API int csa_head_row(const float* h, int M, int K, int in_act, float in_alpha, const float* w, const float* b,
                         const int64_t* labels, const int64_t* idx, const int64_t* cursor, int loss,
                         float grad_scale, float* dh, float* dl, float* rloss, int* rcorr, int64_t* step,
                         int64_t* adv_cursor, long wrap, hipStream_t st) {
  if (!csa_head_row_ok(M, K) || !dh || !dl || !rloss || !rcorr) return -1;
  HeadRowArgs a{h, M, K, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dh, dl, rloss, rcorr,
                step, adv_cursor, wrap};
  if (K <= HR_T) hipLaunchKernelGGL(head_row_kernel<1>, dim3((unsigned)M), dim3(HR_T), 0, st, a);
  else if (K <= 2 * HR_T) hipLaunchKernelGGL(head_row_kernel<2>, dim3((unsigned)M), dim3(HR_T), 0, st, a);
  else hipLaunchKernelGGL(head_row_kernel<HR_KPT>, dim3((unsigned)M), dim3(HR_T), 0, st, a);
  return (int)hipGetLastError();
}

CSA_API int csa_head_part(const float* h, int M, int K, int in_act, float in_alpha, const float* w,
                          const float* b, const int64_t* labels, const int64_t* idx, const int64_t* cursor,
                          int loss, float grad_scale, float* dh, float* part, float* mpart, int* mcorr,
                          float* logits_out, int64_t* step, hipStream_t st) {
  return csa_head_part2(h, M, K, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dh, part, mpart,
                        mcorr, logits_out, step, nullptr, 0, st);
}

// idx == null: labels are the staged [M] labels of the step; adv_cursor != null: block 0
// advances the batch-stream cursor after the step counter.
CSA_API int csa_head_part2(const float* h, int M, int K, int in_act, float in_alpha, const float* w,
                           const float* b, const int64_t* labels, const int64_t* idx, const int64_t* cursor,
                           int loss, float grad_scale, float* dh, float* part, float* mpart, int* mcorr,
                           float* logits_out, int64_t* step, int64_t* adv_cursor, long wrap, hipStream_t st) {
  const int rg = csa_head_part_rows(M, K);
  if (!rg) return -1;
  HeadPartArgs a{h, M, K, rg, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dh, part,
                 mpart, mcorr, logits_out, step, adv_cursor, wrap};
  const size_t shm = head_part_lds(rg, K);
  if (shm > 64 * 1024) {
    static bool attr = hipFuncSetAttribute((const void*)head_part_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)PHEAD_LDS_MAX) == hipSuccess;
    if (!attr) return -3;
  }
  hipLaunchKernelGGL(head_part_kernel, dim3((unsigned)((M + rg - 1) / rg)), dim3(256), shm, st, a);
  return (int)hipGetLastError();
}

CSA_API int csa_head(const float* h, int M, int K, int in_act, float in_alpha, const float* w,
                     const float* b, const int64_t* labels, const int64_t* idx, int loss,
                     float grad_scale, float* dw, float* db, float* dh, float* logits_out,
                     int64_t* step, float* ring_loss, int* ring_correct, int ring,
                     const int64_t* cursor, int* ws, hipStream_t st) {
  if (M <= 0 || M > 4096) return -1;
  HeadArgs a{h, M, K, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dw, db, dh,
             logits_out, step, ring_loss, ring_correct, ring};
  // dW/db are ACCUMULATED (the caller zeroes them every step); ws = int[4] zeroed once
  const size_t rows_lds =
      ((size_t)RG * NCLS + 4 * 256 + 8 + (size_t)K * NCLS + (size_t)RG * (K + 1)) * sizeof(float);
  // deterministic mode: the single-workgroup generic kernel (fixed-order sums, plain
  // stores; the row-group kernel accumulates dW with atomics)
  if (K % 4 == 0 && rows_lds <= HEAD_LDS_MAX && ws && !g_csa_det) {
    if (rows_lds > 64 * 1024) {
      static bool attr_set = hipFuncSetAttribute((const void*)head_rows_kernel,
                                                 hipFuncAttributeMaxDynamicSharedMemorySize,
                                                 (int)HEAD_LDS_MAX) == hipSuccess;
      if (!attr_set) return -3;
    }
    hipLaunchKernelGGL(head_rows_kernel, dim3((M + RG - 1) / RG), dim3(RT), rows_lds, st, a, ws);
  } else {
    const size_t base = ((size_t)M * NCLS + 32) * sizeof(float);
    if (base > 64 * 1024) {
      if (base > HEAD_LDS_MAX) return -4;
      static bool attr_g = hipFuncSetAttribute((const void*)head_generic_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)HEAD_LDS_MAX) == hipSuccess;
      if (!attr_g) return -3;
    }
    hipLaunchKernelGGL(head_generic_kernel, dim3(1), dim3(HT), base, st, a);
  }
  return (int)hipGetLastError();
}

// Head + last dense layer input gradient (see head_dgrad_kernel): 0 when outside its
// family (Kh a multiple of 64 up to 1024; K1 any).
CSA_API int csa_head_dgrad_ok(int M, int Kh, int K1) {
  return M >= 1 && K1 >= 1 && Kh >= 64 && Kh <= 1024 && Kh % 64 == 0 ? 1 : 0;
}

CSA_API int csa_head_dgrad(const float* h, int M, int Kh, int in_act, float in_alpha, const float* w,
                           const float* b, const int64_t* labels, const int64_t* idx, const int64_t* cursor,
                           int loss, float grad_scale, float* dh, float* dl, float* rloss, int* rcorr,
                           int64_t* step, int64_t* adv_cursor, long wrap, const float* W, int K1,
                           const float* x_fwd, int act, float alpha, float* dX, hipStream_t st) {
  if (!csa_head_dgrad_ok(M, Kh, K1) || !dh || !dl || !rloss || !rcorr || !W || !dX || !step) return -1;
  if (act && !x_fwd) return -2;
  HeadDgradArgs a{h, M, Kh, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dh, dl, rloss, rcorr,
                  step, adv_cursor, wrap, W, K1, x_fwd, act, alpha, dX};
  if (g_hd_rec.on) {                     // the fused forward chain launches it (dense_direct.hip)
    g_hd_rec.a = a; g_hd_rec.kq = Kh / 64; g_hd_rec.has = 1;
    return 0;
  }
  const int blocks = ((M + HD_R - 1) / HD_R) * ((K1 + HD_FS - 1) / HD_FS);
  const dim3 grid((unsigned)blocks), blk(HD_T);
  const int kq = Kh / 64;
#define HD_CASE(KQ)                                                                         \
  case KQ:                                                                                  \
    hipLaunchKernelGGL((head_dgrad_kernel<(KQ * 64 + HD_T - 1) / HD_T, KQ>), grid, blk, 0, st, a); \
    break;
  switch (kq) {
    HD_CASE(1) HD_CASE(2) HD_CASE(3) HD_CASE(4) HD_CASE(5) HD_CASE(6) HD_CASE(7) HD_CASE(8)
    HD_CASE(9) HD_CASE(10) HD_CASE(11) HD_CASE(12) HD_CASE(13) HD_CASE(14) HD_CASE(15) HD_CASE(16)
    default: return -1;
  }
#undef HD_CASE
  return (int)hipGetLastError();
}
