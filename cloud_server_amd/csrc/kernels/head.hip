// Fused classifier head + loss + head backward + step bookkeeping (one workgroup).
//
// Reference: the fixed 10-way head (construct_distribute.py:252-264), the loss
// (softmax-xent 'entropy' or 'mse', :285-298), the accuracy op (:381-382) and the
// global_step increment done by minimize() (:372-373).  At B = 50 the whole head is
// ~0.8 MFLOP, less than one launch's fixed cost, so ONE 1024-thread workgroup does it:
//   stage T(h) (T = optional activation of the head input; rows padded to K+1 floats so
//   MFMA operand reads are bank-conflict free) and Wh in LDS,
//   logits = T(h) @ Wh + bh      — f32 MFMA 32x32x2, K split over the 16 waves,
//   loss, dlogits (scaled by grad_scale = 1/world), #correct,
//   dWh = T(h)^T dlogits, dbh    — MFMA, one 32-row tile of Wh per wave,
//   dh  = (dlogits @ Wh^T) * T'  — MFMA, two 32x32 tiles per wave,
//   ring_loss[step % R] = loss, ring_correct[step % R] = #correct, step += 1
// so metrics never force a host sync inside the training loop.  (A VALU version with
// both dot-product operands in LDS was LDS-bandwidth bound at ~38 µs.)
//
// MFMA 32x32x2 f32 operand map: A lane l = A[l&31][l>>5], B lane l = B[l>>5][l&31],
// D reg r of lane l = D[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31].
#include "common.h"
#include <cstdlib>

namespace csa {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int HT = 1024;
constexpr int NW = HT / 64;
constexpr int NCLS = 10;
constexpr int MPAD = 64;                  // batch rows handled by the MFMA path
constexpr size_t HEAD_LDS_MAX = 160 * 1024;

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
  long long* dbg;                          // optional s_memtime stamps (diagnostics)
};

#define HEAD_STAMP(i) \
  do { if (a.dbg && threadIdx.x == 0) a.dbg[i] = (long long)__builtin_amdgcn_s_memtime(); } while (0)

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

// M <= 64 and M*(K+1) + 10K floats fit in LDS: the MFMA path (v_mfma_f32_16x16x4_f32:
// 10 classes pad to 16 columns instead of 32).  16x16x4 map: A lane l = A[l&15][l>>4],
// B lane l = B[l>>4][l&15], D reg r of lane l = D[4*(l>>4) + r][l&15].
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(HT) void head_mfma_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int M = a.M, K = a.K, KP = K + 1;
  float* s_log = smem;                     // [64][10] logits, then dlogits (rows >= M zero)
  float* s_red = s_log + MPAD * NCLS;      // [16]
  int* s_cor = (int*)(s_red + 16);
  float* s_part = s_red + 32;              // [16 waves][16 rows][16 cols] logits partials
  float* s_w = s_part + NW * 256;          // [K][10]
  float* s_h = s_w + K * NCLS;             // [M][K+1]  T(h)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * M : a.idx;
  HEAD_STAMP(0);
  // labels / bias early: their latency hides under the staging
  int my_label = 0;
  if (tid < M) my_label = (int)a.labels[idx[tid]];

  for (int i = tid; i < MPAD * NCLS; i += HT) s_log[i] = 0.f;
  if (tid == 0) *s_cor = 0;
  stage_to_lds<4>(s_w, a.w, K * NCLS, [](float v, int) { return v; });
  {  // T(h) into padded rows: float4 loads, all of a thread's loads in flight together
    const int act = a.in_act;
    const float alpha = a.in_alpha;
    const int n4 = (M * K) >> 2;            // K % 4 == 0 on this path
    const int K4 = K >> 2;
    const FastDiv dk4(K4);
    for (int base = 0; base < n4; base += HT * 8) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * HT + tid;
        v[u] = reinterpret_cast<const float4*>(a.h)[i < n4 ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = base + u * HT + tid;
        if (i < n4) {
          int m, k4;
          dk4.divmod(i, m, k4);
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
  HEAD_STAMP(1);

  // ---- 1) logits: wave = (16-row M tile mt, K quarter kq); partials in LDS ----
  {
    const int mt = wave & 3, kq = wave >> 2;
    const int r = lane & 15, hk = lane >> 4;
    const int kper = ((K + 3) / 4 + 3) & ~3;
    const int kb = kq * kper, ke = min(K, kb + kper);
    const int m = min(mt * 16 + r, M - 1);
    const bool okm = mt * 16 + r < M, okj = r < NCLS;
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
  for (int e = tid; e < MPAD * NCLS; e += HT) {   // reduce the 4 K quarters
    const int row = e / NCLS, j = e % NCLS, mt = row >> 4, rr = row & 15;
    float v = 0.f;
#pragma unroll
    for (int kq = 0; kq < 4; ++kq) v += s_part[(kq * 4 + mt) * 256 + rr * 16 + j];
    s_log[e] = row < M ? v : 0.f;
  }
  __syncthreads();
  HEAD_STAMP(2);

  // ---- 2) loss / dlogits / accuracy / bookkeeping ----
  head_loss(a, idx, s_log, s_red, s_cor, my_label);
  __syncthreads();
  HEAD_STAMP(3);

  // ---- 3) dWh[k][j] = sum_m T(h)[m][k] dl[m][j]: 16-row k tiles over the waves ----
  {
    const int r = lane & 15, hk = lane >> 4;
    for (int kt = wave; kt * 16 < K; kt += NW) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int k = kt * 16 + r;
      const int kc = min(k, K - 1);
      for (int m = 0; m < M; m += 4) {
        const int mm = m + hk;                     // s_log rows >= M are zero
        const float hv = s_h[min(mm, M - 1) * KP + kc];
        const float lv = s_log[mm * NCLS + (r < NCLS ? r : 0)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(hv, r < NCLS ? lv : 0.f, acc, 0, 0, 0);
      }
      if (r < NCLS) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int kr = kt * 16 + 4 * hk + i;
          if (kr < K) a.dw[kr * NCLS + r] = acc[i];
        }
      }
    }
  }
  HEAD_STAMP(4);

  // ---- 4) dh[m][k] = (sum_j dl[m][j] Wh[k][j]) * T'(h): (16-row m, 16-col k) tiles ----
  if (a.dh) {
    const int r = lane & 15, hk = lane >> 4;
    const int nkt = (K + 15) / 16;
    const int nmt = (M + 15) / 16;
    for (int t = wave; t < nmt * nkt; t += NW) {
      const int mt = t / nkt, kt = t % nkt;
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      const int m = mt * 16 + r, k = kt * 16 + r;
#pragma unroll
      for (int j = 0; j < 12; j += 4) {            // 10 classes -> 3 k-steps of 4
        const int jj = j + hk;
        const bool okj = jj < NCLS;
        const float lv = s_log[m * NCLS + (okj ? jj : 0)];    // m < 64: rows >= M zero
        const float wv = s_w[min(k, K - 1) * NCLS + (okj ? jj : 0)];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(okj ? lv : 0.f, (okj && k < K) ? wv : 0.f, acc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int mr = mt * 16 + 4 * hk + i;
        if (mr < M && k < K) {
          float g = acc[i];
          if (a.in_act) {  // post-activation value decides every supported derivative
            const float y = s_h[mr * KP + k];
            g = act_bwd(g, y, y, a.in_act, a.in_alpha);
          }
          a.dh[(long)mr * K + k] = g;
        }
      }
    }
  }
  HEAD_STAMP(5);
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

CSA_API int csa_head(const float* h, int M, int K, int in_act, float in_alpha, const float* w,
                     const float* b, const int64_t* labels, const int64_t* idx, int loss,
                     float grad_scale, float* dw, float* db, float* dh, float* logits_out,
                     int64_t* step, float* ring_loss, int* ring_correct, int ring,
                     const int64_t* cursor, hipStream_t st) {
  if (M <= 0 || M > 4096) return -1;
  HeadArgs a{h, M, K, in_act, in_alpha, w, b, labels, idx, cursor, loss, grad_scale, dw, db, dh,
             logits_out, step, ring_loss, ring_correct, ring, nullptr};
  if (const char* e = getenv("CSA_HEAD_DBG")) a.dbg = (long long*)strtoull(e, nullptr, 0);
  const size_t mfma_lds =
      ((size_t)MPAD * NCLS + 32 + NW * 256 + (size_t)K * NCLS + (size_t)M * (K + 1)) * sizeof(float);
  if (M <= MPAD && K % 4 == 0 && mfma_lds <= HEAD_LDS_MAX) {
    static bool attr_set = hipFuncSetAttribute((const void*)head_mfma_kernel,
                                               hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)HEAD_LDS_MAX) == hipSuccess;
    (void)attr_set;
    hipLaunchKernelGGL(head_mfma_kernel, dim3(1), dim3(HT), mfma_lds, st, a);
  } else {
    const size_t base = ((size_t)M * NCLS + 32) * sizeof(float);
    hipLaunchKernelGGL(head_generic_kernel, dim3(1), dim3(HT), base, st, a);
  }
  return (int)hipGetLastError();
}
