// Fused classifier head + loss + head backward + step bookkeeping (one workgroup).
//
// Reference: the fixed 10-way head (construct_distribute.py:252-264), the loss
// (softmax-xent 'entropy' or 'mse', :285-298), the accuracy op (:381-382) and the
// global_step increment done by minimize() (:372-373).  At B = 50 the whole head is
// ~0.8 MFLOP — far less than one launch's fixed cost — so ONE 1024-thread workgroup:
//   stages T(h) (T = optional activation of the head input) and Wh in LDS (122 KB of
//   the CU's 160 KB at B=50, K=512; larger shapes read through L2 instead),
//   logits = T(h) @ Wh + bh; loss, dlogits (scaled by grad_scale = 1/world), #correct;
//   dWh = T(h)^T dlogits, dbh = colsum(dlogits) -> gradient buffer;
//   dh  = (dlogits @ Wh^T) * T'(h) -> input grad of the previous layer;
//   ring_loss[step % R] = loss, ring_correct[step % R] = #correct, step += 1
// so metrics never force a host sync inside the training loop.
#include "common.h"

namespace csa {

constexpr int HT = 1024;
constexpr int NCLS = 10;
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

template <bool STAGED>
__global__ __launch_bounds__(HT) void head_kernel(HeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* s_log = smem;                          // [M][10] logits, then dlogits
  float* s_red = s_log + a.M * NCLS;            // [16] partial loss
  int* s_cor = (int*)(s_red + 16);
  float* s_w = s_red + 32;                      // [K][10]   (STAGED)
  float* s_h = s_w + a.K * NCLS;                // [M][K]    T(h) (STAGED)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, nw = HT / 64;
  const int64_t* idx = a.cursor ? a.idx + a.cursor[0] * a.M : a.idx;
  if (tid == 0) *s_cor = 0;
  if (STAGED) {
    stage_to_lds<4>(s_w, a.w, a.K * NCLS, [](float v, int) { return v; });
    const int act = a.in_act;
    const float alpha = a.in_alpha;
    stage_to_lds<8>(s_h, a.h, a.M * a.K, [&](float v, int) { return act_fwd(v, act, alpha); });
    __syncthreads();
  }
  auto TH = [&](int m, int k) -> float {
    return STAGED ? s_h[(long)m * a.K + k] : act_fwd(a.h[(long)m * a.K + k], a.in_act, a.in_alpha);
  };
  auto WW = [&](int k, int j) -> float { return STAGED ? s_w[k * NCLS + j] : a.w[(long)k * NCLS + j]; };

  // 1) logits: one wave per batch row, lanes split K
  for (int m = wave; m < a.M; m += nw) {
    float acc[NCLS];
#pragma unroll
    for (int j = 0; j < NCLS; ++j) acc[j] = 0.f;
    for (int k = lane; k < a.K; k += 64) {
      const float v = TH(m, k);
#pragma unroll
      for (int j = 0; j < NCLS; ++j) acc[j] = fmaf(v, WW(k, j), acc[j]);
    }
#pragma unroll
    for (int j = 0; j < NCLS; ++j) {
      const float s = wave_sum(acc[j]);
      if (lane == j) s_log[m * NCLS + j] = s + a.b[j];
    }
  }
  __syncthreads();

  // 2) loss / dlogits / accuracy: one lane per row
  float lsum = 0.f;
  for (int m = tid; m < a.M; m += HT) {
    const int y = (int)a.labels[idx[m]];
    float* row = s_log + m * NCLS;
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
      const float inv = a.grad_scale / (float)a.M;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) row[j] = (__expf(row[j] - lse) - (j == y ? 1.f : 0.f)) * inv;
    } else {
      const float inv = 2.f * a.grad_scale / (float)(a.M * NCLS);
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
    for (int i = 0; i < nw; ++i) t += s_red[i];
    t = (a.loss == 0) ? t / a.M : t / (a.M * NCLS);
    const int64_t st = *a.step;
    const int pos = (int)(st % a.ring);
    a.ring_loss[pos] = t;
    a.ring_correct[pos] = *s_cor;
    *a.step = st + 1;
  }

  // 3) dWh[k][j] = sum_m T(h)[m][k] * dl[m][j];  dbh
  for (int e = tid; e < a.K * NCLS; e += HT) {
    const int k = e / NCLS, j = e % NCLS;
    float acc = 0.f;
    int m = 0;
    for (; m + 8 <= a.M; m += 8) {     // 16 LDS reads in flight per step
      float hv[8], lv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) { hv[u] = TH(m + u, k); lv[u] = s_log[(m + u) * NCLS + j]; }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = fmaf(hv[u], lv[u], acc);
    }
    for (; m < a.M; ++m) acc = fmaf(TH(m, k), s_log[m * NCLS + j], acc);
    a.dw[e] = acc;
  }
  if (tid < NCLS) {
    float acc = 0.f;
    for (int m = 0; m < a.M; ++m) acc += s_log[m * NCLS + tid];
    a.db[tid] = acc;
  }
  // 4) dh[m][k] = (sum_j dl[m][j] * Wh[k][j]) * T'(h)
  if (a.dh) {
    for (long e = tid; e < (long)a.M * a.K; e += HT) {
      const int m = (int)(e / a.K), k = (int)(e % a.K);
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < NCLS; ++j) acc = fmaf(s_log[m * NCLS + j], WW(k, j), acc);
      if (a.in_act) {
        if (STAGED) {   // post-activation value decides every supported derivative
          const float y = s_h[e];
          acc = act_bwd(acc, y, y, a.in_act, a.in_alpha);
        } else {
          const float x = a.h[e];
          acc = act_bwd(acc, x, act_fwd(x, a.in_act, a.in_alpha), a.in_act, a.in_alpha);
        }
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
             logits_out, step, ring_loss, ring_correct, ring};
  const size_t base = ((size_t)M * NCLS + 32) * sizeof(float);
  const size_t staged = base + ((size_t)K * NCLS + (size_t)M * K) * sizeof(float);
  if (staged <= HEAD_LDS_MAX) {
    static bool attr_set = false;
    if (!attr_set) {
      hipFuncSetAttribute((const void*)head_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)HEAD_LDS_MAX);
      attr_set = true;
    }
    hipLaunchKernelGGL(head_kernel<true>, dim3(1), dim3(HT), staged, st, a);
  } else {
    hipLaunchKernelGGL(head_kernel<false>, dim3(1), dim3(HT), base, st, a);
  }
  return (int)hipGetLastError();
}
