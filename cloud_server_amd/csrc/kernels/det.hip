// Deterministic mode (CSA_DETERMINISTIC=1) for the hand-written kernels.
//
// The fast path accumulates partial results across workgroups with float atomics:
// split-K GEMM outputs, BatchNorm statistic slabs (rows shared by many workgroups) and
// weight-gradient stripes.  fp32 addition is not associative, so the arrival order of
// those atomics changes the last bits of a step from run to run.  The reference's train
// op (construct_distribute.py:372-373) ran on TF's CPU kernels, which reduce in a fixed
// order; deterministic mode restores that property on the GPU without leaving HIP:
//
//   * every cross-workgroup accumulation gets EXCLUSIVE destinations — one slab row or
//     one stripe per producing workgroup (an atomic onto a zeroed slot with a single
//     contributor is exact), split-K is off;
//   * ``csa_rows_fold`` then reduces the R rows in a fixed order (row slices in order,
//     then the slices in order) — the result depends only on the data, never on timing;
//   * every reduction INSIDE a workgroup on those paths is already fixed-order.
//
// The flag is per-thread host state read by the launch-configuration helpers (split-K
// factors, slab row counts); the step program sets it around its own planning and launches.
#include "common.h"

namespace csa {

thread_local int g_csa_det = 0;
thread_local int g_csa_packed = 0;
thread_local int g_csa_shared = 0;

constexpr int RF_COLS = 64;      // columns per workgroup
constexpr int RF_SL = 4;         // row slices per column (one per wave)
constexpr int RF_U = 8;          // loads in flight per thread

// dst[j] = sum_{r < R} src[r * ld + j] for j < n, rows in slices [s * per, (s + 1) * per)
// summed in order, then the RF_SL slices in order.  zero_src: the rows are re-zeroed
// after they were read (accumulators whose only reader is this fold).  dst may alias
// row 0 of src (each column is read completely before its result is written).
__global__ __launch_bounds__(RF_COLS * RF_SL) void rows_fold_kernel(const float* src, long ld, int R, long n,
                                                                    float* dst, int zero_src) {
  __shared__ float s_part[RF_SL][RF_COLS];
  const int c = threadIdx.x % RF_COLS, sl = threadIdx.x / RF_COLS;
  const long j = (long)blockIdx.x * RF_COLS + c;
  const int per = (R + RF_SL - 1) / RF_SL;
  const int r0 = sl * per, r1 = min(R, r0 + per);
  const long jj = j < n ? j : n - 1;
  float acc = 0.f;
  for (int r = r0; r < r1; r += RF_U) {
    float v[RF_U];
#pragma unroll
    for (int u = 0; u < RF_U; ++u) v[u] = src[(long)min(r + u, r1 - 1) * ld + jj];
#pragma unroll
    for (int u = 0; u < RF_U; ++u) pin(v[u]);
#pragma unroll
    for (int u = 0; u < RF_U; ++u)
      if (r + u < r1) acc += v[u];
  }
  s_part[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && j < n) {
    float t = 0.f;
#pragma unroll
    for (int s = 0; s < RF_SL; ++s) t += s_part[s][c];
    dst[j] = t;
  }
  if (zero_src && j < n)
    for (int r = r0; r < r1; ++r) const_cast<float*>(src)[(long)r * ld + j] = 0.f;
}

// Several folds in ONE launch (the data-parallel program folds the conv pair's four striped
// gradients into the flat gradient before their bucket is exchanged: four launches of a
// couple of µs each were serial links of the step).  Block b belongs to the job whose
// block range holds it; the job is chosen by uniform selects of named fields (no argument
// arrays indexed at run time: those are copied to scratch by every workgroup).
struct RFJob { const float* src; long ld; long n; float* dst; int R; int zero; int blk0; int pad; };
struct RFMulti { RFJob j0, j1, j2, j3; int njobs; };

__global__ __launch_bounds__(RF_COLS * RF_SL) void rows_fold_multi_kernel(RFMulti a) {
  __shared__ float s_part[RF_SL][RF_COLS];
  const int b = blockIdx.x;
  RFJob J = a.j0;
  if (a.njobs > 1 && b >= a.j1.blk0) J = a.j1;
  if (a.njobs > 2 && b >= a.j2.blk0) J = a.j2;
  if (a.njobs > 3 && b >= a.j3.blk0) J = a.j3;
  const int c = threadIdx.x % RF_COLS, sl = threadIdx.x / RF_COLS;
  const long j = (long)(b - J.blk0) * RF_COLS + c;
  const int per = (J.R + RF_SL - 1) / RF_SL;
  const int r0 = sl * per, r1 = min(J.R, r0 + per);
  const long jj = j < J.n ? j : J.n - 1;
  float acc = 0.f;
  for (int r = r0; r < r1; r += RF_U) {
    float v[RF_U];
#pragma unroll
    for (int u = 0; u < RF_U; ++u) v[u] = J.src[(long)min(r + u, r1 - 1) * J.ld + jj];
#pragma unroll
    for (int u = 0; u < RF_U; ++u) pin(v[u]);
#pragma unroll
    for (int u = 0; u < RF_U; ++u)
      if (r + u < r1) acc += v[u];
  }
  s_part[sl][c] = acc;
  __syncthreads();
  if (sl == 0 && j < J.n) {
    float t = 0.f;
#pragma unroll
    for (int s2 = 0; s2 < RF_SL; ++s2) t += s_part[s2][c];
    J.dst[j] = t;
  }
  if (J.zero && j < J.n)
    for (int r = r0; r < r1; ++r) const_cast<float*>(J.src)[(long)r * J.ld + j] = 0.f;
}

}  // namespace csa

using namespace csa;

// Up to 4 csa_rows_fold jobs as one launch (same arithmetic, same fixed order).
CSA_API int csa_rows_fold_multi(int njobs, const float* const* src, const long* ld, const int* R, const long* n,
                                float* const* dst, const int* zero_src, hipStream_t st) {
  if (njobs < 1 || njobs > 4) return -1;
  RFMulti a{};
  RFJob* js[4] = {&a.j0, &a.j1, &a.j2, &a.j3};
  int blk = 0;
  for (int k = 0; k < njobs; ++k) {
    if (!src[k] || !dst[k] || R[k] < 1 || n[k] < 1 || ld[k] < n[k]) return -1;
    if (zero_src[k] && dst[k] >= src[k] && dst[k] < src[k] + (long)R[k] * ld[k]) return -2;
    *js[k] = RFJob{src[k], ld[k], n[k], dst[k], R[k], zero_src[k], blk, 0};
    blk += (int)((n[k] + RF_COLS - 1) / RF_COLS);
  }
  a.njobs = njobs;
  hipLaunchKernelGGL(rows_fold_multi_kernel, dim3((unsigned)blk), dim3(RF_COLS * RF_SL), 0, st, a);
  return (int)hipGetLastError();
}

CSA_API void csa_set_deterministic(int on) { g_csa_det = on ? 1 : 0; }
CSA_API int csa_deterministic() { return g_csa_det; }
CSA_API void csa_set_packed(int on) { g_csa_packed = on ? 1 : 0; }
CSA_API int csa_packed() { return g_csa_packed; }
CSA_API void csa_set_shared_gpu(int on) { g_csa_shared = on ? 1 : 0; }
CSA_API int csa_shared_gpu() { return g_csa_shared; }

CSA_API int csa_rows_fold(const float* src, long ld, int R, long n, float* dst, int zero_src, hipStream_t st) {
  if (!src || !dst || R < 1 || n < 1 || ld < n) return -1;
  if (zero_src && dst >= src && dst < src + (long)R * ld) return -2;   // would zero the result
  hipLaunchKernelGGL(rows_fold_kernel, dim3((unsigned)((n + RF_COLS - 1) / RF_COLS)), dim3(RF_COLS * RF_SL), 0, st,
                     src, ld, R, n, dst, zero_src);
  return (int)hipGetLastError();
}
