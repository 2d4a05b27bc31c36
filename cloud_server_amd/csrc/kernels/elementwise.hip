// Elementwise kernels of the training step (gfx950 / CDNA4).
//
// csa_bn_act_apply: y = act(x * a[c] + b[c]) with (a, b) from the BatchNorm forward
// slab (common.h) — the reference's tf.nn.batch_normalization + activation
// (construct_distribute.py:155-165, 133-152) materialised ONCE for a dense consumer,
// so the GEMM prologues of its forward and weight-gradient launches stream plain float4
// operands instead of recomputing BN + sigmoid per N-tile (measured: the recompute made
// those GEMMs VALU-bound).
#include "common.h"

namespace csa {

struct ApplyArgs {
  const float* x; float* y; long n; int C; BNRef bn; int act; float alpha;
  float* tab;   // optional [4][C] mean | rstd | a | b for later consumers (block 0 writes)
  unsigned* clear;   // optional word block 0 zeroes (the carried update's pending flag)
};

// diagnostics: per-workgroup start / end (s_memrealtime, 100 MHz) at [2 b], [2 b + 1]
// (csa_ew_life_debug; scripts/mb/graph_life.py)
__constant__ long long* g_ew_life = nullptr;

__global__ __launch_bounds__(256) void bn_act_apply_kernel(ApplyArgs a) {
  __shared__ float s_bn[4 * 128 + 2 * 128];
  if (g_ew_life && threadIdx.x == 0) g_ew_life[2 * blockIdx.x] = (long long)__builtin_amdgcn_s_memrealtime();
  // the element loads go out before the slab reduction (overlapping round trips)
  const long i4 = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n4 = a.n >> 2;
  float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) v = reinterpret_cast<const float4*>(a.x)[i4];
  bn_reduce_to_lds(a.bn, s_bn, s_bn + 128, s_bn + 256, s_bn + 384, s_bn + 512);
  __syncthreads();
  if (a.clear && blockIdx.x == 0 && threadIdx.x == 0) *a.clear = 0u;
  if (a.tab && blockIdx.x == 0)
    for (int c = threadIdx.x; c < 4 * a.C; c += blockDim.x) a.tab[c] = s_bn[(c / a.C) * 128 + c % a.C];
  if (g_ew_life && threadIdx.x == 0) g_ew_life[2 * blockIdx.x + 1] = (long long)__builtin_amdgcn_s_memrealtime();
  if (i4 >= n4) return;
  const FastDiv dc(a.C);
  int q, c0;
  dc.divmod((int)((i4 * 4) % (long)a.C), q, c0);
  float o[4] = {v.x, v.y, v.z, v.w};
  int c = c0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    o[u] = act_fwd(o[u] * s_bn[256 + c] + s_bn[384 + c], a.act, a.alpha);
    c = (c + 1 == a.C) ? 0 : c + 1;
  }
  out_store4(a.y + 4 * i4, make_float4(o[0], o[1], o[2], o[3]));
}

}  // namespace csa

using namespace csa;

CSA_NT_SETTER(csa_nt_out_ew)

CSA_API int csa_ew_life_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_ew_life), &p, sizeof(p));
}

// The next bn_act_apply launched by this thread also zeroes *p (block 0): the carried dense
// update's pending flag, retired right after the carrying pair forward (conv_pair.hip).
static thread_local unsigned* g_ew_clear = nullptr;
CSA_API void csa_ew_clear_next(unsigned* p) { g_ew_clear = p; }

// n % 4 == 0; channel of element e is e % C (NHWC flattened).
CSA_API int csa_bn_act_apply(const float* x, float* y, long n, int C, const float* bn_slab,
                             int bn_nslab, float bn_count, float bn_eps, const float* bn_scale,
                             const float* bn_offset, int act, float alpha, float* tab, hipStream_t st) {
  if (n % 4 || C > 128 || C <= 0) return -1;
  ApplyArgs a{x, y, n, C, BNRef{bn_slab, bn_nslab, C, bn_count, bn_eps, bn_scale, bn_offset}, act, alpha, tab,
              g_ew_clear};
  g_ew_clear = nullptr;
  const long n4 = n / 4;
  hipLaunchKernelGGL(bn_act_apply_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
