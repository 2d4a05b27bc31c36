// Shared device helpers for the cloud_server_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//  * activations are NHWC fp32, conv weights HWIO, dense weights [in, out] row-major
//    (the reference's TF layouts, construct_distribute.py:91-118, 168-182);
//  * wave = 64 lanes; block sizes are multiples of 64;
//  * a launcher never allocates, copies or synchronises (everything is HIP-graph
//    capturable); scratch comes from a caller-owned workspace;
//  * every launcher returns hipGetLastError() as an int (0 == ok).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define CSA_API extern "C" __attribute__((visibility("default")))

// Non-temporal stores for the activations one launch writes for the next (A/B knob,
// CSA_NT_OUT): each code object has its own flag and setter (CSA_NT_SETTER).
typedef float csa_f2v __attribute__((ext_vector_type(2)));
typedef float csa_f4v __attribute__((ext_vector_type(4)));
static __constant__ int g_nt_out = 0;
#define CSA_NT_SETTER(name)                                                                   \
  CSA_API int name(int on) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_nt_out), &on, sizeof(on)); }
__device__ __forceinline__ void out_store(float* p, float v) {
  if (g_nt_out) __builtin_nontemporal_store(v, p); else *p = v;
}
__device__ __forceinline__ void out_store2(float* p, float a, float b) {
  if (g_nt_out) { csa_f2v w = {a, b}; __builtin_nontemporal_store(w, reinterpret_cast<csa_f2v*>(p)); }
  else *reinterpret_cast<float2*>(p) = make_float2(a, b);
}
__device__ __forceinline__ void out_store4(float* p, float4 v) {
  if (g_nt_out) { csa_f4v w = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(w, reinterpret_cast<csa_f4v*>(p)); }
  else *reinterpret_cast<float4*>(p) = v;
}

namespace csa {

enum Act : int { ACT_NONE = 0, ACT_SIGMOID = 1, ACT_RELU = 2, ACT_LEAKY = 3 };

// Deterministic mode (det.hip, host state of the CALLING thread: a job planned on a builder
// thread never changes the launch shapes of a job stepping on another): launch helpers
// choose exclusive destinations and no split-K, so no float atomic has more than one
// contributor per slot.
extern thread_local int g_csa_det;
// Packed profile (det.hip, host state): a process that packs several jobs onto one GPU
// prefers launch shapes with less CU-time per job-step over the lowest latency alone.
extern thread_local int g_csa_packed;
// Shared-GPU profile (det.hip, host state): several ranks of one job run on ONE GPU (the
// multi-process tests); no launch may depend on a 16-wave workgroup being placed while a
// peer rank's kernel spins in a peer wait.
extern thread_local int g_csa_shared;

__device__ __forceinline__ float act_fwd(float x, int act, float alpha) {
  switch (act) {
    case ACT_SIGMOID: return __builtin_amdgcn_rcpf(1.0f + __expf(-x));   // v_exp + v_rcp
    case ACT_RELU: return x > 0.f ? x : 0.f;
    case ACT_LEAKY: return fmaxf(x, alpha * x);  // tf.maximum(x, a*x)
    default: return x;
  }
}

// derivative expressed through the pre-activation x and the output y
__device__ __forceinline__ float act_bwd(float g, float x, float y, int act, float alpha) {
  switch (act) {
    case ACT_SIGMOID: return g * y * (1.0f - y);
    case ACT_RELU: return x > 0.f ? g : 0.f;
    case ACT_LEAKY: return (x >= alpha * x) ? g : g * alpha;
    default: return g;
  }
}

// Division by a runtime constant through a float reciprocal (exact for 0 <= x < 2^22
// after a +-1 fix-up): ~6 VALU ops instead of the ~40-op integer division sequence.
struct FastDiv {
  int d; float inv;
  __host__ __device__ FastDiv() : d(1), inv(1.f) {}
  __host__ __device__ explicit FastDiv(int dd) : d(dd < 1 ? 1 : dd), inv(1.0f / (float)(dd < 1 ? 1 : dd)) {}
  __device__ __forceinline__ int div(int x) const {
    int q = __float2int_rz((float)x * inv);
    if ((q + 1) * d <= x) ++q;
    if (q * d > x) --q;
    return q;
  }
  __device__ __forceinline__ void divmod(int x, int& q, int& r) const {
    q = div(x);
    r = x - q * d;
  }
};

// Materialise loaded values here (the empty asm "reads and writes" them): hipcc otherwise
// sinks each load into the conditional block that consumes it and waits for it there, one
// serial memory round trip per element.  Pin a batch of loads after issuing all of them.
__device__ __forceinline__ void pin(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void pin(float& v) { asm volatile("" : "+v"(v)); }
__device__ __forceinline__ void pin(int& v) { asm volatile("" : "+v"(v)); }

// Block-cooperative copy global -> LDS with a per-element transform, issuing UNROLL
// independent loads per thread before any store (branch-free clamped addresses), so a
// thread waits for one memory round trip per UNROLL elements instead of one per element
// (hipcc otherwise emits load -> s_waitcnt vmcnt(0) -> store for every iteration).
template <int UNROLL, class T, class F>
__device__ __forceinline__ void stage_to_lds(float* dst, const T* src, int n, F f) {
  const int step = blockDim.x * UNROLL;
  for (int base = 0; base < n; base += step) {
    T v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int i = base + u * blockDim.x + threadIdx.x;
      v[u] = src[i < n ? i : 0];
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int i = base + u * blockDim.x + threadIdx.x;
      if (i < n) dst[i] = f(v[u], i);
    }
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Wave64 sum with DPP inside each row of 16 lanes (quad swaps, half-row and row mirrors:
// VALU data movement, no LDS round trip) and two cross-row shuffles; every lane gets it.
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xb1, 0xf, 0xf, false));   // quad_perm 1,0,3,2
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4e, 0xf, 0xf, false));   // quad_perm 2,3,0,1
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xf, 0xf, false));  // row_half_mirror
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xf, 0xf, false));  // row_mirror
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---------------------------------------------------------------------------------
// BatchNorm statistics travel between kernels as per-workgroup partial slabs
// [nslab][2][C] = {sum x, sum x^2} (forward) or {sum dz, sum dz*xhat} (backward).
// A consumer reduces the slab itself at kernel start (a few KB, L2-resident), which
// removes the separate "finalize" launch a textbook BN needs.
// ---------------------------------------------------------------------------------
struct BNRef {
  const float* slab;    // [nslab][2][C] forward partial sums
  int nslab;
  int C;
  float count;          // elements per channel (B*H*W)
  float eps;
  const float* scale;   // [C]
  const float* offset;  // [C]
};

// Sum a partial slab [nslab][2C] over its rows into s_out[2C], using the whole block.
// Each thread owns one fixed column (t % 2C) so it sums locally and issues ONE LDS atomic
// (a serial per-channel loop over the rows was latency-bound: ~60 µs per launch).
// Must be called by every thread of the block; ends with a barrier.
__device__ __forceinline__ void slab_sum_to_lds(const float* slab, int nslab, int C2, float* s_out) {
  for (int i = threadIdx.x; i < C2; i += blockDim.x) s_out[i] = 0.f;
  __syncthreads();
  const int per = (int)blockDim.x / C2;          // threads per column
  if (per > 0) {
    const int col = threadIdx.x % C2, lane_row = threadIdx.x / C2;
    if (lane_row < per) {
      // batches of 16 loads in flight per thread (a load -> add chain is one memory round
      // trip per row; a 32-row slab over 2 threads per column is then ONE round trip)
      constexpr int U = 16;
      float acc = 0.f;
      for (int r0 = lane_row; r0 < nslab; r0 += U * per) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int r = r0 + u * per;
          v[u] = slab[(size_t)(r < nslab ? r : 0) * C2 + col];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) pin(v[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) acc += (r0 + u * per < nslab) ? v[u] : 0.f;
      }
      atomicAdd(&s_out[col], acc);
    }
  } else {
    for (int col = threadIdx.x; col < C2; col += blockDim.x) {
      float acc = 0.f;
      for (int r = 0; r < nslab; ++r) acc += slab[(size_t)r * C2 + col];
      s_out[col] = acc;
    }
  }
  __syncthreads();
}

// Deterministic-mode replacement of the per-thread LDS atomics that fold channel partials:
// thread t holds partials v1[c], v2[c] of channel (t % G) * CB + c; out[ch] / out[C + ch]
// receive the sums over t = g, g + G, g + 2G, ... in ascending order (plain stores, every
// channel < C written once).  s_scr holds 2 * blockDim.x floats.  Every thread must call;
// ends with a barrier.
template <int CB>
__device__ __forceinline__ void det_fold_groups(const float (&v1)[CB], const float (&v2)[CB], int G, int C,
                                                float* s_scr, float* out) {
  const int t = threadIdx.x, nt = blockDim.x;
#pragma unroll
  for (int c = 0; c < CB; ++c) {
    s_scr[t] = v1[c];
    s_scr[nt + t] = v2[c];
    __syncthreads();
    const int ch = t * CB + c;
    if (t < G && ch < C) {
      float s1 = 0.f, s2 = 0.f;
      for (int u = t; u < nt; u += G) { s1 += s_scr[u]; s2 += s_scr[nt + u]; }
      out[ch] = s1;
      out[C + ch] = s2;
    }
    __syncthreads();
  }
}

// Reduce the forward slab into LDS tables with y = x * s_a[c] + s_b[c]
// (a = scale*rstd, b = offset - mean*a).  s_tmp needs 2C floats.  Every thread must call.
__device__ __forceinline__ void bn_reduce_to_lds(const BNRef& bn, float* s_mean, float* s_rstd,
                                                 float* s_a, float* s_b, float* s_tmp) {
  slab_sum_to_lds(bn.slab, bn.nslab, 2 * bn.C, s_tmp);
  for (int c = threadIdx.x; c < bn.C; c += blockDim.x) {
    float mean = s_tmp[c] / bn.count;
    float var = fmaxf(s_tmp[bn.C + c] / bn.count - mean * mean, 0.f);
    float rstd = rsqrtf(var + bn.eps);
    float a = bn.scale[c] * rstd;
    s_mean[c] = mean;
    s_rstd[c] = rstd;
    s_a[c] = a;
    s_b[c] = bn.offset[c] - mean * a;
  }
}

}  // namespace csa
