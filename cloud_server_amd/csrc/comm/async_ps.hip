// Asynchronous bounded-staleness parameter server over xGMI peer buffers (gfx950).
//
// The reference's data parallelism (construct_distribute.py:344-357, 402-414): workers
// push gradients to the PS with no barrier between them and the PS applies ApplyAdagrad
// to each push as it arrives.  Here every rank owns one shard of the flat parameters (and
// its optimizer slots) and ONE launch per step does, per workgroup b (chunk b of a shard):
//
//   push    chunk b of every OTHER owner's part of my gradient -> owner's inbox[t % R][me],
//           then a system-scope flag (value t + 1) in that owner.  My own part never leaves
//           the GPU: the same workgroup applies it straight from the gradient when its turn
//           comes in this launch, else copies it to a local (cached) selfbox[t % R] at the
//           end of the apply phase for a later launch — no uncached round trip, no flag;
//   apply   as owner: pushes in (clock, source) order, each its own optimizer update —
//           must wait (bounded) for every push with clock <= t - s, applies newer ones only
//           if their flag is already up (arrival order = "as they arrive");
//   publish chunk b of my shard -> my outbox[t & 1] under a seqlock word (0 while written,
//           t + 1 when complete) and my applied-through clock (world > 1: a reader exists);
//   pull    chunk b of every other owner's latest complete publication whose
//           applied-through clock is >= t - 2s (bounded wait), re-validated after the copy.
//
// R = 2s + 2 inbox slots per source: a source can only get 2s + 1 clocks ahead of the
// slowest owner's applied-through clock (its pull needs t - 2s), so a slot is never
// rewritten before it was applied.  Receive buffers and flags are uncached IPC memory
// (parallel/xgmi.py rules: plain payload stores -> system release -> flag store; one
// relaxed poll -> system acquire -> payload loads); every wait is bounded and a timeout
// poisons the state word instead of hanging the GPU.  Clocks and per-workgroup progress
// live on the device, so the launch replays inside a HIP graph.
#include "../kernels/common.h"
#include "../kernels/optim_common.h"

namespace csa {

constexpr int APS_MAXR = 8;       // ranks
constexpr int APS_T = 256;
constexpr int APS_PROG = 5;

struct ApsArgs {
  int rank, world, R, s;          // ranks, inbox ring slots, staleness bound
  long sh;                        // shard floats (multiple of 4)
  int nb; long chunk;             // workgroups, floats per workgroup chunk (multiple of 4)
  float* inbox[APS_MAXR];         // rank p's [R][world][sh] (mapped)
  unsigned* inflag[APS_MAXR];     // rank p's [R][world][nb]
  float* outbox[APS_MAXR];        // rank p's [2][sh]
  unsigned* outver[APS_MAXR];     // rank p's [2][nb] seqlock words (0 = being written)
  int* outat[APS_MAXR];           // rank p's [2][nb] applied-through clock of that copy
  const float* grad;              // my flat gradient [world * sh]
  float* flat;                    // my flat parameters [world * sh] (my shard updated in place)
  float* s0; float* s1;           // optimizer slots of my shard
  float* selfbox;                 // my own pushes not applied in their launch: [R][sh] (local)
  int opt; float lr;
  int* prog;                      // [nb][APS_PROG]: next clock, next source, pushes applied,
                                  //   this rank's clock t, max staleness seen — per workgroup:
                                  //   every launch runs every workgroup once, so the clocks
                                  //   advance in lockstep with no same-address atomics
  unsigned* state;                // {-, -, err}
  int drain;                      // 1: apply everything through t - 1, pull through t - 1
  unsigned long long timeout_ticks;
};

// dst[c0, c1) = src[c0, c1) by the workgroup, four float4 loads in flight per thread
__device__ __forceinline__ void aps_copy(float* dst, const float* src, long c0, long c1) {
  constexpr long ST = 4L * APS_T;
  auto ld = [&](long i) { return *reinterpret_cast<const float4*>(src + (i < c1 ? i : c0)); };
  auto st = [&](long i, const float4& v) { if (i < c1) *reinterpret_cast<float4*>(dst + i) = v; };
  for (long i0 = c0 + 4 * (long)threadIdx.x; i0 < c1; i0 += 4 * ST) {
    const float4 v0 = ld(i0), v1 = ld(i0 + ST), v2 = ld(i0 + 2 * ST), v3 = ld(i0 + 3 * ST);
    st(i0, v0); st(i0 + ST, v1); st(i0 + 2 * ST, v2); st(i0 + 3 * ST, v3);
  }
}

__device__ __forceinline__ bool aps_poll(const unsigned* f, unsigned want, bool wait, unsigned long long t0,
                                         const ApsArgs& a, int* s_abort) {
  while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
    if (!wait) return false;
    if (wall_clock64() - t0 > a.timeout_ticks) {
      __hip_atomic_store(reinterpret_cast<int*>(a.state + 2), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_abort = 1;
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  return true;
}

__global__ __launch_bounds__(APS_T) void aps_kernel(ApsArgs a) {
  __shared__ int s_abort, s_go, s_c, s_q, s_n, s_par, s_t, s_st;
  const int tid = threadIdx.x, b = blockIdx.x, W = a.world, me = a.rank;
  if (tid == 0) {
    s_abort = __hip_atomic_load(reinterpret_cast<int*>(a.state + 2), __ATOMIC_RELAXED,
                                __HIP_MEMORY_SCOPE_AGENT) != 0;
    // this workgroup's own clock (written by this workgroup index in the previous launch;
    // a kernel boundary in between)
    s_t = a.prog[APS_PROG * b + 3];
    s_st = a.prog[APS_PROG * b + 4];
  }
  __syncthreads();
  if (s_abort) return;
  const int t = s_t;                                   // this rank's clock
  const long c0 = (long)b * a.chunk;
  const long c1 = c0 + a.chunk < a.sh ? c0 + a.chunk : a.sh;
  const unsigned long long t0 = wall_clock64();

  // ---- push (skipped when draining: every clock was pushed already; one rank: nothing
  // leaves the GPU, and the two system-scope release fences — an L2 write-back each — go)
  if (!a.drain && W > 1) {
    const int slot = t % a.R;
    for (int p = 0; p < W; ++p) {
      if (p == me) continue;                           // (own part: applied / kept locally)
      aps_copy(a.inbox[p] + ((long)slot * W + me) * a.sh, a.grad + (long)p * a.sh, c0, c1);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      for (int p = 0; p < W; ++p)
        if (p != me) __hip_atomic_store(a.inflag[p] + ((long)slot * W + me) * a.nb + b, (unsigned)(t + 1),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");      // flag lines written back (xgmi.hip)
    }
  }

  // ---- apply (owner): arrived pushes in (clock, source) order
  const int last = a.drain ? t - 1 : t;                // highest clock that may be applied
  const int must = a.drain ? t - 1 : t - a.s;          // every push up to here is waited for
  int* pg = a.prog + APS_PROG * b;
  if (tid == 0) { s_c = pg[0]; s_q = pg[1]; s_n = pg[2]; }
  __syncthreads();
  float* w = a.flat + (long)me * a.sh;
  for (;;) {
    if (tid == 0) {
      s_go = 0;
      if (s_c <= last && s_q == me) {
        s_go = 1;                                      // own push: always here (this workgroup)
      } else if (s_c <= last) {
        const unsigned* f = a.inflag[me] + ((long)(s_c % a.R) * W + s_q) * a.nb + b;
        if (aps_poll(f, (unsigned)(s_c + 1), s_c <= must, t0, a, &s_abort)) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
          s_go = 1;
        }
      }
    }
    __syncthreads();
    if (!s_go || s_abort) break;
    // own push of THIS clock: the gradient itself; of an earlier clock: the selfbox copy
    const float* g = s_q != me ? a.inbox[me] + ((long)(s_c % a.R) * W + s_q) * a.sh
                     : (s_c == t && !a.drain ? a.grad + (long)me * a.sh : a.selfbox + (long)(s_c % a.R) * a.sh);
    const int n = s_n + 1;                              // 1-based update count of this chunk
    const float lr = a.opt == OPT_ADAM
                         ? a.lr * sqrtf(1.f - powf(0.999f, (float)n)) / (1.f - powf(0.9f, (float)n))
                         : a.lr;
    // float4 over the chunk (chunk and shard are multiples of 4): one 16-byte load of
    // the uncached inbox per lane instead of four dependent 4-byte round trips
    // four float4s per thread per round, every load of the round issued first (named
    // registers: an indexed array here was promoted to LDS / scratch by the compiler)
    const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
    auto ld = [&](long i, float4& wv, float4& gv, float4& z0, float4& z1) {
      const long j = i < c1 ? i : c0;
      wv = *reinterpret_cast<const float4*>(w + j);
      gv = *reinterpret_cast<const float4*>(g + j);
      z0 = a.s0 ? *reinterpret_cast<const float4*>(a.s0 + j) : z4;
      z1 = a.s1 ? *reinterpret_cast<const float4*>(a.s1 + j) : z4;
    };
    auto up = [&](long i, float4& wv, const float4& gv, float4& z0, float4& z1) {
      if (i >= c1) return;
      opt_update(a.opt, lr, wv.x, gv.x, z0.x, z1.x);
      opt_update(a.opt, lr, wv.y, gv.y, z0.y, z1.y);
      opt_update(a.opt, lr, wv.z, gv.z, z0.z, z1.z);
      opt_update(a.opt, lr, wv.w, gv.w, z0.w, z1.w);
      *reinterpret_cast<float4*>(w + i) = wv;
      if (a.s0) *reinterpret_cast<float4*>(a.s0 + i) = z0;
      if (a.s1) *reinterpret_cast<float4*>(a.s1 + i) = z1;
    };
    constexpr long ST = 4L * APS_T;
    for (long i0 = c0 + 4 * tid; i0 < c1; i0 += 4 * ST) {
      float4 w0, g0, a0, b0, w1, g1, a1, b1, w2, g2, a2, b2, w3, g3, a3, b3;
      ld(i0, w0, g0, a0, b0);
      ld(i0 + ST, w1, g1, a1, b1);
      ld(i0 + 2 * ST, w2, g2, a2, b2);
      ld(i0 + 3 * ST, w3, g3, a3, b3);
      up(i0, w0, g0, a0, b0);
      up(i0 + ST, w1, g1, a1, b1);
      up(i0 + 2 * ST, w2, g2, a2, b2);
      up(i0 + 3 * ST, w3, g3, a3, b3);
    }
    __syncthreads();
    if (tid == 0) {
      s_n = n;
      if (++s_q == W) { s_q = 0; ++s_c; }
    }
    __syncthreads();
  }
  if (s_abort) return;
  const int at = s_c - 1;                                // applied-through clock of this chunk
  // my own push of this clock not applied yet (an earlier push it must follow has not
  // arrived): keep it for a later launch (written and read by this workgroup only)
  if (!a.drain && (s_c < t || (s_c == t && s_q <= me))) {
    aps_copy(a.selfbox + (long)(t % a.R) * a.sh, a.grad + (long)me * a.sh, c0, c1);
  }
  if (tid == 0) { pg[0] = s_c; pg[1] = s_q; pg[2] = s_n; }

  // ---- publish my chunk (seqlock: 0 while the copy is written; one rank: nobody reads it)
  if (W > 1) {
    const int par = t & 1;
    if (tid == 0)
      __hip_atomic_store(a.outver[me] + par * a.nb + b, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");          // the invalidation is visible first
    aps_copy(a.outbox[me] + (long)par * a.sh, w, c0, c1);
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.outat[me] + par * a.nb + b, at, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(a.outver[me] + par * a.nb + b, (unsigned)(t + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    }
  }

  // ---- pull every other owner's chunk (latest complete copy with applied-through >= need)
  const int need = a.drain ? t - 1 : t - 2 * a.s;
  int worst = t - at;
  for (int p = 0; p < W; ++p) {
    if (p == me) continue;
    for (int tries = 0;; ++tries) {
      if (tid == 0) {
        s_par = -1;
        for (;;) {
          unsigned best = 0; int bp = -1, bat = -1;
          for (int q = 0; q < 2; ++q) {
            const unsigned v = __hip_atomic_load(a.outver[p] + q * a.nb + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (v > best) { best = v; bp = q; }
          }
          if (bp >= 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            bat = __hip_atomic_load(a.outat[p] + bp * a.nb + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          if (bp >= 0 && bat >= need) { s_par = bp; s_n = (int)best; s_c = bat; break; }
          if (wall_clock64() - t0 > a.timeout_ticks) {
            __hip_atomic_store(reinterpret_cast<int*>(a.state + 2), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_abort = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
      if (s_abort) return;
      aps_copy(a.flat + (long)p * a.sh, a.outbox[p] + (long)s_par * a.sh, c0, c1);
      __builtin_amdgcn_s_waitcnt(0);
      __syncthreads();
      if (tid == 0) {                                    // unchanged while copied?
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        const unsigned v = __hip_atomic_load(a.outver[p] + s_par * a.nb + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s_go = v == (unsigned)s_n;
      }
      __syncthreads();
      if (s_go) break;
    }
    if (t - s_c > worst) worst = t - s_c;
  }
  // (the drain launch has no gradient of its own: t - at there is not a staleness)
  // ---- this workgroup's clock advances (the next launch's workgroup b reads it) and its
  // staleness record (the host takes the max over workgroups)
  if (tid == 0 && !a.drain) {
    pg[3] = t + 1;
    pg[4] = worst > s_st ? worst : s_st;
  }
}

}  // namespace csa

using namespace csa;

// bufs: per rank {inbox, inflag, outbox, outver, outat} (mapped pointers, rank-major).
CSA_API int csa_aps_step(int rank, int world, int R, int s, long sh, int nb, void* const* bufs, const float* grad,
                         float* flat, float* s0, float* s1, float* selfbox, int opt, float lr, int* prog,
                         unsigned* state, int drain, double timeout_s, hipStream_t st) {
  if (world < 1 || world > APS_MAXR || rank < 0 || rank >= world || R < 2 || s < 0 || sh <= 0 || sh % 4 || nb < 1)
    return -1;
  if (((uintptr_t)grad & 15) || ((uintptr_t)flat & 15) || !selfbox || ((uintptr_t)selfbox & 15)) return -2;
  ApsArgs a{};
  a.rank = rank; a.world = world; a.R = R; a.s = s; a.sh = sh; a.nb = nb;
  a.chunk = ((sh + nb - 1) / nb + 3) / 4 * 4;
  for (int p = 0; p < world; ++p) {
    a.inbox[p] = static_cast<float*>(bufs[5 * p + 0]);
    a.inflag[p] = static_cast<unsigned*>(bufs[5 * p + 1]);
    a.outbox[p] = static_cast<float*>(bufs[5 * p + 2]);
    a.outver[p] = static_cast<unsigned*>(bufs[5 * p + 3]);
    a.outat[p] = static_cast<int*>(bufs[5 * p + 4]);
  }
  a.grad = grad; a.flat = flat; a.s0 = s0; a.s1 = s1; a.selfbox = selfbox; a.opt = opt; a.lr = lr;
  a.prog = prog; a.state = state; a.drain = drain;
  a.timeout_ticks = (unsigned long long)(timeout_s * 1.0e8);     // wall_clock64: 100 MHz
  hipLaunchKernelGGL(aps_kernel, dim3((unsigned)nb), dim3(APS_T), 0, st, a);
  return (int)hipGetLastError();
}
