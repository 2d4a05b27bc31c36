// Intra-node collectives over xGMI through IPC-mapped peer buffers (gfx950).
//
// Replaces the reference's per-step PS pull/push over TF gRPC (construct_distribute.py:
// 355-357, 413) for the small, latency-bound messages of this
// workload.  RCCL rings move a message hop by hop over ONE xGMI link per step; an
// MI355X has 7 point-to-point links per GPU, so here every rank PUSHES its whole message
// into a slot of every peer's receive buffer at once (7 links busy, posted writes), then
// raises a per-(block, source) flag in each peer.  A receiving block waits only for the
// flags of the chunk it owns and then works from LOCAL memory:
//
//   * all-gather  — copy the world slots of its chunk into the rank-major output;
//   * all-reduce  — sum the world slots of its chunk (fp32) into the in/out tensor.
//
// One-shot all-reduce sends (W-1) x the message out of every GPU: right for small,
// latency-bound messages.  For large ones (a whole 9.1 MB gradient: 63.7 MB of egress at
// W=8) the TWO-SHOT all-reduce (op 2) sends 2 (W-1)/W x the message instead:
//   phase 1 (reduce-scatter): shard j of the message goes ONLY to rank j, which sums the
//     W contributions of its shard in fixed rank order;
//   phase 2 (all-gather): rank j pushes its reduced shard to every peer.
// Block b owns sub-chunk b of EVERY shard in both phases, so the shard a block reduces is
// exactly the one it broadcasts: no cross-block dependency on either side.  Same flag /
// epoch / parity protocol, one flag array per phase; bitwise identical on every rank.
//
// Protocol details
//   * receive buffers and flags are allocated uncached (hipDeviceMallocUncached), so a
//     reader never hits a stale L2 line written by a peer (XCD/L2 non-coherence);
//   * data stores -> __threadfence_system() -> __syncthreads() -> flag store with
//     release/system scope; the waiter does an acquire/system load of the flag;
//   * the epoch e = (device sequence counter + 1) is the flag value; the buffer parity
//     e & 1 double-buffers the slots: a rank can write epoch e+2 into a peer only after
//     it saw that peer's epoch e+1 push, which the peer issues after finishing epoch e;
//   * the counter advances in the launch's last-finishing block, so the same kernel
//     node replays correctly inside a HIP graph (no host-side epoch);
//   * every wait is bounded (wall clock): on timeout the kernel raises `err` and every
//     later call returns at once, so a missing peer can never hang the GPU.
// One channel (buffers + flags + counter) serves ONE device-ordered sequence of calls;
// call sites that may run concurrently on different streams use different channels.
#include "../kernels/common.h"
#include <cstring>

namespace csa {

constexpr int XG_MAXR = 8;     // ranks per node
constexpr int XG_MAXB = 256;   // blocks per launch (all co-resident: 256 CUs)
constexpr int XG_MAXSEG = 8;

struct XgSeg { const char* src; char* dst; long bytes; long off; };

struct XgArgs {
  int op, rank, world, nseg;
  long msg_bytes, slot_bytes;
  char* buf[XG_MAXR];           // rank r's receive buffer [2][world][slot_bytes] (mapped);
                                // two-shot: [2 parity][2 phase][world][shard] in the same bytes
  unsigned* flags[XG_MAXR];     // rank r's flags [2 phase][2 parity][XG_MAXB][XG_MAXR] (mapped)
  XgSeg seg[XG_MAXSEG];
  // op 3 (reduce-scatter of a range with GLOBAL ownership): the message is units
  // [rs_lo, rs_lo + msg) of a flat buffer whose unit g belongs to rank g / rs_sh; the
  // owner writes the sum of its units to rs_dst[g - rank * rs_sh]
  long rs_lo, rs_sh; char* rs_dst;
  unsigned* seq; unsigned* done; int* err;
  unsigned long long timeout_ticks;
  // per-block record of the last call (nullable), [XG_MAXB][XG_DIAG] u64:
  //   {epoch, t_start, t_published, t_waited, status (1 ok / 2 timeout), missing source,
  //    last flag value seen from it, that source's OWN copy of the flag}
  // wall_clock64 is one device-wide 100 MHz clock, so ranks sharing a GPU (the one-GPU
  // multi-process tests) can be lined up block by block after a timeout
  unsigned long long* diag;
};

constexpr int XG_DIAG = 8;

// native 16-byte vectors for the per-rank register arrays (HIP's uint4 / float4 classes
// kept those arrays in scratch)
typedef unsigned xu4 __attribute__((ext_vector_type(4)));
typedef float xf4 __attribute__((ext_vector_type(4)));

// Element i of a kernarg pointer table without indexing it dynamically: a runtime index
// into the by-value XgArgs made the compiler copy the struct to scratch in every lane
// (144 B/lane; a scratch-using spinning kernel beside another process's queue is what the
// round-5 stall traces point at).  With a uniform i this is a chain of scalar selects.
template <class T>
__device__ __forceinline__ T xg_pick(T const (&v)[XG_MAXR], int i) {
  T x = v[0];
#pragma unroll
  for (int k = 1; k < XG_MAXR; ++k)
    if (i == k) x = v[k];
  return x;
}

// The segment holding byte `off` of the packed message (per lane: unrolled selects, no
// dynamic index into the kernarg segment table).
struct XgPos { const char* src; char* dst; long so; long bytes; };
__device__ __forceinline__ XgPos xg_pos(const XgArgs& a, long off) {
  XgPos p{a.seg[0].src, a.seg[0].dst, off - a.seg[0].off, a.seg[0].bytes};
#pragma unroll
  for (int k = 1; k < XG_MAXSEG; ++k)
    if (k < a.nseg && off >= a.seg[k].off) p = XgPos{a.seg[k].src, a.seg[k].dst, off - a.seg[k].off, a.seg[k].bytes};
  return p;
}

__device__ __forceinline__ void xg_note(const XgArgs& a, int k, unsigned long long v) {
  if (a.diag) a.diag[(long)blockIdx.x * XG_DIAG + k] = v;
}

// The channel epoch of this call: the device counter + 1, read ONCE per block by thread 0
// at agent scope (a plain load could hit a stale line in this XCD's L2: the counter is
// advanced by whichever block finished last, on any XCD) and broadcast through LDS.
__device__ __forceinline__ unsigned xg_epoch(const XgArgs& a, int* s_abort, unsigned* s_e) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();
    *s_abort = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    *s_e = __hip_atomic_load(a.seq, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    if (a.diag && !*s_abort) {       // (a poisoned channel keeps the failing call's record)
      unsigned long long* d = a.diag + (long)blockIdx.x * XG_DIAG;
      d[0] = *s_e; d[1] = t0; d[2] = 0; d[3] = 0; d[4] = 0; d[5] = 0; d[6] = 0; d[7] = 0;
    }
  }
  __syncthreads();
  return *s_e;
}

// The last block to finish advances the epoch for the next call on this channel (agent-
// scope RMW / release store: visible to every XCD's blocks of the next launch).
__device__ __forceinline__ void xg_finish(const XgArgs& a, unsigned e) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1u) {
      __hip_atomic_store(a.done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.seq, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Byte offset of parity half `par` of a receive buffer [2][world][slot + 32]: every
// protocol (one-shot slots, two-shot phases, range reduce-scatter) stays inside its half.
__host__ __device__ __forceinline__ long xg_par_base(const XgArgs& a, int par) {
  return (long)par * ((long)a.world * a.slot_bytes + 32L * a.world);
}

// Publish this block's stores of one phase, then raise its flags (value e) in every rank.
__device__ __forceinline__ void xg_publish(const XgArgs& a, long fidx, unsigned e) {
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#pragma unroll
    for (int p = 0; p < XG_MAXR; ++p)
      if (p < a.world) __hip_atomic_store(a.flags[p] + fidx + a.rank, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // write the flag lines back too: ranks sharing ONE GPU map each other's buffers as
    // local memory, where a flag store can stay in this XCD's L2 until the next release
    // (a waiting peer then never sees it: intermittent timeouts in the one-GPU tests)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    xg_note(a, 2, wall_clock64());
  }
}

// Wait (bounded) until every source raised flag value e at fidx in this rank; returns
// false (and poisons the channel) on timeout.  Every thread must call.
__device__ __forceinline__ bool xg_wait(const XgArgs& a, long fidx, unsigned e, int* s_abort) {
  if (threadIdx.x == 0) {
    const unsigned* f = xg_pick(a.flags, a.rank) + fidx;
    const unsigned long long t0 = wall_clock64();
    for (int r = 0; r < a.world && !*s_abort; ++r) {
      unsigned v;
      while ((v = __hip_atomic_load(f + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != e) {
        if (wall_clock64() - t0 > a.timeout_ticks) {
          __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *s_abort = 1;
          // the failure record: who never arrived, what was seen, and what the missing
          // source's OWN copy of that flag says (it publishes to itself too): e there but
          // not here = a lost store; not there either = that block never published
          if (a.diag) {
            unsigned long long* d = a.diag + (long)blockIdx.x * XG_DIAG;
            d[3] = wall_clock64(); d[4] = 2; d[5] = (unsigned long long)r; d[6] = v;
            d[7] = __hip_atomic_load(xg_pick(a.flags, r) + fidx + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          }
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (!*s_abort && a.diag) {
      unsigned long long* d = a.diag + (long)blockIdx.x * XG_DIAG;
      d[3] = wall_clock64(); d[4] = 1;
    }
  }
  __syncthreads();
  return !*s_abort;
}

__device__ __forceinline__ const char* xg_src(const XgArgs& a, long off) {
  const XgPos p = xg_pos(a, off);
  return p.src + p.so;
}

__device__ __forceinline__ char* xg_dst(const XgArgs& a, long off) {
  const XgPos p = xg_pos(a, off);
  return p.dst + p.so;
}

// Two-shot fp32 sum all-reduce (op 2): see the header comment.  W = a.world as a template
// parameter: the per-rank register arrays then have constant bounds (with a runtime bound
// the compiler kept them in scratch, 144 B/lane).
template <int W>
__device__ __forceinline__ void xg_twoshot(const XgArgs& a, unsigned e, int* s_abort) {
  const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const int par = e & 1u;
  const long units = a.msg_bytes >> 4;
  const long S = (units + W - 1) / W;                 // 16-byte units per shard
  const long shard = S << 4;
  const long per = (S + nb - 1) / nb;
  const long v0 = b * per < S ? b * per : S;
  const long v1 = v0 + per < S ? v0 + per : S;
  // inside THIS parity's half of the buffer, exactly where the one-shot layout keeps its
  // parity: a channel may mix the protocols, and the double-buffer guarantee (a peer one
  // epoch ahead writes only the OTHER half) must hold across them
  const long area0 = xg_par_base(a, par);                // phase-1 slots [src][shard]
  const long area1 = area0 + (long)W * shard;            // phase-2 slots [owner][shard]
  const long f1 = ((long)(0 * 2 + par) * XG_MAXB + b) * XG_MAXR;
  const long f2 = ((long)(1 * 2 + par) * XG_MAXB + b) * XG_MAXR;

  // phase 1: my contribution to shard p -> rank p's slot [my rank]
  for (long v = v0 + t; v < v1; v += blockDim.x) {
#pragma unroll
    for (int p = 0; p < W; ++p) {
      const long u = p * S + v;
      if (u < units) {
        const xu4 x = *reinterpret_cast<const xu4*>(xg_src(a, u << 4));
        *reinterpret_cast<xu4*>(a.buf[p] + area0 + (long)a.rank * shard + (v << 4)) = x;
      }
    }
  }
  xg_publish(a, f1, e);
  if (!xg_wait(a, f1, e, s_abort)) return;

  // reduce my shard's sub-chunk (fixed rank order), push the sum to every rank's slot [me]
  const char* mine0 = xg_pick(a.buf, a.rank) + area0;
  for (long v = v0 + t; v < v1; v += blockDim.x) {
    const long u = (long)a.rank * S + v;
    if (u >= units) break;
    xf4 x[W];
#pragma unroll
    for (int r = 0; r < W; ++r) x[r] = *reinterpret_cast<const xf4*>(mine0 + (long)r * shard + (v << 4));
    xf4 acc = x[0];
#pragma unroll
    for (int r = 1; r < W; ++r) { acc += x[r]; }
#pragma unroll
    for (int p = 0; p < W; ++p)
      *reinterpret_cast<xf4*>(a.buf[p] + area1 + (long)a.rank * shard + (v << 4)) = acc;
  }
  xg_publish(a, f2, e);
  if (!xg_wait(a, f2, e, s_abort)) return;

  // phase 2 consume: every owner's reduced sub-chunk -> the output
  const char* mine1 = xg_pick(a.buf, a.rank) + area1;
  for (long v = v0 + t; v < v1; v += blockDim.x) {
    xu4 x[W];
#pragma unroll
    for (int r = 0; r < W; ++r)           // in the buffer for every r (v < S); only the stores are guarded
      x[r] = *reinterpret_cast<const xu4*>(mine1 + (long)r * shard + (v << 4));
#pragma unroll
    for (int r = 0; r < W; ++r)
      if (r * S + v < units) *reinterpret_cast<xu4*>(xg_dst(a, (r * S + v) << 4)) = x[r];
  }
}

// One-shot all-gather / all-reduce (ops 0 / 1) for W = a.world ranks.
template <int W>
__device__ __forceinline__ void xg_oneshot(const XgArgs& a, unsigned e, int* s_abort) {
  const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const int par = e & 1u;
  // this block's chunk of the packed per-rank message, in 16-byte units
  const long units = a.msg_bytes >> 4;
  const long per = (units + nb - 1) / nb;
  const long u0 = b * per < units ? b * per : units;
  const long u1 = u0 + per < units ? u0 + per : units;
  const long my_slot = xg_par_base(a, par) + (long)a.rank * a.slot_bytes;

  // 1) push: load each 16 B once, store it into every rank's slot [rank] (own included)
  for (long u = u0 + t; u < u1; u += blockDim.x) {
    const long off = u << 4;
    const xu4 v = *reinterpret_cast<const xu4*>(xg_src(a, off));
#pragma unroll
    for (int p = 0; p < W; ++p) *reinterpret_cast<xu4*>(a.buf[p] + my_slot + off) = v;
  }
  // publish (every wave drains its stores, the barrier, ONE system-scope release per
  // block, the flags), then wait for every source's flag of this chunk (one lane polls,
  // bounded) and ONE system-scope acquire for the block (the vector L1 is per CU)
  const long fidx = ((long)par * XG_MAXB + b) * XG_MAXR;
  xg_publish(a, fidx, e);
  // 3) consume from local memory
  if (xg_wait(a, fidx, e, s_abort)) {
    const char* mine = xg_pick(a.buf, a.rank) + xg_par_base(a, par);
    for (long u = u0 + t; u < u1; u += blockDim.x) {
      const long off = u << 4;
      const XgPos s = xg_pos(a, off);
      const long so = s.so;
      if (a.op == 0) {           // all-gather: out is rank-major [world][seg.bytes]
        xu4 v[W];
#pragma unroll
        for (int r = 0; r < W; ++r) v[r] = *reinterpret_cast<const xu4*>(mine + (long)r * a.slot_bytes + off);
#pragma unroll
        for (int r = 0; r < W; ++r) *reinterpret_cast<xu4*>(s.dst + (long)r * s.bytes + so) = v[r];
      } else {                   // all-reduce (fp32 sum), rank order fixed -> bitwise identical on all ranks
        xf4 v[W];
#pragma unroll
        for (int r = 0; r < W; ++r) v[r] = *reinterpret_cast<const xf4*>(mine + (long)r * a.slot_bytes + off);
        xf4 acc = v[0];
#pragma unroll
        for (int r = 1; r < W; ++r) { acc += v[r]; }
        *reinterpret_cast<xf4*>(s.dst + so) = acc;
      }
    }
  }
}

template <int W>
__device__ __forceinline__ void xg_body(const XgArgs& a, unsigned e, int* s_abort) {
  if (a.op == 2) xg_twoshot<W>(a, e, s_abort);
  else xg_oneshot<W>(a, e, s_abort);
}

__global__ __launch_bounds__(256) void xgmi_kernel(XgArgs) {
  // the arguments are read in place from the kernarg segment: through the by-value
  // parameter the compiler copied the whole struct into scratch in every lane (488 B)
  const XgArgs& a = *(const XgArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  __shared__ int s_abort;
  __shared__ unsigned s_e;
  const unsigned e = xg_epoch(a, &s_abort, &s_e);
  if (s_abort) return;
  switch (a.world) {
    case 1: xg_body<1>(a, e, &s_abort); break;
    case 2: xg_body<2>(a, e, &s_abort); break;
    case 3: xg_body<3>(a, e, &s_abort); break;
    case 4: xg_body<4>(a, e, &s_abort); break;
    case 5: xg_body<5>(a, e, &s_abort); break;
    case 6: xg_body<6>(a, e, &s_abort); break;
    case 7: xg_body<7>(a, e, &s_abort); break;
    default: xg_body<8>(a, e, &s_abort); break;
  }
  // 4) the last block to finish advances the epoch for the next call on this channel
  xg_finish(a, e);
}

// op 3: reduce-scatter of a range with GLOBAL ownership (its own kernel: the extra code
// raised the shared kernel's registers from 89 to 149, which cut its residency to 3
// blocks per CU — several ranks sharing one GPU then no longer fit co-resident and their
// peer waits time out).  Same slot / flag / epoch protocol as the one-shot path: every
// unit goes only to its OWNER's slot [rank] (it leaves the GPU at most once), flags go to
// every rank, the owner sums its units of the range in fixed rank order.
__global__ __launch_bounds__(256) void xgmi_rs_kernel(XgArgs a) {
  __shared__ int s_abort;
  __shared__ unsigned s_e;
  const int t = threadIdx.x, b = blockIdx.x, nb = gridDim.x;
  const unsigned e = xg_epoch(a, &s_abort, &s_e);
  if (s_abort) return;
  const int par = e & 1u;
  const long units = a.msg_bytes >> 4;
  const long per = (units + nb - 1) / nb;
  const long u0 = b * per < units ? b * per : units;
  const long u1 = u0 + per < units ? u0 + per : units;
  const long my_slot = xg_par_base(a, par) + (long)a.rank * a.slot_bytes;
  const char* src = a.seg[0].src;
  for (long u = u0 + t; u < u1; u += blockDim.x) {
    const int p = (int)((a.rs_lo + u) / a.rs_sh);
    *reinterpret_cast<uint4*>(a.buf[p] + my_slot + (u << 4)) = *reinterpret_cast<const uint4*>(src + (u << 4));
  }
  const long fidx = ((long)par * XG_MAXB + b) * XG_MAXR;
  xg_publish(a, fidx, e);
  if (xg_wait(a, fidx, e, &s_abort)) {
    const char* mine = xg_pick(a.buf, a.rank) + xg_par_base(a, par);
    // my units of this block's chunk: [max(u0, own_lo), min(u1, own_hi))
    const long own_lo = (long)a.rank * a.rs_sh - a.rs_lo, own_hi = own_lo + a.rs_sh;
    const long c0 = u0 > own_lo ? u0 : own_lo, c1 = u1 < own_hi ? u1 : own_hi;
    for (long u = c0 + t; u < c1; u += blockDim.x) {
      const long off = u << 4;
      float4 acc = *reinterpret_cast<const float4*>(mine + off);
      for (int r = 1; r < a.world; ++r) {
        const float4 v = *reinterpret_cast<const float4*>(mine + (long)r * a.slot_bytes + off);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
      *reinterpret_cast<float4*>(a.rs_dst + ((u - own_lo) << 4)) = acc;
    }
  }
  xg_finish(a, e);
}

}  // namespace csa

using namespace csa;

// Uncached device allocation + its IPC handle (64 bytes written to `handle`).
CSA_API int csa_xgmi_alloc(long bytes, void** ptr, void* handle) {
  hipError_t e = hipExtMallocWithFlags(ptr, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  if ((e = hipMemset(*ptr, 0, (size_t)bytes)) != hipSuccess) return (int)e;
  if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), *ptr);
}

// A pooled buffer handed to a new channel: zeroed again, its IPC handle re-exported.
CSA_API int csa_xgmi_reuse(void* ptr, long bytes, void* handle) {
  hipError_t e = hipMemset(ptr, 0, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  if ((e = hipDeviceSynchronize()) != hipSuccess) return (int)e;
  return (int)hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), ptr);
}

CSA_API int csa_xgmi_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  return (int)hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

CSA_API int csa_xgmi_close(void* ptr) { return (int)hipIpcCloseMemHandle(ptr); }
CSA_API int csa_xgmi_free(void* ptr) { return (int)hipFree(ptr); }
CSA_API int csa_xgmi_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }
CSA_API int csa_xgmi_max_blocks() { return XG_MAXB; }
CSA_API int csa_xgmi_diag_words() { return XG_DIAG; }

// op 0 = all-gather (dst[r] = src of rank r, rank-major per segment), 1 = fp32 sum all-reduce
// (src == dst allowed).  Segments are packed back to back into one per-rank message of
// sum(bytes) <= slot_bytes; every segment size and pointer must be 16-byte aligned.
// state = 3 x uint32 on the device: {seq, done, err}.
CSA_API int csa_xgmi_run(int op, int rank, int world, long slot_bytes, void* const* bufs, void* const* flags,
                         int nseg, void* const* srcs, void* const* dsts, const long* seg_bytes,
                         unsigned* state, double timeout_s, int nblocks, void* diag, hipStream_t st) {
  if (world < 1 || world > XG_MAXR || rank < 0 || rank >= world || nseg < 1 || nseg > XG_MAXSEG) return -1;
  XgArgs a{};
  a.op = op; a.rank = rank; a.world = world; a.nseg = nseg; a.slot_bytes = slot_bytes;
  long off = 0;
  for (int i = 0; i < nseg; ++i) {
    if (seg_bytes[i] <= 0 || (seg_bytes[i] & 15) || ((uintptr_t)srcs[i] & 15) || ((uintptr_t)dsts[i] & 15)) return -2;
    a.seg[i] = XgSeg{static_cast<const char*>(srcs[i]), static_cast<char*>(dsts[i]), seg_bytes[i], off};
    off += seg_bytes[i];
  }
  if (off > slot_bytes) return -3;
  if (op == 2) {                // [2 phase][world][shard] must fit one parity half
    const long S = ((off >> 4) + world - 1) / world;
    if (2L * world * (S << 4) > (long)world * slot_bytes + 32L * world) return -4;
  }
  a.msg_bytes = off;
  for (int r = 0; r < world; ++r) {
    a.buf[r] = static_cast<char*>(bufs[r]);
    a.flags[r] = static_cast<unsigned*>(flags[r]);
  }
  a.seq = state; a.done = state + 1; a.err = reinterpret_cast<int*>(state + 2);
  a.timeout_ticks = (unsigned long long)(timeout_s * 1.0e8);   // wall_clock64: 100 MHz
  a.diag = static_cast<unsigned long long*>(diag);
  const long units = off >> 4;
  // ~8 KB per block: measured 9.6 us vs 16.9 (32 KB) / 52.5 (128 KB) for the 0.9 MB
  // lowrank gather (profiles/r1s4_xgmi_collectives.md)
  int nb = nblocks > 0 ? nblocks : (int)((units + 511) / 512);
  nb = nb < 1 ? 1 : (nb > XG_MAXB ? XG_MAXB : nb);
  hipLaunchKernelGGL(xgmi_kernel, dim3(nb), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// Reduce-scatter of the range [lo, lo + bytes) of a flat fp32 buffer (src = its start,
// lo and bytes in bytes, 16-aligned) whose shard of shard_bytes belongs to rank
// offset / shard_bytes: this rank receives the fixed-rank-order sum of its part of the
// range in dst_shard (the start of ITS shard's buffer).  Issued per gradient bucket as the
// backward produces it (the "ps" strategy: construct_distribute.py:355-357, 413).
CSA_API int csa_xgmi_reduce_scatter(int rank, int world, long slot_bytes, void* const* bufs, void* const* flags,
                                    const void* src, long lo, long bytes, long shard_bytes, void* dst_shard,
                                    unsigned* state, double timeout_s, int nblocks, void* diag, hipStream_t st) {
  if (world < 1 || world > XG_MAXR || rank < 0 || rank >= world) return -1;
  if ((lo & 15) || bytes <= 0 || (bytes & 15) || (shard_bytes & 15) || shard_bytes <= 0) return -2;
  if (((uintptr_t)src & 15) || ((uintptr_t)dst_shard & 15)) return -2;
  if (bytes > slot_bytes) return -3;
  if ((lo + bytes + shard_bytes - 1) / shard_bytes > world) return -4;     // range beyond the last shard
  XgArgs a{};
  a.op = 3; a.rank = rank; a.world = world; a.nseg = 1; a.slot_bytes = slot_bytes;
  a.seg[0] = XgSeg{static_cast<const char*>(src) + lo, nullptr, bytes, 0};
  a.msg_bytes = bytes;
  a.rs_lo = lo >> 4; a.rs_sh = shard_bytes >> 4; a.rs_dst = static_cast<char*>(dst_shard);
  for (int r = 0; r < world; ++r) {
    a.buf[r] = static_cast<char*>(bufs[r]);
    a.flags[r] = static_cast<unsigned*>(flags[r]);
  }
  a.seq = state; a.done = state + 1; a.err = reinterpret_cast<int*>(state + 2);
  a.timeout_ticks = (unsigned long long)(timeout_s * 1.0e8);
  a.diag = static_cast<unsigned long long*>(diag);
  const long units = bytes >> 4;
  int nb = nblocks > 0 ? nblocks : (int)((units + 511) / 512);
  nb = nb < 1 ? 1 : (nb > XG_MAXB ? XG_MAXB : nb);
  hipLaunchKernelGGL(xgmi_rs_kernel, dim3(nb), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}
