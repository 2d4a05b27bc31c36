// Fused multi-tensor optimizer over the flat parameter buffer (gfx950 / CDNA4).
//
// Reference: tf.train.AdagradOptimizer(1e-4).minimize (construct_distribute.py:372-373)
// running ApplyAdagrad on the parameter server, plus the GD / Adam / Adadelta choices of
// the option catalog (apps/construction/util/options.py:26-37).  All parameters of a
// model live in one contiguous buffer, so the update is ONE launch of a float4-vectorised
// streaming kernel over a list of flat SEGMENTS — the whole buffer, or (with the fused
// dense updates of dense_update.hip) only what those kernels did not already update.
// The per-element rule is shared with the fused kernels (optim_common.h).
//
// Side jobs folded into the same launch (each would otherwise be its own tiny launch):
//   * zero the split-K / atomic accumulators the NEXT step's kernels add into,
//   * fold striped / partial gradients: a conv weight gradient accumulated by hundreds of
//     workgroups into S stripes, or the head's per-row-group partial dWh / dbh; the update
//     of those parameters reads g = sum of the S rows,
//   * write the step's metric-ring entry from the head's per-group loss / #correct,
//   * advance the batch-stream cursor (mod its wrap).
#include "common.h"
#include "optim_common.h"
#include <cstdlib>

namespace csa {

constexpr int MAXZ = 16;
constexpr int MAXF = 8;
constexpr int MAXSEG = 16;

struct ZeroList { float* p[MAXZ]; long n[MAXZ]; int count; };

// g[off + e] = sum_s src[s * ld + e] for e < n (flat-buffer offsets; off % 4 == 0);
// zero != 0: the rows are accumulators that the fold re-zeroes (their only reader)
struct Fold { long off, n, ld; float* src; int S; int zero; };
struct FoldList { Fold f[MAXF]; int count; long lo, hi; };

constexpr int MAXK = 32;
// Gradient ranges whose producer STORES every element each step: the update need not
// re-zero them.
struct KeepList { long lo[MAXK], hi[MAXK]; int count; };

struct SegList { long lo[MAXSEG]; long start4[MAXSEG + 1]; int count; };

// The fast path's segments (no folds): flat [lo, lo + 4 n) with a per-segment rule for the
// gradient — zero it after reading (an accumulator) or keep it (stored whole every step) —
// instead of a per-element search of the keep list.
constexpr int MAXFS = 32;
struct FastSegs { long lo4[MAXFS]; long start4[MAXFS + 1]; int zero[MAXFS]; int count; };

struct MetricFold {        // head partials -> ring[(step - 1) % ring]
  const float* loss; const int* corr; int parts; float div;
  float* ring_loss; int* ring_correct; int ring;
};

// The NEXT step's batch (rows[*cursor]) copied into fixed staging buffers, so the step's
// kernels read their images / labels at fixed addresses instead of walking the cursor ->
// row index -> image chain (two dependent round trips at the start of each kernel).  The
// cursor was already advanced by this step's head kernel.
struct BatchStage {
  const uint32_t* img; const int64_t* labels; const int64_t* rows; const int64_t* cursor;
  int B; long words;               // 32-bit words per image
  uint32_t* out_img; int64_t* out_lbl;
  int blocks;                      // trailing workgroups doing the copy (0: off)
};

__device__ __forceinline__ void stage_gather(const BatchStage& s, int blk) {
  const long i = (long)blk * 256 + threadIdx.x;
  const long total = (long)s.B * s.words;
  const int64_t c = *s.cursor;
  if (i < s.B) s.out_lbl[i] = s.labels[s.rows[c * s.B + i]];
  if (i >= total) return;
  const long b = i / s.words, off = i - b * s.words;
  s.out_img[i] = s.img[s.rows[c * s.B + b] * s.words + off];
}

__global__ __launch_bounds__(256) void gather_batch_kernel(BatchStage s) { stage_gather(s, blockIdx.x); }

struct OptArgs {
  int opt; float* w; const float* g; float* s0; float* s1;
  SegList seg;                     // flat segments to update
  float* gz;                       // if set (== g): each thread zeroes the gradient it read
  KeepList keep;                   // ... except inside these ranges (float4-aligned)
  float lr; const int64_t* step;   // 1-based step (the head kernel already advanced it)
  ZeroList z; FoldList fold; MetricFold met;
  int64_t* cursor;                 // batch-stream cursor: += 1 (mod cursor_wrap) per step
  long cursor_wrap;
  BatchStage stage;                // next step's batch gathered by the trailing blocks
  int fast;                        // no folds: the FastSegs loop (two float4 per thread in flight)
  FastSegs fs;
  unsigned* set_pending;           // data parallel: raise the deferred dense update's flag
};                                 // (csa_conv_pair_fwd_carry: the next pair forward applies it)

constexpr int MAXS = 16;   // stripes / partial rows per folded gradient

__device__ __forceinline__ float4 fold_grad(const FoldList& fl, long e, float4 g) {
  float gs[4] = {g.x, g.y, g.z, g.w};
  for (int k = 0; k < fl.count; ++k) {
    const Fold& f = fl.f[k];
    if (e + 3 < f.off || e >= f.off + f.n) continue;
    const long i0 = e - f.off;
    if (i0 >= 0 && i0 + 4 <= f.n && (f.ld & 3) == 0) {
      // whole float4 inside the segment: all stripes' loads in flight together
      float4 v[MAXS];
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2)
        v[s2] = s2 < f.S ? *reinterpret_cast<const float4*>(f.src + s2 * f.ld + i0) : make_float4(0.f, 0.f, 0.f, 0.f);
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) {
        acc.x += v[s2].x; acc.y += v[s2].y; acc.z += v[s2].z; acc.w += v[s2].w;
        if (f.zero && s2 < f.S) *reinterpret_cast<float4*>(f.src + s2 * f.ld + i0) = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      gs[0] = acc.x; gs[1] = acc.y; gs[2] = acc.z; gs[3] = acc.w;
      continue;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // segment edge: per element
      const long i = i0 + j;
      if (i < 0 || i >= f.n) continue;
      float v[MAXS];
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) v[s2] = s2 < f.S ? f.src[s2 * f.ld + i] : 0.f;
      float acc = 0.f;
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) {
        acc += v[s2];
        if (f.zero && s2 < f.S) f.src[s2 * f.ld + i] = 0.f;
      }
      gs[j] = acc;
    }
  }
  return make_float4(gs[0], gs[1], gs[2], gs[3]);
}

// diagnostics: s_memrealtime stamps (100 MHz) of every block, [block][4] = start, main
// loop done, zero lists done, end (scripts/microbench.py MB_OPT)
__constant__ long long* g_opt_dbg = nullptr;
#define OPT_STAMP(i)                                                                         \
  do {                                                                                       \
    if (g_opt_dbg && threadIdx.x == 0) g_opt_dbg[blockIdx.x * 4 + (i)] = (long long)__builtin_amdgcn_s_memrealtime(); \
  } while (0)

// The launch's side jobs after the update: zero the next step's accumulators, write the
// metric ring, advance the cursor.
__device__ __forceinline__ void opt_duties(const OptArgs& a, long tid, long nth) {
  // zero accumulators for the next step
  for (int z = 0; z < a.z.count; ++z) {
    float* p = a.z.p[z];
    const long n = a.z.n[z];
    for (long i = tid; i < n; i += nth) p[i] = 0.f;
  }
  OPT_STAMP(2);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (a.met.parts > 0) {
      // MAXS partials' loads in flight together per round (a serial load -> add loop is one
      // memory round trip per partial on the critical path of the whole step)
      float ls = 0.f;
      int nc = 0;
      for (int p0 = 0; p0 < a.met.parts; p0 += MAXS) {
        float lv[MAXS];
        int cv[MAXS];
#pragma unroll
        for (int p = 0; p < MAXS; ++p) {
          const int pp = p0 + p < a.met.parts ? p0 + p : 0;
          lv[p] = a.met.loss[pp];
          cv[p] = a.met.corr[pp];
        }
#pragma unroll
        for (int p = 0; p < MAXS; ++p)
          if (p0 + p < a.met.parts) { ls += lv[p]; nc += cv[p]; }
      }
      const int pos = (int)((*a.step - 1) % a.met.ring);
      a.met.ring_loss[pos] = ls / a.met.div;
      a.met.ring_correct[pos] = nc;
    }
    if (a.cursor) {
      const int64_t c = *a.cursor + 1;
      *a.cursor = (a.cursor_wrap > 0 && c >= a.cursor_wrap) ? 0 : c;
    }
  }
}

__global__ __launch_bounds__(256) void optim_kernel(OptArgs a) {
  OPT_STAMP(0);
  if (a.set_pending && blockIdx.x == 0 && threadIdx.x == 0) *a.set_pending = 1u;
  const int nmain = (int)gridDim.x - a.stage.blocks;
  if ((int)blockIdx.x >= nmain) {
    stage_gather(a.stage, (int)blockIdx.x - nmain);
    OPT_STAMP(3);
    return;
  }
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nth = (long)nmain * blockDim.x;
  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  const long n4 = a.seg.start4[a.seg.count];
  float4* w4 = (float4*)a.w;
  const float4* g4 = (const float4*)a.g;
  float4* s04 = (float4*)a.s0;
  float4* s14 = (float4*)a.s1;
  const int nslot = opt_nslots(a.opt);
  for (long t = tid; t < n4; t += nth) {
    int k = 0;
    for (int j = 1; j < a.seg.count; ++j) k = t >= a.seg.start4[j] ? j : k;
    const long i = (a.seg.lo[k] >> 2) + (t - a.seg.start4[k]);   // float4 index in the flat buffer
    // a float4 lying wholly inside one folded gradient: its S stripe loads are issued with
    // the parameter / slot loads, one memory round trip for all of them (a fold after the
    // w / g / slot loads cost block 0 — the conv weights — three dependent round trips)
    int fk = -1;
    for (int k2 = 0; k2 < a.fold.count; ++k2) {
      const Fold& f = a.fold.f[k2];
      const long i0 = i * 4 - f.off;
      if (i0 >= 0 && i0 + 4 <= f.n && (f.ld & 3) == 0) fk = k2;
    }
    float4 sv[MAXS];
    if (fk >= 0) {
      const Fold& f = a.fold.f[fk];
      const long i0 = i * 4 - f.off;
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2)
        sv[s2] = *reinterpret_cast<const float4*>(f.src + (s2 < f.S ? s2 : 0) * f.ld + i0);
    }
    float4 w = w4[i];
    float4 g = g4[i];
    float4 s0 = nslot >= 1 ? s04[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 s1 = nslot >= 2 ? s14[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (fk >= 0) {
      const Fold& f = a.fold.f[fk];
      const long i0 = i * 4 - f.off;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int s2 = 0; s2 < MAXS; ++s2) {
        if (s2 >= f.S) break;
        acc.x += sv[s2].x; acc.y += sv[s2].y; acc.z += sv[s2].z; acc.w += sv[s2].w;
      }
      if (f.zero)
        for (int s2 = 0; s2 < f.S; ++s2) *reinterpret_cast<float4*>(f.src + s2 * f.ld + i0) = make_float4(0.f, 0.f, 0.f, 0.f);
      g = acc;
    }
    // Zeroing the accumulators the next step adds into must not race with this read:
    // a zero-list pass over flat-gradient ranges run by OTHER threads could clear an
    // element before its owner read it, so the owner clears what it read.
    if (a.gz) {
      bool keep = false;
      for (int q = 0; q < a.keep.count; ++q) keep |= (i * 4 >= a.keep.lo[q]) & (i * 4 < a.keep.hi[q]);
      if (!keep) reinterpret_cast<float4*>(a.gz)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (fk < 0 && i * 4 + 3 >= a.fold.lo && i * 4 < a.fold.hi) g = fold_grad(a.fold, i * 4, g);   // edges
    float* wp = (float*)&w;
    const float* gp = (const float*)&g;
    float* sp0 = (float*)&s0;
    float* sp1 = (float*)&s1;
#pragma unroll
    for (int j = 0; j < 4; ++j) opt_update(a.opt, lr, wp[j], gp[j], sp0[j], sp1[j]);
    w4[i] = w;
    if (nslot >= 1) s04[i] = s0;
    if (nslot >= 2) s14[i] = s1;
  }
  OPT_STAMP(1);
  opt_duties(a, tid, nth);
  OPT_STAMP(3);
}

// No folds (the data-parallel programs): a streaming update over FastSegs, two float4s of
// every operand in flight per thread, then the same side jobs.  Its own kernel: inside
// optim_kernel the extra live registers cut that kernel's occupancy to two waves per SIMD.
__global__ __launch_bounds__(256) void optim_fast_kernel(OptArgs a) {
  OPT_STAMP(0);
  if (a.set_pending && blockIdx.x == 0 && threadIdx.x == 0) *a.set_pending = 1u;
  const int nmain = (int)gridDim.x - a.stage.blocks;
  if ((int)blockIdx.x >= nmain) {
    stage_gather(a.stage, (int)blockIdx.x - nmain);
    OPT_STAMP(3);
    return;
  }
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nth = (long)nmain * blockDim.x;
  const float lr = opt_step_lr(a.opt, a.lr, a.step);
  float4* w4 = (float4*)a.w;
  const float4* g4 = (const float4*)a.g;
  float4* s04 = (float4*)a.s0;
  float4* s14 = (float4*)a.s1;
  const int nslot = opt_nslots(a.opt);
  {
    // streaming update: each thread keeps two float4s of every operand in flight (the loop
    // below was one dependent round trip per float4 with a per-element keep search)
    const long m4 = a.fs.start4[a.fs.count];
    for (long t0 = tid; t0 < m4; t0 += 2 * nth) {
      long idx[2];
      int zg[2];
      bool ok[2];
      float4 w[2], g[2], s0[2], s1[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const long t = t0 + u * nth;
        ok[u] = t < m4;
        const long tc = ok[u] ? t : m4 - 1;
        int k = 0;
        for (int j = 1; j < a.fs.count; ++j) k = tc >= a.fs.start4[j] ? j : k;
        idx[u] = a.fs.lo4[k] + (tc - a.fs.start4[k]);
        zg[u] = a.fs.zero[k];
        w[u] = w4[idx[u]];
        g[u] = g4[idx[u]];
        s0[u] = nslot >= 1 ? s04[idx[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
        s1[u] = nslot >= 2 ? s14[idx[u]] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!ok[u]) continue;
        float* wp = (float*)&w[u];
        const float* gp = (const float*)&g[u];
        float* sp0 = (float*)&s0[u];
        float* sp1 = (float*)&s1[u];
#pragma unroll
        for (int j = 0; j < 4; ++j) opt_update(a.opt, lr, wp[j], gp[j], sp0[j], sp1[j]);
        w4[idx[u]] = w[u];
        if (nslot >= 1) s04[idx[u]] = s0[u];
        if (nslot >= 2) s14[idx[u]] = s1[u];
        if (a.gz && zg[u]) reinterpret_cast<float4*>(a.gz)[idx[u]] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  }
  OPT_STAMP(1);
  opt_duties(a, tid, nth);
  OPT_STAMP(3);
}

}  // namespace csa

using namespace csa;

CSA_API int csa_opt_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_opt_dbg), &p, sizeof(p));
}

// Segments seg_lo/seg_hi (count <= 16, float4-aligned; nseg == 0: the whole [0, n)).
// zero_ptrs/zero_ns: count <= 16 regions; fold_*: count <= 8 striped/partial descriptors.
// zero_grad != 0: the update clears g[i] after reading it (g is then an accumulator that
// must start the next step at zero); zero_ptrs must NOT overlap g or the fold stripes.
// met_parts > 0: write the metric ring from the head's partial loss / #correct.
static BatchStage make_stage(const uint8_t* img, const int64_t* labels, const int64_t* rows, const int64_t* cursor,
                             int B, long imsz, uint8_t* out_img, int64_t* out_lbl) {
  BatchStage s{};
  if (!out_img) return s;
  s.img = reinterpret_cast<const uint32_t*>(img);
  s.labels = labels; s.rows = rows; s.cursor = cursor; s.B = B; s.words = imsz / 4;
  s.out_img = reinterpret_cast<uint32_t*>(out_img); s.out_lbl = out_lbl;
  const long total = (long)B * s.words > B ? (long)B * s.words : B;
  s.blocks = (int)((total + 255) / 256);
  return s;
}

// Prime the staging buffers for the current cursor (before the first step, after the
// host moved the cursor).  imsz % 4 == 0.
CSA_API int csa_gather_batch(const uint8_t* img, const int64_t* labels, const int64_t* rows, const int64_t* cursor,
                             int B, long imsz, uint8_t* out_img, int64_t* out_lbl, hipStream_t st) {
  if (B <= 0 || imsz <= 0 || imsz % 4 || !out_img || !out_lbl) return -1;
  const BatchStage s = make_stage(img, labels, rows, cursor, B, imsz, out_img, out_lbl);
  hipLaunchKernelGGL(gather_batch_kernel, dim3(s.blocks), dim3(256), 0, st, s);
  return (int)hipGetLastError();
}

CSA_API int csa_optimizer2s(int opt, float* w, float* g, float* s0, float* s1, long n, const long* seg_lo,
                            const long* seg_hi, int nseg, int zero_grad, float lr, const int64_t* step,
                            float* const* zero_ptrs, const long* zero_ns, int nzero, const long* fold_off,
                            const long* fold_n, float* const* fold_src, const int* fold_S, const long* fold_ld,
                            const int* fold_zero, int nfold, const long* keep_lo, const long* keep_hi, int nkeep,
                            const float* met_loss, const int* met_corr, int met_parts, float met_div,
                            float* ring_loss, int* ring_correct, int ring, int64_t* cursor, long cursor_wrap,
                            const uint8_t* st_img, const int64_t* st_labels, const int64_t* st_rows,
                            const int64_t* st_cursor, int st_B, long st_imsz, uint8_t* st_out_img,
                            int64_t* st_out_lbl, hipStream_t st);

// The flag the NEXT csa_optimizer2s launch on this thread raises (host state, consumed by
// that call): the data-parallel programs' deferred dense update (conv_pair.hip CPOptCarry).
static thread_local unsigned* g_opt_set_pending = nullptr;
CSA_API void csa_optimizer_set_pending(unsigned* flag) { g_opt_set_pending = flag; }

// A network whose first unit reads no raw images (a dense / standalone norm / pool first
// layer) takes its float input [B][D] = images[rows[cursor]] / 255 from this one launch
// (was index_select + to(float) + mul: three torch kernels per step).  One thread per
// 4 pixels: a uint32 load, a float4 store.
__global__ __launch_bounds__(256) void gather_f32_kernel(const uint32_t* img, const int64_t* rows,
                                                         const int64_t* cursor, int B, long words, float4* out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)B * words) return;
  const long b = i / words, off = i - b * words;
  const int64_t r = rows[*cursor * B + b];
  const uint32_t v = img[r * words + off];
  constexpr float k = 1.0f / 255.0f;
  out[i] = make_float4((float)(v & 255u) * k, (float)((v >> 8) & 255u) * k, (float)((v >> 16) & 255u) * k,
                       (float)(v >> 24) * k);
}

CSA_API int csa_gather_images_f32(const uint8_t* img, const int64_t* rows, const int64_t* cursor, int B, long imsz,
                                  float* out, hipStream_t st) {
  if (B <= 0 || imsz <= 0 || imsz % 4 || !img || !rows || !cursor || !out) return -1;
  const long words = imsz / 4, total = (long)B * words;
  hipLaunchKernelGGL(gather_f32_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st,
                     reinterpret_cast<const uint32_t*>(img), rows, cursor, B, words, reinterpret_cast<float4*>(out));
  return (int)hipGetLastError();
}

CSA_API int csa_optimizer2(int opt, float* w, float* g, float* s0, float* s1, long n, const long* seg_lo,
                           const long* seg_hi, int nseg, int zero_grad, float lr, const int64_t* step,
                           float* const* zero_ptrs, const long* zero_ns, int nzero, const long* fold_off,
                           const long* fold_n, float* const* fold_src, const int* fold_S, const long* fold_ld,
                           const int* fold_zero, int nfold, const long* keep_lo, const long* keep_hi, int nkeep,
                           const float* met_loss, const int* met_corr, int met_parts, float met_div,
                           float* ring_loss, int* ring_correct, int ring, int64_t* cursor, long cursor_wrap,
                           hipStream_t st) {
  return csa_optimizer2s(opt, w, g, s0, s1, n, seg_lo, seg_hi, nseg, zero_grad, lr, step, zero_ptrs, zero_ns, nzero,
                         fold_off, fold_n, fold_src, fold_S, fold_ld, fold_zero, nfold, keep_lo, keep_hi, nkeep,
                         met_loss, met_corr, met_parts, met_div, ring_loss, ring_correct, ring, cursor, cursor_wrap,
                         nullptr, nullptr, nullptr, nullptr, 0, 0, nullptr, nullptr, st);
}

// ... plus the next step's batch staging (st_out_img != null; the head advanced the
// cursor, so pass cursor = null here).
CSA_API int csa_optimizer2s(int opt, float* w, float* g, float* s0, float* s1, long n, const long* seg_lo,
                            const long* seg_hi, int nseg, int zero_grad, float lr, const int64_t* step,
                            float* const* zero_ptrs, const long* zero_ns, int nzero, const long* fold_off,
                            const long* fold_n, float* const* fold_src, const int* fold_S, const long* fold_ld,
                            const int* fold_zero, int nfold, const long* keep_lo, const long* keep_hi, int nkeep,
                            const float* met_loss, const int* met_corr, int met_parts, float met_div,
                            float* ring_loss, int* ring_correct, int ring, int64_t* cursor, long cursor_wrap,
                            const uint8_t* st_img, const int64_t* st_labels, const int64_t* st_rows,
                            const int64_t* st_cursor, int st_B, long st_imsz, uint8_t* st_out_img,
                            int64_t* st_out_lbl, hipStream_t st) {
  if (st_out_img && (st_imsz % 4 || st_B <= 0)) return -1;
  if (n % 4 || nzero > MAXZ || nfold > MAXF || nkeep > MAXK || nseg > MAXSEG) return -1;
  OptArgs a{};
  a.set_pending = g_opt_set_pending;
  g_opt_set_pending = nullptr;
  a.keep.count = nkeep;
  for (int i = 0; i < nkeep; ++i) {
    if (keep_lo[i] % 4 || keep_hi[i] % 4) return -1;
    a.keep.lo[i] = keep_lo[i];
    a.keep.hi[i] = keep_hi[i];
  }
  a.seg.count = nseg > 0 ? nseg : 1;
  a.seg.start4[0] = 0;
  for (int i = 0; i < a.seg.count; ++i) {
    const long lo = nseg > 0 ? seg_lo[i] : 0, hi = nseg > 0 ? seg_hi[i] : n;
    if (lo % 4 || hi % 4 || hi < lo || hi > n) return -4;
    a.seg.lo[i] = lo;
    a.seg.start4[i + 1] = a.seg.start4[i] + (hi - lo) / 4;
  }
  a.cursor = cursor;
  a.cursor_wrap = cursor_wrap;
  a.opt = opt; a.w = w; a.g = g; a.s0 = s0; a.s1 = s1; a.lr = lr; a.step = step;
  a.gz = zero_grad ? g : nullptr;
  a.z.count = nzero;
  for (int i = 0; i < nzero; ++i) { a.z.p[i] = zero_ptrs[i]; a.z.n[i] = zero_ns[i]; }
  a.fold.count = nfold;
  a.fold.lo = nfold ? fold_off[0] : 0;
  a.fold.hi = 0;
  for (int i = 0; i < nfold; ++i) {
    if (fold_off[i] % 4 || fold_S[i] > MAXS || fold_S[i] < 1) return -1;
    a.fold.f[i] = Fold{fold_off[i], fold_n[i], fold_ld[i], fold_src[i], fold_S[i], fold_zero ? fold_zero[i] : 1};
    a.fold.lo = fold_off[i] < a.fold.lo ? fold_off[i] : a.fold.lo;
    a.fold.hi = fold_off[i] + fold_n[i] > a.fold.hi ? fold_off[i] + fold_n[i] : a.fold.hi;
  }
  a.met = MetricFold{met_loss, met_corr, met_parts, met_div, ring_loss, ring_correct, ring};
  // fast path: no folds -> split the segments at the keep ranges' edges (float4 units)
  if (nfold == 0) {
    FastSegs f{};
    bool fits = true;
    f.start4[0] = 0;
    for (int i = 0; i < a.seg.count && fits; ++i) {
      long x = a.seg.lo[i], end = a.seg.lo[i] + 4 * (a.seg.start4[i + 1] - a.seg.start4[i]);
      while (x < end && fits) {
        // the piece [x, y) lies wholly inside a keep range (zero = 0) or wholly outside (1)
        int inside = -1;
        long y = end;
        for (int q = 0; q < nkeep; ++q) {
          if (x >= keep_lo[q] && x < keep_hi[q]) { inside = q; y = y < keep_hi[q] ? y : keep_hi[q]; }
          else if (keep_lo[q] > x && keep_lo[q] < y) y = keep_lo[q];
        }
        if (f.count >= MAXFS) { fits = false; break; }
        f.lo4[f.count] = x / 4;
        f.zero[f.count] = inside < 0 ? 1 : 0;
        f.start4[f.count + 1] = f.start4[f.count] + (y - x) / 4;
        ++f.count;
        x = y;
      }
    }
    if (fits && f.count > 0) { a.fast = 1; a.fs = f; }
  }
  const long n4 = a.seg.start4[a.seg.count];
  long zmax = 0;
  for (int i = 0; i < nzero; ++i) zmax = zero_ns[i] > zmax ? zero_ns[i] : zmax;
  const long work = n4 > zmax ? n4 : zmax;
  // block cap: swept on MI355X for the 2.28 M-parameter sample (graph step, µs): 512 ->
  // 122.8, 1024 -> 121.0, 1536 -> 120.2, 2048 -> 120.3, 8192 (one float4 per thread) ->
  // 121.6 — more blocks cost more than the grid-stride second iteration saves
  constexpr int cap = 2048;
  int blocks = (int)((work + 255) / 256);
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  a.stage = make_stage(st_img, st_labels, st_rows, st_cursor, st_B, st_imsz, st_out_img, st_out_lbl);
  if (a.fast) {
    // half the threads: each keeps two float4s of every operand in flight
    const long fwork = ((a.fs.start4[a.fs.count] + 1) / 2) > zmax ? (a.fs.start4[a.fs.count] + 1) / 2 : zmax;
    int fb = (int)((fwork + 255) / 256);
    fb = fb > cap ? cap : (fb < 1 ? 1 : fb);
    hipLaunchKernelGGL(optim_fast_kernel, dim3(fb + a.stage.blocks), dim3(256), 0, st, a);
  } else {
    hipLaunchKernelGGL(optim_kernel, dim3(blocks + a.stage.blocks), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

// Backward-compatible entry: the whole buffer, the head wrote the metric ring itself.
CSA_API int csa_optimizer(int opt, float* w, float* g, float* s0, float* s1, long n, int zero_grad,
                          float lr, const int64_t* step, float* const* zero_ptrs, const long* zero_ns,
                          int nzero, const long* fold_off, const long* fold_n, float* const* fold_src,
                          const int* fold_S, const long* fold_ld, int nfold, const long* keep_lo,
                          const long* keep_hi, int nkeep, int64_t* cursor, long cursor_wrap, hipStream_t st) {
  return csa_optimizer2(opt, w, g, s0, s1, n, nullptr, nullptr, 0, zero_grad, lr, step, zero_ptrs, zero_ns, nzero,
                        fold_off, fold_n, fold_src, fold_S, fold_ld, nullptr, nfold, keep_lo, keep_hi, nkeep,
                        nullptr, nullptr, 0, 1.f, nullptr, nullptr, 1, cursor, cursor_wrap, st);
}

// Zero a list of regions (used once at init and by tests).
__global__ void zero_kernel(ZeroList z) {
  const long tid = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long nth = (long)gridDim.x * blockDim.x;
  for (int k = 0; k < z.count; ++k)
    for (long i = tid; i < z.n[k]; i += nth) z.p[k][i] = 0.f;
}

CSA_API int csa_zero(float* const* ptrs, const long* ns, int count, hipStream_t st) {
  if (count > MAXZ) return -1;
  ZeroList z{};
  z.count = count;
  for (int i = 0; i < count; ++i) { z.p[i] = ptrs[i]; z.n[i] = ns[i]; }
  hipLaunchKernelGGL(zero_kernel, dim3(256), dim3(256), 0, st, z);
  return (int)hipGetLastError();
}
