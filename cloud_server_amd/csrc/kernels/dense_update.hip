// Dense-layer backward + optimizer update in ONE launch (gfx950 / CDNA4).
//
// Reference: the train op minimize() of construct_distribute.py:372-373 — gradients of
// the dense layers (:168-182) followed by ApplyAdagrad on the parameter server.  On one
// GPU nothing needs a dense weight gradient except the optimizer, so it is never written
// to memory.
//
// Decomposition (round 2, v4).  W is [K][N] (input x output features).  One 1024-thread
// workgroup per ROW GROUP of 16 input features (f0 .. f0+15) owns those W rows across ALL
// N columns, so the input gradient of its features is complete inside the workgroup (no
// split-K, no cross-workgroup hand-off) and every W element has exactly one owner (the
// in-place update is race-free).  fc1 of the sample config: 245 workgroups = one round
// on 256 CUs; everything is issued as ONE batch of loads at kernel start:
//
//   dY           the whole [M][N] batch gradient -> LDS (row stride N + 4);
//   W / slots    lane (i = lane & 15, q = lane >> 4) of wave w, column sub-tile
//                j in {w, w + 16} (16 columns each): W[f0 + i][16j + 4q .. +3] as one float4
//                straight into registers (the "update layout");
//   Xw           the weight-gradient operand Xw[4s + q][f0 + i] (13 k-steps at M = 50);
//   x_fwd, BN    the epilogue's forward input and BatchNorm tables (precomputed by
//                csa_bn_act_apply, so the epilogue needs no slab reduction).
//
// Per sub-tile: wgrad  dW[f][n] = sum_m dY[m][n] Xw[m][f]  (v_mfma_f32_16x16x4_f32,
// A = dY[4s + q][16j + i] from LDS, B = Xw) lands in the update layout, so the optimizer
// update is register-local; dgrad partial  dX[m][f] += sum_n dY[m][n] W[f][n]  (A = one
// LDS float4 dY[16t + i][16j + 4q ..], B = the OLD W float4, consumed before the update).
// The 16 waves' partials fold in LDS in fixed order, then the forward input transform's
// backward (activation; BatchNorm partial statistics into the backward slab) and dX.
// Bias gradients (column sums of dY) are spread over the workgroups, a few columns each.
//
// Earlier designs measured slower (profiles/r2_dense_fused.md): one 256-thread workgroup
// per row group walking N in 8 dependent chunks (23 us for fc1), and 16 x 64 tiles with a
// write-through partial hand-off to the row group's last arriving tile (31 us: 1960 tiles
// queue for slots and the elected tile's epilogue is a second chain).
//
// HBM per step for the sample fc1 (3920 x 512): W and the Adagrad accumulator read once
// and written once (32 MB) — instead of the split-K backward pair (dW written) plus the
// flat optimizer pass (dW, W, acc re-read).
#include "dense_update.h"
#include <cstdlib>

namespace csa {

template <int NSLOT, int WAVES, bool HEAD, bool DGO = false>
__global__ __launch_bounds__(64 * WAVES) void dense_bwd_update_kernel(DUArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  du_body<NSLOT, WAVES, HEAD, DGO>(a, (int)blockIdx.x, (int)gridDim.x, smem);
}

// Deferred weight-gradient + update segments (see csa_dense_update_defer).
thread_local DUDeferred g_du_def{};

}  // namespace csa


using namespace csa;

// gradient-mode outputs of the next launch on this thread (set by csa_dense_bwd_grad_head only)
static thread_local float* g_du_grad_w = nullptr;
static thread_local float* g_du_grad_b = nullptr;

CSA_NT_SETTER(csa_nt_out_du)

CSA_API int csa_du_debug(long long* p) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_du_dbg), &p, sizeof(p));
}

// Shape family of the fused kernel (0 = outside: the caller uses the separate backward
// kernels + the flat optimizer).  M <= 64, K % 4 == 0, N % 16 == 0; N <= 512 (one block
// per row group) or N % 128 == 0 (column blocks of 128).
CSA_API int csa_dense_bwd_update_ok(int M, int K, int N, int bn_C) {
  if (M < 1 || M > DU_MAXM || K < 4 || K % 4 || N < 16 || N % 16) return 0;
  if (bn_C > MAXC_DU) return 0;
  if (N > 512 && N % 128) return 0;
  return du_lds_floats(M, 16) * sizeof(float) <= DU_LDS_MAX ? 1 : 0;
}

// BN-backward slab rows the kernel accumulates into (atomically; the caller zeroes them).
// Deterministic mode: one exclusive row per row group.
CSA_API int csa_dense_bwd_update_slabs(int K) {
  const int groups = (K + DU_FT - 1) / DU_FT;
  return g_csa_det || groups < DU_SLAB ? groups : DU_SLAB;
}

// Column blocks per row group the launcher picks: one 1024-thread block when the row groups
// fill the chip (fc1: 245) and N <= 512 (one process per GPU), else 128-column blocks of
// 256 threads.
static int du_cs(int K, int N) {
  const int groups = (K + DU_FT - 1) / DU_FT;
  // packed profile: always 128-column blocks (256 threads, 33 KB LDS: four per CU beside
  // other jobs' kernels): K = 4 805.5k vs 743.0k samples/s (profiles/r2_multitenant.md)
  // ranks sharing ONE GPU (g_csa_shared): a 16-wave workgroup of one process was seen
  // not to be placed for as long as another process's kernel spun in a peer wait (the
  // round-5 world-2 stall: profiles/r5_notes.md); 256-thread blocks always were
  // CSA_DU_WIDE=0: 128-column blocks everywhere (an A/B knob for the one-GPU programs)
  // CSA_DU_WIDE=1: the wide blocks in the packed profile too (A/B knob)
  static const int wide_env = [] { const char* e = getenv("CSA_DU_WIDE"); return e ? (e[0] == '0' ? 0 : 1) : -1; }();
  const bool narrow = wide_env == 0 || g_csa_shared || (g_csa_packed && wide_env != 1);
  const int minb = narrow ? (1 << 30) : 128;
  if (N <= 512 && groups >= minb) return 1;
  return (N + 127) / 128;
}

// Workspace of the partial hand-off: floats of the slabs (ws[0]), arrival counters (ws[1]).
CSA_API int csa_dense_bwd_update_ws(int K, int N, long long* ws) {
  const long long groups = (K + DU_FT - 1) / DU_FT, cs = du_cs(K, N);
  ws[0] = cs > 1 ? groups * cs * DU_PART : 0;
  ws[1] = cs > 1 ? groups : 0;
  return (int)cs;
}

template <int NSLOT, int WAVES, bool HEAD>
static void du_launch3(const DUArgs& a, int blocks, hipStream_t st) {
  static const bool attr = hipFuncSetAttribute((const void*)dense_bwd_update_kernel<NSLOT, WAVES, HEAD>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL((dense_bwd_update_kernel<NSLOT, WAVES, HEAD>), dim3((unsigned)blocks), dim3(64 * WAVES),
                     du_lds_floats(a.M, WAVES) * sizeof(float), st, a);
}

template <int WAVES>
static void du_launch3_dgo(const DUArgs& a, int blocks, hipStream_t st) {
  static const bool attr = hipFuncSetAttribute((const void*)dense_bwd_update_kernel<0, WAVES, false, true>,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)DU_LDS_MAX) == hipSuccess;
  (void)attr;
  hipLaunchKernelGGL((dense_bwd_update_kernel<0, WAVES, false, true>), dim3((unsigned)blocks), dim3(64 * WAVES),
                     du_lds_floats(a.M, WAVES) * sizeof(float), st, a);
}

template <int NSLOT, int WAVES>
static void du_launch(const DUArgs& a, int blocks, hipStream_t st) {
  if (a.hy) du_launch3<NSLOT, WAVES, true>(a, blocks, st);
  else du_launch3<NSLOT, WAVES, false>(a, blocks, st);
}

CSA_API int csa_dense_bwd_update_head(const float* dY, float* W, float* bias, float* dX, int M, int K, int N,
                                      const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                      int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                      const float* bn_offset, float* bwd_slab, const float* Xw, int opt, float lr,
                                      const int64_t* step, float* s0w, float* s1w, float* s0b, float* s1b,
                                      float scale, const float* bn_tab, float* part, unsigned* cnt,
                                      const float* hy, const float* hdl, float* hgw, float* hgb, const float* hrl,
                                      const int* hrc, float* ring_loss, int* ring_correct, int ring, float ldiv,
                                      int hact, float halpha, hipStream_t st);

CSA_API int csa_dense_bwd_update(const float* dY, float* W, float* bias, float* dX, int M, int K, int N,
                                 const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                 int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                 const float* bn_offset, float* bwd_slab, const float* Xw, int opt, float lr,
                                 const int64_t* step, float* s0w, float* s1w, float* s0b, float* s1b,
                                 float scale, const float* bn_tab, float* part, unsigned* cnt, hipStream_t st) {
  return csa_dense_bwd_update_head(dY, W, bias, dX, M, K, N, x_fwd, act, alpha, bn_slab, bn_nslab, bn_C, bn_count,
                                   bn_eps, bn_scale, bn_offset, bwd_slab, Xw, opt, lr, step, s0w, s1w, s0b, s1b,
                                   scale, bn_tab, part, cnt, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                   nullptr, nullptr, 1, 1.f, 0, 0.f, st);
}

CSA_API int csa_dense_bwd_grad_head(const float* dY, const float* W, float* dX, int M, int K, int N,
                                    const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                    int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                    const float* bn_offset, float* bwd_slab, const float* Xw, float scale,
                                    const float* bn_tab, float* part, unsigned* cnt, float* gW, float* gb,
                                    const float* hy, const float* hdl, float* hgw, float* hgb, const float* hrl,
                                    const int* hrc, float* ring_loss, int* ring_correct, int ring, float ldiv,
                                    int hact, float halpha, const int64_t* step, hipStream_t st);

// ... plus the head epilogue (hy != null): dWh / dbh of the row-per-workgroup head and the
// step's metric ring entry are reduced by this launch (see DUArgs).
CSA_API int csa_dense_bwd_update_head(const float* dY, float* W, float* bias, float* dX, int M, int K, int N,
                                 const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                 int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                 const float* bn_offset, float* bwd_slab, const float* Xw, int opt, float lr,
                                 const int64_t* step, float* s0w, float* s1w, float* s0b, float* s1b,
                                 float scale, const float* bn_tab, float* part, unsigned* cnt,
                                      const float* hy, const float* hdl, float* hgw, float* hgb, const float* hrl,
                                      const int* hrc, float* ring_loss, int* ring_correct, int ring, float ldiv,
                                      int hact, float halpha, hipStream_t st) {
  if (!csa_dense_bwd_update_ok(M, K, N, bn_slab ? bn_C : 0)) return -1;
  if (hy && (!hdl || !hgw || !hgb || !hrl || !hrc || !ring_loss || !ring_correct || ring < 1 || !step)) return -2;
  if (!Xw || !W || !dY) return -2;
  DUArgs a{};
  a.M = M; a.K = K; a.N = N; a.dY = dY; a.W = W; a.bias = bias; a.dX = dX; a.x_fwd = x_fwd;
  a.act = act; a.alpha = alpha;
  a.bn = BNRef{bn_slab, bn_nslab, bn_slab ? bn_C : 1, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr; a.bn_tab = bn_slab ? bn_tab : nullptr;
  a.bwd_slab = bwd_slab; a.Xw = Xw; a.det = g_csa_det;
  a.opt = opt; a.lr = lr; a.step = step; a.s0w = s0w; a.s1w = s1w; a.s0b = s0b; a.s1b = s1b; a.scale = scale;
  const int groups = (K + DU_FT - 1) / DU_FT;
  a.cs = du_cs(K, N);
  a.part = part; a.cnt = cnt;
  a.hy = hy; a.hdl = hdl; a.hgw = hgw; a.hgb = hgb; a.hrl = hrl; a.hrc = hrc;
  a.ring_loss = ring_loss; a.ring_correct = ring_correct; a.ring = ring; a.ldiv = ldiv;
  a.hact = hact; a.halpha = halpha;
  a.gW = g_du_grad_w; a.gb = g_du_grad_b;
  if (a.cs > 1 && dX && (!part || !cnt)) return -2;
  const int blocks = groups * a.cs;
  const int ns = a.gW ? 0 : opt_nslots(opt);
  if (a.cs == 1) {
    if (ns == 0) du_launch<0, 16>(a, blocks, st);
    else if (ns == 1) du_launch<1, 16>(a, blocks, st);
    else du_launch<2, 16>(a, blocks, st);
  } else {
    if (ns == 0) du_launch<0, 4>(a, blocks, st);
    else if (ns == 1) du_launch<1, 4>(a, blocks, st);
    else du_launch<2, 4>(a, blocks, st);
  }
  return (int)hipGetLastError();
}

// Data-parallel form: the same fused launch (input gradient + transform backward + BN
// statistics + the head epilogue) with the weight / bias GRADIENTS stored whole into
// gW / gb instead of the in-kernel update — the gradient must be all-reduced first.
CSA_API int csa_dense_bwd_grad_head(const float* dY, const float* W, float* dX, int M, int K, int N,
                                    const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                    int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                    const float* bn_offset, float* bwd_slab, const float* Xw, float scale,
                                    const float* bn_tab, float* part, unsigned* cnt, float* gW, float* gb,
                                    const float* hy, const float* hdl, float* hgw, float* hgb, const float* hrl,
                                    const int* hrc, float* ring_loss, int* ring_correct, int ring, float ldiv,
                                    int hact, float halpha, const int64_t* step, hipStream_t st) {
  if (!gW || !gb) return -2;
  g_du_grad_w = gW;
  g_du_grad_b = gb;
  const int rc = csa_dense_bwd_update_head(dY, const_cast<float*>(W), nullptr, dX, M, K, N, x_fwd, act, alpha,
                                           bn_slab, bn_nslab, bn_C, bn_count, bn_eps, bn_scale, bn_offset,
                                           bwd_slab, Xw, OPT_SGD, 0.f, step, nullptr, nullptr, nullptr, nullptr,
                                           scale, bn_tab, part, cnt, hy, hdl, hgw, hgb, hrl, hrc, ring_loss,
                                           ring_correct, ring, ldiv, hact, halpha, st);
  g_du_grad_w = g_du_grad_b = nullptr;
  return rc;
}

// ---------------------------------------------------------------------------------------
// Horizontal fusion (round 4).  On one GPU a dense layer's weight gradient + update feeds
// nothing but the NEXT step's forward of that layer, while its input gradient is on the
// step's critical path.  So the backward is split: the input gradient (+ transform
// backward + BN statistics) runs as its own launch (csa_dense_bwd_dgrad), and the weight
// gradient + update is DEFERRED — recorded here and carried as extra workgroups of a later
// launch that is on the critical path anyway (the conv-pair backward, conv_pair.hip), where
// it fills CUs that launch leaves idle instead of adding a kernel boundary and a serial
// 10-15 us to the chain.  Reference: the train op of construct_distribute.py:372-373.

// Input gradient only: same shapes / outputs as csa_dense_bwd_update minus the update.
CSA_API int csa_dense_bwd_dgrad(const float* dY, const float* W, float* dX, int M, int K, int N,
                                const float* x_fwd, int act, float alpha, const float* bn_slab, int bn_nslab,
                                int bn_C, float bn_count, float bn_eps, const float* bn_scale,
                                const float* bn_offset, float* bwd_slab, const float* bn_tab, float* part,
                                unsigned* cnt, hipStream_t st) {
  if (!csa_dense_bwd_update_ok(M, K, N, bn_slab ? bn_C : 0) || !dX || !dY || !W) return -1;
  DUArgs a{};
  a.M = M; a.K = K; a.N = N; a.dY = dY; a.W = const_cast<float*>(W); a.dX = dX; a.x_fwd = x_fwd;
  a.act = act; a.alpha = alpha;
  a.bn = BNRef{bn_slab, bn_nslab, bn_slab ? bn_C : 1, bn_count, bn_eps, bn_scale, bn_offset};
  a.bn_on = bn_slab != nullptr; a.bn_tab = bn_slab ? bn_tab : nullptr;
  // Xw is not read in this mode, but it is the epilogue's address-select fallback for
  // x_fwd, so it must have the [M][K] shape: the input gradient buffer itself
  a.bwd_slab = bwd_slab; a.Xw = x_fwd ? x_fwd : dX; a.det = g_csa_det; a.scale = 1.f;
  const int groups = (K + DU_FT - 1) / DU_FT;
  a.cs = du_cs(K, N);
  a.part = part; a.cnt = cnt;
  if (a.cs > 1 && (!part || !cnt)) return -2;
  const int blocks = groups * a.cs;
  if (a.cs == 1) du_launch3_dgo<16>(a, blocks, st);
  else du_launch3_dgo<4>(a, blocks, st);
  return (int)hipGetLastError();
}

// Record the weight gradient + optimizer update of a dense layer (dW = Xw^T dY, K x N)
// for the next launch that carries deferred segments (csa_conv_pair_bwd), as 128-column
// workgroups of 256 threads.  hy != null: the head epilogue rides along (dWh / dbh into the
// flat gradient, the step's metric ring entry; see DUArgs).  Returns the segment count, or
// < 0 when the shape is outside the family or the list is full.
CSA_API int csa_dense_update_defer(const float* dY, float* W, float* bias, int M, int K, int N, const float* Xw,
                                   int opt, float lr, const int64_t* step, float* s0w, float* s1w, float* s0b,
                                   float* s1b, float scale, const float* hy, const float* hdl, float* hgw,
                                   float* hgb, const float* hrl, const int* hrc, float* ring_loss,
                                   int* ring_correct, int ring, float ldiv, int hact, float halpha) {
  if (!csa_dense_bwd_update_ok(M, K, N, 0) || N % 128 || !Xw || !W || !dY || !step) return -1;
  if (g_du_def.n >= DU_MAXDEF) return -3;
  if (hy && (g_du_def.head >= 0 || !hdl || !hgw || !hgb || !hrl || !hrc || !ring_loss || !ring_correct || ring < 1))
    return -2;
  if (g_du_def.n > 0 && opt_nslots(g_du_def.seg[0].opt) != opt_nslots(opt)) return -4;   // one NSLOT per launch
  DUArgs a{};
  a.M = M; a.K = K; a.N = N; a.dY = dY; a.W = W; a.bias = bias; a.dX = nullptr; a.x_fwd = nullptr;
  a.bn = BNRef{nullptr, 0, 1, 1.f, 0.f, nullptr, nullptr};
  a.Xw = Xw; a.det = g_csa_det;
  a.opt = opt; a.lr = lr; a.step = step; a.s0w = s0w; a.s1w = s1w; a.s0b = s0b; a.s1b = s1b; a.scale = scale;
  a.cs = N / 128;
  a.hy = hy; a.hdl = hdl; a.hgw = hgw; a.hgb = hgb; a.hrl = hrl; a.hrc = hrc;
  a.ring_loss = ring_loss; a.ring_correct = ring_correct; a.ring = ring; a.ldiv = ldiv;
  a.hact = hact; a.halpha = halpha;
  if (g_du_def.n == 0) g_du_def.head = -1;
  if (hy) g_du_def.head = g_du_def.n;
  g_du_def.blocks[g_du_def.n] = ((K + DU_FT - 1) / DU_FT) * a.cs;
  g_du_def.seg[g_du_def.n++] = a;
  return g_du_def.n;
}

CSA_API int csa_dense_update_pending() { return g_du_def.n; }

// The LAST deferred segment in gradient mode (data parallel): its weight / bias gradients
// are stored whole into gW / gb (the flat gradient, exchanged before the optimizer) instead
// of updating W / b.  Defer it with the slot-free rule (opt 0): no slot is read.
CSA_API int csa_dense_update_grad_mode(float* gW, float* gb) {
  if (g_du_def.n < 1 || !gW || !gb) return -1;
  DUArgs& a = g_du_def.seg[g_du_def.n - 1];
  if (opt_nslots(a.opt) != 0) return -2;
  a.gW = gW; a.gb = gb;
  return 0;
}

// The deferred head segment updates the head's parameters in place (w [K][10], b [10] and
// their optimizer slots) instead of storing dWh / dbh: the pair-backward tail program.
CSA_API int csa_dense_update_head_params(float* hw, float* hb, float* hs0w, float* hs1w, float* hs0b, float* hs1b) {
  if (g_du_def.head < 0 || !hw || !hb) return -1;
  DUArgs& a = g_du_def.seg[g_du_def.head];
  const int ns = opt_nslots(a.opt);
  if ((ns >= 1 && (!hs0w || !hs0b)) || (ns >= 2 && (!hs1w || !hs1b))) return -2;
  a.hw = hw; a.hb = hb; a.hs0w = hs0w; a.hs1w = hs1w; a.hs0b = hs0b; a.hs1b = hs1b;
  return 0;
}

namespace csa {
int du_take(DUSegs& out) {
  out = DUSegs{};
  out.head = g_du_def.head;
  out.nseg = g_du_def.n;
  for (int s = 0; s < DU_MAXDEF; ++s) {
    if (s < out.nseg) out.seg[s] = g_du_def.seg[s];
    out.start[s + 1] = out.start[s] + (s < out.nseg ? g_du_def.blocks[s] : 0);
  }
  g_du_def.n = 0;
  g_du_def.head = -1;
  return out.nseg;
}
}  // namespace csa

// Launch the deferred segments on their own (one 256-thread launch per segment): the
// fallback when no carrying launch consumed them.
namespace csa {
int du_flush_segs(const DUSegs& u, hipStream_t st) {
  for (int s = 0; s < u.nseg; ++s) {
    const DUArgs& a = u.seg[s];
    const int ns = opt_nslots(a.opt), blocks = u.start[s + 1] - u.start[s];
    const bool head = s == u.head;
    if (ns == 0) head ? du_launch3<0, 4, true>(a, blocks, st) : du_launch3<0, 4, false>(a, blocks, st);
    else if (ns == 1) head ? du_launch3<1, 4, true>(a, blocks, st) : du_launch3<1, 4, false>(a, blocks, st);
    else head ? du_launch3<2, 4, true>(a, blocks, st) : du_launch3<2, 4, false>(a, blocks, st);
  }
  return (int)hipGetLastError();
}
}  // namespace csa

CSA_API int csa_dense_update_flush(hipStream_t st) {
  DUSegs u;
  return du_take(u) > 0 ? du_flush_segs(u, st) : 0;
}

CSA_API void csa_dense_update_clear() { g_du_def.n = 0; g_du_def.head = -1; }

// Launch only the LAST deferred segment now, on ``st`` (its own stream: a graph branch that
// overlaps the carrying launch and the next step's first launch), and drop it from the list.
CSA_API int csa_dense_update_flush_last(hipStream_t st) {
  const int n = g_du_def.n;
  if (n < 1) return 0;
  DUSegs u{};
  u.nseg = 1;
  u.head = g_du_def.head == n - 1 ? 0 : -1;
  u.seg[0] = g_du_def.seg[n - 1];
  u.start[0] = 0;
  for (int s2 = 1; s2 <= DU_MAXDEF; ++s2) u.start[s2] = g_du_def.blocks[n - 1];
  g_du_def.n = n - 1;
  if (g_du_def.head == n - 1) g_du_def.head = -1;
  return du_flush_segs(u, st);
}
