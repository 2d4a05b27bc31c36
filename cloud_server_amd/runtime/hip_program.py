"""Lower a DSL network to the hand-written gfx950 kernels (the MI355X training step).

Lowering groups the reference layer list (construct_distribute.py:208-265) into:

* **conv units** ``conv [act] [pool]`` — one ``csa_conv_fwd`` launch each (bias, act and
  max-pool fused, argmax kept for backward, BN partial statistics emitted when a norm
  follows);
* **transforms** ``[norm] [act]`` between units — never materialised: the CONSUMER applies
  BN-apply + activation while loading its input (conv input read, GEMM A-prologue,
  im2col loader) and its dgrad epilogue applies the activation backward and emits the
  BN-backward statistics;
* **dense units** ``connect`` — MFMA GEMMs (``csa_dense_fwd/_dgrad/_wgrad``);
* the **head** — one single-workgroup kernel: logits, loss, accuracy, head gradients,
  input gradient and the step/metric bookkeeping.

Backward runs the units in reverse (``csa_route_bwd`` = BN backward + act backward +
max-pool routing; ``csa_conv_dgrad``; ``csa_conv_wgrad`` as an implicit MFMA GEMM),
then gradient all-reduce (data parallel) and ONE fused optimizer launch which also
zeroes next step's atomic accumulators and updates BN running statistics.

A conv with more than 128 input or output channels (beyond the direct kernels' LDS
tables) is a **gconv unit**: forward, input gradient and weight gradient as implicit
MFMA GEMMs whose loaders gather the im2col / transposed operands on the fly
(``csa_gconv_*`` in gemm.hip); its activation, pool and norm run as standalone units.

Layer orders the consumer transform cannot express — a 2-D norm after a dense layer, a
norm over > 128 channels or directly before the head, a pool that does not directly
follow a conv, act/norm sequences like ``act norm`` — become **standalone units**
(``norm_pool.hip``): ``bn`` (materialised ``[norm] [act]``: stats -> finalize -> apply,
with its own backward) and ``pool`` (max pool + gather-form backward).  So every DSL the
reference accepts (construct_distribute.py:155-165, 208-265) lowers to HIP kernels.
"""
from __future__ import annotations

import ctypes as C
import ctypes as _ctypes   # (C is shadowed by channel counts in _alloc)
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..models.dsl import ActSpec, ConvSpec, DenseSpec, LayerPlan, NormSpec, PoolSpec
from ..ops import fused as K
from ..ops import fused as _FK      # (K is shadowed by feature counts inside _alloc)
from ..ops import optim_ref
from ..utils.streams import dedicated_stream


def _opt_call(lib, name: str, *args):
    """Call an entry point that an A/B baseline library (CSA_KERNEL_LIB, an older revision)
    may lack; the in-tree library has them all (ops.fused.load checks)."""
    try:
        fn = getattr(lib, name)
    except AttributeError:
        return None
    return fn(*args)


_NT_SET = [None]


def _set_nt_out(lib) -> None:
    """``CSA_NT_OUT=1``: the activations a launch writes for the next one (pair forward y,
    bn_act xt, head dh / dX, fc1's dX) go out as non-temporal stores (A/B knob; once per
    process and value)."""
    want = int(os.environ.get("CSA_NT_OUT", "0") == "1")
    if _NT_SET[0] == want:
        return
    for name in ("csa_nt_out_ew", "csa_nt_out_cp", "csa_nt_out_head", "csa_nt_out_du"):
        try:
            getattr(lib, name)(want)
        except AttributeError:          # an A/B baseline library without the knob
            pass
    _NT_SET[0] = want


class Unsupported(Exception):
    pass


def _act_id(sp: Optional[ActSpec]) -> int:
    if sp is None:
        return 0
    if sp.func == "leaky_relu" and sp.alpha == 0:
        return K.ACT_IDS["relu"]        # tf.maximum(x, 0 * x) IS relu
    return K.ACT_IDS[sp.func]


def _y_ok(sp: Optional[ActSpec]) -> bool:
    """Can this activation's backward be formed from its OUTPUT alone?  The kernels that
    fuse an activation into a producer's epilogue (conv / pair outputs, the row head's
    input) keep only y; ``maximum(x, a x)`` with a < 0 maps x > 0 and x < 0 both to y > 0,
    so such an activation is lowered where x is at hand instead: as a consumer transform
    (the dgrad epilogues read the pre-transform input) or a standalone act unit
    (construct_distribute.py:147-150 accepts any alpha)."""
    return sp is None or not (sp.func == "leaky_relu" and sp.alpha < 0)


def _alpha(sp: Optional[ActSpec]) -> float:
    return float(sp.alpha) if sp is not None else 0.0


@dataclass
class Transform:
    """Pending ``[norm] [act]`` applied by the consumer of a tensor."""
    norm: Optional[LayerPlan] = None
    act: Optional[ActSpec] = None
    slab: Optional[torch.Tensor] = None     # forward BN partial slab of the tensor
    nslab: int = 0
    count: float = 0.0
    bwd_slab: Optional[torch.Tensor] = None  # filled by the consumer's dgrad
    bwd_nslab: int = 0
    # deterministic mode: rows the producer writes (one per workgroup, folded to row 0 in
    # fixed order by csa_rows_fold; consumers then read nslab = 1)
    prod_rows: int = 0
    bwd_prod_rows: int = 0

    @property
    def has_bn(self) -> bool:
        return self.norm is not None


@dataclass
class Unit:
    kind: str                               # "conv" | "dense" | "gconv" | "bn" | "pool"
    layer: LayerPlan
    act: Optional[ActSpec] = None           # conv: fused output act
    pool: Optional[LayerPlan] = None        # conv: fused pool
    in_tf: Transform = field(default_factory=Transform)   # transform of this unit's INPUT
    x: Optional[torch.Tensor] = None        # input tensor (pre-transform), None = raw images
    y: Optional[torch.Tensor] = None        # output (post act/pool)
    argmax: Optional[torch.Tensor] = None
    dy: Optional[torch.Tensor] = None       # grad wrt output (or wrt the next BN output)
    dc: Optional[torch.Tensor] = None       # conv: grad wrt pre-act conv output
    splits_fwd: int = 1
    xt: Optional[torch.Tensor] = None       # dense: materialised act(bn(x)) (BN inputs)
    wg_stripes: int = 1                     # conv: weight-gradient accumulator stripes
    dw_acc: Optional[torch.Tensor] = None   # conv: [stripes][taps*Cout] (or the flat-grad view)
    db_acc: Optional[torch.Tensor] = None   # conv: [stripes][Cout] (or the flat-grad view)
    norm: Optional[LayerPlan] = None        # bn unit: the norm layer (None: activation only)


class HipProgram:
    WGRAD_STRIPES = int(os.environ.get("CSA_WGRAD_STRIPES", "16"))   # (A/B knob; <= 16: the tail's loads)

    def __init__(self, eng, forward_only: bool = False):
        """``forward_only``: the serving program (``serve.hip_infer``) — the same forward
        launches over another engine's weights, with no gradient, optimizer, staging or
        collective state (``eng`` then needs only cfg/device/model/flat/ctx/data/stream)."""
        self.e = eng
        self.forward_only = forward_only
        self.lib = K.load(required=True)
        _set_nt_out(self.lib)
        if eng.device.type != "cuda":
            raise Unsupported("HIP program needs a GPU device")
        # CSA_DETERMINISTIC=1: bitwise-reproducible steps on the same kernels (det.hip):
        # exclusive slab rows / weight-gradient stripes per workgroup, fixed-order folds,
        # no split-K.  The library flag is process state: set around every planning and
        # launch sequence of this program, restored afterwards.
        self.det = bool(getattr(eng, "deterministic", False)) and not forward_only
        # packed profile (engines built to run as branches of one multi-job graph): launch
        # shapes with less CU-time per step (conv_pair.hip, dense_update.hip)
        # (CSA_PACKED_PROFILE=0: packed engines keep the one-job launch shapes — A/B knob)
        self.packed = bool(getattr(eng, "packed", False)) and os.environ.get("CSA_PACKED_PROFILE", "1") == "1"
        # shared-GPU profile (several ranks of this job on ONE device): no 16-wave
        # workgroups (dense_update.hip du_cs; profiles/r5_notes.md, the world-2 stall)
        self.shared_gpu = bool(getattr(eng, "shared_gpu", False))
        with self._det_scope():
            self._init_plan(eng, forward_only)

    def _det_scope(self):
        prog = self

        class _Scope:
            def __enter__(self_):
                self_.prev = (int(prog.lib.csa_deterministic()), int(prog.lib.csa_packed()),
                              int(prog.lib.csa_shared_gpu()))
                prog.lib.csa_set_deterministic(1 if prog.det else 0)
                prog.lib.csa_set_packed(1 if prog.packed else 0)
                prog.lib.csa_set_shared_gpu(1 if prog.shared_gpu else 0)

            def __exit__(self_, *exc):
                prog.lib.csa_set_deterministic(self_.prev[0])
                prog.lib.csa_set_packed(self_.prev[1])
                prog.lib.csa_set_shared_gpu(self_.prev[2])
                return False
        return _Scope()

    def _init_plan(self, eng, forward_only: bool) -> None:
        self.B = eng.cfg.batch_size
        self.model = eng.model
        # SyncBN under DP: forward {sum, sumsq} slabs and backward {sum dz, sum dz*xhat}
        # slabs are all-reduced between their producer and consumer launches, counts
        # become global, and the BN parameter gradients (formed from the GLOBAL backward
        # sums) are scaled by 1/world before the gradient all-reduce adds them up again
        self.sync_bn = bool(eng.model.sync_bn)
        self.W = eng.ctx.world if self.sync_bn else 1
        self.views = eng.model.state.views(eng.flat)
        self.gviews = {} if forward_only else eng.model.state.views(eng.flat_grad)
        self._lower()
        self._plan_fused()
        self._plan_pair()
        self._plan_hfuse()
        if self.det:
            self._check_det()
        self._alloc()
        self._plan_splits()
        # the pair backward's per-band index tables, computed once (csa_conv_pair_bwd_tables)
        self.pair_tabs = None
        if self.pair is not None and not forward_only:
            n = int(self.lib.csa_conv_pair_bwd_tables_size(K.ints(self.pair)))
            if n > 0:
                self.pair_tabs = torch.zeros(n, dtype=torch.int32, device=eng.device)
                self._rc(self.lib.csa_conv_pair_bwd_tables(K.ints(self.pair), K.ptr(self.pair_tabs), K.stream()),
                         "conv_pair_bwd_tables")
        if forward_only:
            self.staged = False
            return
        self._plan_lowrank()
        self.zero_regions: List[torch.Tensor] = []
        self._collect_zero_regions()
        self._zero_now()
        self._plan_stage()
        self._plan_grad_buckets()
        self._plan_carry()
        self.opt_segments = self._opt_segments()
        self._plan_tail()
        self._plan_chain()

    def _plan_chain(self) -> None:
        """One-GPU program: fc1's forward, fc2's forward and the head launch run as ONE
        launch (``csa_chain_begin`` / ``csa_chain_end``: dense_direct.hip fwd_chain_kernel,
        stages handed over by tickets) instead of three — each launch boundary cost ~2-3 us
        between one launch's last workgroup and the next one's first (scripts/mb/
        graph_life.py, profiles/r6_notes.md).  MEASURED SLOWER, so opt-in (``CSA_FWD_CHAIN=1``):
        a stage hand-off inside the launch — the producer's atomics drained, its ticket RMW,
        the go flag, the consumer's poll and acquire — took 4.5-5.8 us, against ~2.4 us for
        the kernel boundary it replaces (0.0889 vs 0.0753 ms/step, profiles/r6_notes.md)."""
        e = self.e
        self.chain = False
        try:
            chain_ok = self.lib.csa_chain_ok
        except AttributeError:              # an A/B baseline library (CSA_KERNEL_LIB) without it
            return
        dense = [u for u in self.units if u.kind == "dense"]
        if (e.ctx.enabled or self.det or self.packed or self.forward_only
                or not getattr(self, "head_dgrad", False) or os.environ.get("CSA_FWD_CHAIN", "0") != "1"
                or len(dense) != 2 or self.units[-2:] != dense or not all(u.direct for u in dense)
                or getattr(self, "br_unit", None) is not None
                or not chain_ok(self.units[-1].layer.spec.hidden)):
            return
        # counts and spread go flags, each on its own line
        self.chain_tk = torch.zeros(int(self.lib.csa_chain_words()), dtype=torch.int32, device=e.device)
        self.chain_err = torch.zeros(1, dtype=torch.int32, device=e.device)
        self.chain = True

    # ------------------------------------------------------------------ DP deferred update
    def _plan_carry(self) -> None:
        """Data-parallel all-reduce programs: the dense layers' parameter update, which must
        follow the gradient exchange, runs as extra workgroups of the NEXT step's pair
        forward (conv_pair.hip ``CPOptCarry``) instead of in the flat optimizer launch after
        the exchange — those parameters are read again only by that step's dense forwards.
        The flat optimizer launch keeps the rest (conv, BatchNorm, head parameters and the
        side jobs) and raises a device flag; ``flush`` applies a pending update before any
        host read of the parameters (TrainEngine.flush_params).  Only gradients stored whole
        every step (keep ranges) are carried: the carry does not zero accumulators."""
        self.carry = None
        e = self.e
        if (not e.ctx.enabled or e.sync.strategy != "allreduce" or e.aps is not None or self.pair is None
                or os.environ.get("CSA_DP_CARRY", "1") != "1"
                or not self.lib.csa_conv_pair_valu_ok(K.ints(self.pair))):
            return
        offs = self.model.state.offsets
        keep = set(self.keep_ranges)
        n = self.e.flat.numel()
        spans = sorted(offs.values())
        ends = {o: (spans[i + 1] if i + 1 < len(spans) else n) for i, o in enumerate(spans)}
        carried, segs = set(), []
        for u in self.units:
            if u.kind != "dense" or (u.fused and self.fused) or u.lr_update:
                continue
            names = [f"{u.layer.name}.weight", f"{u.layer.name}.bias"]
            if not all((offs[nm], offs[nm] + (self.gviews[nm].numel() // 4) * 4) in keep for nm in names):
                continue
            for nm in names:
                carried.add(offs[nm])
        if not carried:
            return
        for o in spans:
            if o not in carried:
                continue
            lo, hi = o - o % 4, -(-ends[o] // 4) * 4
            if segs and segs[-1][1] >= lo:
                segs[-1][1] = max(segs[-1][1], hi)
            else:
                segs.append([lo, hi])
        if len(segs) > 4:
            return
        m4 = sum(hi - lo for lo, hi in segs) // 4
        self.carry = segs
        self.carry_offsets = carried
        self.carry_blocks = max(1, min(1024, -(-m4 // 256)))
        # the pending flag: set by the optimizer launch, read by the carrying forward, cleared
        # by the launch right after it (bn_act_apply, when the first dense layer takes the
        # pair's BatchNorm output; else only by a flush)
        self.carry_pending = torch.zeros(1, dtype=torch.int32, device=e.device)
        u2 = self.units[2] if len(self.units) > 2 else None
        self.carry_clear = bool(u2 is not None and u2.kind == "dense" and u2.xt is not None)

    def _carry_args(self):
        e = self.e
        s0 = e.slots[0] if e.slots.shape[0] > 0 else None
        s1 = e.slots[1] if e.slots.shape[0] > 1 else None
        lo = (C.c_long * 4)(*[x[0] for x in self.carry])
        hi = (C.c_long * 4)(*[x[1] for x in self.carry])
        return (e.opt_id, float(e.lr), K.ptr(e.dstep), K.ptr(e.flat), K.ptr(e.flat_grad), K.ptr(s0), K.ptr(s1),
                K.ptr(self.carry_pending), len(self.carry), lo, hi, self.carry_blocks)

    def flush(self, st=None) -> None:
        """Apply a pending deferred dense update now (stream-ordered; a no-op on the device
        when none is pending) and clear its flag."""
        if getattr(self, "carry", None) is None:
            return
        self._rc(self.lib.csa_opt_carry_flush(*self._carry_args(), st if st is not None else K.stream()),
                 "opt_carry_flush")

    # ------------------------------------------------------------------ DP overlap
    def _plan_grad_buckets(self) -> None:
        """Overlap the RCCL gradient all-reduce with the rest of the backward pass.

        The flat buffer holds layers in DSL order with the head last, and backward runs
        from the head down, so after unit k's backward every parameter of layer index
        >= unit k's main layer is final: a growing contiguous SUFFIX of ``flat_grad``.
        (A norm layer's scale/offset grads come from the route kernel of the conv unit
        BEFORE it, so they join the suffix one unit later — the rule still holds.)
        Each time the ready suffix has grown by >= ``min_bucket`` bytes it is all-reduced
        on a side stream (captured into the same HIP graph) while the main stream keeps
        computing conv gradients; the optimizer waits for the side stream.  With the
        sample config that is one ~1 MB bucket (head+fc2) launched after fc2, the 8 MB
        fc1 bucket launched right after fc1's weight gradient, and a small tail."""
        e = self.e
        # ps (the parameter-server capability): the same suffix buckets are REDUCE-SCATTERED
        # to their owner shards (GradSync.reduce_scatter_range; xGMI: one launch per bucket,
        # every element leaves its GPU at most once) while the backward continues — only
        # when EVERY bucket's range reduce-scatter measured faster on the xGMI kernel than
        # on RCCL (GradSync.rs_choice, decided below): on RCCL the per-owner reduces per
        # bucket measured 0.156 ms/step at world 1 against 0.107 for one reduce-scatter
        # after the backward (profiles/r4_notes.md)
        # (the ":hf" program forms every dense gradient inside the pair backward launch:
        # nothing is ready early, one exchange after the backward)
        self.overlap = (e.ctx.enabled and e.sync.strategy in ("allreduce", "ps")
                        and (e.sync.strategy == "allreduce" or e.sync.xgmi is not None)
                        and not getattr(self, "dp_hf", False)
                        and os.environ.get("CSA_DP_OVERLAP", "1") == "1")
        self.bucket_at: Dict[object, tuple] = {}
        if not self.overlap:
            return
        self.side = dedicated_stream(e.device)      # (captured: outside torch's stream pool)
        offs = e.model.state.offsets
        end = e.flat.numel()

        def frontier(layer_index: int) -> int:
            c = [o for n, o in offs.items()
                 if n.startswith("head.") or int(n.split(".")[1]) >= layer_index]
            return min(c) if c else end

        min_elems = int(os.environ.get("CSA_DP_MIN_BUCKET", str(512 << 10))) // 4
        hi = end
        points = [("head", frontier(10 ** 9))] + [(k, frontier(self.units[k].layer.index))
                                                  for k in range(len(self.units) - 1, -1, -1)]
        for i, (key, f) in enumerate(points):
            last = i == len(points) - 1
            lo = 0 if last else f
            if hi - lo >= min_elems or (last and hi > lo):
                self.bucket_at[key] = (lo, hi)
                hi = lo
        if e.sync.strategy == "ps":
            # every bucket's path decided now (collectively, timed under CSA_XGMI=auto)
            paths = [e.sync.rs_choice(e.flat_grad, e.grad_shard, lo, hi) for lo, hi in self.bucket_at.values()]
            if any(ch is None for ch in paths):
                self.overlap, self.bucket_at = False, {}
                return

    # ------------------------------------------------------------------ DP "lowrank"
    def _plan_lowrank(self) -> None:
        """Exact data parallelism for the dense layers without all-reducing their weights.

        A dense weight gradient is ``Σ_ranks T(x_r)ᵀ·dy_r`` — a GEMM whose reduction
        dimension is the per-rank batch (50).  So instead of an RCCL all-reduce of the
        [in, out] gradient (8 MB for fc1 of the sample config; ring collectives over xGMI
        are per-link bound), every rank all-gathers the [B, in] GEMM inputs and the
        [B, out] output gradients (0.9 MB for fc1) and forms the global gradient locally
        with K = world·B on a side stream that overlaps the conv backward.  The 1/world
        mean is already folded into the loss-gradient seed.  Only the small remainder
        (conv, BatchNorm, head: ~25 KB for the sample config) is all-reduced.  A dense
        layer whose input goes through a BatchNorm that is not materialised per rank
        (batch statistics differ between ranks) stays on the all-reduce path."""
        e = self.e
        self.lr_units: List[Unit] = []
        self.lr_ranges: List[tuple] = []
        if not (e.ctx.enabled and e.sync.strategy == "lowrank"):
            return
        W, B, dev = e.ctx.world, self.B, e.device
        offs = self.model.state.offsets
        taken = []
        for u in self.units:
            if u.kind != "dense" or (u.in_tf.has_bn and u.xt is None):
                continue
            fin, fout = u.layer.in_shape.numel, u.layer.spec.hidden
            u.lr_src = u.xt if u.xt is not None else u.x.view(B, fin)
            u.lr_act = (0, 0.0) if u.xt is not None else (_act_id(u.in_tf.act), _alpha(u.in_tf.act))
            u.lr_x = torch.zeros(W * B, fin, device=dev)
            u.lr_dy = torch.zeros(W * B, fout, device=dev)
            # every rank forms the SAME global dW, so the optimizer update of W / b runs
            # inside that weight-gradient launch (csa_dd_wgrad update mode: dW never exists)
            # where the variables live — as ApplyAdagrad on the PS did
            # (construct_distribute.py:355-357, 372-373)
            u.lr_update = True
            for p in ("weight", "bias"):
                n = f"{u.layer.name}.{p}"
                taken.append((offs[n], offs[n] + self.gviews[n].numel()))
            self.lr_units.append(u)
        # everything else is all-reduced: the other parameters' spans, merged across
        # alignment padding (with the dense-last flat layout that is ONE leading range)
        lr_spans = set(taken)
        spans = sorted((o, o + self.gviews[n].numel()) for n, o in offs.items())
        open_range = False
        for a, b in spans:
            if (a, b) in lr_spans:
                open_range = False
            elif open_range:
                self.lr_ranges[-1] = (self.lr_ranges[-1][0], b)
            else:
                self.lr_ranges.append((a, b))
                open_range = True
        # each range's end rounded up to 16 bytes through the alignment padding behind it
        # (never-written zeros): the xGMI kernels take 16-byte multiples only, and a range
        # left on RCCL would be the one collective of this program inside the graph that the
        # peer-buffer path does not carry
        starts = sorted(a for a, _ in spans) + [e.flat.numel()]
        self.lr_ranges = [(a, min(-(-b // 4) * 4, min(x for x in starts if x >= b))) for a, b in self.lr_ranges]
        if self.lr_units:
            self.lr_side = dedicated_stream(dev)
            self.lr_first = min(self.units.index(u) for u in self.lr_units)

    def _lowrank_gather_inputs(self) -> None:
        """After the forward pass: all-gather the dense GEMM inputs on the side stream
        (overlaps the head and the dense input-gradient GEMMs)."""
        if not self.lr_units:
            return
        self.lr_side.wait_stream(torch.cuda.current_stream(self.e.device))
        with torch.cuda.stream(self.lr_side):
            self.e.sync.all_gather_rows_many([(u.lr_src, u.lr_x) for u in self.lr_units], tag="lr_x")

    def _lowrank_wgrads(self) -> None:
        """Once every lowrank unit's output gradient is final: gather them and form the
        global weight gradients (K = world·B) on the side stream."""
        lib, W, B, G = self.lib, self.e.ctx.world, self.B, self.gviews
        self.lr_side.wait_stream(torch.cuda.current_stream(self.e.device))
        with torch.cuda.stream(self.lr_side):
            ss = self.lr_side.cuda_stream
            self.e.sync.all_gather_rows_many([(u.dy.view(B, -1), u.lr_dy) for u in self.lr_units], tag="lr_dy")
            for u in self.lr_units:
                lp = u.layer
                fin, fout = lp.in_shape.numel, lp.spec.hidden
                if u.lr_update:
                    self._dd_wgrad_update(u, u.lr_x, u.lr_dy, W * B, u.lr_act, ss)
                    continue
                self._rc(lib.csa_dense_wgrad(
                    K.ptr(u.lr_x), K.ptr(u.lr_dy), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]),
                    W * B, fin, fout, None, 0, 0, 0.0, 0.0, None, None, u.lr_act[0], u.lr_act[1], 1.0, ss),
                    "dense_wgrad(lowrank)")

    def _grad_ready(self, key) -> None:
        b = self.bucket_at.get(key)
        if b is None:
            return
        cur = torch.cuda.current_stream(self.e.device)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            if self.e.sync.strategy == "ps":
                self.e.sync.reduce_scatter_range(self.e.flat_grad, self.e.grad_shard, b[0], b[1])
            else:
                self.e.sync.allreduce(self.e.flat_grad, b[0], b[1])


    # ------------------------------------------------------------------ fused updates
    def _plan_fused(self) -> None:
        """On one GPU the dense weight gradients feed nothing but the optimizer: such a
        layer's backward becomes ``csa_dense_bwd_update`` (dgrad + wgrad + the optimizer
        update of its W rows in one launch, dense_update.hip) and the head writes
        per-row-group partial gradients + metrics that the (now small) optimizer launch
        folds (``csa_head_part``).  Data parallel (all-reduce / ps) runs the SAME fused
        launch in gradient mode (``csa_dense_bwd_grad_head``): the dense weight / bias
        gradients are stored whole into the flat gradient for the all-reduce and the flat
        optimizer updates them (``fused_grad``); lowrank forms them from gathered operands."""
        e, B = self.e, self.B
        on = os.environ.get("CSA_FUSED_UPDATE", "1") == "1" and not self.forward_only
        self.fused = on and not e.ctx.enabled
        self.fused_grad = on and e.ctx.enabled and e.sync.strategy in ("allreduce", "ps", "async_ps")
        # measured on MI355X (profiles/r2_dense_fused.md): the row-group kernel (one
        # 1024-thread workgroup per 16 input features) replaces fc1's split-K pair + its
        # share of the flat optimizer (bench 0.1166 -> 0.1107 ms/step); CSA_FUSED_DENSE=0
        # restores the separate kernels
        fuse_dense = (self.fused or self.fused_grad) and os.environ.get("CSA_FUSED_DENSE", "1") == "1"
        for u in self.units:
            u.fused = False
            if not fuse_dense or u.kind != "dense":
                continue
            tf = u.in_tf
            fin, fout = u.layer.in_shape.numel, u.layer.spec.hidden
            if tf.has_bn and fin % 4:            # the BN'd input is not materialised (see _alloc)
                continue
            if tf.act is not None and not tf.has_bn:
                continue                         # weight-gradient operand would need the act
            C = tf.norm.in_shape.c if tf.has_bn else 0
            # (a narrow layer's row groups are split over 128-column blocks with a partial
            # hand-off, so fc2's 32 row groups still use 128 CUs: profiles/r2_dense_fused.md)
            groups = (fin + 15) // 16
            u.fused = bool(self.lib.csa_dense_bwd_update_ok(B, fin, fout, C)) and groups >= 1
        # the flat optimizer launch updates at most 16 spans between the fused layers' own
        # parameters: beyond 15 fused layers the rest take the materialised-gradient path
        nf = 0
        for u in self.units:
            if getattr(u, "fused", False):
                nf += 1
                u.fused = nf <= 15
        self.head_rg = 0
        self.head_row = False
        self.head_sep = False
        last = self.units[-1]
        if (not self.fused and not self.forward_only and self.head_tf.norm is None
                and not (self.fused_grad and last.kind == "dense" and last.fused)):
            # data parallel without a fused last dense layer (lowrank, or the unfused
            # program): the row-per-workgroup head, its weight gradient as a register-direct
            # wgrad launch (dWh = act(h)^T dlogits) into the flat gradient before the
            # all-reduce, its metrics folded by the optimizer launch (the atomic
            # 4-workgroup head took 15.6 us per DP step)
            if last.kind == "dense" and self.lib.csa_head_row_ok(B, last.layer.spec.hidden):
                self.head_row = self.head_sep = True
        if (self.fused or self.fused_grad) and self.head_tf.norm is None and not self.head_sep:
            last = self.units[-1]
            K = last.layer.spec.hidden if last.kind == "dense" else last.layer.out_shape.numel
            if last.kind == "conv" and last.pool is not None:
                K = last.pool.out_shape.numel
            # one batch row per workgroup; the head's batch reductions (dWh, dbh, metrics)
            # ride in the last dense layer's fused backward (csa_head_row + the head epilogue
            # of csa_dense_bwd_update_head) — no partial rows for the optimizer to fold
            self.head_row = last.kind == "dense" and last.fused and bool(self.lib.csa_head_row_ok(B, K))
            if not self.head_row and self.fused:
                self.head_rg = int(self.lib.csa_head_part_rows(B, K))
        # register-direct MFMA dense forward (dense_direct.hip); the backward of a dense layer
        # is the fused backward + update (one GPU), the LDS-staged dgrad + wgrad pair (data
        # parallel: the gradient is all-reduced), or under lowrank the gathered-operand
        # weight gradient with the update in-kernel (profiles/r2_dense_direct.md measured
        # the register-direct backward slower than the paired kernels)
        for u in self.units:
            u.direct = u.lr_update = False
            if u.kind != "dense":
                continue
            fin = u.layer.in_shape.numel
            if u.in_tf.has_bn and fin % 4:
                continue                         # BN'd input not materialised: LDS-staged GEMM
            u.direct = True

    # ------------------------------------------------------------------ conv pair
    def _plan_pair(self) -> None:
        """``conv [act] conv [act] [pool]`` on the raw images (the sample's conv1 -> conv2
        -> pool) runs as ONE forward and ONE backward launch (conv_pair.hip): c1 stays in
        LDS, the backward recomputes it and never writes dc2 / dc1."""
        self.pair = None
        if len(self.units) < 2:
            return
        ua, ub = self.units[0], self.units[1]
        if ua.kind != "conv" or ub.kind != "conv" or ua.pool is not None:
            return
        if ub.in_tf.norm is not None or ub.in_tf.act is not None:
            return
        la, lb = ua.layer, ub.layer
        if tuple(la.spec.stride) != (1, 1) or tuple(lb.spec.stride) != (1, 1):
            return
        pool = 0
        if ub.pool is not None:
            ps = ub.pool.spec
            if tuple(ps.kernel) != (2, 2) or tuple(ps.stride) != (2, 2) or ub.pool.pads[0] or ub.pool.pads[2]:
                return
            pool = 1
        h, w = la.in_shape.hw
        h1, w1 = la.out_shape.hw
        h2, w2 = lb.out_shape.hw
        ph, pw = ub.pool.out_shape.hw if pool else (h2, w2)
        geom = [self.B, h, w, la.in_shape.c, la.spec.kh, la.spec.kw, la.pads[0], la.pads[2], la.spec.cout,
                h1, w1, lb.spec.kh, lb.spec.kw, lb.pads[0], lb.pads[2], lb.spec.cout, h2, w2, pool, ph, pw]
        if not self.lib.csa_conv_pair_ok(K.ints(geom)):
            return
        if not (_y_ok(ua.act) and _y_ok(ub.act)):
            return
        if self.det and not self.lib.csa_conv_pair_valu_ok(K.ints(geom)):
            return                       # deterministic mode: two conv units instead
        self.pair = geom

    # ------------------------------------------------------------------ horizontal fusion
    def _plan_hfuse(self) -> None:
        """One-GPU fused program with a conv pair: split every fused dense backward into its
        input gradient (``csa_dense_bwd_dgrad``, on the step's critical path) and its weight
        gradient + optimizer update, which is DEFERRED (``csa_dense_update_defer``) and runs
        as extra workgroups of the pair backward launch (conv_pair.hip,
        ``conv_pair_bwd_upd_kernel``).  The update only has to land before the next step's
        forward of its layer; inside the pair backward — a latency chain at 3 % of HBM and
        8 % of MFMA (profiles/r3_roofline.md) — it uses idle CUs instead of adding 10-15 us
        of serial work per dense layer.  The head's batch reductions ride in the last dense
        layer's deferred segment exactly as they rode in its fused backward."""
        self.hfuse = False
        self.head_dgrad = False
        # Packed profile too (round 6): with the round-6 carrier (5 workgroups per CU, the
        # tail program) K = 4 / 8 packs measured 1.295 / 1.313 M samples/s with the deferred
        # updates against 1.249 / 1.264 M without (scripts/archive/gpu_r6q.sh, profiles/
        # r6_multitenant.md; rounds 4-5 measured the opposite with the older carriers).
        # CSA_PACKED_HFUSE=0 restores the packed profile without it.
        # data parallel ("<strategy>:hf"): the same split in GRADIENT mode — the deferred
        # segments store dW / db whole into the flat gradient, the pair backward's tail folds
        # the conv stripes into it, then the exchange and the flat optimizer follow
        self.dp_hf = bool(self.fused_grad and getattr(self.e, "dp_variant", "") == "hf"
                          and self.e.sync.strategy in ("allreduce", "ps", "async_ps"))
        packed_ok = os.environ.get("CSA_PACKED_HFUSE", "1") == "1"
        if (self.forward_only or not (self.fused or self.dp_hf) or self.det or self.pair is None
                or (self.packed and not packed_ok) or os.environ.get("CSA_HFUSE", "1") != "1"):
            self.dp_hf = False
            return
        dense = [u for u in self.units if u.kind == "dense" and u.fused]
        if not dense or len(dense) > 4 or any(u.layer.spec.hidden % 128 for u in dense):
            self.dp_hf = False
            return
        self.hfuse = True
        # the last dense layer's input gradient rides in the head launch (csa_head_dgrad:
        # every workgroup recomputes the head for its rows, no batch reduction), when that
        # layer's input transform is at most an activation
        last = self.units[-1]
        self.head_dgrad = bool(
            self.head_row and last.kind == "dense" and last.fused and len(self.units) > 2
            and not last.in_tf.has_bn
            and self.lib.csa_head_dgrad_ok(self.B, last.layer.spec.hidden, last.layer.in_shape.numel))
        # CSA_DENSE_BRANCH=1: the FIRST dense layer's deferred update (fc1: 980 of the
        # carrying launch's ~1 700 workgroups) runs as its own launch on a side stream — a
        # graph branch from after its input-gradient launch to before the next step's
        # BatchNorm apply that rewrites its operand — instead of inside the pair backward
        self.br_unit = None
        self._br_pending = False
        # (its weight-gradient operand must be the materialised BatchNorm output, which only
        # the next step's bn_act_apply rewrites: _alloc's xt)
        d0 = dense[0]
        if (not self.dp_hf and os.environ.get("CSA_DENSE_BRANCH", "0") == "1" and d0.in_tf.has_bn
                and d0.layer.in_shape.numel % 4 == 0 and d0 is not self.units[-1]):
            self.br_unit = d0
            self.br_side = dedicated_stream(self.e.device)

    def join_branch(self) -> None:
        """Join a pending dense-update branch into the current stream (a capture ends with
        every forked stream joined; the next step's BatchNorm apply needs it done)."""
        if getattr(self, "_br_pending", False):
            torch.cuda.current_stream(self.e.device).wait_stream(self.br_side)
            self._br_pending = False

    # ------------------------------------------------------------------ pair-backward tail
    def _plan_tail(self) -> None:
        """Round 5: the one-GPU fused program without an optimizer launch.

        After horizontal fusion the flat optimizer launch only updated the conv pair's
        (striped) and the BatchNorm's parameters, zeroed the next step's accumulators and
        staged the next batch — 8.1 us of a ~88 us step (profiles/r4_step_trace.md).  Now:

        * the conv / BN updates, the statistic-slab zeroing and the batch staging run as
          TAIL workgroups of the pair backward launch (``csa_conv_pair_tail_set``), which
          wait (bounded) for the pair workgroups — done ~7 us before that launch's dense
          update workgroups;
        * the head's parameters are updated in place by the last dense segment's head
          epilogue (``csa_dense_update_head_params``), which also writes the metric ring;
        * the dense forwards' split-K outputs, read until the end of the pair backward, are
          zeroed by the NEXT step's pair forward threads (its zero list).

        Applies to the horizontal-fusion program with the staged batch and the row head
        when every other parameter and accumulator is one of those (``CSA_PAIR_TAIL=0``
        restores the optimizer launch)."""
        self.tail = False
        self.tail_update = False
        self.fwd_zero: List[torch.Tensor] = []
        if getattr(self, "dp_hf", False):
            self._plan_tail_fold()
            return
        if not (getattr(self, "hfuse", False) and getattr(self, "staged", False) and self.head_row
                and self.pair is not None and os.environ.get("CSA_PAIR_TAIL", "1") == "1"):
            return
        e = self.e
        ua, ub = self.units[0], self.units[1]
        if not (ua.wg_stripes > 1 and ub.wg_stripes == ua.wg_stripes and not getattr(ua, "row_fold", False)
                and ua.wg_stripes <= 16):
            return
        nt = self.units[2].in_tf if len(self.units) > 2 else self.head_tf
        offs = self.model.state.offsets
        fused = {f"{u.layer.name}.{p}" for u in self.units if u.kind == "dense" and u.fused for p in ("weight", "bias")}
        params = []           # (name, src tensor, S, ld, zero)
        for u, acc, nm in ((ua, ua.dw_acc, "weight"), (ua, ua.db_acc, "bias"), (ub, ub.dw_acc, "weight"),
                           (ub, ub.db_acc, "bias")):
            if acc is not None:
                params.append((f"{u.layer.name}.{nm}", acc, u.wg_stripes, acc.shape[1], 1))
        if nt.has_bn:
            for pn in ("scale", "offset"):
                n = f"{nt.norm.name}.{pn}"
                params.append((n, self.gviews[n], 1, self.gviews[n].numel(), 0))
        rest = set(offs) - fused - {p[0] for p in params} - {"head.weight", "head.bias"}
        if rest or len(params) > 8:
            return                      # parameters the tail does not know about
        # zero regions: the BN statistic slabs (read by every pair workgroup) in the tail,
        # the dense split-K outputs at the next pair forward; anything else: no tail
        slabs = []
        for u in self.units:
            if u.in_tf.has_bn:
                slabs += [u.in_tf.slab.view(-1), u.in_tf.bwd_slab.view(-1)]
        ys = [u.y.view(-1) for u in self.units if u.kind == "dense" and u.splits_fwd > 1]
        regions = self.zero_regions + self.zero_early
        ptrs = {t.data_ptr() for t in slabs} | {t.data_ptr() for t in ys}
        if any(r.data_ptr() not in ptrs for r in regions) or len(slabs) > 4 or len(ys) > 4:
            return
        if any(t.numel() % 4 or t.data_ptr() % 16 for t in ys):
            return
        sl = e.slots
        s0 = sl[0] if sl.shape[0] > 0 else None
        s1 = sl[1] if sl.shape[0] > 1 else None

        def slot(s, name):
            return None if s is None else s[offs[name]:]

        self.tail_params = [(self.views[n], slot(s0, n), slot(s1, n), src, S, ld, self.views[n].numel(), z)
                            for n, src, S, ld, z in params]
        self.tail_zero = [t for t in slabs if any(r.data_ptr() == t.data_ptr() for r in regions)]
        self.fwd_zero = [t for t in ys if any(r.data_ptr() == t.data_ptr() for r in regions)]
        self.head_params = (self.views["head.weight"], self.views["head.bias"], slot(s0, "head.weight"),
                            slot(s1, "head.weight"), slot(s0, "head.bias"), slot(s1, "head.bias"))
        self.tail_tk = torch.zeros(int(self.lib.csa_conv_pair_tail_ticket_words()), dtype=torch.int32,
                                   device=e.device)                           # spread tickets
        # the tickets are zeroed by the NEXT step's pair forward (no closing reset counter in
        # the carrier's tail: conv_pair.hip cp_tail_body)
        self.fwd_zero.append(self.tail_tk)
        self.tail_err = torch.zeros(1, dtype=torch.int32, device=e.device)
        self.tail_force = torch.zeros(1, dtype=torch.int32, device=e.device)   # debug: arm_tail_timeout
        # the parameter workgroups' table (one entry per 256 elements of a parameter)
        tp = self.tail_params
        n = len(tp)
        P = C.c_void_p
        ns = (C.c_int * 8)(*[t[6] for t in tp])
        nbytes = int(self.lib.csa_conv_pair_tail_table_bytes(ns, n))
        self.tail_table = torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=e.device)
        torch.cuda.synchronize(e.device)
        self.tail_blocks = int(self.lib.csa_conv_pair_tail_plan(
            K.ptr(self.tail_table), e.opt_id, n, (P * 8)(*[t[0].data_ptr() for t in tp]),
            (P * 8)(*[K.ptr(t[1]) for t in tp]), (P * 8)(*[K.ptr(t[2]) for t in tp]),
            (P * 8)(*[t[3].data_ptr() for t in tp]), (C.c_int * 8)(*[t[4] for t in tp]),
            (C.c_int * 8)(*[t[5] for t in tp]), ns, (C.c_int * 8)(*[t[7] for t in tp]), 0))
        if self.tail_blocks < 1:
            raise RuntimeError(f"conv_pair_tail_plan failed: {self.tail_blocks}")
        self.tail = self.tail_update = True

    def _plan_tail_fold(self) -> None:
        """The ":hf" data-parallel program's tail: fold the pair's weight-gradient stripes
        into the flat gradient (stored sums, no update) before the exchange — the optimizer
        launch after the exchange keeps the updates, zeroing and staging."""
        e = self.e
        ua, ub = self.units[0], self.units[1]
        if not (getattr(ua, "tail_fold", False) and ua.wg_stripes > 1 and ua.wg_stripes <= 16):
            raise Unsupported("data-parallel :hf program: the pair stripes need the tail fold")
        G = self.gviews
        jobs = []
        for u in (ua, ub):
            lp = u.layer
            jobs.append((G[f"{lp.name}.weight"].view(-1), u.dw_acc, u.wg_stripes, u.dw_acc.shape[1]))
            if u.db_acc is not None:
                jobs.append((G[f"{lp.name}.bias"].view(-1), u.db_acc, u.wg_stripes, u.db_acc.shape[1]))
        self.tail_tk = torch.zeros(int(self.lib.csa_conv_pair_tail_ticket_words()), dtype=torch.int32,
                                   device=e.device)
        self.fwd_zero = [self.tail_tk]            # (zeroed by the next step's pair forward)
        self.tail_err = torch.zeros(1, dtype=torch.int32, device=e.device)
        self.tail_force = torch.zeros(1, dtype=torch.int32, device=e.device)   # debug: arm_tail_timeout
        P = C.c_void_p
        n = len(jobs)
        ns = (C.c_int * 8)(*[j[0].numel() for j in jobs])
        nbytes = int(self.lib.csa_conv_pair_tail_table_bytes(ns, n))
        self.tail_table = torch.zeros((nbytes + 15) // 16 * 4, dtype=torch.float32, device=e.device)
        torch.cuda.synchronize(e.device)
        self.tail_blocks = int(self.lib.csa_conv_pair_tail_plan(
            K.ptr(self.tail_table), 0, n, (P * 8)(*[j[0].data_ptr() for j in jobs]), (P * 8)(), (P * 8)(),
            (P * 8)(*[j[1].data_ptr() for j in jobs]), (C.c_int * 8)(*[j[2] for j in jobs]),
            (C.c_int * 8)(*[j[3] for j in jobs]), ns, (C.c_int * 8)(*([1] * n)), 1))
        if self.tail_blocks < 1:
            raise RuntimeError(f"conv_pair_tail_plan failed: {self.tail_blocks}")
        self.tail_zero = []
        self.tail = True

    def _tail_set(self) -> None:
        """Record the tail of this step's pair backward launch (host state, like the
        deferred dense segments) and switch the head segment to in-place updates."""
        e, lib = self.e, self.lib
        P = C.c_void_p
        _opt_call(lib, "csa_conv_pair_tail_force", K.ptr(self.tail_force))
        if not self.tail_update:           # the ":hf" data-parallel fold: nothing else
            self._rc(lib.csa_conv_pair_tail_set(
                K.ptr(self.tail_tk), K.ptr(self.tail_err), 0, 0.0, K.ptr(e.dstep), K.ptr(self.tail_table),
                self.tail_blocks, 0, (P * 4)(), (C.c_long * 4)(), None, None, None, None, 0, 0, None, None),
                "conv_pair_tail_set")
            return
        hw, hb, hs0w, hs1w, hs0b, hs1b = self.head_params
        self._rc(lib.csa_dense_update_head_params(K.ptr(hw), K.ptr(hb), K.ptr(hs0w), K.ptr(hs1w), K.ptr(hs0b),
                                                  K.ptr(hs1b)), "dense_update_head_params")
        rc = lib.csa_conv_pair_tail_set(
            K.ptr(self.tail_tk), K.ptr(self.tail_err), e.opt_id, float(e.lr), K.ptr(e.dstep),
            K.ptr(self.tail_table), self.tail_blocks,
            len(self.tail_zero), (P * 4)(*[t.data_ptr() for t in self.tail_zero]),
            (C.c_long * 4)(*[t.numel() for t in self.tail_zero]),
            K.ptr(e.data.images), K.ptr(e.data.labels), K.ptr(e.stream.rows), K.ptr(e.stream.cursor), self.B,
            self.stage_img.shape[1], K.ptr(self.stage_img), K.ptr(self.stage_lbl))
        self._rc(rc, "conv_pair_tail_set")

    def tail_error(self) -> int:
        """Nonzero when a tail workgroup's bounded wait timed out (its work did not run).

        STICKY by design: a timed-out tail skipped parameter updates, the statistic-slab
        zeroing and the next batch's staging, so the engine's state is no longer a valid
        training state — nothing resets the word; the job fails (``TrainEngine.check_health``)
        and restarts from its last checkpoint in a fresh engine."""
        return int(self.tail_err.item()) if getattr(self, "tail", False) else 0

    def health_words(self):
        """Device int32 words that are nonzero once an in-kernel bounded wait timed out
        (read without a host sync by the job loop's metric drain): the pair-backward tail's
        and the forward chain's."""
        words = [self.tail_err] if getattr(self, "tail", False) else []
        if getattr(self, "chain", False):
            words.append(self.chain_err)
        return words

    def arm_tail_timeout(self) -> bool:
        """Debug / fault injection: the NEXT pair-backward launch's tail waits
        for one ticket more than exists, times out after its 1 s bound and sets the error
        word, as a starved or hung pair workgroup would.  Stream-ordered (a fill before the
        launch); the launch's closing tail disarms it.  False when this program has no tail."""
        if not getattr(self, "tail", False):
            return False
        self.tail_force.fill_(1)
        return True

    # ------------------------------------------------------------------ deterministic mode
    def _check_det(self) -> None:
        """Deterministic mode covers every one-GPU lowering and allreduce / ps data
        parallelism: the VALU conv pair and the conv units (fixed-order in-workgroup folds;
        one exclusive statistic row and weight-gradient stripe per workgroup, folded in row
        order by csa_rows_fold), standalone BatchNorm units (exclusive statistic rows summed
        in row order by the finalize kernels), gather-form pools (overlapping pools are never
        fused), gconv units (implicit GEMM without split-K), fused dense backward + update
        units (exclusive BN-backward rows, fixed-order column-block hand-off), materialised-
        gradient dense units and dense forwards (no split-K; a BatchNorm'd input's backward
        statistics go to one exclusive slab row per GEMM workgroup, folded in (wave, lane)
        order: gemm.hip), and the row-per-workgroup, partial-row or single-workgroup generic
        heads (head.hip csa_head picks the generic kernel: fixed-order sums, plain stores).
        Only async_ps data parallelism stays outside (pushes applied in arrival order)."""
        e = self.e
        # data parallel: every collective of the step is fixed-order (GradSync.det: the xGMI
        # kernels or an exact all-gather + rank-ordered fold), the stripes are exclusive rows
        # folded in order before the exchange, the dense layers run the fused backward in
        # gradient mode (exclusive BN-backward rows)
        if e.ctx.enabled and e.sync.strategy not in ("allreduce", "ps"):
            # (async_ps applies pushes in arrival order: nondeterministic by definition)
            raise Unsupported(f"deterministic mode: {e.sync.strategy} data parallelism")

    def _row_fold(self, t: torch.Tensor, rows: int, width: int, dst: torch.Tensor, zero_src: int, st) -> None:
        """dst[:width] = fixed-order sum of the first ``rows`` rows of ``t`` (row stride width)."""
        self._rc(self.lib.csa_rows_fold(K.ptr(t), width, rows, width, K.ptr(dst), zero_src, st), "rows_fold")

    # ------------------------------------------------------------------ lowering
    def _lower(self) -> None:
        layers = self.e.model.plan.layers
        units: List[Unit] = []
        pending: List[LayerPlan] = []            # norm / act layers since the last unit

        def as_transform(consumer: str) -> Optional[Transform]:
            """``pending`` as a transform the consumer applies while loading, or None."""
            tf = Transform()
            for lp in pending:
                if isinstance(lp.spec, NormSpec):
                    if tf.norm is not None or tf.act is not None:
                        return None              # norm after norm / act
                    tf.norm = lp
                else:
                    if tf.act is not None:
                        return None              # two activations in a row
                    tf.act = lp.spec
            if consumer == "head" and not _y_ok(tf.act):
                return None                      # the row head's backward reads y only
            if tf.norm is not None:
                # the forward statistics come from a conv unit's epilogue, the tables live
                # in LDS (<= 128 channels), and the head has no BN-apply prologue
                if (consumer == "head" or not units or units[-1].kind != "conv"
                        or not tf.norm.in_shape.is_spatial or tf.norm.in_shape.c > 128):
                    return None
            return tf

        def materialise() -> None:
            """``pending`` as standalone units: [norm][act] groups and lone activations."""
            i = 0
            while i < len(pending):
                lp = pending[i]
                if isinstance(lp.spec, NormSpec):
                    nxt = pending[i + 1] if i + 1 < len(pending) else None
                    act = nxt.spec if nxt is not None and isinstance(nxt.spec, ActSpec) else None
                    units.append(Unit("bn", lp, act=act, norm=lp))
                    i += 2 if act is not None else 1
                else:
                    units.append(Unit("bn", lp, act=lp.spec))
                    i += 1
            pending.clear()

        i = 0
        while i < len(layers):
            lp = layers[i]
            sp = lp.spec
            if isinstance(sp, ConvSpec) and (lp.in_shape.c > 128 or sp.cout > 128):
                # wide conv: implicit-GEMM unit on a materialised input; the act / pool /
                # norm after it become standalone units
                materialise()
                units.append(Unit("gconv", lp))
                i += 1
                continue
            if isinstance(sp, (ConvSpec, DenseSpec)):
                kind = "conv" if isinstance(sp, ConvSpec) else "dense"
                tf = as_transform(kind)
                if tf is None:
                    materialise()
                    tf = Transform()
                pending.clear()
                u = Unit(kind, lp, in_tf=tf)
                j = i + 1
                if kind == "conv":
                    if j < len(layers) and isinstance(layers[j].spec, ActSpec) and _y_ok(layers[j].spec):
                        u.act = layers[j].spec
                        j += 1
                    if (j < len(layers) and isinstance(layers[j].spec, PoolSpec)
                            and not (self.det and tuple(layers[j].spec.kernel) != tuple(layers[j].spec.stride))):
                        # (deterministic mode: an overlapping pool's routing adds windows into
                        # dc with atomics — it stays a standalone gather-form pool unit)
                        u.pool = layers[j]
                        j += 1
                units.append(u)
                i = j
            elif isinstance(sp, PoolSpec):
                materialise()                    # pool(act(norm(x))): the transform first
                units.append(Unit("pool", lp))
                i += 1
            elif isinstance(sp, (NormSpec, ActSpec)):
                if isinstance(sp, ActSpec):
                    _act_id(sp)
                pending.append(lp)
                i += 1
            else:  # pragma: no cover
                raise Unsupported(str(sp))
        tf = as_transform("head")
        if tf is None:
            materialise()
            tf = Transform()
        if not units:
            raise Unsupported("no conv/dense layers")
        self.units = units
        self.head_tf = tf

    @staticmethod
    def _bn_channels(u: Unit) -> int:
        """Channel count of a bn unit: C of an NHWC tensor, the features of a 2-D one."""
        sh = u.layer.in_shape
        return sh.c if sh.is_spatial else sh.numel

    # ------------------------------------------------------------------ buffers
    def _alloc(self) -> None:
        dev, B = self.e.device, self.B
        f32 = dict(device=dev, dtype=torch.float32)
        fo = self.forward_only
        prev: Optional[Unit] = None
        for u in self.units:
            u.x = prev.y if prev is not None else None
            if prev is None and u.kind != "conv":
                # first unit reads no raw images: materialise the gathered float input once
                # per step (NHWC [B, 28, 28, 1] for a bn / pool unit)
                self.x_dense_in = torch.zeros(B, u.layer.in_shape.numel, **f32)
                ish = u.layer.in_shape
                u.x = (self.x_dense_in if u.kind == "dense" or not ish.is_spatial
                       else self.x_dense_in.view(B, ish.hw[0], ish.hw[1], ish.c))
            lp = u.layer
            if u.kind == "bn":
                u.y = torch.zeros_like(u.x)
                C_ = self._bn_channels(u)
                if u.norm is not None:
                    R = self.lib.csa_bn_stat_rows(u.x.numel() // C_)
                    u.bn_tab = torch.zeros(4, C_, **f32)
                    u.bn_slab = torch.zeros(R, 2, C_, **f32)
                    if not fo:
                        u.bn_bslab = torch.zeros(R, 2, C_, **f32)
                        u.bn_k = torch.zeros(2, C_, **f32)
            elif u.kind == "pool":
                ph, pw = lp.out_shape.hw
                u.y = torch.zeros(B, ph, pw, lp.out_shape.c, **f32)
                u.argmax = torch.zeros(B, ph, pw, lp.out_shape.c, device=dev, dtype=torch.uint8)
            elif u.kind == "gconv":
                oh, ow = lp.out_shape.hw
                u.y = torch.zeros(B, oh, ow, lp.spec.cout, **f32)
            elif u.kind == "conv":
                oh, ow = lp.out_shape.hw
                if u.pool is not None:
                    ph, pw = u.pool.out_shape.hw
                    u.y = torch.zeros(B, ph, pw, lp.out_shape.c, **f32)
                    u.argmax = torch.zeros(B, ph, pw, lp.out_shape.c, device=dev, dtype=torch.uint8)
                else:
                    u.y = torch.zeros(B, oh, ow, lp.out_shape.c, **f32)
                u.dc = None if fo else torch.zeros(B, oh, ow, lp.out_shape.c, **f32)
            else:
                u.y = torch.zeros(B, lp.spec.hidden, **f32)
            u.dy = None if fo else torch.zeros_like(u.y)
            # forward BN slab for the transform consuming this unit's output
            prev = u
        # forward stat slabs: the unit BEFORE a transform with norm produces the slab
        for k, u in enumerate(self.units):
            tf = u.in_tf
            if tf.has_bn:
                src = self.units[k - 1]
                ph, pw = src.y.shape[1], src.y.shape[2]
                # (deterministic mode: one row per producer workgroup, folded to row 0)
                if self.det and self.pair is not None and k == 2:
                    nslab = int(self.lib.csa_conv_pair_grid(_FK.ints(self.pair)))
                else:
                    nslab = self.lib.csa_conv_fwd_nslab(self._conv_geom(src.layer, B), self._pool_geom(src))
                tf.prod_rows = nslab
                tf.slab = torch.zeros(nslab, 2, src.y.shape[3], **f32)
                tf.nslab = 1 if self.det else nslab
                tf.count = float(B * ph * pw * self.W)
                if fo:
                    continue
                # backward slab is produced by THIS unit's dgrad
                C = src.y.shape[3]
                if u.kind == "dense" and u.fused:
                    nb = self.lib.csa_dense_bwd_update_slabs(u.layer.in_shape.numel)
                elif u.kind == "dense":
                    nb = self.lib.csa_dense_dgrad_slabs(B, u.layer.in_shape.numel, u.layer.spec.hidden)
                else:
                    nb = self.lib.csa_conv_dgrad_nslab(self._conv_geom(u.layer, B))
                tf.bwd_slab = torch.zeros(nb, 2, C, **f32)
                tf.bwd_nslab = nb
                if self.det:            # one row per row group (csa_dense_bwd_update_slabs)
                    tf.bwd_prod_rows, tf.bwd_nslab = nb, 1
        # dense consumers of a BatchNorm'd tensor get it materialised once per step
        for u in self.units:
            u.xt = None
            if u.kind == "dense" and u.in_tf.has_bn and u.layer.in_shape.numel % 4 == 0:
                u.xt = torch.zeros(B, u.layer.in_shape.numel, **f32)
            # BatchNorm tables [mean | rstd | a | b][C] written once per step by the
            # bn_act_apply that materialises xt (the fused dense backward's epilogue reads
            # them instead of reducing the statistic slab again)
            if u.kind == "dense" and u.fused and not fo:
                # partial input-gradient slabs + per-row-group arrival tickets when the
                # kernel splits a row group over column blocks (the last arriver resets
                # its ticket; zero-initialised here)
                ws = (_ctypes.c_longlong * 2)()
                self.lib.csa_dense_bwd_update_ws(u.layer.in_shape.numel, u.layer.spec.hidden, ws)
                u.du_part = torch.zeros(max(int(ws[0]), 1), **f32)
                u.du_cnt = torch.zeros(max(int(ws[1]), 1), dtype=torch.int32, device=dev)
            u.in_tf.bn_tab = torch.zeros(4, u.in_tf.slab.shape[2], **f32) if u.xt is not None else None
        self.dlast = self.units[-1].dy     # head input grad (None: forward only)
        if getattr(self, "head_row", False):
            self.hdl = torch.zeros(B, 10, **f32)                            # dlogits rows
            self.hrl = torch.zeros(B, **f32)                                # per-row loss
            self.hrc = torch.zeros(B, dtype=torch.int32, device=dev)        # per-row correct
        self.idx = None
        if self.head_rg:
            K = self.dlast[0].numel()
            G = -(-B // self.head_rg)
            # per-group dWh | dbh, rows padded to float4 (the optimizer's fold then reads
            # whole float4s: an odd row stride sent every head float4 down the per-element
            # path, 4 dependent round trips, 7 us of the 8.6 us launch)
            self.head_part = torch.zeros(G, (K * 10 + 10 + 3) // 4 * 4, **f32)
            self.head_kw = K * 10
            self.head_mloss = torch.zeros(G, **f32)
            self.head_mcorr = torch.zeros(G, dtype=torch.int32, device=dev)

    def _plan_splits(self) -> None:
        """Split-K factor of each dense forward (> 1: its output is an atomic accumulator
        that must start at zero)."""
        B = self.B
        for u in self.units:
            if u.kind == "dense":
                fin, fout = u.layer.in_shape.numel, u.layer.spec.hidden
                u.splits_fwd = (self.lib.csa_dd_fwd_splits(B, fout, fin) if u.direct
                                else self.lib.csa_dense_fwd_splits(B, fout, fin))
            elif u.kind == "gconv":
                u.splits_fwd = self.lib.csa_gconv_fwd_splits(self._conv_geom(u.layer, B))

    def _collect_zero_regions(self) -> None:
        """Accumulators that must start every step at zero.  ``zero_regions`` are cleared
        by the optimizer's zero-list pass; flat-gradient accumulators are cleared by the
        update itself (each thread zeroes the gradient it read — a separate pass over the
        same memory would race with the reads), except under the sharded "ps" strategy,
        where the update reads the reduce-scattered shard and the flat ranges go to the
        zero list; conv weight-gradient stripes are cleared by the fold that reads them."""
        B = self.B
        regs: List[torch.Tensor] = []
        flat: List[torch.Tensor] = []
        self.stripe_bufs: List[torch.Tensor] = []
        fold_budget = 8 - (2 if self.head_rg else 0)
        for k, u in enumerate(self.units):
            lp = u.layer
            if u.kind == "dense":
                fin, fout = lp.in_shape.numel, lp.spec.hidden
                if u.splits_fwd > 1:
                    regs.append(u.y)
                if u.fused:
                    continue                     # plain stores; W never has a gradient buffer
                if k > 0:
                    tfm = u.in_tf.has_bn or u.in_tf.act is not None
                    if self.lib.csa_dense_dgrad_splits(B, fin, fout, int(tfm)) > 1:
                        regs.append(self.units[k - 1].dy)
                if self.lib.csa_dense_wgrad_splits(B, fin, fout) > 1:
                    flat.append(self.gviews[f"{lp.name}.weight"].view(-1))
                    flat.append(self.gviews[f"{lp.name}.bias"])
            elif u.kind == "gconv":
                geom = self._conv_geom(lp, B)
                if u.splits_fwd > 1:
                    regs.append(u.y.view(-1))
                if k > 0 and self.lib.csa_gconv_dgrad_splits(geom) > 1:
                    regs.append(self.units[k - 1].dy.view(-1))
                if self.lib.csa_gconv_wgrad_splits(geom, int(bool(lp.spec.bias))) > 1:
                    flat.append(self.gviews[f"{lp.name}.weight"].view(-1))
                    if lp.spec.bias:
                        flat.append(self.gviews[f"{lp.name}.bias"])
            elif u.kind == "bn":
                if u.norm is not None:        # atomic stat rows (forward and backward)
                    regs += [u.bn_slab.view(-1), u.bn_bslab.view(-1)]
            elif u.kind == "conv":
                # conv weight gradients: S stripes on one GPU (folded by the optimizer:
                # at most 8 folds, the head's partials included), otherwise accumulated
                # straight into the flat gradient (data parallelism, or beyond that budget)
                nf = 1 + (1 if lp.spec.bias else 0)
                S = 1 if self.e.ctx.enabled or fold_budget < nf else self.WGRAD_STRIPES
                # the conv pair's stripes are folded right after the pair backward (fixed-order
                # csa_rows_fold into the flat gradient) in deterministic mode — one stripe per
                # workgroup — and under data parallelism, where the gradient must be complete
                # before its all-reduce (700 workgroups adding into ONE copy contend: the pair
                # backward took 37 us instead of 25)
                # — and every conv unit's in deterministic mode (one stripe per wgrad workgroup)
                in_pair = self.pair is not None and k < 2
                # (":hf": the pair backward's tail folds the stripes into the flat gradient)
                u.tail_fold = in_pair and getattr(self, "dp_hf", False)
                u.row_fold = self.det or (in_pair and self.e.ctx.enabled and not u.tail_fold)
                if u.tail_fold:
                    S = self.WGRAD_STRIPES
                if u.row_fold:
                    if not self.det:
                        S = self.WGRAD_STRIPES
                    elif in_pair:
                        S = int(self.lib.csa_conv_pair_grid(_FK.ints(self.pair)))
                    else:
                        S = int(self.lib.csa_conv_wgrad_blocks(self._conv_geom(lp, B), int(bool(lp.spec.bias))))
                        if S <= 0:
                            raise Unsupported(f"conv unit {lp.name}: no weight-gradient plan")
                elif S > 1:
                    fold_budget -= nf
                u.wg_stripes = S
                nw = self.gviews[f"{lp.name}.weight"].numel()
                if S > 1:       # zeroed by the fold that reads them (their only reader)
                    u.dw_acc = torch.zeros(S, nw, device=self.e.device)
                    u.db_acc = torch.zeros(S, lp.spec.cout, device=self.e.device) if lp.spec.bias else None
                    self.stripe_bufs += [t for t in (u.dw_acc, u.db_acc) if t is not None]
                else:
                    u.dw_acc = self.gviews[f"{lp.name}.weight"]
                    u.db_acc = self.gviews[f"{lp.name}.bias"] if lp.spec.bias else None
                    flat.append(u.dw_acc.view(-1))
                    if lp.spec.bias:
                        flat.append(u.db_acc.view(-1))
                if u.pool is not None:
                    pk, ps = u.pool.spec.kernel, u.pool.spec.stride
                    if tuple(pk) != tuple(ps):
                        regs.append(u.dc.view(-1))
        # the atomic head accumulates dWh/dbh across its row-group workgroups (the
        # partial-output head of the fused program writes per-group rows instead)
        if not self.head_rg:
            flat.append(self.e.flat_grad[self.e.model.state.offsets["head.weight"]:])
        self.head_ws = torch.zeros(4, dtype=torch.int32, device=self.e.device)   # arrival counter + sums
        for u in self.units:
            if u.in_tf.has_bn:
                regs.append(u.in_tf.slab.view(-1))          # forward stats (atomic rows)
                regs.append(u.in_tf.bwd_slab.view(-1))      # every producer folds rows atomically
        # dense weight gradients produced without split-K are STORED whole every step (by the
        # fused dense backward, the separate wgrad or the lowrank wgrad), so the optimizer
        # skips re-zeroing them (keep ranges, float4-aligned: the flat layout aligns to 64)
        self.keep_ranges = []
        offs = self.model.state.offsets
        for u in self.units:
            if u.kind != "dense" or (u.fused and self.fused) or u.lr_update:
                continue                         # (updated in-kernel: no gradient in memory)
            fin, fout = u.layer.in_shape.numel, u.layer.spec.hidden
            m = B * (self.e.ctx.world if u in getattr(self, "lr_units", []) else 1)
            # the fused backward in gradient mode stores dW / db whole every step
            if (u.fused and self.fused_grad) or self.lib.csa_dense_wgrad_splits(m, fin, fout) == 1:
                for p in ("weight", "bias"):
                    n = f"{u.layer.name}.{p}"
                    lo = offs[n]
                    self.keep_ranges.append((lo, lo + (self.gviews[n].numel() // 4) * 4))
        if getattr(self, "head_row", False):
            for n in ("head.weight", "head.bias"):
                lo = offs[n]
                if self.gviews[n].numel() >= 4:
                    self.keep_ranges.append((lo, lo + (self.gviews[n].numel() // 4) * 4))
        # sharded parameters (ps, async_ps): the update reads a shard, the flat gradient is
        # zeroed through the zero list after the exchange consumed it
        self.ps_mode = self.e.sync.sharded
        regions = regs + (flat if self.ps_mode else [])
        # the optimizer's zero list holds 16; any further accumulators are cleared at the
        # start of the step instead (one fill launch each, inside the same graph)
        self.zero_regions, self.zero_early = regions[:16], regions[16:]

    def _zero_now(self) -> None:
        for r in self.zero_regions + self.zero_early + self.stripe_bufs:
            r.zero_()
        self.e.flat_grad.zero_()
        if getattr(self, "tail", False):
            self.tail_tk.zero_()            # (an aborted launch must not leave tickets behind)

    # ------------------------------------------------------------------ batch staging
    def _plan_stage(self) -> None:
        """Stage each step's batch at fixed addresses (one-GPU fused program).  The head
        advances the stream cursor and the optimizer's trailing workgroups copy the NEXT
        step's images and labels (rows[cursor]) into ``stage_img`` / ``stage_lbl``, so the
        conv pair and head kernels start with one memory round trip instead of the
        cursor -> row index -> image chain.  ``prime()`` fills them for the current cursor
        whenever the host moved it (construction, warm-up restore, seek).

        Default on (``CSA_STAGE_BATCH=0`` turns it off): 3 alternating bench pairs on
        MI355X, 0.1169 vs 0.1175 ms/step (scripts/ab_env.sh) — small, because the conv
        pair's start-up phase is mostly bound by 700 workgroups reading the same weights
        at once, but consistent."""
        e = self.e
        img = e.data.images
        imsz = img[0].numel() if img.dim() > 1 else 0
        self.staged = (self.pair is not None and bool(self.head_rg or self.head_row) and img.dtype == torch.uint8
                       and imsz % 4 == 0 and os.environ.get("CSA_STAGE_BATCH", "1") == "1")
        self.stage_img = self.stage_lbl = None
        if self.staged:
            self.stage_img = torch.zeros(self.B, imsz, dtype=torch.uint8, device=e.device)
            self.stage_lbl = torch.zeros(self.B, dtype=torch.int64, device=e.device)
            self.prime()

    def prime(self) -> None:
        if not getattr(self, "staged", False):
            return
        e = self.e
        self._rc(self.lib.csa_gather_batch(
            K.ptr(e.data.images), K.ptr(e.data.labels), K.ptr(e.stream.rows), K.ptr(e.stream.cursor), self.B,
            self.stage_img.shape[1], K.ptr(self.stage_img), K.ptr(self.stage_lbl), K.stream()), "gather_batch")

    def _batch_src(self):
        """(images, rows, cursor) for a kernel reading this step's batch: the staged batch
        (rows = cursor = None) or the dataset through the device cursor."""
        e = self.e
        if getattr(self, "staged", False) and not getattr(self, "_predicting", False):
            return self.stage_img, None, None
        return e.data.images, e.stream.rows, e.stream.cursor

    def reset_after_warmup(self) -> None:
        self._zero_now()
        if getattr(self, "carry", None) is not None:
            self.carry_pending.zero_()      # the restored parameters have no pending update
        self.prime()

    # ------------------------------------------------------------------ helpers
    @staticmethod
    def _conv_geom(lp: LayerPlan, B: int):
        sp = lp.spec
        h, w = lp.in_shape.hw
        oh, ow = lp.out_shape.hw
        return K.ints([B, h, w, lp.in_shape.c, sp.kh, sp.kw, sp.stride[0], sp.stride[1],
                       lp.pads[0], lp.pads[2], oh, ow, sp.cout])

    @staticmethod
    def _pool_geom(u: Unit):
        if u.pool is None:
            return K.ints([0] * 9)
        lp = u.pool
        sp = lp.spec
        oh, ow = lp.out_shape.hw
        return K.ints([1, sp.kernel[0], sp.kernel[1], sp.stride[0], sp.stride[1],
                       lp.pads[0], lp.pads[2], oh, ow])

    def _bn_args(self, tf: Transform):
        if not tf.has_bn:
            return (None, 0, 0.0, 0.0, None, None)
        name = tf.norm.name
        if self._eval_bn:
            return (K.ptr(tf.eval_slab), 1, 1.0, float(tf.norm.spec.epsilon),
                    K.ptr(self.views[f"{name}.scale"]), K.ptr(self.views[f"{name}.offset"]))
        return (K.ptr(tf.slab), tf.nslab, tf.count, float(tf.norm.spec.epsilon),
                K.ptr(self.views[f"{name}.scale"]), K.ptr(self.views[f"{name}.offset"]))

    def _bn_args_c(self, tf: Transform):
        """BN args with the channel count (dense launchers: channel = feature % C)."""
        a = self._bn_args(tf)
        C_ = tf.slab.shape[2] if tf.has_bn else 0
        return (a[0], a[1], C_, a[2], a[3], a[4], a[5])

    def _rc(self, rc: int, what: str) -> int:
        if rc < 0 or (rc > 0 and not what.startswith("slabs:")):
            raise RuntimeError(f"{what} failed: {rc}")
        return rc

    # ------------------------------------------------------------------ the step
    def run(self) -> None:
        with self._det_scope():
            self._run()

    def _run(self) -> None:
        e, lib, B = self.e, self.lib, self.B
        st = K.stream()
        # this step's dataset rows = stream.rows[cursor]; the kernels resolve the cursor on
        # device and the optimizer launch advances it (no torch index/add launches).
        rows, cur = e.stream.rows, e.stream.cursor
        img = e.data.images
        V, G = self.views, self.gviews
        for r in self.zero_early:
            r.zero_()
        if getattr(self, "hfuse", False):
            lib.csa_dense_update_clear()        # no stale segment from an aborted step
        chain = getattr(self, "chain", False)
        if chain:
            lib.csa_chain_begin()               # the two dense forwards + the head: recorded
        try:
            self._forward(st)
        except BaseException:
            if chain:
                lib.csa_chain_reset()
            raise

        self._lowrank_gather_inputs()

        # ---------------- head (loss, head grads, input grad, metrics) ----------------
        last = self.units[-1]
        hin = last.y.view(B, -1)
        if getattr(self, "head_dgrad", False):
            staged = getattr(self, "staged", False)
            ltf = last.in_tf
            rc_hd = (lib.csa_head_dgrad(
                K.ptr(hin), B, hin.shape[1], _act_id(self.head_tf.act), _alpha(self.head_tf.act),
                K.ptr(V["head.weight"]), K.ptr(V["head.bias"]),
                K.ptr(self.stage_lbl if staged else e.data.labels), None if staged else K.ptr(rows),
                None if staged else K.ptr(cur), 0 if e.cfg.loss_name == "entropy" else 1, float(e.sync.grad_scale),
                K.ptr(last.dy), K.ptr(self.hdl), K.ptr(self.hrl), K.ptr(self.hrc), K.ptr(e.dstep),
                K.ptr(cur) if staged else None, e.stream.wrap if staged else 0,
                K.ptr(V[f"{last.layer.name}.weight"]), last.layer.in_shape.numel, K.ptr(last.x.view(B, -1)),
                _act_id(ltf.act), _alpha(ltf.act), K.ptr(self.units[-2].dy), st))
            if chain:                           # fc1 forward | fc2 forward | head: one launch
                rc = lib.csa_chain_end(K.ptr(self.chain_tk), K.ptr(self.chain_err), st) if rc_hd >= 0 else 0
                if rc_hd < 0:
                    lib.csa_chain_reset()
                self._rc(rc, "fwd_chain")
            self._rc(rc_hd, "head_dgrad")
        elif self.head_row:
            staged = getattr(self, "staged", False)
            self._rc(lib.csa_head_row(
                K.ptr(hin), B, hin.shape[1], _act_id(self.head_tf.act), _alpha(self.head_tf.act),
                K.ptr(V["head.weight"]), K.ptr(V["head.bias"]),
                K.ptr(self.stage_lbl if staged else e.data.labels), None if staged else K.ptr(rows),
                None if staged else K.ptr(cur), 0 if e.cfg.loss_name == "entropy" else 1, float(e.sync.grad_scale),
                K.ptr(last.dy), K.ptr(self.hdl), K.ptr(self.hrl), K.ptr(self.hrc), K.ptr(e.dstep),
                K.ptr(cur) if staged else None, e.stream.wrap if staged else 0, st), "head_row")
            if self.head_sep:
                # dWh = act(h)^T dlogits, dbh = colsum(dlogits) into the flat gradient
                self._rc(lib.csa_dd_wgrad(
                    K.ptr(hin), K.ptr(self.hdl), B, hin.shape[1], 10, _act_id(self.head_tf.act),
                    _alpha(self.head_tf.act), 1.0, K.ptr(G["head.weight"]), K.ptr(G["head.bias"]),
                    None, None, None, None, None, None, -1, 0.0, None, st), "dd_wgrad(head)")
        elif self.head_rg:
            staged = getattr(self, "staged", False)
            self._rc(lib.csa_head_part2(
                K.ptr(hin), B, hin.shape[1], _act_id(self.head_tf.act), _alpha(self.head_tf.act),
                K.ptr(V["head.weight"]), K.ptr(V["head.bias"]),
                K.ptr(self.stage_lbl if staged else e.data.labels), None if staged else K.ptr(rows),
                None if staged else K.ptr(cur),
                0 if e.cfg.loss_name == "entropy" else 1, float(e.sync.grad_scale), K.ptr(last.dy),
                K.ptr(self.head_part), K.ptr(self.head_mloss), K.ptr(self.head_mcorr), None, K.ptr(e.dstep),
                K.ptr(cur) if staged else None, e.stream.wrap if staged else 0, st),
                "head_part")
        else:
            self._rc(lib.csa_head(
                K.ptr(hin), B, hin.shape[1], _act_id(self.head_tf.act), _alpha(self.head_tf.act),
                K.ptr(V["head.weight"]), K.ptr(V["head.bias"]), K.ptr(e.data.labels), K.ptr(rows),
                0 if e.cfg.loss_name == "entropy" else 1, float(e.sync.grad_scale),
                K.ptr(G["head.weight"]), K.ptr(G["head.bias"]), K.ptr(last.dy), None,
                K.ptr(e.dstep), K.ptr(e.ring_loss), K.ptr(e.ring_correct), e.ring_correct.numel(),
                K.ptr(cur), K.ptr(self.head_ws), st), "head")
        self._grad_ready("head")

        # ---------------- backward ----------------
        for k in range(len(self.units) - 1, -1, -1):
            u = self.units[k]
            if self.pair is not None and k < 2:
                if k == 1:
                    self._pair_bwd(st)
                    self._grad_ready(1)
                else:
                    self._grad_ready(0)
                continue
            if u.kind in ("bn", "pool"):
                self._standalone_bwd(u, self.units[k - 1] if k > 0 else None, st)
                self._grad_ready(k)
                continue
            if u.kind == "gconv":
                self._gconv_bwd(u, self.units[k - 1] if k > 0 else None, st)
                self._grad_ready(k)
                continue
            lp, tf = u.layer, u.in_tf
            bn = self._bn_args(tf)
            in_act, in_alpha = _act_id(tf.act), _alpha(tf.act)
            prev = self.units[k - 1] if k > 0 else None
            if self.sync_bn and k + 1 < len(self.units) and self.units[k + 1].in_tf.has_bn:
                # unit k+1's dgrad produced its input transform's backward slab; this
                # unit's route consumes it: make it the global sum first
                e.sync.allreduce_tensors([self.units[k + 1].in_tf.bwd_slab], tag=f"bnb{k + 1}")
            if u.kind == "dense":
                fin, fout = lp.in_shape.numel, lp.spec.hidden
                if u.fused:
                    self._dense_bwd_update(u, prev, st)
                    if self.fused_grad:
                        self._grad_ready(k)
                    continue
                if (prev is not None and u not in self.lr_units
                        and self._dense_bwd_fused(u, prev, st)):
                    self._grad_ready(k)          # dgrad + wgrad in one launch
                    continue
                if prev is not None:
                    xf = u.x.view(B, -1)
                    self._rc(lib.csa_dense_dgrad(
                        K.ptr(u.dy), K.ptr(V[f"{lp.name}.weight"]), K.ptr(prev.dy), B, fin, fout,
                        K.ptr(xf), in_act, in_alpha, *self._bn_args_c(tf), K.ptr(tf.bwd_slab), st),
                        "slabs:dense_dgrad")
                    self._dense_det_fold(u, st)
                if u in self.lr_units:          # global wgrad formed after the gathers
                    if k == self.lr_first:
                        self._lowrank_wgrads()
                    self._grad_ready(k)
                    continue
                ws = st
                if u.xt is not None:
                    self._rc(lib.csa_dense_wgrad(
                        K.ptr(u.xt), K.ptr(u.dy), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]),
                        B, fin, fout, None, 0, 0, 0.0, 0.0, None, None, 0, 0.0, 1.0, ws), "dense_wgrad")
                else:
                    self._rc(lib.csa_dense_wgrad(
                        K.ptr(u.x), K.ptr(u.dy), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]),
                        B, fin, fout, *self._bn_args_c(tf), in_act, in_alpha, 1.0, ws), "dense_wgrad")
            else:
                # output side: (BN backward of the NEXT transform) + act backward + pool routing
                next_tf = self.units[k + 1].in_tf if k + 1 < len(self.units) else self.head_tf
                need_route = next_tf.has_bn or u.act is not None or u.pool is not None
                if need_route:
                    oh, ow = lp.out_shape.hw
                    g = [B, u.y.shape[1], u.y.shape[2], u.y.shape[3], oh, ow,
                         1 if u.pool is not None else 0]
                    if u.pool is not None:
                        ps = u.pool.spec
                        g += [ps.kernel[0], ps.kernel[1], ps.stride[0], ps.stride[1],
                              u.pool.pads[0], u.pool.pads[2]]
                    else:
                        g += [1, 1, 1, 1, 0, 0]
                    nbn = self._bn_args(next_tf)
                    dsc = G[f"{next_tf.norm.name}.scale"] if next_tf.has_bn else None
                    dof = G[f"{next_tf.norm.name}.offset"] if next_tf.has_bn else None
                    rm = rv = None
                    if next_tf.has_bn:
                        rm = getattr(self.model, f"bn{next_tf.norm.index}_mean")
                        rv = getattr(self.model, f"bn{next_tf.norm.index}_var")
                    self._rc(lib.csa_route_bwd(
                        K.ptr(u.dy), K.ptr(u.y), K.ptr(u.argmax), K.ptr(u.dc), K.ints(g),
                        _act_id(u.act), _alpha(u.act), *nbn, K.ptr(next_tf.bwd_slab), next_tf.bwd_nslab,
                        K.ptr(dsc), K.ptr(dof), K.ptr(rm), K.ptr(rv), float(self.model.bn_momentum), st),
                        "route_bwd")
                    self._sync_bn_param_grads(next_tf)
                    dc = u.dc
                else:
                    dc = u.dy
                geom = self._conv_geom(lp, B)
                raw = u.x is None
                sp = lp.spec
                h, w = lp.in_shape.hw
                oh, ow = lp.out_shape.hw
                if prev is not None:
                    # input gradient + weight gradient in one launch
                    self._rc(lib.csa_conv_bwd(
                        K.ptr(dc), K.ptr(V[f"{lp.name}.weight"]), K.ptr(prev.dy), geom,
                        K.ptr(u.x), in_act, in_alpha, *bn, K.ptr(tf.bwd_slab),
                        K.ptr(u.dw_acc), K.ptr(u.db_acc) if sp.bias else None, u.wg_stripes, st), "conv_bwd")
                    self._conv_det_folds(u, tf, st)
                    self._grad_ready(k)
                    continue
                ws = st
                self._rc(lib.csa_conv_wgrad(
                    None if raw else K.ptr(u.x), K.ptr(img) if raw else None, K.ptr(rows) if raw else None,
                    K.ptr(dc), K.ptr(u.dw_acc), K.ptr(u.db_acc) if sp.bias else None, u.wg_stripes,
                    B, h, w, lp.in_shape.c, sp.kh, sp.kw, sp.stride[0], sp.stride[1], lp.pads[0], lp.pads[2],
                    oh, ow, sp.cout, bn[0], bn[1], bn[2], bn[3], bn[4], bn[5], in_act, in_alpha,
                    K.ptr(cur) if raw else None, ws), "conv_wgrad")
                if prev is not None:
                    self._rc(lib.csa_conv_dgrad(
                        K.ptr(dc), K.ptr(V[f"{lp.name}.weight"]), K.ptr(prev.dy), geom,
                        K.ptr(u.x), in_act, in_alpha, *bn, K.ptr(tf.bwd_slab), st), "conv_dgrad")
                self._conv_det_folds(u, tf, st)
            self._grad_ready(k)

        # ---------------- gradient sync + optimizer ----------------
        main = torch.cuda.current_stream(e.device)
        if e.aps is not None:
            # async_ps: push / apply-on-arrival / publish / pull in one launch; the optimizer
            # launch below keeps only its side jobs (zeroing, metrics, batch staging)
            e.aps.step(e.flat_grad, e.flat, e.slots)
            self._optimizer(st)
            return
        if self.overlap:
            main.wait_stream(self.side)
        elif e.ctx.enabled and e.sync.strategy == "lowrank":
            e.sync.allreduce_ranges(e.flat_grad, self.lr_ranges, tag="lr_rem")
            if self.lr_units:
                main.wait_stream(self.lr_side)
        else:
            e.after_backward_sync()
        if getattr(self, "tail", False):
            if lib.csa_dense_update_pending() or lib.csa_conv_pair_tail_pending():
                raise RuntimeError("pair-backward tail / deferred updates not consumed")
            if self.tail_update:
                return                      # the pair backward's tail did the optimizer's work
        self._optimizer(st)

    # ------------------------------------------------------------------ forward
    _eval_bn = False          # predict: BN with running statistics (no batch-stat slabs)

    def _forward(self, st) -> None:
        """Every unit's forward launch (the first half of ``run``; ``predict`` reuses it)."""
        e, lib, B = self.e, self.lib, self.B
        rows, cur = e.stream.rows, e.stream.cursor
        if self.__dict__.get("x_dense_in") is not None:
            D = self.x_dense_in.shape[1]
            if e.data.images.dtype == torch.uint8 and D % 4 == 0:
                self._rc(lib.csa_gather_images_f32(K.ptr(e.data.images), K.ptr(rows), K.ptr(cur), B, D,
                                                   K.ptr(self.x_dense_in), st), "gather_images_f32")
            else:
                idx = rows.index_select(0, cur).view(-1)
                self.x_dense_in.copy_(e.data.images.index_select(0, idx).to(torch.float32).mul_(1.0 / 255.0))
        img = e.data.images
        V = self.views
        # ---------------- forward ----------------
        if self.pair is not None:
            ua, ub = self.units[0], self.units[1]
            nt = self.units[2].in_tf if len(self.units) > 2 else self.head_tf
            oslab = nt.slab if nt.has_bn and not self._eval_bn else None
            simg, srows, scur = self._batch_src()
            # (the tail program: the dense split-K outputs of this step, zeroed by the pair
            # forward's threads — not when predicting, which zeroes them itself)
            fz = [] if getattr(self, "_predicting", False) else getattr(self, "fwd_zero", [])
            carrying = getattr(self, "carry", None) is not None and not getattr(self, "_predicting", False)
            if carrying:
                self._rc(lib.csa_conv_pair_fwd_carry(*self._carry_args()), "conv_pair_fwd_carry")
            self._rc(lib.csa_conv_pair_fwd(
                K.ints(self.pair), K.ptr(simg), K.ptr(srows), K.ptr(scur),
                K.ptr(V[f"{ua.layer.name}.weight"]), K.ptr(V.get(f"{ua.layer.name}.bias")) if ua.layer.spec.bias else None,
                _act_id(ua.act), _alpha(ua.act),
                K.ptr(V[f"{ub.layer.name}.weight"]), K.ptr(V.get(f"{ub.layer.name}.bias")) if ub.layer.spec.bias else None,
                _act_id(ub.act), _alpha(ub.act), K.ptr(ub.y), K.ptr(ub.argmax), K.ptr(oslab),
                nt.prod_rows if self.det else self.lib.csa_conv_fwd_nslab(None, None),
                (C.c_void_p * 4)(*[t.data_ptr() for t in fz]), (C.c_long * 4)(*[t.numel() for t in fz]), len(fz),
                st), "conv_pair_fwd")
            if carrying and self.carry_clear:
                _opt_call(lib, "csa_ew_clear_next", K.ptr(self.carry_pending))   # (next: bn_act_apply)
            if oslab is not None and self.det:
                self._row_fold(oslab, nt.prod_rows, oslab.shape[1] * oslab.shape[2], oslab, 0, st)
            if oslab is not None and self.sync_bn:
                e.sync.allreduce_tensors([oslab], tag="bnf1")
        for k, u in enumerate(self.units):
            if self.pair is not None and k < 2:
                continue
            if u.kind in ("bn", "pool"):
                self._standalone_fwd(u, st)
                continue
            if u.kind == "gconv":
                self._gconv_fwd(u, st)
                continue
            lp, tf = u.layer, u.in_tf
            bn = self._bn_args(tf)
            in_act, in_alpha = _act_id(tf.act), _alpha(tf.act)
            next_tf = self.units[k + 1].in_tf if k + 1 < len(self.units) else self.head_tf
            if u.kind == "conv":
                oslab = next_tf.slab if next_tf.has_bn and not self._eval_bn else None
                raw = u.x is None
                self._rc(lib.csa_conv_fwd(
                    None if raw else K.ptr(u.x), K.ptr(img) if raw else None, K.ptr(rows) if raw else None,
                    K.ptr(V[f"{lp.name}.weight"]), K.ptr(V.get(f"{lp.name}.bias")) if lp.spec.bias else None,
                    K.ptr(u.y), K.ptr(u.argmax), K.ptr(oslab),
                    self._conv_geom(lp, B), self._pool_geom(u), *bn, in_act, in_alpha,
                    _act_id(u.act), _alpha(u.act), K.ptr(cur) if raw else None, st), "conv_fwd")
                if oslab is not None and self.det:        # exclusive rows -> row 0, in order
                    self._row_fold(oslab, next_tf.prod_rows, oslab.shape[1] * oslab.shape[2], oslab, 0, st)
                if oslab is not None and self.sync_bn:
                    e.sync.allreduce_tensors([oslab], tag=f"bnf{k}")
            else:
                fin, fout = lp.in_shape.numel, lp.spec.hidden
                if u is getattr(self, "br_unit", None):
                    self.join_branch()          # the previous step's update read u.xt and W
                if u.xt is not None:
                    self._rc(lib.csa_bn_act_apply(
                        K.ptr(u.x), K.ptr(u.xt), B * fin, tf.slab.shape[2], *bn, in_act, in_alpha,
                        K.ptr(getattr(tf, "bn_tab", None)), st),
                        "bn_act_apply")
                if u.direct:
                    xin = u.xt if u.xt is not None else u.x.view(B, -1)
                    act = (0, 0.0) if u.xt is not None else (in_act, in_alpha)
                    self._rc(lib.csa_dd_fwd(
                        K.ptr(xin), K.ptr(V[f"{lp.name}.weight"]), K.ptr(V[f"{lp.name}.bias"]), K.ptr(u.y),
                        B, fout, fin, act[0], act[1], st), "dd_fwd")
                elif u.xt is not None:
                    self._rc(lib.csa_dense_fwd(
                        K.ptr(u.xt), K.ptr(V[f"{lp.name}.weight"]), K.ptr(V[f"{lp.name}.bias"]), K.ptr(u.y),
                        B, fout, fin, None, 0, 0, 0.0, 0.0, None, None, 0, 0.0, st), "dense_fwd")
                else:
                    self._rc(lib.csa_dense_fwd(
                        K.ptr(u.x), K.ptr(V[f"{lp.name}.weight"]), K.ptr(V[f"{lp.name}.bias"]), K.ptr(u.y),
                        B, fout, fin, *self._bn_args_c(tf), in_act, in_alpha, st), "dense_fwd")


    # ------------------------------------------------------------------ standalone units
    def _pool_geom_full(self, u: Unit):
        lp = u.layer
        sp = lp.spec
        h, w = lp.in_shape.hw
        oh, ow = lp.out_shape.hw
        return K.ints([self.B, h, w, lp.in_shape.c, sp.kernel[0], sp.kernel[1], sp.stride[0], sp.stride[1],
                       lp.pads[0], lp.pads[2], oh, ow])

    def _standalone_fwd(self, u: Unit, st) -> None:
        lib = self.lib
        if u.kind == "pool":
            self._rc(lib.csa_maxpool_fwd(K.ptr(u.x), K.ptr(u.y), K.ptr(u.argmax), self._pool_geom_full(u), st),
                     "maxpool_fwd")
            return
        n = u.x.numel()
        C_ = self._bn_channels(u)
        act, alpha = _act_id(u.act), _alpha(u.act)
        if u.norm is None:
            self._rc(lib.csa_bn_apply(K.ptr(u.x), K.ptr(u.y), n, C_, None, act, alpha, st), "act_apply")
            return
        nm = u.norm.name
        rm = getattr(self.model, f"bn{u.norm.index}_mean")
        rv = getattr(self.model, f"bn{u.norm.index}_var")
        eps = float(u.norm.spec.epsilon)
        if self._eval_bn:
            self._rc(lib.csa_bn_finalize(None, 0, C_, 1.0, eps, K.ptr(self.views[f"{nm}.scale"]),
                                         K.ptr(self.views[f"{nm}.offset"]), K.ptr(rm), K.ptr(rv), 0.0, 1,
                                         K.ptr(u.bn_tab), st), "bn_finalize(eval)")
        else:
            R = u.bn_slab.shape[0]
            self._rc(lib.csa_bn_stats(K.ptr(u.x), n // C_, C_, K.ptr(u.bn_slab), R, st), "bn_stats")
            if self.sync_bn:
                self.e.sync.allreduce_tensors([u.bn_slab], tag=f"bns{u.norm.index}")
            upd = self.model.training and not getattr(self, "_predicting", False)
            self._rc(lib.csa_bn_finalize(K.ptr(u.bn_slab), R, C_, float(n // C_ * self.W), eps,
                                         K.ptr(self.views[f"{nm}.scale"]), K.ptr(self.views[f"{nm}.offset"]),
                                         K.ptr(rm) if upd else None, K.ptr(rv) if upd else None,
                                         float(self.model.bn_momentum), 0, K.ptr(u.bn_tab), st), "bn_finalize")
        self._rc(lib.csa_bn_apply(K.ptr(u.x), K.ptr(u.y), n, C_, K.ptr(u.bn_tab), act, alpha, st), "bn_apply")

    def _gconv_fwd(self, u: Unit, st) -> None:
        lp = u.layer
        V = self.views
        self._rc(self.lib.csa_gconv_fwd(
            K.ptr(u.x), K.ptr(V[f"{lp.name}.weight"]), K.ptr(V[f"{lp.name}.bias"]) if lp.spec.bias else None,
            K.ptr(u.y), self._conv_geom(lp, self.B), st), "gconv_fwd")

    def _gconv_bwd(self, u: Unit, prev: Optional[Unit], st) -> None:
        """Input gradient (reads the pre-update weights) then weight gradient."""
        lp = u.layer
        geom = self._conv_geom(lp, self.B)
        if prev is not None:
            self._rc(self.lib.csa_gconv_dgrad(K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]),
                                              K.ptr(prev.dy), geom, st), "gconv_dgrad")
        G = self.gviews
        self._rc(self.lib.csa_gconv_wgrad(
            K.ptr(u.x), K.ptr(u.dy), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]) if lp.spec.bias else None,
            geom, 1.0, st), "gconv_wgrad")

    def _standalone_bwd(self, u: Unit, prev: Optional[Unit], st) -> None:
        lib = self.lib
        dx = prev.dy if prev is not None else None
        if u.kind == "pool":
            if dx is not None:
                self._rc(lib.csa_maxpool_bwd(K.ptr(u.dy), K.ptr(u.argmax), K.ptr(dx), self._pool_geom_full(u), st),
                         "maxpool_bwd")
            return
        n = u.x.numel()
        C_ = self._bn_channels(u)
        act, alpha = _act_id(u.act), _alpha(u.act)
        if u.norm is None:
            if dx is not None:
                self._rc(lib.csa_bn_bwd_apply(K.ptr(u.x), K.ptr(u.y), K.ptr(u.dy), K.ptr(dx), n, C_, None, None,
                                              act, alpha, st), "act_bwd")
            return
        nm = u.norm.name
        R = u.bn_bslab.shape[0]
        self._rc(lib.csa_bn_bwd_reduce(K.ptr(u.x), K.ptr(u.y), K.ptr(u.dy), n // C_, C_, K.ptr(u.bn_tab), act, alpha,
                                       K.ptr(u.bn_bslab), R, st), "bn_bwd_reduce")
        if self.sync_bn:
            self.e.sync.allreduce_tensors([u.bn_bslab], tag=f"bnbs{u.norm.index}")
        # under SyncBN the slab is already the global sum, so the parameter gradients are
        # scaled by 1/world before the gradient all-reduce adds them up again
        self._rc(lib.csa_bn_bwd_finalize(K.ptr(u.bn_bslab), R, C_, float(n // C_ * self.W), 1.0 / self.W,
                                         K.ptr(self.gviews[f"{nm}.scale"]), K.ptr(self.gviews[f"{nm}.offset"]),
                                         K.ptr(u.bn_k), st), "bn_bwd_finalize")
        if dx is not None:
            self._rc(lib.csa_bn_bwd_apply(K.ptr(u.x), K.ptr(u.y), K.ptr(u.dy), K.ptr(dx), n, C_, K.ptr(u.bn_tab),
                                          K.ptr(u.bn_k), act, alpha, st), "bn_bwd_apply")

    def predict_logits_into(self, logits: torch.Tensor) -> None:
        with self._det_scope():
            self._predict_logits_into(logits)

    def _predict_logits_into(self, logits: torch.Tensor) -> None:
        """Forward-only pass over this program's input rows -> ``logits`` [B, 10] (graph
        capturable; ``serve.hip_infer`` captures it per batch bucket).  BatchNorm uses the
        running statistics unless the model normalises with batch statistics in eval
        (``bn_mode == "batch"``), exactly as ``DigitNet.forward`` in eval mode."""
        st = K.stream()
        self.flush(st)                      # a deferred dense update lands before the forward
        self._eval_bn = self.model.bn_mode != "batch"
        self._predicting = True
        # split-K forward outputs (and, with batch statistics, the forward BN slabs) are
        # atomic accumulators that the training step's optimizer launch re-zeroes
        for u in self.units:
            if u.kind in ("dense", "gconv") and u.splits_fwd > 1:
                u.y.zero_()
            if not self._eval_bn and u.in_tf.has_bn:
                u.in_tf.slab.zero_()
            if not self._eval_bn and u.kind == "bn" and u.norm is not None:
                u.bn_slab.zero_()
        try:
            if self._eval_bn:
                for tf in [u.in_tf for u in self.units] + [self.head_tf]:
                    if tf.has_bn:
                        # a 1-row slab whose {sum, sumsq} / count=1 IS {mean, var + mean^2}
                        if getattr(tf, "eval_slab", None) is None:
                            tf.eval_slab = torch.zeros(1, 2, tf.slab.shape[2], device=self.e.device)
                        rm = getattr(self.model, f"bn{tf.norm.index}_mean")
                        rv = getattr(self.model, f"bn{tf.norm.index}_var")
                        tf.eval_slab[0, 0].copy_(rm)
                        torch.addcmul(rv, rm, rm, out=tf.eval_slab[0, 1])
            self._forward(st)
        finally:
            self._eval_bn = False
            self._predicting = False
        last = self.units[-1]
        hin = last.y.view(self.B, -1)
        Kh = hin.shape[1]
        if self.lib.csa_dense_fwd_splits(self.B, 10, Kh) > 1:
            logits.zero_()
        self._rc(self.lib.csa_dense_fwd(
            K.ptr(hin), K.ptr(self.views["head.weight"]), K.ptr(self.views["head.bias"]), K.ptr(logits),
            self.B, 10, Kh, None, 0, 0, 0.0, 0.0, None, None,
            _act_id(self.head_tf.act), _alpha(self.head_tf.act), st), "head_fwd")

    def _pair_bwd(self, st) -> None:
        e, lib = self.e, self.lib
        ua, ub = self.units[0], self.units[1]
        V, G = self.views, self.gviews
        nt = self.units[2].in_tf if len(self.units) > 2 else self.head_tf
        if self.sync_bn and nt.has_bn:
            e.sync.allreduce_tensors([nt.bwd_slab], tag="bnb2")
        nbn = self._bn_args(nt)
        dsc = G[f"{nt.norm.name}.scale"] if nt.has_bn else None
        dof = G[f"{nt.norm.name}.offset"] if nt.has_bn else None
        rm = rv = None
        if nt.has_bn:
            rm = getattr(self.model, f"bn{nt.norm.index}_mean")
            rv = getattr(self.model, f"bn{nt.norm.index}_var")
        simg, srows, scur = self._batch_src()
        if getattr(self, "tail", False):
            self._tail_set()
        # this step's forward BatchNorm tables (bn_act_apply wrote them for the dense
        # consumer): the pair's workgroups load them instead of each folding the slab
        tab = getattr(nt, "bn_tab", None) if nt.has_bn else None
        if tab is not None and os.environ.get("CSA_PAIR_BN_TAB", "1") == "1":
            lib.csa_conv_pair_bn_tab(K.ptr(tab))
        self._rc(lib.csa_conv_pair_bwd(
            K.ints(self.pair), K.ptr(simg), K.ptr(srows), K.ptr(scur),
            K.ptr(V[f"{ua.layer.name}.weight"]), K.ptr(V.get(f"{ua.layer.name}.bias")) if ua.layer.spec.bias else None,
            _act_id(ua.act), _alpha(ua.act), K.ptr(V[f"{ub.layer.name}.weight"]), 1 if ub.layer.spec.bias else 0,
            _act_id(ub.act), _alpha(ub.act), K.ptr(ub.dy), K.ptr(ub.y), K.ptr(ub.argmax),
            *nbn, K.ptr(nt.bwd_slab) if nt.has_bn else None, nt.bwd_nslab if nt.has_bn else 0,
            K.ptr(dsc), K.ptr(dof), K.ptr(rm), K.ptr(rv), float(self.model.bn_momentum),
            K.ptr(ua.dw_acc), K.ptr(ua.db_acc) if ua.layer.spec.bias else None,
            K.ptr(ub.dw_acc), K.ptr(ub.db_acc) if ub.layer.spec.bias else None,
            min(ua.wg_stripes, ub.wg_stripes), K.ptr(self.pair_tabs), st), "conv_pair_bwd")
        self._sync_bn_param_grads(nt)
        if ua.row_fold:
            # the pair's (up to) four striped gradients into the flat gradient: ONE launch
            jobs = []
            for u in (ua, ub):
                lp = u.layer
                jobs.append((u.dw_acc, u.wg_stripes, u.dw_acc.shape[1], G[f"{lp.name}.weight"]))
                if u.db_acc is not None:
                    jobs.append((u.db_acc, u.wg_stripes, u.db_acc.shape[1], G[f"{lp.name}.bias"]))
            n = len(jobs)
            self._rc(lib.csa_rows_fold_multi(
                n, (C.c_void_p * 4)(*[j[0].data_ptr() for j in jobs]), (C.c_long * 4)(*[j[2] for j in jobs]),
                (C.c_int * 4)(*[j[1] for j in jobs]), (C.c_long * 4)(*[j[2] for j in jobs]),
                (C.c_void_p * 4)(*[j[3].data_ptr() for j in jobs]), (C.c_int * 4)(*([1] * n)), st), "rows_fold_multi")

    def _conv_det_folds(self, u: Unit, tf, st) -> None:
        """Deterministic mode, after a conv unit's backward: its BN-backward rows (one per
        dgrad workgroup) to row 0 and its weight-gradient stripes (one per wgrad workgroup)
        into the flat gradient, both in row order (the stripes are re-zeroed by the fold)."""
        if not self.det:
            return
        if tf.has_bn and u.x is not None:
            self._row_fold(tf.bwd_slab, tf.bwd_prod_rows, tf.bwd_slab.shape[1] * tf.bwd_slab.shape[2],
                           tf.bwd_slab, 0, st)
        if u.row_fold and u.wg_stripes > 1:
            G, lp = self.gviews, u.layer
            self._row_fold(u.dw_acc, u.wg_stripes, u.dw_acc.shape[1], G[f"{lp.name}.weight"], 1, st)
            if u.db_acc is not None:
                self._row_fold(u.db_acc, u.wg_stripes, u.db_acc.shape[1], G[f"{lp.name}.bias"], 1, st)

    def _route_geom(self, u: Unit):
        lp, B = u.layer, self.B
        oh, ow = lp.out_shape.hw
        g = [B, u.y.shape[1], u.y.shape[2], u.y.shape[3], oh, ow, 1 if u.pool is not None else 0]
        if u.pool is not None:
            ps = u.pool.spec
            g += [ps.kernel[0], ps.kernel[1], ps.stride[0], ps.stride[1], u.pool.pads[0], u.pool.pads[2]]
        else:
            g += [1, 1, 1, 1, 0, 0]
        return g

    def _sync_bn_param_grads(self, tf: Transform) -> None:
        if self.sync_bn and tf.has_bn and self.W > 1:
            for p in ("scale", "offset"):
                self.gviews[f"{tf.norm.name}.{p}"].mul_(1.0 / self.W)

    def _dense_bwd_fused(self, u: Unit, prev: Unit, st) -> bool:
        """Input gradient + weight gradient of a dense unit as ONE launch
        (``csa_dense_bwd``) when its weight-gradient operand needs no transform (a
        materialised BN/act input, or an identity transform).  False: not applicable."""
        tf, lp, B = u.in_tf, u.layer, self.B
        if u.xt is None and (tf.has_bn or tf.act is not None):
            return False
        V, G = self.views, self.gviews
        fin, fout = lp.in_shape.numel, lp.spec.hidden
        xw = u.xt if u.xt is not None else u.x.view(B, -1)
        rc = self.lib.csa_dense_bwd(
            K.ptr(u.dy), K.ptr(V[f"{lp.name}.weight"]), K.ptr(prev.dy), B, fin, fout,
            K.ptr(u.x.view(B, -1)), _act_id(tf.act), _alpha(tf.act), *self._bn_args_c(tf),
            K.ptr(tf.bwd_slab), K.ptr(xw), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]),
            1.0, st)
        if rc < 0:
            raise RuntimeError(f"dense_bwd failed: {rc}")
        if rc > 0:
            self._dense_det_fold(u, st)
        return rc > 0

    def _dense_det_fold(self, u: Unit, st) -> None:
        """Deterministic mode, after a materialised-gradient dense unit's input gradient: its
        BN-backward rows (one per GEMM workgroup, gemm.hip) to row 0 in row order."""
        tf = u.in_tf
        if self.det and tf.has_bn:
            self._row_fold(tf.bwd_slab, tf.bwd_prod_rows, tf.bwd_slab.shape[1] * tf.bwd_slab.shape[2],
                           tf.bwd_slab, 0, st)

    def _dd_wgrad_update(self, u: Unit, x: torch.Tensor, dy: torch.Tensor, M: int, act, st) -> None:
        """Weight gradient X^T dY over ``M`` rows with the optimizer update of W / b applied
        in the same launch (csa_dd_wgrad update mode; the head advanced the step counter)."""
        e, lp = self.e, u.layer
        fin, fout = lp.in_shape.numel, lp.spec.hidden
        offs = self.model.state.offsets
        ow, ob = offs[f"{lp.name}.weight"], offs[f"{lp.name}.bias"]
        sl = e.slots
        s0 = sl[0] if sl.shape[0] > 0 else None
        s1 = sl[1] if sl.shape[0] > 1 else None
        V = self.views
        self._rc(self.lib.csa_dd_wgrad(
            K.ptr(x), K.ptr(dy), M, fin, fout, act[0], act[1], 1.0, None, None,
            K.ptr(V[f"{lp.name}.weight"]), K.ptr(V[f"{lp.name}.bias"]),
            K.ptr(s0[ow:]) if s0 is not None else None, K.ptr(s1[ow:]) if s1 is not None else None,
            K.ptr(s0[ob:]) if s0 is not None else None, K.ptr(s1[ob:]) if s1 is not None else None,
            e.opt_id, float(e.lr), K.ptr(e.dstep), st), "dd_wgrad(update)")

    def _dense_bwd_update(self, u: Unit, prev: Optional[Unit], st) -> None:
        """Dense backward + optimizer update of W / b in one launch (dense_update.hip)."""
        e, lib, B = self.e, self.lib, self.B
        lp, tf = u.layer, u.in_tf
        fin, fout = lp.in_shape.numel, lp.spec.hidden
        offs = self.model.state.offsets
        ow, ob = offs[f"{lp.name}.weight"], offs[f"{lp.name}.bias"]
        sl = e.slots
        s0 = sl[0] if sl.shape[0] > 0 else None
        s1 = sl[1] if sl.shape[0] > 1 else None
        xw = u.xt if u.xt is not None else u.x.view(B, -1)
        if self.head_row and u is self.units[-1]:
            # the head's batch reductions ride along: dWh / dbh into the flat gradient (the
            # optimizer updates them), the step's loss / #correct into the metric ring
            G = self.gviews
            head = (K.ptr(u.y), K.ptr(self.hdl), K.ptr(G["head.weight"]), K.ptr(G["head.bias"]),
                    K.ptr(self.hrl), K.ptr(self.hrc), K.ptr(e.ring_loss), K.ptr(e.ring_correct),
                    e.ring_correct.numel(), float(B if e.cfg.loss_name == "entropy" else B * 10),
                    _act_id(self.head_tf.act), _alpha(self.head_tf.act))
        else:
            head = (None, None, None, None, None, None, None, None, 1, 1.0, 0, 0.0)
        if self.hfuse:
            # weight gradient + update deferred into the pair backward launch; the input
            # gradient (+ transform backward + BN statistics) now
            if self.dp_hf:
                # gradient mode: dW / db stored whole into the flat gradient (slot-free rule)
                G = self.gviews
                rc = lib.csa_dense_update_defer(
                    K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]), K.ptr(self.views[f"{lp.name}.bias"]),
                    B, fin, fout, K.ptr(xw), 0, 0.0, K.ptr(e.dstep), None, None, None, None, 1.0, *head)
                if rc >= 0:
                    rc = lib.csa_dense_update_grad_mode(K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]))
            else:
                rc = lib.csa_dense_update_defer(
                    K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]), K.ptr(self.views[f"{lp.name}.bias"]),
                    B, fin, fout, K.ptr(xw), e.opt_id, float(e.lr), K.ptr(e.dstep),
                    K.ptr(s0[ow:]) if s0 is not None else None, K.ptr(s1[ow:]) if s1 is not None else None,
                    K.ptr(s0[ob:]) if s0 is not None else None, K.ptr(s1[ob:]) if s1 is not None else None,
                    1.0, *head)
            if rc < 0:
                raise RuntimeError(f"dense_update_defer failed: {rc}")
            if prev is not None and not (self.head_dgrad and u is self.units[-1]):
                self._rc(lib.csa_dense_bwd_dgrad(
                    K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]), K.ptr(prev.dy), B, fin, fout,
                    K.ptr(u.x.view(B, -1)), _act_id(tf.act), _alpha(tf.act), *self._bn_args_c(tf),
                    K.ptr(tf.bwd_slab) if tf.has_bn else None, K.ptr(getattr(tf, "bn_tab", None)),
                    K.ptr(u.du_part), K.ptr(u.du_cnt), st), "dense_bwd_dgrad")
            if u is getattr(self, "br_unit", None):
                # the update reads W before nothing else does: fork after the input gradient
                cur = torch.cuda.current_stream(e.device)
                self.br_side.wait_stream(cur)
                self._rc(lib.csa_dense_update_flush_last(self.br_side.cuda_stream), "dense_update_branch")
                self._br_pending = True
            return
        if self.fused_grad:
            # data parallel: the same launch stores dW / db whole into the flat gradient
            G = self.gviews
            self._rc(lib.csa_dense_bwd_grad_head(
                K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]), K.ptr(prev.dy) if prev is not None else None,
                B, fin, fout, K.ptr(u.x.view(B, -1)), _act_id(tf.act), _alpha(tf.act), *self._bn_args_c(tf),
                K.ptr(tf.bwd_slab) if tf.has_bn else None, K.ptr(xw), 1.0, K.ptr(getattr(tf, "bn_tab", None)),
                K.ptr(u.du_part), K.ptr(u.du_cnt), K.ptr(G[f"{lp.name}.weight"]), K.ptr(G[f"{lp.name}.bias"]),
                *head, K.ptr(e.dstep), st), "dense_bwd_grad")
            if self.det and tf.has_bn:        # exclusive rows -> row 0, fixed order
                self._row_fold(tf.bwd_slab, tf.bwd_prod_rows, tf.bwd_slab.shape[1] * tf.bwd_slab.shape[2],
                               tf.bwd_slab, 0, st)
            return
        self._rc(lib.csa_dense_bwd_update_head(
            K.ptr(u.dy), K.ptr(self.views[f"{lp.name}.weight"]), K.ptr(self.views[f"{lp.name}.bias"]),
            K.ptr(prev.dy) if prev is not None else None, B, fin, fout,
            K.ptr(u.x.view(B, -1)), _act_id(tf.act), _alpha(tf.act), *self._bn_args_c(tf),
            K.ptr(tf.bwd_slab) if tf.has_bn else None, K.ptr(xw), e.opt_id, float(e.lr), K.ptr(e.dstep),
            K.ptr(s0[ow:]) if s0 is not None else None, K.ptr(s1[ow:]) if s1 is not None else None,
            K.ptr(s0[ob:]) if s0 is not None else None, K.ptr(s1[ob:]) if s1 is not None else None,
            1.0, K.ptr(getattr(tf, "bn_tab", None)), K.ptr(u.du_part), K.ptr(u.du_cnt), *head, st),
            "dense_bwd_update")
        if self.det and tf.has_bn:
            self._row_fold(tf.bwd_slab, tf.bwd_prod_rows, tf.bwd_slab.shape[1] * tf.bwd_slab.shape[2],
                           tf.bwd_slab, 0, st)

    def _opt_segments(self):
        """Flat [lo, hi) spans the optimizer launch updates: everything except the
        parameters a fused dense backward already updated (spans padded to float4; the
        flat layout's alignment padding is zero and stays zero)."""
        n = self.e.flat.numel()
        offs = self.model.state.offsets
        spans = sorted(offs.values())
        ends = {o: (spans[i + 1] if i + 1 < len(spans) else n) for i, o in enumerate(spans)}
        skip = set(getattr(self, "carry_offsets", set()) if getattr(self, "carry", None) else set())
        for u in self.units:
            if u.kind == "dense" and ((u.fused and self.fused) or u.lr_update):
                skip |= {offs[f"{u.layer.name}.weight"], offs[f"{u.layer.name}.bias"]}
        if not skip:
            return []
        segs: List[list] = []
        for o in spans:
            if o in skip:
                continue
            lo, hi = o - o % 4, -(-ends[o] // 4) * 4
            if segs and segs[-1][1] >= lo:
                segs[-1][1] = max(segs[-1][1], hi)
            else:
                segs.append([lo, hi])
        assert len(segs) <= 16, "at most 15 fused dense layers (_plan_fused)"
        return segs

    def _optimizer(self, st) -> None:
        """The flat optimizer launch: the update of every parameter no fused kernel updated
        plus the step's side jobs (accumulator zeroing, folds, metrics, cursor, staging).
        (Round 5 measured per-bucket updates on the DP side stream, each right after its
        bucket's exchange: 0.137 against 0.102 ms/step at world 1 — the graph's branches
        serialised behind them: profiles/r5_notes.md.)"""
        e, lib = self.e, self.lib
        lo, hi = e.sync.shard_range()
        s0 = e.slots[0] if e.slots.shape[0] > 0 else None
        s1 = e.slots[1] if e.slots.shape[0] > 1 else None
        if e.aps is not None:
            # parameters / slots were updated by the async_ps launch: the update part of this
            # launch runs on four scratch floats (w, g, two slots) and changes nothing real
            if getattr(self, "_aps_dummy", None) is None:
                self._aps_dummy = torch.zeros(4, 4, device=e.device)
            w, g, s0, s1 = self._aps_dummy[0], self._aps_dummy[1], self._aps_dummy[2], self._aps_dummy[3]
        elif e.sync.strategy == "ps" and e.ctx.enabled:
            w, g = e.flat[lo:hi], e.grad_shard
        else:
            w, g = e.flat, e.flat_grad
        zregs = self.zero_regions
        zp = (C.c_void_p * 16)(*[r.data_ptr() for r in zregs])
        zn = (C.c_long * 16)(*[r.numel() for r in zregs])
        folds = []          # striped conv weight gradients / head partials -> summed inside the update
        offs = self.model.state.offsets
        for u in self.units:
            if (u.kind == "conv" and u.wg_stripes > 1 and not getattr(u, "row_fold", False)
                    and not getattr(u, "tail_fold", False)):
                lp = u.layer
                folds.append((offs[f"{lp.name}.weight"], u.dw_acc.shape[1], u.dw_acc, u.wg_stripes, u.dw_acc.shape[1], 1))
                if u.db_acc is not None:
                    folds.append((offs[f"{lp.name}.bias"], u.db_acc.shape[1], u.db_acc, u.wg_stripes, u.db_acc.shape[1], 1))
        if self.head_rg:
            hp = self.head_part
            kw = self.head_kw
            folds.append((offs["head.weight"], kw, hp, hp.shape[0], hp.shape[1], 0))
            # the bias span rounded up to a float4: the partial rows' padding and the flat
            # layout's padding are zero, so the extra lanes update zero parameters by zero
            # (no per-element edge path: one round trip instead of four)
            nb = 12 if hp.shape[1] >= kw + 12 and self.e.flat.numel() >= offs["head.bias"] + 12 else 10
            folds.append((offs["head.bias"], nb, hp[:, kw:], hp.shape[0], hp.shape[1], 0))
        if len(folds) > 8:
            raise Unsupported("more than 8 striped gradients")
        fo = (C.c_long * 8)(*[f[0] for f in folds])
        fn = (C.c_long * 8)(*[f[1] for f in folds])
        fs = (C.c_void_p * 8)(*[f[2].data_ptr() for f in folds])
        fS = (C.c_int * 8)(*[f[3] for f in folds])
        fl = (C.c_long * 8)(*[f[4] for f in folds])
        fz = (C.c_int * 8)(*[f[5] for f in folds])
        keep = self.keep_ranges
        if len(keep) > 32:
            raise RuntimeError(f"{len(keep)} stored dense gradient ranges (optimizer holds 32)")
        klo = (C.c_long * 32)(*[k[0] for k in keep])
        khi = (C.c_long * 32)(*[k[1] for k in keep])
        segs = self.opt_segments
        slo = (C.c_long * 16)(*[x[0] for x in segs])
        shi = (C.c_long * 16)(*[x[1] for x in segs])
        div = float(self.B if e.cfg.loss_name == "entropy" else self.B * 10)
        if self.head_rg:
            met = (K.ptr(self.head_mloss), K.ptr(self.head_mcorr), self.head_mloss.numel(), div,
                   K.ptr(e.ring_loss), K.ptr(e.ring_correct), e.ring_correct.numel())
        elif self.head_sep:             # the row head's per-row loss / #correct
            met = (K.ptr(self.hrl), K.ptr(self.hrc), self.B, div,
                   K.ptr(e.ring_loss), K.ptr(e.ring_correct), e.ring_correct.numel())
        else:
            met = (None, None, 0, 1.0, None, None, 1)
        if getattr(self, "staged", False):
            # the head advanced the cursor; the trailing workgroups stage the next batch
            stage = (K.ptr(e.data.images), K.ptr(e.data.labels), K.ptr(e.stream.rows), K.ptr(e.stream.cursor),
                     self.B, self.stage_img.shape[1], K.ptr(self.stage_img), K.ptr(self.stage_lbl))
            cursor_args = (None, 0)
        else:
            stage = (None, None, None, None, 0, 0, None, None)
            cursor_args = (K.ptr(e.stream.cursor), e.stream.wrap)
        if getattr(self, "carry", None) is not None:
            lib.csa_optimizer_set_pending(K.ptr(self.carry_pending))
        self._rc(lib.csa_optimizer2s(
            e.opt_id, K.ptr(w), K.ptr(g), K.ptr(s0), K.ptr(s1), w.numel(), slo, shi, len(segs),
            0 if self.ps_mode else 1, float(e.lr), K.ptr(e.dstep),
            zp, zn, len(zregs), fo, fn, fs, fS, fl, fz, len(folds), klo, khi, len(keep),
            *met, *cursor_args, *stage, st), "optimizer")
        if getattr(self, "hfuse", False) and lib.csa_dense_update_pending():
            raise RuntimeError("deferred dense updates were not consumed by the pair backward")
        if e.sync.strategy == "ps" and e.ctx.enabled:
            e.sync.all_gather_params(e.flat)
