"""ctypes bindings for ``libcsa_kernels.so`` (the hand-written gfx950 kernels).

The library is plain HIP with a C ABI (no torch C++ extension, no hipify): tensors are
passed as raw device pointers and every launcher takes the current HIP stream, so calls
made while ``torch.cuda.graph`` is capturing become graph nodes.  ``import torch`` must
come first so the library binds to the HIP runtime torch already loaded (same SONAME).

``load(required=True)`` raises if the library is missing — a GPU run never silently
falls back to PyTorch ops.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import torch

from . import build as _build

_LIB: Optional[C.CDLL] = None

P = C.c_void_p
I = C.c_int
L = C.c_long
F = C.c_float

ACT_IDS = {None: 0, "none": 0, "sigmoid": 1, "relu": 2, "leaky_relu": 3}

_SIGS = {
    "csa_dense_fwd_splits": (I, [I, I, I]),
    "csa_dense_fwd": (I, [P, P, P, P, I, I, I, P, I, I, F, F, P, P, I, F, P]),
    "csa_dense_dgrad": (I, [P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P]),
    "csa_dense_dgrad_splits": (I, [I, I, I, I]),
    "csa_dense_dgrad_slabs": (I, [I, I, I]),
    "csa_dense_wgrad_splits": (I, [I, I, I]),
    "csa_dense_bwd": (I, [P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P, P, P, F, P]),
    "csa_dense_wgrad": (I, [P, P, P, P, I, I, I, P, I, I, F, F, P, P, I, F, F, P]),
    "csa_conv_wgrad": (I, [P, P, P, P, P, P, I, I, I, I, I, I, I, I, I, I, I, I, I, I,
                           P, I, F, F, P, P, I, F, P, P]),
    "csa_conv_fwd_nslab": (I, [P, P]),
    "csa_conv_fwd": (I, [P, P, P, P, P, P, P, P, P, P, P, I, F, F, P, P, I, F, I, F, P, P]),
    "csa_route_bwd": (I, [P, P, P, P, P, I, F, P, I, F, F, P, P, P, I, P, P, P, P, F, P]),
    "csa_conv_dgrad_nslab": (I, [P]),
    "csa_conv_wgrad_blocks": (I, [P, I]),
    "csa_conv_dgrad": (I, [P, P, P, P, P, I, F, P, I, F, F, P, P, P, P]),
    "csa_conv_bwd": (I, [P, P, P, P, P, I, F, P, I, F, F, P, P, P, P, P, I, P]),
    "csa_head": (I, [P, I, I, I, F, P, P, P, P, I, F, P, P, P, P, P, P, P, I, P, P, P]),
    "csa_optimizer": (I, [I, P, P, P, P, L, I, F, P, P, P, I, P, P, P, P, P, I, P, P, I, P, L, P]),
    "csa_optimizer2": (I, [I, P, P, P, P, L, P, P, I, I, F, P, P, P, I, P, P, P, P, P, P, I, P, P, I,
                           P, P, I, F, P, P, I, P, L, P]),
    "csa_optimizer2s": (I, [I, P, P, P, P, L, P, P, I, I, F, P, P, P, I, P, P, P, P, P, P, I, P, P, I,
                           P, P, I, F, P, P, I, P, L,
                                P, P, P, P, I, L, P, P, P]),
    "csa_dense_bwd_update_ok": (I, [I, I, I, I]),
    "csa_dense_bwd_update_slabs": (I, [I]),
    "csa_dense_bwd_update": (I, [P, P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P, I, F, P,
                                 P, P, P, P, F, P, P, P, P]),
    "csa_dense_bwd_update_ws": (I, [I, I, P]),
    "csa_dense_bwd_grad_head": (I, [P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P, F, P, P, P, P, P,
                                    P, P, P, P, P, P, P, P, I, F, I, F, P, P]),
    "csa_dense_bwd_update_head": (I, [P, P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P, I, F, P,
                                      P, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, I, F, I, F, P]),
    # horizontal fusion (round 4): dgrad-only dense backward + deferred update segments
    "csa_dense_bwd_dgrad": (I, [P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P, P, P, P]),
    "csa_dense_update_defer": (I, [P, P, P, I, I, I, P, I, F, P, P, P, P, P, F, P, P, P, P, P, P, P, P, I, F,
                                   I, F]),
    "csa_dense_update_pending": (I, []),
    "csa_head_dgrad_ok": (I, [I, I, I]),
    "csa_head_dgrad": (I, [P, I, I, I, F, P, P, P, P, P, I, F, P, P, P, P, P, P, L, P, I, P, I, F, P, P]),
    "csa_dense_update_flush": (I, [P]),
    "csa_dense_update_clear": (None, []),
    "csa_head_row_ok": (I, [I, I]),
    "csa_head_row": (I, [P, I, I, I, F, P, P, P, P, P, I, F, P, P, P, P, P, P, L, P]),
    "csa_head_part_rows": (I, [I, I]),
    "csa_du_debug": (I, [P]),
    "csa_opt_debug": (I, [P]),
    "csa_conv_pair_ok": (I, [P]),
    "csa_cp_debug": (I, [P]),
    "csa_cp_debug_block": (I, [I]),
    "csa_cp_life_debug": (I, [P]),
    "csa_cpv_life_debug": (I, [P]),
    "csa_dd_group_begin": (None, []),
    "csa_chain_begin": (None, []),
    "csa_nt_out_ew": (I, [I]),
    "csa_ew_clear_next": (None, [P]),
    "csa_nt_out_cp": (I, [I]),
    "csa_nt_out_head": (I, [I]),
    "csa_nt_out_du": (I, [I]),
    "csa_chain_reset": (None, []),
    "csa_chain_ok": (I, [I]),
    "csa_chain_words": (I, []),
    "csa_chain_end": (I, [P, P, P]),
    "csa_chain_head_debug": (I, [P]),
    "csa_dd_life_debug": (I, [P]),
    "csa_ew_life_debug": (I, [P]),
    "csa_dd_group_end": (I, [P]),
    "csa_cp_du_debug": (I, [P]),
    "csa_conv_pair_bn_tab": (None, [P]),
    "csa_head_debug": (I, [P]),
    "csa_conv_pair_fwd": (I, [P, P, P, P, P, P, I, F, P, P, I, F, P, P, P, I, P, P, I, P]),
    "csa_conv_pair_fwd_carry": (I, [I, F, P, P, P, P, P, P, I, P, P, I]),
    "csa_opt_carry_flush": (I, [I, F, P, P, P, P, P, P, I, P, P, I, P]),
    "csa_optimizer_set_pending": (None, [P]),
    "csa_dense_update_flush_last": (I, [P]),
    "csa_conv_pair_tail_table_bytes": (L, [P, I]),
    "csa_conv_pair_tail_plan": (I, [P, I, I, P, P, P, P, P, P, P, P, I]),
    "csa_dense_update_grad_mode": (I, [P, P]),
    "csa_conv_pair_tail_set": (I, [P, P, I, F, P, P, I, I, P, P, P, P, P, P, I, L, P, P]),
    "csa_conv_pair_tail_force": (None, [P]),
    "csa_conv_pair_tail_pending": (I, []),
    "csa_conv_pair_tail_ticket_words": (I, []),
    "csa_dense_update_head_params": (I, [P, P, P, P, P, P]),
    "csa_conv_pair_valu_ok": (I, [P]),
    "csa_conv_pair_grid": (I, [P]),
    "csa_set_deterministic": (None, [I]),
    "csa_deterministic": (I, []),
    "csa_set_packed": (None, [I]),
    "csa_packed": (I, []),
    "csa_set_shared_gpu": (None, [I]),
    "csa_shared_gpu": (I, []),
    "csa_rows_fold": (I, [P, L, I, L, P, I, P]),
    "csa_rows_fold_multi": (I, [I, P, P, P, P, P, P, P]),
    "csa_conv_pair_bwd": (I, [P, P, P, P, P, P, I, F, P, I, I, F, P, P, P, P, I, F, F, P, P, P, I, P, P, P, P, F,
                              P, P, P, P, I, P, P]),
    "csa_conv_pair_bwd_tables_size": (L, [P]),
    "csa_conv_pair_bwd_tables": (I, [P, P, P]),
    "csa_head_part": (I, [P, I, I, I, F, P, P, P, P, P, I, F, P, P, P, P, P, P, P]),
    "csa_head_part2": (I, [P, I, I, I, F, P, P, P, P, P, I, F, P, P, P, P, P, P, P, L, P]),
    "csa_gather_batch": (I, [P, P, P, P, I, L, P, P, P]),
    "csa_gather_images_f32": (I, [P, P, P, I, L, P, P]),
    "csa_zero": (I, [P, P, I, P]),
    "csa_gemm_debug": (I, [P]),
    "csa_conv_debug": (I, [P]),
    "csa_bn_act_apply": (I, [P, P, L, I, P, I, F, F, P, P, I, F, P, P]),
    # register-direct MFMA dense kernels (dense_direct.hip)
    "csa_dd_debug": (I, [P]),
    "csa_dd_fwd_splits": (I, [I, I, I]),
    "csa_dd_fwd": (I, [P, P, P, P, I, I, I, I, F, P]),
    "csa_dd_dgrad_splits": (I, [I, I, I]),
    "csa_dd_dgrad_slabs": (I, []),
    "csa_dd_dgrad": (I, [P, P, P, I, I, I, P, I, F, P, I, I, F, F, P, P, P, P]),
    "csa_dd_wgrad": (I, [P, P, I, I, I, I, F, F, P, P, P, P, P, P, P, P, I, F, P, P]),
    # wide convolutions (> 128 channels) as implicit MFMA GEMMs (gemm.hip)
    "csa_gconv_fwd_splits": (I, [P]),
    "csa_gconv_fwd": (I, [P, P, P, P, P, P]),
    "csa_gconv_wgrad_splits": (I, [P, I]),
    "csa_gconv_wgrad": (I, [P, P, P, P, P, F, P]),
    "csa_gconv_dgrad_splits": (I, [P]),
    "csa_gconv_dgrad": (I, [P, P, P, P, P]),
    # standalone BatchNorm / activation / max-pool units (norm_pool.hip)
    "csa_bn_slab_rows": (I, []),
    "csa_bn_stat_rows": (I, [L]),
    "csa_bn_stats": (I, [P, L, I, P, I, P]),
    "csa_bn_finalize": (I, [P, I, I, F, F, P, P, P, P, F, I, P, P]),
    "csa_bn_apply": (I, [P, P, L, I, P, I, F, P]),
    "csa_bn_bwd_reduce": (I, [P, P, P, L, I, P, I, F, P, I, P]),
    "csa_bn_bwd_finalize": (I, [P, I, I, F, F, P, P, P, P]),
    "csa_bn_bwd_apply": (I, [P, P, P, P, L, I, P, P, I, F, P]),
    "csa_maxpool_fwd": (I, [P, P, P, P, P]),
    "csa_maxpool_bwd": (I, [P, P, P, P, P]),
    "csa_xgmi_alloc": (I, [L, C.POINTER(P), P]),
    "csa_xgmi_open": (I, [P, C.POINTER(P)]),
    "csa_xgmi_reuse": (I, [P, L, P]),
    "csa_xgmi_close": (I, [P]),
    "csa_xgmi_free": (I, [P]),
    "csa_xgmi_handle_bytes": (I, []),
    "csa_xgmi_max_blocks": (I, []),
    "csa_xgmi_diag_words": (I, []),
    "csa_xgmi_run": (I, [I, I, I, L, P, P, I, P, P, P, P, C.c_double, I, P, P]),
    "csa_xgmi_reduce_scatter": (I, [I, I, L, P, P, P, L, L, L, P, P, C.c_double, I, P, P]),
    "csa_aps_step": (I, [I, I, I, I, L, I, P, P, P, P, P, P, I, F, P, P, I, C.c_double, P]),
}


def lib_path() -> str:
    """The in-tree kernel library (``CSA_KERNEL_LIB`` overrides it: A/B runs of a kernel
    variant built beside it, e.g. scripts/xgmi_stress.py)."""
    return os.environ.get("CSA_KERNEL_LIB") or _build.KERNEL_LIB


def available() -> bool:
    return os.path.exists(lib_path())


def load(required: bool = True) -> Optional[C.CDLL]:
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        if os.environ.get("CSA_AUTOBUILD", "1") == "1":
            try:
                _build.build_kernels()
            except Exception as e:  # pragma: no cover - reported below
                if required:
                    raise RuntimeError(f"cannot build {path}: {e}") from e
        if not os.path.exists(path):
            if required:
                raise RuntimeError(f"HIP kernel library missing: {path} (run python -m cloud_server_amd.ops.build)")
            return None
    lib = C.CDLL(path)
    variant = bool(os.environ.get("CSA_KERNEL_LIB"))
    for name, (res, args) in _SIGS.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an A/B baseline built from an older revision (CSA_KERNEL_LIB) may lack entry
            # points added since; the in-tree library must have every one
            if variant:
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def check(rc: int, what: str) -> int:
    if rc < 0 or (rc > 0 and what.endswith("!")):
        raise RuntimeError(f"{what.rstrip('!')} failed with code {rc}")
    return rc


def ints(vals: Sequence[int]):
    arr = (C.c_int * len(vals))(*[int(v) for v in vals])
    return arr
