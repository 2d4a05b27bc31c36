"""Device backend of the preprocessing pipeline: the 14 ops + resize + inference prep as
batched gfx950 kernels (``csrc/kernels/image_ops.hip``) over a uint8 [N, H, W] tensor.

Same entry point and parameter semantics as ``ops_ref.apply_op`` (which is the spec and
the CPU path).  Host-side parameter preparation mirrors the reference exactly — default
values, Gaussian taps, and the random draws of ``random_brightness_contrast`` and
``add_salt_pepper_noise`` are taken from the same NumPy generator in the same order —
so the device result equals the CPU result for a given seed.

``apply_op`` accepts a NumPy batch (uploaded, processed, downloaded) or a CUDA uint8
tensor (processed in place on the device, nothing copied) — the pipeline keeps its
image set resident on the GPU across all operations.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Union

import numpy as np
import torch

from ..ops import fused as K
from . import ops_ref

Batch = Union[np.ndarray, torch.Tensor]

_SIGS = {
    "csa_img_flip": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.I, K.P]),
    "csa_img_affine": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.P, K.P, K.I, K.P]),
    "csa_img_sep_filter": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.P, K.I, K.P]),
    "csa_img_rank_filter": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.I, K.I, K.P]),
    "csa_img_equalize": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.P]),
    "csa_img_clahe": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.I, K.F, K.P]),
    "csa_img_nlmeans": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.F, K.I, K.I, K.P]),
    "csa_img_salt_pepper": (C.c_int, [K.P, K.I, K.I, K.I, K.P, K.I, K.P]),
    "csa_img_resize": (C.c_int, [K.P, K.P, K.I, K.I, K.I, K.I, K.P, K.P, K.P, K.P, K.P]),
    "csa_img_infer_prep": (C.c_int, [K.P, K.P, K.I, K.P]),
    "csa_img_infer_prep_u8": (C.c_int, [K.P, K.P, K.I, K.P]),
    "csa_img_affine_rand": (C.c_int, [K.P, K.P, K.I, K.I, K.I, C.c_ulonglong, C.c_double, K.I, K.I, K.P]),
    "csa_img_salt_pepper_rand": (C.c_int, [K.P, K.P, K.I, K.I, K.I, C.c_ulonglong, K.I, K.P]),
}
_bound = False


def _lib():
    global _bound
    lib = K.load(required=True)
    if not _bound:
        for name, (res, args) in _SIGS.items():
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _bound = True
    return lib


def available() -> bool:
    try:
        return torch.cuda.is_available() and K.load(required=False) is not None
    except Exception:
        return False


def _dev() -> torch.device:
    return torch.device("cuda", torch.cuda.current_device())


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed (rc={rc})")


def to_device(batch: Batch) -> torch.Tensor:
    if isinstance(batch, torch.Tensor):
        t = batch if batch.is_cuda else batch.to(_dev())
    else:
        t = torch.from_numpy(np.ascontiguousarray(ops_ref._as_batch(batch), dtype=np.uint8)).to(_dev())
    if t.dtype != torch.uint8 or t.dim() != 3:
        raise ValueError("expected a uint8 [N, H, W] batch")
    return t.contiguous()


def _d(arr, dtype) -> torch.Tensor:
    return torch.as_tensor(np.ascontiguousarray(arr), dtype=dtype).to(_dev())


def resize(batch: Batch, size: int = 28) -> Batch:
    """Bicubic (a=-0.75, REPLICATE) resize of a same-shape batch to size x size."""
    x = to_device(batch)
    n, h, w = x.shape
    if (h, w) == (size, size):
        out = x.clone()
    else:
        iy, wy = ops_ref._resize_axis_weights(h, size)
        ix, wx = ops_ref._resize_axis_weights(w, size)
        out = torch.empty(n, size, size, dtype=torch.uint8, device=x.device)
        tabs = [_d(iy, torch.int32), _d(wy, torch.float64), _d(ix, torch.int32), _d(wx, torch.float64)]
        _check(_lib().csa_img_resize(x.data_ptr(), out.data_ptr(), n, h, w, size, *[t.data_ptr() for t in tabs],
                                     K.stream()), "csa_img_resize")
    return out.cpu().numpy() if isinstance(batch, np.ndarray) else out


def infer_prep(img20: Batch) -> torch.Tensor:
    """[N, 20, 20] uint8 -> [N, 784] float32 on the device (construct_inference.py:312-330)."""
    x = to_device(img20)
    if tuple(x.shape[1:]) != (20, 20):
        raise ValueError("infer_prep expects [N, 20, 20]")
    out = torch.empty(x.shape[0], 784, dtype=torch.float32, device=x.device)
    _check(_lib().csa_img_infer_prep(x.data_ptr(), out.data_ptr(), x.shape[0], K.stream()), "csa_img_infer_prep")
    return out


def apply_op(name: str, batch: Batch, value1=None, value2=None, *, mode: str = "saturate",
             rng: Optional[np.random.Generator] = None, seed: Optional[int] = None) -> Batch:
    """``ops_ref.apply_op`` on the device.  Returns the same container type as ``batch``."""
    name = ops_ref.OP_MAP.get(name, name)
    lib = _lib()
    x = to_device(batch)
    n, H, W = x.shape
    st = K.stream()
    out = torch.empty_like(x)
    xp, op = x.data_ptr(), out.data_ptr()
    if name in ("flip_up_down", "flip_left_right", "transpose_image"):
        m = {"flip_up_down": 0, "flip_left_right": 1, "transpose_image": 2}[name]
        _check(lib.csa_img_flip(xp, op, n, H, W, m, st), name)
    elif name == "adjust_brightness_contrast":
        a = np.full(n, 1.0 if value1 is None else float(value1))
        b = np.full(n, 0.0 if value2 is None else float(value2))
        da, db = _d(a, torch.float64), _d(b, torch.float64)
        _check(lib.csa_img_affine(xp, op, n, H, W, da.data_ptr(), db.data_ptr(), int(mode == "wrap"), st), name)
    elif name == "random_brightness_contrast":
        # per-image draws from the counter RNG inside the kernel (ops_ref.crng)
        s = ops_ref.seed_from(rng, seed)
        max_alpha = 1.0 if value1 is None else float(value1)
        max_beta = 0 if value2 is None else int(value2)
        _check(lib.csa_img_affine_rand(xp, op, n, H, W, s, max_alpha, max_beta, int(mode == "wrap"), st), name)
    elif name in ("mean_filter", "gaussian_blur"):
        k = int(value1 or 3)
        if name == "gaussian_blur" and (k % 2 == 0 or k < 1):
            raise ValueError("gaussian kernel size must be odd")
        taps = np.full(k, 1.0 / k) if name == "mean_filter" else ops_ref.gaussian_kernel(k)
        dt = _d(taps, torch.float64)
        _check(lib.csa_img_sep_filter(xp, op, n, H, W, dt.data_ptr(), k, st), name)
    elif name in ("median_filter", "erode", "dilate"):
        k = int(value1 or 3)
        if name == "median_filter" and (k % 2 == 0 or k < 1):
            raise ValueError("median kernel size must be odd")
        if name == "median_filter" and k > 7:
            raise ValueError("median kernel size must be <= 7 on the device path")
        _check(lib.csa_img_rank_filter(xp, op, n, H, W, k, {"median_filter": 0, "erode": 1, "dilate": 2}[name],
                                       st), name)
    elif name == "equalize_hist":
        _check(lib.csa_img_equalize(xp, op, n, H, W, st), name)
    elif name == "clahe":
        _check(lib.csa_img_clahe(xp, op, n, H, W, 8, 40.0, st), name)
    elif name == "nl_denoise_gray":
        _check(lib.csa_img_nlmeans(xp, op, n, H, W, float(value1 or 10), 7, 21, st), name)
    elif name == "add_salt_pepper_noise":
        s = ops_ref.seed_from(rng, seed)
        m = int(H * W * float(value1 or 0))
        _check(lib.csa_img_salt_pepper_rand(xp, op, n, H, W, s, m, st), name)
    else:
        raise ValueError(f"unknown preprocessing op {name!r}")
    return _finish(batch, out)


def _finish(batch: Batch, out: torch.Tensor) -> Batch:
    return out.cpu().numpy() if isinstance(batch, np.ndarray) else out
