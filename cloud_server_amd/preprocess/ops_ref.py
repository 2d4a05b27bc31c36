"""The 14 image-preprocessing ops (+ resize) — NumPy reference implementations.

Reference: apps/preprocess/preprocess.py:18-227 (OpenCV, one JPEG file per call,
Python per-pixel loops in three of them) and the UI label -> op map at
apps/preprocess/views.py:15-40.  OpenCV is not available here, so every op is
re-specified from OpenCV's documented semantics and implemented on a whole batch
``uint8 [N, H, W]`` at once:

==========================  =========================================================
op                          semantics (border handling as in OpenCV)
==========================  =========================================================
resize                      bicubic (a = -0.75), half-pixel centres, replicate border
flip_up_down / left_right   cv2.flip(img, 0) / cv2.flip(img, 1)
transpose_image             cv2.flip(img, -1): a 180-degree rotation (reference quirk 12)
adjust_brightness_contrast  img*alpha + beta; ``saturate`` (intended) or ``wrap`` (what
                            the reference's uint8 loop actually does, quirk 11)
random_brightness_contrast  alpha ~ U(0, max_alpha), beta ~ randint(-max_beta, max_beta)
                            drawn once per image
mean_filter                 cv2.blur k x k, BORDER_REFLECT_101
gaussian_blur               cv2.GaussianBlur k x k, sigma from k (OpenCV's fixed small
                            kernels for k <= 7), BORDER_REFLECT_101
median_filter               cv2.medianBlur k, BORDER_REPLICATE
nl_denoise_gray             fastNlMeansDenoising(h, 7x7 template, 21x21 search)
add_salt_pepper_noise       int(H*W*p) white pixels then as many black pixels
equalize_hist               cv2.equalizeHist
clahe                       cv2.createCLAHE() defaults: clip 40, 8x8 tiles
erode / dilate              min / max over a k x k window (outside pixels ignored)
==========================  =========================================================

The GPU path (``preprocess.gpu``) runs the same ops as batched HIP kernels and is
tested against these functions.
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np

# UI label (Chinese) -> op name: apps/preprocess/views.py:15-40 (live entries only)
OP_MAP = {
    "上下翻转": "flip_up_down",
    "左右翻转": "flip_left_right",
    "对角线翻转": "transpose_image",
    "对比度亮度调整": "adjust_brightness_contrast",
    "随机对比度亮度调整": "random_brightness_contrast",
    "直方图均衡化": "equalize_hist",
    "CLAHE均衡化": "clahe",
    "腐蚀": "erode",
    "膨胀": "dilate",
    "均值滤波": "mean_filter",
    "高斯模糊": "gaussian_blur",
    "中值滤波": "median_filter",
    "灰度非局部平均值去噪": "nl_denoise_gray",
    "添加椒盐噪声": "add_salt_pepper_noise",
}
OP_NAMES = tuple(OP_MAP.values())


def _sat(x: np.ndarray) -> np.ndarray:
    return np.clip(np.rint(x), 0, 255).astype(np.uint8)


def _pad_reflect101(img: np.ndarray, r: int) -> np.ndarray:
    return np.pad(img, ((0, 0), (r, r), (r, r)), mode="reflect")  # numpy 'reflect' == REFLECT_101


def _as_batch(img: np.ndarray) -> np.ndarray:
    a = np.asarray(img)
    return a[None] if a.ndim == 2 else a


# ------------------------------------------------------------------------ resize
def _cubic_w(t: np.ndarray, a: float = -0.75) -> np.ndarray:
    t = np.abs(t)
    w = np.where(t <= 1, ((a + 2) * t - (a + 3)) * t * t + 1,
                 np.where(t < 2, ((a * t - 5 * a) * t + 8 * a) * t - 4 * a, 0.0))
    return w


def _resize_axis_weights(src: int, dst: int):
    scale = src / dst
    x = (np.arange(dst) + 0.5) * scale - 0.5
    x0 = np.floor(x).astype(np.int64)
    fx = x - x0
    idx = np.stack([x0 - 1, x0, x0 + 1, x0 + 2], 1)
    w = np.stack([_cubic_w(1 + fx), _cubic_w(fx), _cubic_w(1 - fx), _cubic_w(2 - fx)], 1)
    idx = np.clip(idx, 0, src - 1)
    return idx, w


def resize(img: np.ndarray, size: int = 28) -> np.ndarray:
    """cv2.resize(..., (size, size), INTER_CUBIC) for a uint8 batch (preprocess.py:18-30)."""
    b = _as_batch(img).astype(np.float64)
    n, h, w = b.shape
    if (h, w) == (size, size):
        return _as_batch(img).copy()
    iy, wy = _resize_axis_weights(h, size)
    ix, wx = _resize_axis_weights(w, size)
    rows = (b[:, iy, :] * wy[None, :, :, None]).sum(2)            # [n, size, w]
    out = (rows[:, :, ix] * wx[None, None, :, :]).sum(3)           # [n, size, size]
    return _sat(out)


# ------------------------------------------------------------------------ flips / affine
def flip_up_down(img, *_):
    return _as_batch(img)[:, ::-1, :].copy()


def flip_left_right(img, *_):
    return _as_batch(img)[:, :, ::-1].copy()


def transpose_image(img, *_):
    """The reference calls cv2.flip(img, -1): both axes, i.e. a 180-degree rotation."""
    return _as_batch(img)[:, ::-1, ::-1].copy()


def adjust_brightness_contrast(img, alpha=1.0, beta=0.0, mode: str = "saturate"):
    b = _as_batch(img).astype(np.float64)
    alpha = 1.0 if alpha is None else float(alpha)
    beta = 0.0 if beta is None else float(beta)
    v = b * alpha + beta
    if mode == "wrap":   # numpy uint8 element assignment in the reference loop
        return (np.trunc(v).astype(np.int64) % 256).astype(np.uint8)
    return _sat(v)


# ------------------------------------------------------------------------ counter RNG
# Stateless draws shared bit for bit with the device kernels (image_ops.hip `crng`):
# image i, draw j -> splitmix64(splitmix64((i << 32) | j) ^ seed) >> 32.  A batch's
# random parameters are a pure function of (seed, image, draw), so the GPU computes them
# in-kernel and this spec reproduces them exactly.
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _smix(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def crng(seed: int, i, j) -> np.ndarray:
    """uint32 draws for image indices ``i`` and draw indices ``j`` (broadcast)."""
    i = np.asarray(i, np.uint64)
    j = np.asarray(j, np.uint64)
    with np.errstate(over="ignore"):
        z = _smix((i << np.uint64(32)) | j) ^ np.uint64(int(seed) & 0xFFFFFFFFFFFFFFFF)
        return (_smix(z) >> np.uint64(32)).astype(np.uint64)


def crng_uniform(seed: int, i, j) -> np.ndarray:
    return (crng(seed, i, j) >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)


def crng_below(seed: int, i, j, n: int) -> np.ndarray:
    return ((crng(seed, i, j) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def seed_from(rng: Optional[np.random.Generator] = None, seed: Optional[int] = None) -> int:
    """The counter-RNG seed of one op application: ``seed`` if given, else one draw of
    ``rng`` (so a seeded pipeline is reproducible and CPU == GPU for the same rng)."""
    if seed is not None:
        return int(seed) & ((1 << 63) - 1)
    return int((rng or np.random.default_rng()).integers(0, 1 << 62))


def random_brightness_contrast(img, max_alpha=1.0, max_beta=0, mode: str = "saturate",
                               rng: Optional[np.random.Generator] = None, seed: Optional[int] = None):
    """alpha ~ U(0, max_alpha), beta ~ randint(-max_beta, max_beta), one draw per image
    (preprocess.py:105-106), from the counter RNG (draws 0 and 1 of each image)."""
    s = seed_from(rng, seed)
    b = _as_batch(img)
    max_alpha = 1.0 if max_alpha is None else float(max_alpha)
    max_beta = 0 if max_beta is None else int(max_beta)
    idx = np.arange(b.shape[0])
    a = crng_uniform(s, idx, 0) * max_alpha
    be = (crng_below(s, idx, 1, 2 * max_beta + 1) - max_beta).astype(np.float64)
    v = b.astype(np.float64) * a[:, None, None] + be[:, None, None]
    if mode == "wrap":
        return (np.trunc(v).astype(np.int64) % 256).astype(np.uint8)
    return _sat(v)


# ------------------------------------------------------------------------ linear filters
def _box_or_sep(img: np.ndarray, k1d: np.ndarray) -> np.ndarray:
    r = len(k1d) // 2
    b = _pad_reflect101(_as_batch(img).astype(np.float64), r)
    n, h, w = _as_batch(img).shape
    tmp = sum(k1d[i] * b[:, :, i:i + w] for i in range(len(k1d)))          # rows
    out = sum(k1d[i] * tmp[:, i:i + h, :] for i in range(len(k1d)))        # cols
    return _sat(out)


def mean_filter(img, k=3, *_):
    k = int(k or 3)
    return _box_or_sep(img, np.full(k, 1.0 / k))


_SMALL_GAUSS = {
    1: [1.0],
    3: [0.25, 0.5, 0.25],
    5: [0.0625, 0.25, 0.375, 0.25, 0.0625],
    7: [0.03125, 0.109375, 0.21875, 0.28125, 0.21875, 0.109375, 0.03125],
}


def gaussian_kernel(k: int, sigma: float = 0.0) -> np.ndarray:
    """cv2.getGaussianKernel(k, sigma): fixed tables for odd k <= 7 when sigma <= 0."""
    if sigma <= 0 and k in _SMALL_GAUSS:
        return np.asarray(_SMALL_GAUSS[k])
    if sigma <= 0:
        sigma = 0.3 * ((k - 1) * 0.5 - 1) + 0.8
    x = np.arange(k) - (k - 1) / 2
    g = np.exp(-(x * x) / (2 * sigma * sigma))
    return g / g.sum()


def gaussian_blur(img, k=3, *_):
    k = int(k or 3)
    if k % 2 == 0 or k < 1:
        raise ValueError("gaussian kernel size must be odd")
    return _box_or_sep(img, gaussian_kernel(k))


def _windows(img: np.ndarray, k: int, mode: str, cval=0) -> np.ndarray:
    r = k // 2
    b = _as_batch(img)
    if mode == "constant":
        p = np.pad(b, ((0, 0), (r, r), (r, r)), mode="constant", constant_values=cval)
    else:
        p = np.pad(b, ((0, 0), (r, r), (r, r)), mode=mode)
    n, h, w = b.shape
    return np.lib.stride_tricks.sliding_window_view(p, (k, k), axis=(1, 2))[:, :h, :w]


def median_filter(img, k=3, *_):
    k = int(k or 3)
    if k % 2 == 0 or k < 1:
        raise ValueError("median kernel size must be odd")
    win = _windows(img, k, "edge")
    n, h, w = win.shape[:3]
    return np.median(win.reshape(n, h, w, -1), axis=3).astype(np.uint8)


def erode(img, k=3, *_):
    k = int(k or 3)
    win = _windows(img, k, "constant", 255)
    return win.min(axis=(3, 4)).astype(np.uint8)


def dilate(img, k=3, *_):
    k = int(k or 3)
    win = _windows(img, k, "constant", 0)
    return win.max(axis=(3, 4)).astype(np.uint8)


# ------------------------------------------------------------------------ NL-means
def nl_denoise_gray(img, h=10, *_, template: int = 7, search: int = 21):
    """Non-local means (cv2.fastNlMeansDenoising semantics, float formulation):
    w(p, q) = exp(-max(0, d2(p, q)) / h^2), d2 = mean squared template difference."""
    h = float(h or 10)
    b = _as_batch(img).astype(np.float64)
    n, H, W = b.shape
    tr, sr = template // 2, search // 2
    pad = tr + sr
    P = np.pad(b, ((0, 0), (pad, pad), (pad, pad)), mode="reflect")
    acc = np.zeros_like(b)
    wsum = np.zeros_like(b)
    base = P[:, sr:sr + H + 2 * tr, sr:sr + W + 2 * tr]
    for dy in range(-sr, sr + 1):
        for dx in range(-sr, sr + 1):
            sh = P[:, sr + dy:sr + dy + H + 2 * tr, sr + dx:sr + dx + W + 2 * tr]
            d = (base - sh) ** 2
            # mean over the template window via separable box sums
            c = np.cumsum(np.cumsum(np.pad(d, ((0, 0), (1, 0), (1, 0))), 1), 2)
            t = template
            d2 = (c[:, t:, t:] - c[:, :-t, t:] - c[:, t:, :-t] + c[:, :-t, :-t]) / (t * t)
            wgt = np.exp(-np.maximum(d2, 0) / (h * h))
            acc += wgt * sh[:, tr:tr + H, tr:tr + W]
            wsum += wgt
    return _sat(acc / wsum)


# ------------------------------------------------------------------------ noise
def add_salt_pepper_noise(img, percent=0.05, *_, rng: Optional[np.random.Generator] = None,
                          seed: Optional[int] = None):
    """m = H*W*percent salt pixels (255) then m pepper pixels (0) per image
    (preprocess.py:155-170); coordinates from the counter RNG: salt j = draws (2+4j, 3+4j),
    pepper j = draws (4+4j, 5+4j)."""
    s = seed_from(rng, seed)
    b = _as_batch(img).copy()
    n, H, W = b.shape
    m = int(H * W * float(percent or 0))       # reference assumes 28x28 (preprocess.py:162)
    if m == 0 or n == 0:
        return b
    i = np.arange(n)[:, None]
    j = np.arange(m)[None, :]
    rows = np.broadcast_to(i, (n, m))
    b[rows, crng_below(s, i, 2 + 4 * j, H), crng_below(s, i, 3 + 4 * j, W)] = 255
    b[rows, crng_below(s, i, 4 + 4 * j, H), crng_below(s, i, 5 + 4 * j, W)] = 0
    return b


# ------------------------------------------------------------------------ histograms
def equalize_hist(img, *_):
    b = _as_batch(img)
    out = np.empty_like(b)
    for i in range(b.shape[0]):
        hist = np.bincount(b[i].ravel(), minlength=256)
        total = b[i].size
        nz = np.flatnonzero(hist)
        if len(nz) <= 1 or hist[nz[0]] == total:
            out[i] = b[i]
            continue
        cdf = np.cumsum(hist)
        cmin = hist[nz[0]]
        scale = 255.0 / (total - cmin)
        lut = np.clip(np.rint((cdf - cmin) * scale), 0, 255)
        lut[: nz[0]] = 0
        out[i] = lut.astype(np.uint8)[b[i]]
    return out


def clahe(img, *_, clip_limit: float = 40.0, tiles: int = 8):
    """cv2.createCLAHE(40, (8, 8)).apply: images not divisible by the grid are padded
    with BORDER_REFLECT_101 to a multiple of it; per-tile clipped histograms with
    redistribution; bilinear interpolation between tile LUTs."""
    b = _as_batch(img)
    n, H, W = b.shape
    th, tw = -(-H // tiles), -(-W // tiles)
    ph, pw = th * tiles - H, tw * tiles - W
    P = np.pad(b, ((0, 0), (0, ph), (0, pw)), mode="reflect") if (ph or pw) else b
    area = th * tw
    clip = max(int(clip_limit * area / 256), 1) if clip_limit > 0 else 0
    lut_scale = 255.0 / area
    out = np.empty_like(b)
    for i in range(n):
        luts = np.zeros((tiles, tiles, 256))
        for ty in range(tiles):
            for tx in range(tiles):
                tile = P[i, ty * th:(ty + 1) * th, tx * tw:(tx + 1) * tw]
                hist = np.bincount(tile.ravel(), minlength=256).astype(np.int64)
                if clip > 0:
                    excess = int(np.maximum(hist - clip, 0).sum())
                    hist = np.minimum(hist, clip)
                    add, resid = excess // 256, excess % 256
                    hist += add
                    if resid:
                        step = max(256 // resid, 1)
                        for j in range(0, 256, step):
                            if resid <= 0:
                                break
                            hist[j] += 1
                            resid -= 1
                luts[ty, tx] = np.clip(np.rint(np.cumsum(hist) * lut_scale), 0, 255)
        ys = (np.arange(H) + 0.5) / th - 0.5
        xs = (np.arange(W) + 0.5) / tw - 0.5
        y0 = np.floor(ys).astype(int); fy = ys - y0
        x0 = np.floor(xs).astype(int); fx = xs - x0
        y1 = np.clip(y0 + 1, 0, tiles - 1); y0 = np.clip(y0, 0, tiles - 1)
        x1 = np.clip(x0 + 1, 0, tiles - 1); x0 = np.clip(x0, 0, tiles - 1)
        v = b[i].astype(np.int64)
        l00 = luts[y0[:, None], x0[None, :], v]
        l01 = luts[y0[:, None], x1[None, :], v]
        l10 = luts[y1[:, None], x0[None, :], v]
        l11 = luts[y1[:, None], x1[None, :], v]
        fxm, fym = fx[None, :], fy[:, None]
        res = (l00 * (1 - fxm) + l01 * fxm) * (1 - fym) + (l10 * (1 - fxm) + l11 * fxm) * fym
        out[i] = _sat(res)
    return out


# ------------------------------------------------------------------------ dispatch
def apply_op(name: str, batch: np.ndarray, value1=None, value2=None, *,
             mode: str = "saturate", rng: Optional[np.random.Generator] = None) -> np.ndarray:
    """Apply op ``name`` (English name or UI label) to a uint8 [N, H, W] batch."""
    name = OP_MAP.get(name, name)
    b = _as_batch(batch)
    if name in ("flip_up_down", "flip_left_right", "transpose_image", "equalize_hist", "clahe"):
        return globals()[name](b)
    if name == "adjust_brightness_contrast":
        return adjust_brightness_contrast(b, value1, value2, mode)
    if name == "random_brightness_contrast":
        return random_brightness_contrast(b, value1, value2, mode, rng)
    if name in ("mean_filter", "gaussian_blur", "median_filter", "erode", "dilate"):
        return globals()[name](b, int(value1 or 3))
    if name == "nl_denoise_gray":
        return nl_denoise_gray(b, value1)
    if name == "add_salt_pepper_noise":
        return add_salt_pepper_noise(b, value1, rng=rng)
    raise ValueError(f"unknown preprocessing op {name!r}")
