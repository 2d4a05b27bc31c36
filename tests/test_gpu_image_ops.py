"""HIP image-op kernels (csrc/kernels/image_ops.hip) vs the NumPy reference ops_ref
(GPU only).  Exact equality except NL-means / resize (double exp & tap order: |d| <= 1)."""
import os
import shutil
import zipfile

import numpy as np
import pytest
import torch

from cloud_server_amd.preprocess import gpu, ops_ref, pipeline

pytestmark = pytest.mark.gpu
FIX = os.path.join(os.path.dirname(__file__), "fixtures")


def _imgs(n=64, h=28, w=28, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (n, h, w)).astype(np.uint8)


def _smooth(n=16, seed=1):
    """Digit-like images (smooth blobs) so NL-means weights are non-trivial."""
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:28, 0:28]
    out = np.zeros((n, 28, 28))
    for i in range(n):
        cy, cx, r = rng.uniform(8, 20), rng.uniform(8, 20), rng.uniform(4, 9)
        out[i] = 220 * np.exp(-((yy - cy) ** 2 + (xx - cx) ** 2) / (2 * r * r))
    return np.clip(out + rng.normal(0, 12, out.shape), 0, 255).astype(np.uint8)


EXACT = [
    ("flip_up_down", None, None), ("flip_left_right", None, None), ("transpose_image", None, None),
    ("adjust_brightness_contrast", 1.37, -12), ("adjust_brightness_contrast", 0.5, 40.5),
    ("mean_filter", 3, None), ("mean_filter", 5, None), ("mean_filter", 4, None),
    ("gaussian_blur", 3, None), ("gaussian_blur", 5, None), ("gaussian_blur", 7, None), ("gaussian_blur", 9, None),
    ("median_filter", 3, None), ("median_filter", 5, None), ("median_filter", 7, None),
    ("erode", 3, None), ("erode", 4, None), ("dilate", 3, None), ("dilate", 5, None),
    ("equalize_hist", None, None), ("clahe", None, None),
]


@pytest.mark.parametrize("name,v1,v2", EXACT)
def test_exact_ops(name, v1, v2):
    x = _imgs()
    ref = ops_ref.apply_op(name, x, v1, v2)
    got = gpu.apply_op(name, x, v1, v2)
    assert got.dtype == np.uint8 and got.shape == ref.shape
    assert np.array_equal(got, ref), (np.abs(got.astype(int) - ref).max(), (got != ref).mean())


def test_wrap_mode_and_random_draws_match():
    x = _imgs()
    assert np.array_equal(gpu.apply_op("adjust_brightness_contrast", x, 1.9, 30, mode="wrap"),
                          ops_ref.apply_op("adjust_brightness_contrast", x, 1.9, 30, mode="wrap"))
    for name, v1, v2 in [("random_brightness_contrast", 1.8, 25), ("add_salt_pepper_noise", 0.07, None)]:
        a = gpu.apply_op(name, x, v1, v2, rng=np.random.default_rng(11))
        b = ops_ref.apply_op(name, x, v1, v2, rng=np.random.default_rng(11))
        assert np.array_equal(a, b), name


def test_equalize_constant_and_two_level():
    c = np.full((3, 28, 28), 9, np.uint8)
    c[1, :5] = 200
    assert np.array_equal(gpu.apply_op("equalize_hist", c), ops_ref.equalize_hist(c))


def test_nlmeans_close():
    x = _smooth()
    ref = ops_ref.nl_denoise_gray(x, 15)
    got = gpu.apply_op("nl_denoise_gray", x, 15)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3


@pytest.mark.parametrize("hw", [(56, 56), (40, 33), (20, 20), (100, 64)])
def test_resize_close(hw):
    x = _imgs(8, *hw, seed=3)
    ref = ops_ref.resize(x, 28)
    got = gpu.resize(x, 28)
    d = np.abs(got.astype(int) - ref.astype(int))
    assert d.max() <= 1 and (d > 0).mean() < 1e-3


def test_device_resident_tensor_io():
    x = torch.from_numpy(_imgs(10)).cuda()
    y = gpu.apply_op("左右翻转", x)
    assert y.is_cuda and torch.equal(y.cpu(), torch.from_numpy(_imgs(10)[:, :, ::-1].copy()))


def test_infer_prep_kernel():
    x = _imgs(5, 20, 20)
    got = gpu.infer_prep(x).cpu().numpy()
    ref = np.zeros((5, 28, 28), np.float32)
    ref[:, 4:24, 4:24] = np.where(x > 150, 254.0, 0.0)
    assert np.array_equal(got, (ref / 255.0).reshape(5, 784).astype(np.float32))


def test_pipeline_gpu_equals_cpu(tmp_path):
    ops = [{"operationName": "上下翻转", "overlap": True},
           {"operationName": "高斯模糊", "value1": 5, "overlap": False},
           {"operationName": "随机对比度亮度调整", "value1": 1.5, "value2": 20, "overlap": True},
           {"operationName": "添加椒盐噪声", "value1": 0.03, "overlap": "true"},
           {"operationName": "CLAHE均衡化", "overlap": False}]
    res = {}
    for be in ("cpu", "gpu"):
        d = tmp_path / be
        with zipfile.ZipFile(os.path.join(FIX, "test-pics.zip")) as z:
            z.extractall(d / "data")
        shutil.copyfile(os.path.join(FIX, "tag.json"), d / "tag.json")
        tags = pipeline.run(str(d / "data"), str(d / "tag.json"), ops, backend=be, seed=5)
        res[be] = (tags, {n: pipeline._read(str(d / "data" / n)) for n in tags})
    assert res["cpu"][0] == res["gpu"][0] and len(res["cpu"][0]) == 99 * 4
    for n, a in res["cpu"][1].items():
        assert np.array_equal(a, res["gpu"][1][n]), n
