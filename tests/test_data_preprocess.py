"""Datasets, batch stream, the 14 image ops and the preprocessing pipeline (CPU).

Image-op golden values come from scipy.ndimage (OpenCV is not installed): border modes
map as REFLECT_101 -> 'mirror', REPLICATE -> 'nearest' (SURVEY.md §7.4-5).  The
end-to-end fixture is the reference's own 99-image set (test-data/test-pics.zip +
tag.json, copied to tests/fixtures, read with PIL/JSON only)."""
import json
import os
import zipfile

import numpy as np
import pytest
import scipy.ndimage as ndi
import torch

from cloud_server_amd.data.datasets import (ArrayDataset, load_dataset_for_model, load_mnist_dir,
                                            load_user_data, read_idx, synthetic_mnist, write_idx)
from cloud_server_amd.data.stream import BatchStream
from cloud_server_amd.preprocess import ops_ref, pipeline

FIX = os.path.join(os.path.dirname(__file__), "fixtures")


@pytest.fixture()
def fixture_dir(tmp_path):
    d = tmp_path / "data"
    with zipfile.ZipFile(os.path.join(FIX, "test-pics.zip")) as z:
        z.extractall(d)
    tag = tmp_path / "tag.json"
    tag.write_bytes(open(os.path.join(FIX, "tag.json"), "rb").read())
    return str(d), str(tag)


def _imgs(n=4, seed=0):
    return np.random.default_rng(seed).integers(0, 256, (n, 28, 28)).astype(np.uint8)


# ---------------------------------------------------------------- datasets
def test_user_data_fixture(fixture_dir):
    d, tag = fixture_dir
    ds = load_user_data(d, tag)
    assert len(ds) == 99 and ds.images.shape == (99, 784) and ds.images.dtype == np.uint8
    counts = np.bincount(ds.labels, minlength=10)
    assert counts[4] == 15 and counts[1] == 14 and counts[8] == 3
    tr, te = ds.split(0.8)
    assert len(tr) == 79 and len(te) == 20
    assert np.array_equal(tr.images, ds.images[:79])                  # ordered split


def test_idx_roundtrip(tmp_path):
    ds = synthetic_mnist(50, seed=1)
    write_idx(str(tmp_path / "train-images-idx3-ubyte"), ds.images.reshape(-1, 28, 28))
    write_idx(str(tmp_path / "train-labels-idx1-ubyte"), ds.labels.astype(np.uint8))
    assert np.array_equal(read_idx(str(tmp_path / "train-images-idx3-ubyte")).reshape(50, 784), ds.images)
    tr, te = load_mnist_dir(str(tmp_path))
    assert len(tr) == 50 and te is None
    assert np.array_equal(tr.labels, ds.labels)


def test_synthetic_is_deterministic_and_labelled():
    a, b = synthetic_mnist(100, seed=3), synthetic_mnist(100, seed=3)
    assert np.array_equal(a.images, b.images) and np.array_equal(a.labels, b.labels)
    assert set(np.unique(a.labels)) <= set(range(10))


def test_batch_stream_epoch_and_rank_shards():
    n, B = 100, 10
    seen = []
    for rank in range(2):
        bs = BatchStream(n, B, "cpu", seed=5, chunk=8, rank=rank, world=2)
        rows = []
        for _ in range(5):          # one epoch of this rank's half
            bs.before_step()
            rows.append(bs.current().clone())
        seen.append(torch.cat(rows))
    allidx = torch.cat(seen)
    assert sorted(allidx.tolist()) == list(range(n))   # disjoint, full coverage per epoch


# ---------------------------------------------------------------- image ops
def test_flips_and_transpose():
    x = _imgs()
    assert np.array_equal(ops_ref.flip_up_down(x), x[:, ::-1])
    assert np.array_equal(ops_ref.flip_left_right(x), x[:, :, ::-1])
    assert np.array_equal(ops_ref.transpose_image(x), np.rot90(x, 2, axes=(1, 2)))


def test_brightness_contrast():
    x = _imgs()
    y = ops_ref.adjust_brightness_contrast(x, 1.5, 10)
    assert np.array_equal(y, np.clip(np.rint(x * 1.5 + 10), 0, 255).astype(np.uint8))
    w = ops_ref.adjust_brightness_contrast(x, 1.5, 10, mode="wrap")
    assert np.array_equal(w, (np.trunc(x * 1.5 + 10).astype(np.int64) % 256).astype(np.uint8))
    r = ops_ref.random_brightness_contrast(x, 2.0, 20, rng=np.random.default_rng(0))
    assert r.shape == x.shape and r.dtype == np.uint8


@pytest.mark.parametrize("k", [3, 5])
def test_mean_filter_matches_scipy(k):
    x = _imgs()
    ref = ndi.uniform_filter(x.astype(np.float64), size=(1, k, k), mode="mirror")
    got = ops_ref.mean_filter(x, k).astype(np.int64)
    assert np.abs(got - np.rint(ref)).max() <= 1


@pytest.mark.parametrize("k", [3, 5, 7])
def test_gaussian_matches_scipy_correlate(k):
    x = _imgs()
    g = ops_ref.gaussian_kernel(k)
    assert abs(g.sum() - 1) < 1e-12
    k2 = np.outer(g, g)[None]
    ref = ndi.correlate(x.astype(np.float64), k2, mode="mirror")
    assert np.abs(ops_ref.gaussian_blur(x, k).astype(np.int64) - np.rint(ref)).max() <= 1


@pytest.mark.parametrize("k", [3, 5])
def test_median_erode_dilate_match_scipy(k):
    x = _imgs()
    assert np.array_equal(ops_ref.median_filter(x, k), ndi.median_filter(x, size=(1, k, k), mode="nearest"))
    assert np.array_equal(ops_ref.erode(x, k), ndi.grey_erosion(x, size=(1, k, k), mode="nearest"))
    assert np.array_equal(ops_ref.dilate(x, k), ndi.grey_dilation(x, size=(1, k, k), mode="nearest"))


def test_equalize_hist_properties():
    x = (_imgs(2) // 4 + 60).astype(np.uint8)      # narrow range 60..123
    y = ops_ref.equalize_hist(x)
    for i in range(2):
        assert y[i].max() == 255 and y[i].min() == 0
        order = np.argsort(x[i].ravel(), kind="stable")
        assert np.all(np.diff(y[i].ravel()[order].astype(int)) >= 0)   # monotone mapping
    c = np.full((1, 28, 28), 77, np.uint8)
    assert np.array_equal(ops_ref.equalize_hist(c), c)


def test_clahe_properties():
    x = _imgs(2)
    y = ops_ref.clahe(x)
    assert y.shape == x.shape and y.dtype == np.uint8
    c = np.full((1, 28, 28), 128, np.uint8)
    yc = ops_ref.clahe(c)
    assert np.ptp(yc) == 0


def test_nl_denoise_reduces_noise():
    rng = np.random.default_rng(0)
    clean = np.zeros((1, 28, 28)); clean[:, 8:20, 8:20] = 200
    noisy = np.clip(clean + rng.normal(0, 20, clean.shape), 0, 255).astype(np.uint8)
    den = ops_ref.nl_denoise_gray(noisy, 20)
    assert np.abs(den - clean).mean() < np.abs(noisy - clean).mean()
    const = np.full((1, 28, 28), 90, np.uint8)
    assert np.array_equal(ops_ref.nl_denoise_gray(const, 10), const)


def test_salt_pepper():
    x = np.full((3, 28, 28), 100, np.uint8)
    y = ops_ref.add_salt_pepper_noise(x, 0.1, rng=np.random.default_rng(1))
    changed = y != 100
    assert set(np.unique(y[changed])) <= {0, 255}
    assert 0.1 < changed.mean() < 0.25


def test_resize_bicubic():
    c = np.full((1, 56, 56), 131, np.uint8)
    assert np.array_equal(ops_ref.resize(c, 28), np.full((1, 28, 28), 131, np.uint8))
    x = _imgs(1)
    assert np.array_equal(ops_ref.resize(x, 28), x)
    # downscale by 2 of a smooth ramp stays a ramp (monotone along x)
    ramp = np.tile(np.linspace(0, 255, 56), (56, 1))[None].astype(np.uint8)
    r = ops_ref.resize(ramp, 28)[0]
    assert np.all(np.diff(r[10].astype(int)) >= 0)


def test_apply_op_by_ui_label():
    x = _imgs()
    for label, name in ops_ref.OP_MAP.items():
        y = ops_ref.apply_op(label, x, 3 if "滤波" in label or label in ("腐蚀", "膨胀", "高斯模糊") else None,
                             None, rng=np.random.default_rng(0))
        assert y.shape == x.shape and y.dtype == np.uint8, name
    with pytest.raises(ValueError):
        ops_ref.apply_op("nope", x)


# ---------------------------------------------------------------- pipeline
def test_pipeline_overlap_and_inplace(fixture_dir):
    d, tag = fixture_dir
    before = np.asarray(pipeline._read(os.path.join(d, "test1.jpg")))
    ops = [{"operationName": "上下翻转", "overlap": True},
           {"operationName": "左右翻转", "overlap": False}]
    tags = pipeline.run(d, tag, ops, backend="cpu", seed=0)
    assert len(tags) == 198
    assert tags["test1_copy.jpg"] == tags["test1.jpg"]
    assert json.load(open(tag)) == tags
    a = pipeline._read(os.path.join(d, "test1.jpg")).astype(int)
    # in-place left-right flip of the original (JPEG re-encode: allow small error)
    assert np.abs(a - before[:, ::-1].astype(int)).mean() < 6
    b = pipeline._read(os.path.join(d, "test1_copy.jpg")).astype(int)
    assert np.abs(b - before[::-1, ::-1].astype(int)).mean() < 6
    ds = load_user_data(d, tag)
    assert len(ds) == 198


def test_pipeline_rejects_unknown_op(fixture_dir):
    d, tag = fixture_dir
    with pytest.raises(ValueError):
        pipeline.run(d, tag, [{"operationName": "旋转"}], backend="cpu")


def test_copied_name():
    assert pipeline.copied_name("a/b/test1.jpg") == "a/b/test1_copy.jpg"
