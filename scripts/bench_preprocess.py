"""Throughput of the 14 preprocessing ops: batched HIP kernels (device-resident uint8
batch) vs the NumPy reference path, images/s.  The reference itself ran one OpenCV call
per image per op with a JPEG read+write around each (apps/preprocess/views.py:118-126)
and reported no number."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_server_amd.preprocess import gpu, ops_ref  # noqa: E402

OPS = [("flip_up_down", None), ("transpose_image", None), ("adjust_brightness_contrast", 1.3),
       ("random_brightness_contrast", 1.5), ("mean_filter", 3), ("gaussian_blur", 5), ("median_filter", 5),
       ("erode", 3), ("dilate", 3), ("equalize_hist", None), ("clahe", None), ("nl_denoise_gray", 10),
       ("add_salt_pepper_noise", 0.05)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000)
    ap.add_argument("--cpu-n", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    x = np.random.default_rng(0).integers(0, 256, (a.n, 28, 28)).astype(np.uint8)
    xd = torch.from_numpy(x).cuda()
    rows = []
    for name, v in OPS:
        rng = np.random.default_rng(0)
        gpu.apply_op(name, xd[:64], v, 10, rng=rng)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            gpu.apply_op(name, xd, v, 10, rng=rng)
        torch.cuda.synchronize()
        g = a.n * a.reps / (time.perf_counter() - t0)
        xc = x[: a.cpu_n]
        t0 = time.perf_counter()
        ops_ref.apply_op(name, xc, v, 10, rng=rng)
        c = a.cpu_n / (time.perf_counter() - t0)
        rows.append({"op": name, "gpu_img_per_s": round(g), "cpu_numpy_img_per_s": round(c),
                     "speedup": round(g / c, 1)})
        print(json.dumps(rows[-1]), flush=True)


if __name__ == "__main__":
    main()
