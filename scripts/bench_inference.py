#!/usr/bin/env python3
"""Server-side latency of the warm inference path (POST /construct/inference/<m>/ minus
HTTP): PNG decode + the reference's image prep (construct_inference.py:312-330) + one
forward pass of the cached model on the device + argmax.  The reference started a new
python3 + TF process per request (apps/construction/views.py:231-250) and reported no
number; BASELINE.md's target is <= 2 ms.  Also times a 256-image batch."""
import io
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cloud_server_amd.data.datasets import synthetic_mnist  # noqa: E402
from cloud_server_amd.models.dsl import SAMPLE_CONFIG  # noqa: E402
from cloud_server_amd.runtime.trainer import run_job  # noqa: E402
from cloud_server_amd.serve.inference import InferenceService  # noqa: E402


def main() -> int:
    from PIL import Image
    ds = synthetic_mnist(4000, seed=0)
    mdir = tempfile.mkdtemp(prefix="csa_inf_")
    cfg = json.loads(json.dumps(SAMPLE_CONFIG))
    cfg.update(iter=200, learning_rate=0.01, optimizer_name="AdamOptimizer")
    cfg["options"] = {"log_every": 100, "ckpt_every": 200}
    run_job(mdir, cfg, device="cuda:0" if torch.cuda.is_available() else "cpu", data=ds.split(0.9))
    pngs = []
    for i in range(300):
        b = io.BytesIO()
        Image.fromarray(ds.images[i].reshape(28, 28)).save(b, format="PNG")
        pngs.append(b.getvalue())
    svc = InferenceService()
    for p in pngs[:20]:
        svc.predict(mdir, p)                      # warm: model load, kernels, allocator
    lat = []
    for p in pngs[20:]:
        t0 = time.perf_counter()
        out = svc.predict(mdir, p)
        lat.append((time.perf_counter() - t0) * 1e3)
        assert out["result"] == "success"
    t0 = time.perf_counter()
    svc.predict_many(mdir, pngs[:256])
    tb = (time.perf_counter() - t0) * 1e3
    lat = np.array(lat)
    ent = svc._entry(mdir)
    dev_ips = None
    if ent.hip is not None:                        # device predictor alone: 256-image buckets
        x = ds.images[:256]
        ent.hip.predict_u8(x, "mnist")
        t0 = time.perf_counter()
        for _ in range(200):
            ent.hip.predict_u8(x, "mnist")
        dev_ips = round(256 * 200 / (time.perf_counter() - t0))
    print(json.dumps({"device": str(svc.device), "backend": svc.backend(mdir),
                      "hip_predictor_images_per_s_b256": dev_ips,
                      "single_image_ms_p50": round(float(np.median(lat)), 3),
                      "single_image_ms_p99": round(float(np.percentile(lat, 99)), 3),
                      "single_image_ms_mean": round(float(lat.mean()), 3),
                      "batch256_ms": round(tb, 3), "cache_hits": svc.hits, "cache_misses": svc.misses}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
