"""Training worker entrypoint (one process per GPU rank).

Replaces the reference's shipped TF program started with ``nohup python
construct_distribute.py --job_name=ps|worker --task_index=i ...`` inside docker
containers over SSH (apps/construction/util/cmd.py:54-70, views.py:125-141).

    python -m cloud_server_amd.runtime.worker --model-dir DIR [--datatype file|url]
           [--device cuda:0|cpu] [--backend auto|hip|torch]

Reads ``DIR/model.json`` (the reference DSL, plus an optional ``options`` block), trains
with ``runtime.trainer.run_job`` and exits 0 (done / stopped / paused) or 1 (failed).
Data-parallel jobs run this module under ``torch.distributed.run`` (or
``runtime.jobs``): ranks come from RANK / WORLD_SIZE / LOCAL_RANK, one GPU each.
"""
from __future__ import annotations

import argparse
import json
import os
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="cloud_server_amd.runtime.worker")
    ap.add_argument("--model-dir", required=True)
    ap.add_argument("--datatype", default="file", choices=["file", "url"])
    ap.add_argument("--device", default=None)
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"])
    a = ap.parse_args(argv)

    import torch
    from ..parallel.dist import init_distributed, shutdown
    from .trainer import run_job, write_status

    with open(os.path.join(a.model_dir, "model.json"), encoding="utf-8") as f:
        config = json.load(f)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    ctx = None
    if world > 1:
        ctx = init_distributed("cuda" if (a.device or "").startswith("cuda") or
                               (a.device is None and torch.cuda.is_available()) else "cpu")
    try:
        res = run_job(a.model_dir, config, a.datatype, device=a.device if world == 1 else None,
                      ctx=ctx, backend=a.backend)
        print(json.dumps(res), flush=True)
        return 0
    except Exception as exc:  # status.json already records the failure
        print(f"worker failed: {exc!r}", file=sys.stderr, flush=True)
        return 1
    finally:
        if ctx is not None:
            shutdown(ctx)


if __name__ == "__main__":
    sys.exit(main())
