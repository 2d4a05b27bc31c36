import faulthandler
import os
import sys

import pytest

# (see parallel/dist.py:init_distributed: RCCL works captured into HIP graphs must not
# share end events with eager works the process-group watchdog still polls)
os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# A dup of the real stderr taken before pytest's per-test capture redirects fd 2: output
# written here survives a native abort (SIGABRT inside HIP/RCCL) that loses captured text.
_REAL_ERR = None


@pytest.fixture(autouse=True)
def _gpu_test_cleanup(request):
    """After a @gpu test: retire the inference services it left (their HIP graphs and
    batcher threads) and collect its garbage here, so nothing of it is destroyed while a
    later test captures a graph."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import gc
    import torch
    if not torch.cuda.is_available():
        return
    from cloud_server_amd.serve import inference
    inference.close_all()
    gc.collect()
    torch.cuda.synchronize()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.hookimpl(trylast=True)
def pytest_sessionstart(session):
    """Dump only the faulting thread on a fatal signal, so the test frames stay inside a
    short output tail (pytest's own handler dumps every thread plus the extension list)."""
    global _REAL_ERR
    try:
        _REAL_ERR = os.dup(sys.__stderr__.fileno())
    except (AttributeError, OSError, ValueError):
        _REAL_ERR = None
        return
    faulthandler.enable(file=_REAL_ERR, all_threads=False)


def pytest_runtest_logstart(nodeid, location):
    if _REAL_ERR is not None:
        os.write(_REAL_ERR, f"[csa-test] {nodeid}\n".encode())
    if os.environ.get("CSA_FATAL_TRACE", "0") == "1":
        # native backtrace of the thread that aborts (HIP / RCCL / c10d), chained in front
        # of faulthandler's Python stack (csrc/runtime/fatal_trace.cpp); re-armed before
        # every test because runtimes initialised by a test may install their own handlers
        import ctypes
        from cloud_server_amd.ops import build as _b
        ctypes.CDLL(_b.build_runtime()).csa_install_fatal_trace()


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
