"""The thread fact the RCCL configuration relies on.

``parallel.dist.rccl_env_defaults`` sets ``TORCH_NCCL_BLOCKING_WAIT=1`` and
``utils.graphs.wait_retired`` returns at once in that mode, on the premise that this
torch build then starts NO process-group watchdog thread — the only thread that ever
queried a collective's end event from outside the capturing thread (the round-5
``hipErrorCapturedEvent`` aborts: ``Watchdog::runLoop -> WorkNCCL::isCompleted``).  Measured
here on the installed torch, in fresh processes (the variable is read when the group is
created): with blocking wait, ``pt_nccl_watchdg`` / ``pt_nccl_heartbt`` are absent; without
it, both exist (so the probe can see them)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "scripts", "mb", "watchdog_probe.py")


def _probe(blocking: str) -> dict:
    env = dict(os.environ, TORCH_NCCL_BLOCKING_WAIT=blocking)
    out = subprocess.run([sys.executable, PROBE, "child"], env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    return json.loads(line)


def test_blocking_wait_starts_no_watchdog_thread():
    on, off = _probe("1"), _probe("0")
    assert "pt_nccl_watchdg" in off["all_threads"] and "pt_nccl_heartbt" in off["all_threads"], off
    assert not any("nccl" in t for t in on["all_threads"]), on       # no watchdog, no heartbeat


def test_package_default_is_blocking_wait(monkeypatch):
    from cloud_server_amd.parallel.dist import rccl_env_defaults
    monkeypatch.delenv("TORCH_NCCL_BLOCKING_WAIT", raising=False)
    rccl_env_defaults()
    assert os.environ["TORCH_NCCL_BLOCKING_WAIT"] == "1"
    from cloud_server_amd.utils.graphs import wait_retired
    assert wait_retired() is None                                     # nothing to wait for
