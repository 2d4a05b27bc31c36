"""Node / device status — replaces ``GET /runtime/kubernetes/``.

Reference (C31, apps/runtime/views.py:76-187): SSH to the k8s master, run
``kubectl describe nodes`` and hand-parse the text into ``{Conditions, Addresses,
Capacity, Allocatable, System Info, Non-terminated Pods}`` (API.md:344-447).

Here the same top-level keys are produced for the local node from ``amdsmi`` (the
AMD SMI library: per-GPU utilisation, VRAM, temperature, power — no HIP context is
created, so the API process stays GPU-free) plus ``psutil``; "Non-terminated Pods"
lists the running training jobs with their GPU slots.
"""
from __future__ import annotations

import os
import platform
import socket
import time
from typing import Any, Dict, List, Optional


_TOPOLOGY: List[Any] = []   # [src][dst] link type of the last _gpus() scan (None on the diagonal)


def _gpus() -> List[Dict[str, Any]]:
    out: List[Dict[str, Any]] = []
    try:
        import amdsmi
    except Exception:
        return out
    try:
        amdsmi.amdsmi_init()
    except Exception:
        return out
    try:
        for i, h in enumerate(amdsmi.amdsmi_get_processor_handles()):
            g: Dict[str, Any] = {"index": i}
            for key, fn in (("asic", "amdsmi_get_gpu_asic_info"), ("activity", "amdsmi_get_gpu_activity"),
                            ("vram", "amdsmi_get_gpu_vram_usage")):
                try:
                    g[key] = getattr(amdsmi, fn)(h)
                except Exception:
                    pass
            try:
                g["temperature_c"] = amdsmi.amdsmi_get_temp_metric(
                    h, amdsmi.AmdSmiTemperatureType.EDGE, amdsmi.AmdSmiTemperatureMetric.CURRENT)
            except Exception:
                pass
            # xGMI: per-link up/down status and the data-plane link metrics (the fabric the
            # peer-buffer collectives of parallel/xgmi.py and RCCL run over)
            for key, fn in (("xgmi_link_status", "amdsmi_get_gpu_xgmi_link_status"),
                            ("xgmi_info", "amdsmi_get_xgmi_info"),
                            ("link_metrics", "amdsmi_get_link_metrics")):
                try:
                    g[key] = getattr(amdsmi, fn)(h)
                except Exception:
                    pass
            out.append(_jsonable(g))
        handles = amdsmi.amdsmi_get_processor_handles()
        if len(handles) > 1 and out:
            topo = []
            for i, hs in enumerate(handles):
                row = []
                for j, hd in enumerate(handles):
                    if i == j:
                        row.append(None)
                        continue
                    try:
                        lt = amdsmi.amdsmi_topo_get_link_type(hs, hd)
                        row.append(_jsonable(lt))
                    except Exception:
                        row.append(None)
                topo.append(row)
            _TOPOLOGY[:] = topo
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:
            pass
    return out


def _jsonable(x):
    if isinstance(x, dict):
        return {str(k): _jsonable(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_jsonable(v) for v in x]
    if isinstance(x, (str, int, float, bool)) or x is None:
        return x
    return str(x)


def node_status(jobs: Optional[List[Dict[str, Any]]] = None) -> Dict[str, Any]:
    try:
        import psutil
        mem = psutil.virtual_memory()
        mem_total_kib, mem_avail_kib = mem.total // 1024, mem.available // 1024
    except Exception:
        mem_total_kib = mem_avail_kib = 0
    gpus = _gpus()
    host = socket.gethostname()
    return {
        "Conditions": [{"Type": "Ready", "Status": "True", "LastHeartbeatTime": time.strftime(
            "%a, %d %b %Y %H:%M:%S %z"), "Reason": "GpuRuntimeReady",
            "Message": f"{len(gpus)} AMD GPU(s) visible"}],
        "Addresses": {"Hostname": host},
        "Capacity": {"cpu": str(os.cpu_count() or 0), "memory": f"{mem_total_kib}Ki",
                     "amd.com/gpu": str(len(gpus))},
        "Allocatable": {"cpu": str(os.cpu_count() or 0), "memory": f"{mem_avail_kib}Ki",
                        "amd.com/gpu": str(len(gpus))},
        "System Info": {"Operating System": platform.system(), "Kernel Version": platform.release(),
                        "Architecture": platform.machine(), "Python": platform.python_version()},
        "GPUs": gpus,
        "Topology": list(_TOPOLOGY),
        "Non-terminated Pods": [
            {"Name": f"job-{j['id']}", "Model": j.get("model"), "State": j.get("state"), "GPU": j.get("gpu")}
            for j in (jobs or [])],
    }
