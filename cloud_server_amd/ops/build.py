"""Build the native libraries in-tree with hipcc for gfx950 (no hipify, no JIT cache).

* ``libcsa_kernels.so`` — the HIP/CDNA4 kernels (``csrc/kernels/*.hip``) and the xGMI
  peer-buffer collectives (``csrc/comm/*.hip``), C ABI, called
  through ctypes from ``ops.fused``.  Launchers take a ``hipStream_t`` and never
  allocate or synchronise, so they are captured into HIP graphs by the engine.
* ``libcsa_runtime.so`` — host-side C++ runtime pieces (``csrc/runtime/*.cpp``): the
  GPU-slot job scheduler used by the job manager.

Objects are rebuilt only when a source/header hash changes (stamp file next to the .so),
so ``build()`` on an up-to-date tree is instant.  Built ``.so`` files are git-ignored but
travel to the GPU box with the working tree.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from typing import List

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(PKG, "csrc")
LIBDIR = os.path.join(PKG, "_lib")
ARCH = os.environ.get("CSA_OFFLOAD_ARCH", "gfx950")
KERNEL_LIB = os.path.join(LIBDIR, "libcsa_kernels.so")
RUNTIME_LIB = os.path.join(LIBDIR, "libcsa_runtime.so")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (need ROCm)")


def _hash(files: List[str], extra: str) -> str:
    h = hashlib.sha256(extra.encode())
    for f in sorted(files):
        h.update(f.encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def _sources(sub: str, exts) -> List[str]:
    d = os.path.join(CSRC, sub)
    return sorted(os.path.join(d, f) for f in os.listdir(d) if f.endswith(exts))


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_kernels(verbose: bool = False, force: bool = False) -> str:
    srcs = _sources("kernels", (".hip",)) + _sources("comm", (".hip",))
    hdrs = _sources("kernels", (".h",)) + _sources("comm", (".h",))
    flags = ["-O3", "-fPIC", f"--offload-arch={ARCH}", "-std=c++17", "-ffp-contract=fast-honor-pragmas",
             "-Wno-unused-result"]
    stamp = _hash(srcs + hdrs, " ".join(flags))
    stamp_file = KERNEL_LIB + ".stamp"
    if not force and os.path.exists(KERNEL_LIB) and os.path.exists(stamp_file):
        if open(stamp_file).read().strip() == stamp:
            return KERNEL_LIB
    os.makedirs(os.path.join(LIBDIR, "obj"), exist_ok=True)
    hipcc = _hipcc()
    objs = [os.path.join(LIBDIR, "obj", os.path.basename(s) + ".o") for s in srcs]

    def compile_one(so) -> None:
        # per-object stamp: the source, every header (any may be included) and the flags,
        # so editing one kernel file recompiles that object only
        src, obj = so
        ostamp = _hash([src] + hdrs, " ".join(flags))
        sf = obj + ".stamp"
        if not force and os.path.exists(obj) and os.path.exists(sf) and open(sf).read().strip() == ostamp:
            return
        _run([hipcc, *flags, "-c", src, "-o", obj], verbose)
        with open(sf, "w") as f:
            f.write(ostamp)

    with cf.ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        list(ex.map(compile_one, zip(srcs, objs)))
    tmp = KERNEL_LIB + ".tmp"
    _run([hipcc, "-shared", f"--offload-arch={ARCH}", *objs, "-o", tmp], verbose)
    os.replace(tmp, KERNEL_LIB)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    return KERNEL_LIB


def build_runtime(verbose: bool = False, force: bool = False) -> str:
    srcs = _sources("runtime", (".cpp",))
    hdrs = _sources("runtime", (".h",))
    if not srcs:
        return ""
    flags = ["-O2", "-fPIC", "-std=c++17", "-shared", "-pthread"]
    stamp = _hash(srcs + hdrs, " ".join(flags))
    stamp_file = RUNTIME_LIB + ".stamp"
    if not force and os.path.exists(RUNTIME_LIB) and os.path.exists(stamp_file):
        if open(stamp_file).read().strip() == stamp:
            return RUNTIME_LIB
    os.makedirs(LIBDIR, exist_ok=True)
    cxx = shutil.which("g++") or shutil.which("c++")
    tmp = RUNTIME_LIB + ".tmp"
    _run([cxx, *flags, *srcs, "-o", tmp], verbose)
    os.replace(tmp, RUNTIME_LIB)
    with open(stamp_file, "w") as f:
        f.write(stamp)
    return RUNTIME_LIB


def build_all(verbose: bool = False, force: bool = False) -> None:
    build_kernels(verbose, force)
    build_runtime(verbose, force)


if __name__ == "__main__":
    build_all(verbose=True, force="--force" in sys.argv)
