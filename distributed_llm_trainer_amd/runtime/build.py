"""In-tree build of the native host runtime (``runtime/_dlt_runtime.so``).

Plain C++17 (g++), C ABI, loaded with ctypes -- no torch headers, so it builds in
seconds and never depends on the torch ABI.  Rebuilt only when a source is newer.
``python -m distributed_llm_trainer_amd.runtime.build``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "_dlt_runtime.so")


def _cxx() -> str:
    for cand in (os.environ.get("CXX"), shutil.which("g++"), shutil.which("c++"), "/opt/rocm/llvm/bin/clang++"):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("no C++ compiler found")


def build(verbose: bool = True, extra=()) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.cpp")))
    deps = srcs + glob.glob(os.path.join(CSRC, "*.h"))
    if os.path.exists(LIB) and all(os.path.getmtime(s) <= os.path.getmtime(LIB) for s in deps):
        return LIB
    tmp = LIB + ".tmp"
    cmd = [_cxx(), "-O3", "-std=c++17", "-fPIC", "-shared", "-pthread", "-Wall", *extra, *srcs, "-o", tmp]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native runtime build failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, LIB)
    if verbose:
        print(f"[dlt-build] linked {LIB}", flush=True)
    return LIB


if __name__ == "__main__":
    build()
