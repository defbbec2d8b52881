"""In-tree build of the gfx950 HIP kernel library (no hipify, no torch JIT cache).

Every ``ops/csrc/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` into an
object file and linked into ``ops/_dlt_kernels.so``, a plain C-ABI shared library
loaded with ctypes (``ops/hip.py``).  Incremental: a source is rebuilt only when it
or a header is newer than its object.  ``python -m distributed_llm_trainer_amd.ops.build``.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "_dlt_kernels.so")
DEBUG_LIB = os.path.join(HERE, "_dlt_kernels_debug.so")  # DLT_DEBUG bounds checks (DLT_KERNEL_DEBUG=1)
GEMM_SRC = os.path.join(HERE, "csrc_gemm", "gemm_planner.cpp")
GEMM_LIB = os.path.join(HERE, "_dlt_gemm.so")
ARCH = os.environ.get("DLT_OFFLOAD_ARCH", "gfx950")

# -amdgpu-mfma-vgpr-form: keep MFMA accumulators in arch VGPRs (gfx950 has a unified
# VGPR/AGPR file) -- removes v_accvgpr_read/write copies around the attention softmax.
CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wno-unused-result",
            "-mllvm", "-amdgpu-mfma-vgpr-form"]


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the MI355X kernels)")


def _needs(src: str, obj: str, headers) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or any(os.path.getmtime(hh) > t for hh in headers)


def _compile(src: str, obj: str, extra):
    cmd = [hipcc(), *CXXFLAGS, *extra, "-I", CSRC, "-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr[-6000:]}")
    return obj


def build(verbose: bool = True, jobs: int = 0, extra=(), debug: bool = False) -> str:
    """Compile every ``csrc/*.hip`` for gfx950 and link ``_dlt_kernels.so`` (or, with
    ``debug``, ``_dlt_kernels_debug.so``: -DDLT_DEBUG device bounds checks, -g)."""
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    lib_path = DEBUG_LIB if debug else LIB
    if debug:
        extra = (*extra, "-DDLT_DEBUG", "-g")
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s)[:-4] + (".dbg.o" if debug else ".o"))
        objs.append(o)
        if _needs(s, o, headers):
            todo.append((s, o))
    if todo:
        jobs = jobs or min(len(todo), max(1, min(8, (os.cpu_count() or 2))))
        if verbose:
            print(f"[dlt-build] compiling {len(todo)} HIP sources for {ARCH} (-j{jobs})", flush=True)
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            futs = [ex.submit(_compile, s, o, list(extra)) for s, o in todo]
            for f in futs:
                f.result()
    relink = not os.path.exists(lib_path) or any(os.path.getmtime(o) > os.path.getmtime(lib_path) for o in objs)
    if relink:
        tmp = lib_path + ".tmp"
        cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-4000:]}")
        os.replace(tmp, lib_path)
        if verbose:
            print(f"[dlt-build] linked {lib_path}", flush=True)
    build_gemm(verbose)
    return lib_path


def build_gemm(verbose: bool = True) -> str:
    """Host-side hipBLASLt planner library (links libhipblaslt.so.1; at run time it binds
    to the copy already loaded by torch -- same SONAME)."""
    if os.path.exists(GEMM_LIB) and os.path.getmtime(GEMM_LIB) >= os.path.getmtime(GEMM_SRC):
        return GEMM_LIB
    tmp = GEMM_LIB + ".tmp"
    cmd = [hipcc(), "-O2", "-fPIC", "-shared", "-std=c++17", "-Wno-unused-result", GEMM_SRC, "-o", tmp,
           "-L/opt/rocm/lib", "-lhipblaslt"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"gemm planner build failed:\n{r.stderr[-4000:]}")
    os.replace(tmp, GEMM_LIB)
    if verbose:
        print(f"[dlt-build] linked {GEMM_LIB}", flush=True)
    return GEMM_LIB


if __name__ == "__main__":
    build(verbose=True, debug="--debug" in sys.argv)
    sys.exit(0)
