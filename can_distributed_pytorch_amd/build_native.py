"""Build the native extension in-tree: hipcc --offload-arch=gfx950.

Every ``csrc/*.hip`` translation unit (kernels, no torch headers) and
``csrc/*.cpp`` (bindings / runtime: RCCL communicator, reducer) is compiled to
an object under ``build/`` and linked into
``can_distributed_pytorch_amd/_C.<abi>.so``.  Objects are rebuilt only when a
source or header is newer.  Usage: ``python -m can_distributed_pytorch_amd.build_native [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "native")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("CANNET_OFFLOAD_ARCH", "gfx950")


def ext_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def _newer(src_files, target) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(f) > t for f in src_files)


def _compile(src: str, headers, verbose=False) -> str:
    import pybind11
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if not _newer([src] + headers, obj):
        return obj
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-Wno-unused-result"]
    if src.endswith(".hip"):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-x", "hip", "-c", src, "-o", obj, "-munsafe-fp-atomics"] + common
    else:
        py_inc = sysconfig.get_paths()["include"]
        cmd = [HIPCC, "-c", src, "-o", obj, f"-I{pybind11.get_include()}", f"-I{py_inc}",
               "-D__HIP_PLATFORM_AMD__", "-fvisibility=hidden"] + common
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def build(jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, verbose), srcs))
    out = ext_path()
    if _newer(objs, out):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [
            f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", "-Wl,--no-undefined"]
        py_lib = sysconfig.get_config_var("LIBDIR")
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            # python symbols are resolved at import time; retry without --no-undefined
            cmd = [c for c in cmd if c != "-Wl,--no-undefined"]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"link failed\n{r.stdout}\n{r.stderr}")
        _ = py_lib
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("-v", action="store_true")
    a = ap.parse_args()
    print(build(a.j, a.v))
