"""Build the native extension in-tree: hipcc --offload-arch=gfx950.

Every ``csrc/*.hip`` translation unit (kernels, no torch headers) and
``csrc/*.cpp`` (bindings / runtime: RCCL communicator, reducer) is compiled to
an object under ``build/`` and linked into
``can_distributed_pytorch_amd/_C.<abi>.so``.  Objects are rebuilt only when a
source or header is newer.  Usage: ``python -m can_distributed_pytorch_amd.build_native [-j N]``.

``--asan`` builds the host-AddressSanitizer variant ``_C_asan`` (SURVEY §5 race
detection / sanitizers): the host C++ of the runtime (pybind bindings, RCCL
communicator, bucketed reducer) and the host side of every .hip translation
unit (launch stubs, planning code) compiled with ``-fsanitize=address``; GPU
code is NOT instrumented (``-Xarch_host``: device ASan is not available on this
pool).  Load it with ``CANNET_ASAN=1`` under the ASan runtime, see
``asan_env()`` / ``tests/test_asan_host.py`` (host-only paths: the ROCm ASan
runtime's HSA interceptor aborts HIP allocations on this XNACK-off pool).
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


def ext_path(asan: bool = False) -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, ("_C_asan" if asan else "_C") + suffix)


def asan_runtime() -> str:
    """Path of the clang ASan runtime matching hipcc (to LD_PRELOAD before python)."""
    r = subprocess.run([HIPCC, "-print-file-name=libclang_rt.asan-x86_64.so"], capture_output=True, text=True)
    return r.stdout.strip()


def asan_env(base=None) -> dict:
    """Environment for a child python that imports the ASan build (_C_asan)."""
    env = dict(os.environ if base is None else base)
    env["LD_PRELOAD"] = asan_runtime() + ((":" + env["LD_PRELOAD"]) if env.get("LD_PRELOAD") else "")
    # python itself is not instrumented: no leak report for the interpreter, runtime may not be first
    env["ASAN_OPTIONS"] = "detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:abort_on_error=1"
    env["CANNET_ASAN"] = "1"
    return env


def source_files():
    """Every file the extension is built from (kernels, runtime, headers), sorted."""
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")) +
                  glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc")))


def source_hash(files=None) -> str:
    """sha256 over (name, content) of the csrc/ sources: embedded in _C at build time and recomputed by
    ops/_ext.py at import, so a binary that does not match the tree's sources fails loudly."""
    import hashlib
    h = hashlib.sha256()
    for f in (files if files is not None else source_files()):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()


def extra_flags():
    # CANNET_EXTRA_HIPFLAGS: extra defines for A/B variant builds (scripts/dev/ab_variant_build.sh), e.g.
    # -DCANNET_DMA_ORDER_WG=0.  Objects of a flagged build live in their own directory (build/native_<hash>), so
    # setting or clearing the variable never mixes variant objects into the default build.
    return os.environ.get("CANNET_EXTRA_HIPFLAGS", "").split()


def build_dir(asan: bool = False) -> str:
    import hashlib
    fl = extra_flags()
    tag = ("_" + hashlib.sha256(" ".join(fl).encode()).hexdigest()[:10]) if fl else ""
    return BUILD + tag + ("_asan" if asan else "")


def _newer(src_files, target) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(f) > t for f in src_files)


ASAN_HOST = ["-fsanitize=address", "-fno-omit-frame-pointer", "-g"]


def _compile(src: str, headers, verbose=False, asan: bool = False) -> str:
    import pybind11
    bdir = build_dir(asan)
    obj = os.path.join(bdir, os.path.basename(src) + ".o")
    if not _newer([src] + headers, obj):
        return obj
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-Wno-unused-result"]
    common += extra_flags()
    if src.endswith(".hip"):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-x", "hip", "-c", src, "-o", obj, "-munsafe-fp-atomics"] + common
        if asan:   # host half only: each -fsanitize right after -Xarch_host
            cmd += [f for flag in ASAN_HOST for f in ("-Xarch_host", flag)]
    else:
        py_inc = sysconfig.get_paths()["include"]
        cmd = [HIPCC, "-c", src, "-o", obj, f"-I{pybind11.get_include()}", f"-I{py_inc}",
               "-D__HIP_PLATFORM_AMD__", "-fvisibility=hidden"] + common
        if asan:
            cmd += ASAN_HOST + ["-DCAN_MODULE_NAME=_C_asan"]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{r.stdout}\n{r.stderr}")
    return obj


def _hash_unit(bdir: str) -> str:
    """build/native*/src_hash.cpp: the source hash and build flags as C strings (rewritten only when they change)."""
    path = os.path.join(bdir, "src_hash.cpp")
    text = ('extern "C" const char* can_src_hash() { return "%s"; }\n'
            'extern "C" const char* can_build_flags() { return "%s"; }\n'
            % (source_hash(), " ".join(extra_flags()).replace("\\", "\\\\").replace('"', '\\"')))
    old = open(path).read() if os.path.exists(path) else None
    if old != text:
        with open(path, "w") as f:
            f.write(text)
    return path


def build(jobs: int = 8, verbose: bool = False, asan: bool = False) -> str:
    bdir = build_dir(asan)
    os.makedirs(bdir, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(CSRC, "*.inc"))
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    srcs.append(_hash_unit(bdir))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, headers, verbose, asan), srcs))
    out = ext_path(asan)
    if _newer(objs, out):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out] + objs + [
            f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", "-Wl,--no-undefined"]
        if asan:
            cmd += ["-fsanitize=address", "-shared-libasan"]
        py_lib = sysconfig.get_config_var("LIBDIR")
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            # python symbols are resolved at import time; retry without --no-undefined, but never with an undefined
            # symbol of our own (can_* / can::): that would only surface as an import error on the GPU box
            import re
            if re.search(r"undefined reference to `[^']*can_", r.stderr):
                raise RuntimeError(f"link failed: undefined extension symbol\n{r.stderr[-4000:]}")
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
    ap.add_argument("--asan", action="store_true", help="host-AddressSanitizer variant _C_asan")
    a = ap.parse_args()
    print(build(a.j, a.v, a.asan))
