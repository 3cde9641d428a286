"""Native build driver (no setuptools/hipify): compiles in-tree, in parallel, with content caching.

* ``_hq_kernels<ext>.so`` — ``kernels/*.hip`` + ``runtime/*.cpp`` + ``bindings.cpp`` compiled by
  ``hipcc --offload-arch=gfx950`` and linked against torch + librccl.
* ``_hq_host<ext>.so``    — ``host/*.cpp`` (pure C++17 + pybind11, g++), no GPU dependency.

Usage: ``python -m ml_recipe_distributed_pytorch_amd.csrc.build [--host] [--kernels] [-j N] [--force] [--debug]``
"""
from __future__ import annotations

import argparse
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import List

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
BUILD = os.path.join(HERE, "build")
DEBUG_DIR = os.path.join(PKG, "_debug")   # HQ_KERNELS_DEBUG=1 loads it (_native); in-tree so it reaches the GPU box
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIPCC = os.path.join(ROCM, "bin", "hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _sh(cmd: List[str]):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


def _digest(paths: List[str], flags: List[str]) -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def _headers() -> List[str]:
    inc = os.path.join(HERE, "include")
    return sorted(os.path.join(inc, f) for f in os.listdir(inc) if f.endswith(".h"))


def _compile(src: str, flags: List[str], compiler: str, force: bool, deps: List[str] = ()) -> str:
    os.makedirs(BUILD, exist_ok=True)
    key = _digest([src] + _headers() + list(deps), flags + [compiler])
    obj = os.path.join(BUILD, os.path.basename(src) + f".{key}.o")
    if force or not os.path.exists(obj):
        _sh([compiler] + flags + ["-c", src, "-o", obj + ".tmp"])
        os.replace(obj + ".tmp", obj)
    return obj


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    incs = ce.include_paths(device_type="cuda")
    libdir = os.path.join(os.path.dirname(torch.__file__), "lib")
    return incs, libdir


_PROD_PKG = PKG


def build_kernels(jobs: int = 8, force: bool = False, verbose: bool = True, debug: bool = False,
                  lab_defines: List[str] = ()) -> str:
    """Release build → ``<pkg>/_hq_kernels<ext>``.  ``debug=True`` adds ``-DHQ_DEBUG`` (device-side
    ``HQ_DASSERT`` bounds checks, host line info) and writes ``<pkg>/_debug/_hq_kernels<ext>``,
    which ``_native`` loads instead when ``HQ_KERNELS_DEBUG=1``.

    ``lab_defines`` (``-D...``; tools/build_ab_lib.py only) are lab switches such as ``HQ_EPI_DIAG`` whose builds
    give WRONG results by design: they are refused for the production library path, and nothing is read from
    the environment, so a lab setting left in a shell can never reach the library training loads."""
    if lab_defines and os.path.realpath(PKG) == os.path.realpath(_PROD_PKG):
        raise RuntimeError(f"lab defines {list(lab_defines)} refused for the production kernel library {PKG}")
    if os.environ.get("HQ_KERNEL_CFLAGS"):
        print("[hq-build] note: HQ_KERNEL_CFLAGS is ignored (pass lab defines to tools/build_ab_lib.py)",
              file=sys.stderr)
    incs, torch_lib = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I" + os.path.join(HERE, "include"),
              "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result"]
    if debug:
        common += ["-DHQ_DEBUG=1", "-g1"]
    # lab / A-B builds only (tools/build_ab_lib.py, output outside the package): e.g. -DHQ_EPI_DIAG=1
    bad = [f for f in lab_defines if not f.startswith("-D")]
    if bad:
        raise ValueError(f"lab_defines must be -D flags: {bad}")
    common += list(lab_defines)
    kernel_srcs = sorted(os.path.join(HERE, "kernels", f) for f in os.listdir(os.path.join(HERE, "kernels"))
                         if f.endswith(".hip"))
    runtime_srcs = sorted(os.path.join(HERE, "runtime", f) for f in os.listdir(os.path.join(HERE, "runtime"))
                          if f.endswith(".cpp"))
    torch_flags = (["-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_hq_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
                    "-D_GLIBCXX_USE_CXX11_ABI=1", "-O2", "-fPIC", "-std=c++17", "-I" + os.path.join(HERE, "include"),
                    "-I" + py_inc, "-D__HIP_PLATFORM_AMD__=1", "-Wno-unused-result", "-Wno-deprecated-declarations"]
                   + ["-I" + p for p in incs])
    jobs_list = [(s, common, HIPCC) for s in kernel_srcs]
    jobs_list += [(s, ["-O3", "-fPIC", "-std=c++17", "-I" + os.path.join(HERE, "include"), "-I" + os.path.join(ROCM, "include"),
                       "-D__HIP_PLATFORM_AMD__=1"], HIPCC) for s in runtime_srcs]
    jobs_list.append((os.path.join(HERE, "bindings.cpp"), torch_flags, HIPCC))
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda a: _compile(a[0], a[1], a[2], force), jobs_list))
    out = os.path.join(PKG, "_hq_kernels" + EXT)
    if debug:
        os.makedirs(DEBUG_DIR, exist_ok=True)
        out = os.path.join(DEBUG_DIR, "_hq_kernels" + EXT)
    link = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp"] + objs + [
        "-L" + torch_lib, "-Wl,-rpath," + torch_lib, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip",
        "-ltorch_python", "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-lrccl"]
    _sh(link)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[hq-build] {out}")
    return out


def build_diag(verbose: bool = True) -> str:
    """``tools/diag/_hq_diag.so``: diagnostic kernels that are not part of the production library (the CU-hog
    spin kernel of the GEMM schedule contention test), plain C ABI for ctypes."""
    src = os.path.join(os.path.dirname(PKG), "tools", "diag", "cu_hog.hip")
    out = os.path.join(os.path.dirname(src), "_hq_diag.so")
    obj = _compile(src, ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}"], HIPCC, False)
    _sh([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out + ".tmp", obj,
         "-L" + os.path.join(ROCM, "lib"), "-lamdhip64"])
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[hq-build] {out}")
    return out


def _unicode_tables() -> str:
    gen_dir = os.path.join(BUILD, "gen")
    os.makedirs(gen_dir, exist_ok=True)
    out = os.path.join(gen_dir, "unicode_tables.inc")
    if not os.path.exists(out):
        _sh([sys.executable, os.path.join(HERE, "host", "gen_unicode.py"), out + ".tmp"])
        os.replace(out + ".tmp", out)
    return out


def build_host(jobs: int = 8, force: bool = False, verbose: bool = True) -> str:
    import pybind11
    host_dir = os.path.join(HERE, "host")
    tables = _unicode_tables()
    srcs = sorted(os.path.join(host_dir, f) for f in os.listdir(host_dir) if f.endswith(".cpp"))
    flags = ["-O3", "-fPIC", "-std=c++17", "-pthread", "-I" + host_dir, "-I" + os.path.dirname(tables),
             "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-fvisibility=hidden"]
    cxx = shutil.which("g++") or "c++"
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(lambda s: _compile(s, flags, cxx, force, [tables, os.path.join(host_dir, "hq_host.h")]),
                           srcs))
    out = os.path.join(PKG, "_hq_host" + EXT)
    _sh([cxx, "-shared", "-pthread", "-o", out + ".tmp"] + objs)
    os.replace(out + ".tmp", out)
    if verbose:
        print(f"[hq-build] {out}")
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--host", action="store_true")
    ap.add_argument("--kernels", action="store_true")
    ap.add_argument("-j", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--debug", action="store_true", help="kernels with HQ_DASSERT checks into <pkg>/_debug/")
    a = ap.parse_args(argv)
    both = not a.host and not a.kernels
    if a.host or both:
        build_host(a.j, a.force)
    if a.kernels or both:
        build_kernels(a.j, a.force, debug=a.debug)
        build_diag()


if __name__ == "__main__":
    main()
