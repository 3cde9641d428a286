"""Loader for the in-tree native libraries.

* ``_hq_kernels*.so`` — HIP/CDNA4 kernels (gfx950) + RCCL flat-bucket reducer + torch bindings.
  Built by ``csrc/build.py`` with ``hipcc --offload-arch=gfx950``.
* ``_hq_host*.so``    — pure C++ host runtime (WordPiece tokenizer, dummy-batch synthesiser,
  CRC32C, sentence splitter), pybind11, built with g++.

GPU ops never fall back silently: if the kernel library is missing while a CUDA tensor reaches
a fused op, ``kernels()`` raises with the build command.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys
import threading

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_lock = threading.Lock()
_cache = {}


def _load(name: str):
    with _lock:
        if name in _cache:
            return _cache[name]
        hits = sorted(glob.glob(os.path.join(_PKG_DIR, name + "*.so")))
        if not hits:
            _cache[name] = None
            return None
        import torch  # noqa: F401  (kernels lib resolves libamdhip64/librccl/libtorch from torch's lib dir)
        spec = importlib.util.spec_from_file_location(name, hits[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _cache[name] = mod
        return mod


def kernels():
    mod = _load("_hq_kernels")
    if mod is None:
        raise RuntimeError(
            "HIP kernel library _hq_kernels.so is not built. Run `python -m ml_recipe_distributed_pytorch_amd.csrc.build` "
            "(or __graft_entry__.build()) before running on the GPU.")
    return mod


def kernels_available() -> bool:
    return _load("_hq_kernels") is not None


def host():
    mod = _load("_hq_host")
    if mod is None:
        raise RuntimeError("Host runtime library _hq_host.so is not built. Run "
                           "`python -m ml_recipe_distributed_pytorch_amd.csrc.build --host`.")
    return mod


def host_available() -> bool:
    return _load("_hq_host") is not None


def reset_cache():
    with _lock:
        _cache.clear()
