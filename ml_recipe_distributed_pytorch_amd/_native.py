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


_DEBUG_DIR = os.path.join(_PKG_DIR, "_debug")   # in-tree (travels to the GPU box; csrc/build/ does not)


def _load(name: str, directory: str = _PKG_DIR):
    with _lock:
        ck = (name, directory)
        if ck in _cache:
            return _cache[ck]
        hits = sorted(glob.glob(os.path.join(directory, name + "*.so")))
        if not hits:
            _cache[ck] = None
            return None
        import torch  # noqa: F401  (kernels lib resolves libamdhip64/librccl/libtorch from torch's lib dir)
        spec = importlib.util.spec_from_file_location(name, hits[0])
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _cache[ck] = mod
        return mod


class _SyncedKernels:
    """Debug-build proxy: every kernel entry point is followed by a device synchronisation, so an
    ``HQ_DASSERT`` trap or a memory fault is reported against the op that caused it.  Not while the current
    stream is being captured into a graph (a synchronisation there is illegal; the replay reports faults)."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        attr = getattr(self._mod, name)
        if type(attr).__name__ != "builtin_function_or_method":
            return attr

        def call(*args, **kwargs):
            import torch
            out = attr(*args, **kwargs)
            if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
                return out
            if os.environ.get("HQ_DEBUG_NOSYNC", "0") == "1":   # lab: the debug kernels without the serialisation
                return out
            only, skip = os.environ.get("HQ_DEBUG_SYNC_ONLY"), os.environ.get("HQ_DEBUG_SYNC_SKIP")
            if (only and name not in only.split(",")) or (skip and name in skip.split(",")):   # lab bisection
                return out
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError(f"HIP kernel op {name!r} failed in the debug build: {e}") from e
            return out

        return call


def debug_enabled() -> bool:
    return os.environ.get("HQ_KERNELS_DEBUG", "0") == "1"


def kernels():
    if debug_enabled():
        mod = _load("_hq_kernels", _DEBUG_DIR)
        if mod is None:
            raise RuntimeError("HQ_KERNELS_DEBUG=1 but the debug kernel library is not built. Run "
                               "`python -m ml_recipe_distributed_pytorch_amd.csrc.build --kernels --debug`.")
        return _SyncedKernels(mod)
    # HQ_KERNELS_DIR: load an alternative release build (A/B of two kernel variants in one GPU call)
    mod = _load("_hq_kernels", os.environ.get("HQ_KERNELS_DIR", _PKG_DIR))
    if mod is None:
        raise RuntimeError(
            "HIP kernel library _hq_kernels.so is not built. Run `python -m ml_recipe_distributed_pytorch_amd.csrc.build` "
            "(or __graft_entry__.build()) before running on the GPU.")
    if os.environ.get("HQ_SYNC_PROXY", "0") == "1":   # lab: the release kernels behind the debug build's per-op sync
        return _SyncedKernels(mod)
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
