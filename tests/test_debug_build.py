"""Debug build of the HIP kernels ("debug build of the HIP kernels with bounds asserts").

``csrc/build.py --debug`` compiles every kernel with ``-DHQ_DEBUG`` so the ``HQ_DASSERT`` device checks
(embedding ids vs table sizes, GEMM tile bounds, attention length) are live, and ``HQ_KERNELS_DEBUG=1``
makes ``_native.kernels()`` load that library behind a proxy that synchronises after every op.
The CPU test only cross-compiles (a failing assertion traps the GPU queue, which is never provoked on
the shared GPU pool); the GPU test runs valid inputs through the debug library.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ml_recipe_distributed_pytorch_amd", "csrc")
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")
def test_debug_kernels_compile(tmp_path):
    src = os.path.join(CSRC, "kernels", "norm.hip")
    out = tmp_path / "norm_debug.o"
    r = subprocess.run([HIPCC, "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950", "-DHQ_DEBUG=1",
                        "-I" + os.path.join(CSRC, "include"), "-c", src, "-o", str(out)],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0, r.stdout
    assert out.stat().st_size > 0


def test_debug_proxy_syncs_and_names_op(monkeypatch):
    from ml_recipe_distributed_pytorch_amd import _native

    calls = []

    class Fake:
        Reducer = type("Reducer", (), {})
        op = len  # a builtin, like the pybind11 entry points

    proxy = _native._SyncedKernels(Fake)
    monkeypatch.setattr("torch.cuda.synchronize", lambda: calls.append("sync"))
    assert proxy.op([1, 2]) == 2
    assert calls == ["sync"]
    assert proxy.Reducer is Fake.Reducer  # classes pass through unwrapped


_GPU_SNIPPET = r"""
import torch
from ml_recipe_distributed_pytorch_amd import _native, ops
assert _native.debug_enabled()
k = _native.kernels()
assert type(k).__name__ == "_SyncedKernels"
dev = torch.device("cuda")
T, H = 512, 768
ids = torch.randint(0, 1000, (T,), device=dev)
pids = torch.arange(T, device=dev) % 512
tids = torch.zeros(T, dtype=torch.long, device=dev)
ww = torch.randn(1000, H, device=dev).bfloat16()
wp = torch.randn(512, H, device=dev).bfloat16()
wt = torch.randn(2, H, device=dev).bfloat16()
g = torch.ones(H, device=dev)
b = torch.zeros(H, device=dev)
y, mu, rs = k.embed_fwd(ids, pids, tids, ww, wp, wt, g, b, 1e-12, 0.0, 1, 1)
# 77ab202 regression: the flat layout (seq_len 0 -> L = T = 512 rows, P = 64 positions, L > P): the position
# partial rows exist for l < min(L, P) only — the debug build's asserts check every partial-row, carry-slot and
# word-row index of the backward
P = 64
pf = torch.randint(0, P, (T,), device=dev)
y2, mu2, rs2 = k.embed_fwd(ids, pf, tids, ww, wp[:P].contiguous(), wt, g, b, 1e-12, 0.1, 1, 1)
outs = [torch.zeros(1000, H, device=dev), torch.zeros(P, H, device=dev), torch.zeros(2, H, device=dev),
        torch.zeros(H, device=dev), torch.zeros(H, device=dev)]
k.embed_bwd(torch.randn(T, H, device=dev).bfloat16(), ids, pf, tids, ww, wp[:P].contiguous(), wt, g, mu2, rs2, 0.1, 1,
            1, *outs, False, 0, -1, 0)
pseq = torch.arange(T, device=dev) % P
k.embed_bwd(torch.randn(T, H, device=dev).bfloat16(), ids, pseq, tids, ww, wp[:P].contiguous(), wt, g, mu2, rs2, 0.1,
            1, 1, *outs, True, 0, -1, T)
assert all(bool(torch.isfinite(o).all()) for o in outs)
A = torch.randn(256, 768, device=dev).bfloat16()
B = torch.randn(256, 768, device=dev).bfloat16()
C = torch.empty(256, 256, device=dev, dtype=torch.bfloat16)
k.gemm_nt(A, B, 0, out=C)
ref = A.float() @ B.float().t()
assert (C.float() - ref).abs().max().item() < 0.1 * ref.abs().max().item()
print("DEBUG_OK")
"""


@pytest.mark.gpu
def test_debug_library_runs_valid_inputs(cuda):
    """Valid inputs through the debug library (built beforehand on the CPU host: ``csrc/build.py --kernels
    --debug`` writes ``<pkg>/_debug/``, which travels with the tree; building inside a GPU test is not done)."""
    sys.path.insert(0, ROOT)
    from ml_recipe_distributed_pytorch_amd import _native
    import glob
    if not glob.glob(os.path.join(_native._DEBUG_DIR, "_hq_kernels*.so")):
        pytest.skip("debug kernel library not built (python -m ml_recipe_distributed_pytorch_amd.csrc.build "
                    "--kernels --debug)")
    env = dict(os.environ, HQ_KERNELS_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _GPU_SNIPPET], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0 and "DEBUG_OK" in r.stdout, r.stdout[-4000:]


def test_lab_defines_refused_for_production_library(monkeypatch):
    """Lab switches (HQ_EPI_DIAG & co. give wrong results by design) can reach only an A/B library outside the
    package: the production build refuses them and ignores HQ_KERNEL_CFLAGS in the environment."""
    import pytest
    from ml_recipe_distributed_pytorch_amd.csrc import build
    with pytest.raises(RuntimeError, match="refused"):
        build.build_kernels(1, lab_defines=["-DHQ_EPI_DIAG=1"])
    import inspect
    src = inspect.getsource(build.build_kernels)
    assert 'environ.get("HQ_KERNEL_CFLAGS", "")' not in src
