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
    sys.path.insert(0, ROOT)
    from ml_recipe_distributed_pytorch_amd.csrc import build
    build.build_kernels(jobs=16, debug=True, verbose=False)
    env = dict(os.environ, HQ_KERNELS_DEBUG="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _GPU_SNIPPET], stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0 and "DEBUG_OK" in r.stdout, r.stdout[-4000:]
