"""Out-projection / FFN2 + dropout + residual + LayerNorm with the GEMM's EPI_BDR epilogue (gemm.hip writes
z = dropout(x·Wᵀ + b) + resid, the LayerNorm reads z alone) must be bitwise the unfused pair
``linear_fwd`` → ``ln_fwd`` — every GEMM kernel variant (256-row v1 / v2 / persistent v3, 128² tiles for
M tails), with and without dropout — and match an fp32 reference."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native, ops

SHAPES = [(4096, 768, 768), (4096, 768, 3072), (1000, 768, 768), (2304, 1024, 1024)]


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["auto", "v1", "v2", "v3", "vS"])
def variant(request):
    k = _native.kernels()
    k.gemm_set_variant(request.param)
    yield request.param
    k.gemm_set_variant(0)


def _inputs(dev, M, N, K, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn(M, K, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) * K ** -0.5).bfloat16()
    b32 = torch.randn(N, device=dev, generator=g) * 0.1
    resid = torch.randn(M, N, device=dev, generator=g).bfloat16()
    gamma = 1 + 0.1 * torch.randn(N, device=dev, generator=g)
    beta = 0.1 * torch.randn(N, device=dev, generator=g)
    return x, w, b32, resid, gamma, beta


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_bdr_ln_fused_bitwise_equals_unfused(cuda, variant, M, N, K, p):
    x, w, b32, resid, gamma, beta = _inputs(cuda, M, N, K, seed=M + N + K)
    args = (x, w, b32.bfloat16(), b32, resid, "out", gamma, beta, 1e-12, p, 1234, 7)
    prev = ops.LN_FUSE
    try:
        ops.LN_FUSE = False
        ref = ops.linear_bdr_ln_fwd(*args)
        ops.LN_FUSE = True
        got = ops.linear_bdr_ln_fwd(*args)
    finally:
        ops.LN_FUSE = prev
    for name, r, g in zip(("y", "z", "mean", "rstd"), ref, got):
        assert torch.equal(r, g), f"{name} differs (variant {variant}, p={p})"
    if p == 0.0:   # and it is the right function
        z = (x.float() @ w.float().t() + b32).bfloat16().float() + resid.float()
        y = torch.nn.functional.layer_norm(z, (N,), gamma, beta, 1e-12)
        assert (got[0].float() - y).abs().max().item() < 0.05
    else:          # dropped positions of z are exactly the residual
        zf = got[1].float()
        keep = (zf - resid.float()).abs() > 0
        frac = 1 - keep.float().mean().item()
        assert 0.07 < frac < 0.13, f"dropped fraction {frac}"
