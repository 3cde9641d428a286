"""Own fp8 (OCP e4m3) NT GEMM on the block-scaled MFMA (gemm_fp8.hip) and the delayed-scaling quantiser,
vs fp32 torch references of the dequantised operands."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native

EPI_BIAS, EPI_GELUD = 1, 5


def _q(x):
    k = _native.kernels()
    x8, s = k.fp8_quantize(x)
    return x8, s.reshape(1).float()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 768), (768, 2304, 768), (256, 768, 3072)])
def test_gemm_fp8_bias(cuda, M, N, K):
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g)
    A8, sa = _q(A)
    B8, sb = _q(B)
    assert k.gemm_fp8_supported(M, N, K)
    C = k.gemm_fp8(A8, B8, EPI_BIAS, bias, sa, sb)
    ref = (A8.float() * sa) @ (B8.float() * sb).t() + bias
    err = (C.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err


@pytest.mark.gpu
def test_gemm_fp8_asymmetric_exact(cuda):
    """Small-integer operands (exact in e4m3 and in the fp32 accumulator): catches any lane-map slip."""
    k = _native.kernels()
    M, N, K = 256, 512, 256
    i = torch.arange(M, device=cuda)[:, None]
    kk = torch.arange(K, device=cuda)[None, :]
    n = torch.arange(N, device=cuda)[:, None]
    A = ((i * 7 + kk * 3) % 5 - 2).float()
    B = ((n * 11 + kk * 5 + 1) % 5 - 2).float()
    A8, B8 = A.to(torch.float8_e4m3fn), B.to(torch.float8_e4m3fn)
    one = torch.ones(1, device=cuda)
    C = k.gemm_fp8(A8, B8, EPI_BIAS, torch.zeros(N, device=cuda), one, one)
    assert torch.equal(C.float(), (A @ B.t()).bfloat16().float())


@pytest.mark.gpu
def test_gemm_fp8_gelud_delayed_q8(cuda):
    """FFN1 epilogue: act = gelu(pre), gelu'(pre), and act in e4m3 under delayed scaling (unit scale
    on the first step, 2·amax_prev/448 after; amax tracked in the 3-slot state)."""
    k = _native.kernels()
    M, N, K = 512, 768, 256
    g = torch.Generator(device=cuda).manual_seed(3)
    A = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    A8, sa = _q(A)
    B8, sb = _q(B)
    state = torch.zeros(4, device=cuda)
    pre_ref = ((A8.float() * sa) @ (B8.float() * sb).t() + bias).bfloat16().float()
    x = pre_ref.clone().requires_grad_(True)
    y = torch.nn.functional.gelu(x)
    y.backward(torch.ones_like(y))
    for phase in range(3):
        gd = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        act8 = torch.empty(M, N, device=cuda, dtype=torch.float8_e4m3fn)
        act = k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd, out8=act8, state=state, phase=phase)
        torch.testing.assert_close(act.float(), y.detach(), atol=2e-2, rtol=2e-2)
        torch.testing.assert_close(gd.float(), x.grad, atol=2e-2, rtol=2e-2)
        s = state[3].item()
        assert s == (1.0 if phase == 0 else pytest.approx(2 * act.float().abs().max().item() / 448, rel=1e-3))
        torch.testing.assert_close(act8.float() * s, act.float(), atol=s * 16, rtol=0.07)
        amax = state[:3].view(torch.int32)[phase].view(torch.float32).item()
        assert amax == pytest.approx(act.float().abs().max().item(), rel=1e-6)


@pytest.mark.gpu
def test_fp8_quant_delayed(cuda):
    k = _native.kernels()
    x = (torch.randn(1024, 768, device=cuda) * 3).bfloat16()
    state = torch.zeros(4, device=cuda)
    y0 = k.fp8_quant_delayed(x, state, 0)
    assert state[3].item() == 1.0
    torch.testing.assert_close(y0.float(), x.float().clamp(-448, 448).to(torch.float8_e4m3fn).float())
    y1 = k.fp8_quant_delayed(x, state, 1)
    s = state[3].item()
    assert s == pytest.approx(2 * x.float().abs().max().item() / 448, rel=1e-6)
    torch.testing.assert_close(y1.float() * s, x.float(), atol=s * 16, rtol=0.07)
