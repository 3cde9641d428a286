"""``--precision fp32`` on the GPU (the reference's Apex-off default, trainer.py:23-32,128-133): the exact-f32
MFMA GEMM (gemm_f32.hip) against fp64 products, and the whole fp32 model on the GPU against the CPU fp32 oracle
of the same weights, inputs and dropout masks — forward outputs, every gradient, and optimizer steps."""
import copy

import pytest
import torch

from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
from ml_recipe_distributed_pytorch_amd.models.config import get_config

pytestmark = pytest.mark.gpu


def _ref(A, B, alpha=1.0):
    return alpha * (A.double() @ B.double().t())


def _rel(a, b):
    return float((a.double() - b.double()).abs().max() / (b.double().abs().max() + 1e-30))


@pytest.mark.parametrize("M,N,K", [(256, 768, 768), (200, 132, 68), (4, 128, 4096)])
def test_gemm_f32_layouts(cuda, M, N, K):
    """Forward (A_K B_K), dgrad (A_K, j-contiguous B), weight gradient (both i/j-contiguous, split-K when the
    output is small), with bias and residual epilogues; ragged M/N/K tails."""
    from ml_recipe_distributed_pytorch_amd._native import kernels
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(M, K, device=cuda, generator=g)
    w = torch.randn(N, K, device=cuda, generator=g)
    b = torch.randn(N, device=cuda, generator=g)
    r = torch.randn(M, N, device=cuda, generator=g)
    y = torch.empty(M, N, device=cuda)
    kernels().gemm_f32(x, w, y, M, N, K, [K, 1, 0, 0], [K, 1, 0, 0], [N, 0, 0], bias=b, R=r, ldr=N)
    ref = _ref(x, w) + b.double() + r.double()
    assert _rel(y, ref) < 2e-6
    # dgrad: dx[M, K] = y[M, N]·w[N, K], w read as B(j = k, kk = n) = w[n·K + k]
    dx = torch.empty(M, K, device=cuda)
    kernels().gemm_f32(y, w, dx, M, K, N, [N, 1, 0, 0], [1, K, 0, 0], [K, 0, 0])
    assert _rel(dx, y.double() @ w.double()) < 2e-6
    # weight gradient: dw[N, K] = yᵀ·x (reduction over M rows), accumulated onto a prior value
    dw = torch.randn(N, K, device=cuda, generator=g)
    dw0 = dw.clone()
    kernels().gemm_f32(y, x, dw, N, K, M, [1, N, 0, 0], [1, K, 0, 0], [K, 0, 0], R=dw, ldr=K)
    assert _rel(dw, dw0.double() + y.double().t() @ x.double()) < 2e-6


def test_gemm_f32_batched_attention_layout(cuda):
    """The two-level batch (b, h) over qkv [B·L, 3H] views, as ops.f32.attn_fwd addresses it: S = scale·Q·Kᵀ."""
    from ml_recipe_distributed_pytorch_amd._native import kernels
    B, L, nh, dh = 3, 96, 4, 32
    H = nh * dh
    qkv = torch.randn(B * L, 3 * H, device=cuda)
    s = torch.empty(B, nh, L, L, device=cuda)
    kernels().gemm_f32(qkv, qkv[:, H:], s, L, L, dh, [3 * H, 1, L * 3 * H, dh], [3 * H, 1, L * 3 * H, dh],
                       [L, nh * L * L, L * L], batch=B * nh, nb_in=nh, alpha=0.125)
    t = qkv.double().view(B, L, 3, nh, dh).permute(2, 0, 3, 1, 4)
    ref = 0.125 * t[0] @ t[1].transpose(-1, -2)
    assert _rel(s, ref) < 2e-6


def test_gemm_f32_rejects_out_of_bounds_view(cuda):
    from ml_recipe_distributed_pytorch_amd._native import kernels
    a = torch.randn(64, 64, device=cuda)
    c = torch.empty(64, 64, device=cuda)
    with pytest.raises(RuntimeError, match="exceeds"):
        kernels().gemm_f32(a, a, c, 128, 64, 64, [64, 1, 0, 0], [64, 1, 0, 0], [64, 0, 0])


@pytest.mark.parametrize("train", [False, True])
def test_fp32_model_gpu_matches_cpu(cuda, train):
    """BERT-tiny in fp32 on the GPU (own f32 GEMMs + fp32 oracle row ops) vs the CPU fp32 path: same weights,
    inputs and counter-hash dropout masks — outputs and gradients agree to fp32 rounding."""
    cfg = get_config("bert-tiny-test")
    cpu = BertForQuestionAnswering(cfg, seed=0, precision="fp32")
    gpu = copy.deepcopy(cpu).to(cuda)
    assert gpu.store.compute.dtype == torch.float32 and gpu.store.compute.is_cuda
    cpu.train(train)
    gpu.train(train)
    g = torch.Generator().manual_seed(5)
    B, L = 3, 64
    ids = torch.randint(1, cfg.vocab_size, (B, L), generator=g)
    ids[1, L - 5:] = 0
    tt = torch.zeros_like(ids)
    tt[:, L // 3:] = 1
    mask = ids > 0
    torch.manual_seed(11)
    oc = cpu(ids, mask, tt)
    torch.manual_seed(11)
    og = gpu(ids.to(cuda), mask.to(cuda), tt.to(cuda))
    for k in oc:
        assert og[k].dtype == torch.float32
        assert _rel(og[k].cpu(), oc[k]) < 1e-4, k
    cpu.zero_grad()
    gpu.zero_grad()
    sum(v.sum() for v in oc.values()).backward()
    sum(v.sum() for v in og.values()).backward()
    # relative per tensor, with an absolute floor at 1e-6 of the largest gradient (the key bias gradient is zero
    # up to rounding: softmax is invariant to it)
    gmax = max(float(p.grad.abs().max()) for p in cpu.parameters())
    for (n, pc), (_, pg) in zip(cpu.named_parameters(), gpu.named_parameters()):
        err = float((pg.grad.cpu().double() - pc.grad.double()).abs().max())
        assert err <= 1e-3 * float(pc.grad.abs().max()) + 1e-6 * gmax, (n, err)


def test_fp32_train_steps_gpu(cuda):
    """TrainEngine + FusedAdamW in fp32 on the GPU for a few steps: finite, decreasing loss and the same
    trajectory as the CPU fp32 oracle."""
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    cfg = get_config("bert-tiny-test")
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, w_start=1, w_end=1, w_start_reg=1, w_end_reg=1, w_cls=1)
    batch = synth_batch_native(8, 64, 16, SpecialIds(vocab_size=cfg.vocab_size), seed=0)
    losses = {}
    for dev in ("cpu", cuda):
        m = BertForQuestionAnswering(cfg, seed=0, precision="fp32").to(dev).eval()
        opt = FusedAdamW(optimizer_groups(m.named_parameters(), 1e-4), m.store, lr=1e-3, correct_bias=False,
                         zero_grad_fn=m.zero_grad)
        eng = TrainEngine(m, build_loss(lp), opt)
        inputs, labels = to_device(batch[0], dev), to_device(batch[1], dev)
        losses[str(dev)] = [eng.step([(inputs, labels)]).losses.to_floats()["loss"] for _ in range(4)]
    lc, lg = losses["cpu"], losses[str(cuda)]
    assert all(v == v for v in lg) and lg[-1] < lg[0], lg
    for a, b in zip(lg, lc):
        assert abs(a - b) <= 1e-3 * (1 + abs(b)), (lg, lc)
