"""Own fp8 (OCP e4m3) NT GEMM on the block-scaled MFMA (gemm_fp8.hip) and the delayed-scaling quantiser,
vs fp32 torch references of the dequantised operands."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native

EPI_BIAS, EPI_GELUD = 1, 5


@pytest.fixture(params=[2, 3], ids=["v2", "persistent"])
def variant(request):
    """Run an fp8 GEMM test on both kernel forms (per-tile v2 and persistent), restoring auto afterwards."""
    k = _native.kernels()
    k.gemm_fp8_set_variant(request.param)
    yield request.param
    k.gemm_fp8_set_variant(0)


def _q(x):
    k = _native.kernels()
    x8, s = k.fp8_quantize(x)
    return x8, s.reshape(1).float()


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (512, 768, 768), (768, 2304, 768), (256, 768, 3072)])
def test_gemm_fp8_bias(cuda, variant, M, N, K):
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
def test_gemm_fp8_asymmetric_exact(cuda, variant):
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
def test_gemm_fp8_gelud_delayed_q8(cuda, variant):
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
    from ml_recipe_distributed_pytorch_amd import ops
    lo, step = ops.gelud_code()
    for phase in range(3):
        gd = torch.empty(M, N, device=cuda, dtype=torch.uint8)   # the 8-bit gelu' code (hq_gd_encode8)
        act8 = torch.empty(M, N, device=cuda, dtype=torch.float8_e4m3fn)
        act = k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd, out8=act8, state=state, phase=phase)
        torch.testing.assert_close(act.float(), y.detach(), atol=2e-2, rtol=2e-2)
        # the code's half step plus the bf16 pre the reference differentiates at
        torch.testing.assert_close(ops.gelud_decode(gd, torch.float32), x.grad, atol=step / 2 + 1e-2, rtol=0)
        # rounded to nearest, not truncated: no systematic offset of half a step
        assert abs((ops.gelud_decode(gd, torch.float32) - x.grad).mean().item()) < step / 8
        assert int(gd.min()) >= 0 and int(gd.max()) <= 255
        s = state[3].item()
        assert s == (1.0 if phase == 0 else pytest.approx(2 * act.float().abs().max().item() / 448, rel=1e-3))
        torch.testing.assert_close(act8.float() * s, act.float(), atol=s * 16, rtol=0.07)
        amax = state[:3].view(torch.int32)[phase].view(torch.float32).item()
        assert amax == pytest.approx(act.float().abs().max().item(), rel=1e-6)


@pytest.mark.gpu
def test_gemm_fp8_gelud_bf16_gelu_prime_with_q8(cuda, variant):
    """The fp8 FFN1 when the FFN2 dgrad will run in bf16: the e4m3 act AND gelu' in bf16 (no 8-bit code, so the
    bf16 dgrad reads gelu' at bf16 precision) — same act / act8 bytes as the code-writing form."""
    k = _native.kernels()
    M, N, K = 512, 768, 256
    g = torch.Generator(device=cuda).manual_seed(4)
    A8, sa = _q(torch.randn(M, K, device=cuda, generator=g).bfloat16())
    B8, sb = _q((torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16())
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    x = ((A8.float() * sa) @ (B8.float() * sb).t() + bias).bfloat16().float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(torch.ones(M, N, device=cuda))
    s1, s2 = torch.zeros(4, device=cuda), torch.zeros(4, device=cuda)
    gd16 = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    gd8 = torch.empty(M, N, device=cuda, dtype=torch.uint8)
    a8_16 = torch.empty(M, N, device=cuda, dtype=torch.float8_e4m3fn)
    a8_8 = torch.empty_like(a8_16)
    act16 = k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd16, out8=a8_16, state=s1, phase=0)
    act8 = k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd8, out8=a8_8, state=s2, phase=0)
    assert torch.equal(act16, act8) and torch.equal(a8_16.view(torch.uint8), a8_8.view(torch.uint8))
    assert torch.equal(s1, s2)
    torch.testing.assert_close(gd16.float(), x.grad, atol=1e-2, rtol=1e-2)
    # the device encoder of a bf16 gelu' = the host mirror (one fma; a rounding tie may differ by one code)
    from ml_recipe_distributed_pytorch_amd import ops
    dev = ops.gelud_encode(gd16)
    host = ops.gelud_encode(gd16.cpu())
    d = (dev.cpu().int() - host.int()).abs()
    assert d.max().item() <= 1 and (d > 0).float().mean().item() < 1e-4
    # and within half a step of the code the epilogue wrote from the fp32 gelu'
    d2 = (dev.int() - gd8.int()).abs()
    assert d2.max().item() <= 2, d2.max().item()
    with pytest.raises(RuntimeError, match="write_out"):
        k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd16, out8=a8_16, state=s1, phase=1, write_out=False)


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


@pytest.mark.gpu
@pytest.mark.parametrize("T,H", [(1024, 768), (98304, 768), (1000, 1024), (1003, 768), (5, 768)])
def test_ln_fwd_fp8_output(cuda, T, H):
    """LayerNorm forward with the e4m3 copy of y for the next fp8 GEMM (producer-side quantisation): the
    bf16 outputs equal the plain kernel's bitwise, y8 = e4m3(bf16(y) / s) under the delayed scale, and the
    step's amax lands in the state (second call scales by 2·amax/448 of the first)."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(T)
    a = torch.randn(T, H, device=cuda, generator=g).bfloat16()
    r = torch.randn(T, H, device=cuda, generator=g).bfloat16()
    gamma = torch.rand(H, device=cuda, generator=g) + 0.5
    beta = torch.randn(H, device=cuda, generator=g) * 0.1
    ref = k.ln_fwd(a, r, gamma, beta, 1e-12, 0.1, 7, 3)
    state = torch.zeros(4, device=cuda)
    out = k.ln_fwd(a, r, gamma, beta, 1e-12, 0.1, 7, 3, q8=state, phase=0)
    for x, y in zip(out[:4], ref):
        assert torch.equal(x, y)
    y, y8 = out[0].float(), out[4]
    assert y8.dtype == torch.float8_e4m3fn and state[3].item() == 1.0       # first step: unit scale
    assert torch.equal(y8.view(torch.uint8), y.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8))
    amax = state[:3].view(torch.int32)[0].view(torch.float32).item()
    assert amax == pytest.approx(y.abs().max().item(), rel=0, abs=0)
    out2 = k.ln_fwd(a, r, gamma, beta, 1e-12, 0.1, 7, 3, q8=state, phase=1)
    s = state[3].item()
    assert s == pytest.approx(2 * amax / 448, rel=1e-6)
    exp = (y / s).clamp(-448, 448).to(torch.float8_e4m3fn)
    assert torch.equal(out2[4].view(torch.uint8), exp.view(torch.uint8))


@pytest.mark.gpu
def test_fp8_model_step_runs_on_own_kernels(cuda):
    """--precision fp8 at a tile-aligned shape: every forward projection (QKV, out-projection, FFN1, FFN2)
    on gemm_fp8 with producer-quantised inputs; a training step stays finite and close to bf16."""
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    cfg = get_config("bert-base-uncased", num_hidden_layers=2, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    m = BertForQuestionAnswering(cfg, seed=0).to(cuda).train()
    g = torch.Generator().manual_seed(3)
    ids = torch.randint(1, cfg.vocab_size, (4, 256), generator=g).to(cuda)
    ref = m(ids)
    m.set_precision("fp8")
    for _ in range(3):   # delayed scaling settles after the first step
        out = m(ids)
    for key in ("start_class", "cls"):
        rel = ((out[key].float() - ref[key].float()).norm() / ref[key].float().norm()).item()
        assert rel < 0.1, (key, rel)
    m.zero_grad()
    sum(v.float().mean() for v in out.values()).backward()
    torch.cuda.synchronize()
    assert torch.isfinite(m.store.grad).all()


@pytest.mark.gpu
def test_fp8_quant_delayed_multi_matches_per_tensor(cuda):
    """All weights in one launch (ParamStore.view_fp8): each segment under its own state row, bitwise
    equal to the per-tensor quantiser with the same state, over three phases (amax slots rotate)."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(9)
    sizes = [768 * 2304, 768 * 768, 64, 3072 * 768 + 8]
    offs, o = [], 0
    for n in sizes:
        offs.append(o)
        o += (n + 63) // 64 * 64
    x = (torch.randn(o, device=cuda, generator=g) * 0.05).bfloat16()
    for i, n in enumerate(sizes):   # different magnitudes per segment
        x[offs[i]:offs[i] + n] *= 10.0 ** (i - 1)
    states = torch.zeros(len(sizes), 4, device=cuda)
    states[:, 2] = torch.tensor([0.3, 5.0, 0.0, 40.0], device=cuda)   # seeded "previous amax"
    ref_states = [states[i].clone() for i in range(len(sizes))]
    rows, yo, blk = [], 0, 0
    for off, n in zip(offs, sizes):
        rows.append([off, yo, n // 8, blk])
        blk += k.fp8_quant_multi_blocks(n // 8)
        yo += (n + 255) // 256 * 256
    seg = torch.tensor(rows, dtype=torch.int64, device=cuda)
    y = torch.zeros(yo, dtype=torch.uint8, device=cuda)
    for phase in range(3):
        k.fp8_quant_delayed_multi(x, y, seg, states, blk, phase)
        for i, (off, n) in enumerate(zip(offs, sizes)):
            exp = k.fp8_quant_delayed(x[off:off + n], ref_states[i], phase)
            assert torch.equal(y[rows[i][1]:rows[i][1] + n], exp.view(torch.uint8)), (phase, i)
            assert torch.equal(states[i], ref_states[i]), (phase, i)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_fwd_fp8_ctx_output(cuda, p):
    """Attention forward with the e4m3 copy of ctx for the fp8 out-projection: ctx / lse / keep-bits equal
    the plain call bitwise, ctx8 = e4m3(bf16(ctx) / s) under the delayed scale, amax lands in the state."""
    k = _native.kernels()
    B, L, nh = 4, 384, 12
    g = torch.Generator(device=cuda).manual_seed(11)
    qkv = torch.randn(B * L, 3 * nh * 64, device=cuda, generator=g).bfloat16()
    kb = torch.zeros(B, L, device=cuda)
    kb[2, 300:] = -10000.0
    ref = k.attn_fwd(qkv, kb, B, L, nh, p, 5, 9, 0.125)
    state = torch.zeros(4, device=cuda)
    out = k.attn_fwd(qkv, kb, B, L, nh, p, 5, 9, 0.125, q8=state, phase=0)
    for x, y in zip(out[:3], ref):
        assert torch.equal(x, y)
    ctx, ctx8 = out[0].float(), out[3]
    assert ctx8.dtype == torch.float8_e4m3fn and state[3].item() == 1.0
    assert torch.equal(ctx8.view(torch.uint8), ctx.clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8))
    amax = state[:3].view(torch.int32)[0].view(torch.float32).item()
    assert amax == ctx.abs().max().item()
    out2 = k.attn_fwd(qkv, kb, B, L, nh, p, 5, 9, 0.125, q8=state, phase=1)
    s = state[3].item()
    assert s == pytest.approx(2 * amax / 448, rel=1e-6)
    exp = (ctx / s).clamp(-448, 448).to(torch.float8_e4m3fn)
    diff = (out2[3].view(torch.uint8).int() - exp.view(torch.uint8).int()).abs()
    assert diff.max().item() <= 1 and (diff > 0).float().mean().item() < 1e-4   # x·(1/s) vs x/s rounding


# ----------------------------------------------------------------------------- fp8 backward (e5m2)
EPI_NONE, EPI_DMUL = 0, 6


def _q5(x, s):
    """e5m2(x / s) the way the kernels round it (saturated, RNE)."""
    return (x.float() / s).clamp(-57344, 57344).to(torch.float8_e5m2)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(256, 768, 768), (512, 3072, 768), (512, 768, 3072)])
def test_gemm_fp8_dgrad_e5m2(cuda, variant, M, N, K):
    """dgrad form: A = e5m2 gradient (mixed-format MFMA, blgp = e5m2), B = e4m3 Wᵀ, no epilogue."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(M * 3 + N + K)
    dy = torch.randn(M, K, device=cuda, generator=g) * 1e-3
    sa = torch.full((1,), 1e-3 * 4 / 57344, device=cuda)
    A8 = _q5(dy, sa)
    B8, sb = _q((torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16())
    C = k.gemm_fp8(A8, B8, EPI_NONE, None, sa, sb)
    ref = (A8.float() * sa) @ (B8.float() * sb).t()
    err = (C.float() - ref).abs().max().item()
    assert err <= 1e-2 * ref.abs().max().item(), err


@pytest.mark.gpu
def test_gemm_fp8_dgrad_exact(cuda, variant):
    """Small integers (exact in e5m2, e4m3 and fp32): the e5m2 operand's lane map and format code."""
    k = _native.kernels()
    M, N, K = 256, 512, 256
    i = torch.arange(M, device=cuda)[:, None]
    kk = torch.arange(K, device=cuda)[None, :]
    n = torch.arange(N, device=cuda)[:, None]
    A = ((i * 5 + kk * 3) % 7 - 3).float()     # -3..3: 3 is exact in e5m2 (1.1b × 2^1)
    B = ((n * 11 + kk * 5 + 1) % 5 - 2).float()
    one = torch.ones(1, device=cuda)
    C = k.gemm_fp8(A.to(torch.float8_e5m2), B.to(torch.float8_e4m3fn), EPI_NONE, None, one, one)
    assert torch.equal(C.float(), (A @ B.t()).bfloat16().float())


@pytest.mark.gpu
def test_gemm_fp8_dmul_colsum_q8(cuda, variant):
    """FFN2 dgrad epilogue: dpre = bf16(dy·W) ⊙ gelu', per-256-row column sums (FFN1 bias gradient) and
    dpre in e5m2 under the gradient's delayed scale (64·amax_prev/57344), over three phases."""
    k = _native.kernels()
    M, N, K = 768, 3072, 768
    g = torch.Generator(device=cuda).manual_seed(21)
    sa = torch.full((1,), 1e-2 * 4 / 57344, device=cuda)
    A8 = _q5(torch.randn(M, K, device=cuda, generator=g) * 1e-2, sa)
    B8, sb = _q((torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16())
    from ml_recipe_distributed_pytorch_amd import ops
    gd = ops.gelud_encode(torch.rand(M, N, device=cuda, generator=g) * 1.2 - 0.1)   # the fp8 forward's code
    mm = ((A8.float() * sa) @ (B8.float() * sb).t()).bfloat16().float()
    ref = mm * ops.gelud_decode(gd, torch.float32)
    state = torch.zeros(4, device=cuda)
    for phase in range(3):
        part = torch.empty(M // 256, N, device=cuda)
        out8 = torch.empty(M, N, device=cuda, dtype=torch.float8_e5m2)
        C = k.gemm_fp8(A8, B8, EPI_DMUL, None, sa, sb, pre=gd, out8=out8, state=state, phase=phase, part=part)
        torch.testing.assert_close(C.float(), ref, atol=2e-3 * ref.abs().max().item(), rtol=2e-2)
        torch.testing.assert_close(part, ref.view(M // 256, 256, N).sum(1), atol=1e-2 * ref.abs().max().item(),
                                   rtol=2e-2)
        s = state[3].item()
        amax_c = C.float().abs().max().item()
        assert s == (1.0 if phase == 0 else pytest.approx(64 * amax_c / 57344, rel=1e-3))
        exp = _q5(C, s)
        diff = (out8.view(torch.uint8).int() - exp.view(torch.uint8).int()).abs()
        assert diff.max().item() <= 1 and (diff > 0).float().mean().item() < 1e-3   # x·(1/s) vs x/s
        amax = state[:3].view(torch.int32)[phase].view(torch.float32).item()
        assert amax == pytest.approx(amax_c, rel=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("T,H", [(1024, 768), (2048, 1024)])
def test_ln_bwd_e5m2_output(cuda, T, H):
    """LayerNorm backward with the e5m2 copy of da for the fp8 dgrad: dz / da equal the plain call bitwise
    (the parameter gradients to the last bit), da8 = e5m2(bf16(da) / s) under the delayed scale, amax
    recorded; with write_da=False only the e5m2 copy is written, identical."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(T + H)
    dy = (torch.randn(T, H, device=cuda, generator=g) * 1e-3).bfloat16()
    z = torch.randn(T, H, device=cuda, generator=g).bfloat16()
    gamma = torch.rand(H, device=cuda, generator=g) + 0.5
    mean = z.float().mean(1)
    rstd = torch.rsqrt(z.float().var(1, unbiased=False) + 1e-12)
    grads = [torch.zeros(H, device=cuda) for _ in range(3)]
    ref = k.ln_bwd(dy, None, z, gamma, mean, rstd, 0.1, 7, 3, *grads, False)
    grads8 = [torch.zeros(H, device=cuda) for _ in range(3)]
    state = torch.zeros(4, device=cuda)
    out = k.ln_bwd(dy, None, z, gamma, mean, rstd, 0.1, 7, 3, *grads8, False, q8=state, phase=0)
    assert torch.equal(out[0], ref[0]) and torch.equal(out[1], ref[1])
    for a, b in zip(grads, grads8):   # the variants may contract a·m + acc differently: last-bit differences
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-5 * a.abs().max().item())
    da, da8 = out[1].float(), out[2]
    assert da8.dtype == torch.float8_e5m2 and state[3].item() == 1.0

    def close_codes(got, exp):   # x·(1/s) in the kernel vs x/s here: at most one code apart, rarely
        diff = (got.view(torch.uint8).int() - exp.view(torch.uint8).int()).abs()
        assert diff.max().item() <= 1 and (diff > 0).float().mean().item() < 1e-3
    assert torch.equal(da8.view(torch.uint8), _q5(da, 1.0).view(torch.uint8))
    amax = state[:3].view(torch.int32)[0].view(torch.float32).item()
    assert amax == da.abs().max().item()
    out2 = k.ln_bwd(dy, None, z, gamma, mean, rstd, 0.1, 7, 3, *grads8, True, q8=state, phase=1)
    s = state[3].item()
    assert s == pytest.approx(64 * amax / 57344, rel=1e-6)
    close_codes(out2[2], _q5(da, s))
    state2 = state.clone()
    out3 = k.ln_bwd(dy, None, z, gamma, mean, rstd, 0.1, 7, 3, *grads8, True, q8=state2, phase=1, write_da=False)
    assert out3[1].numel() == 0 and torch.equal(out3[0], out2[0]) and torch.equal(out3[2], out2[2])


@pytest.mark.gpu
def test_view_fp8_t_is_the_transposed_forward_copy(cuda):
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    cfg = get_config("bert-base-uncased", num_hidden_layers=1)
    m = BertForQuestionAnswering(cfg, seed=0, precision="fp8").to(cuda)
    for name in ("qkv.weight", "intermediate.dense.weight", "output.dense.weight"):
        key = "transformer.encoder.layer.0." + name
        w8, s = m.store.view_fp8(key)
        wt8, st = m.store.view_fp8_t(key)
        assert wt8.shape == (w8.shape[1], w8.shape[0]) and wt8.is_contiguous()
        assert torch.equal(wt8.view(torch.uint8), w8.view(torch.uint8).t())
        assert st.data_ptr() == s.data_ptr()


@pytest.mark.gpu
def test_fp8_dgrad_step_close_to_bf16_dgrad(cuda):
    """--precision fp8 with the e5m2 dgrads (FFN2 / FFN1 / out-projection / QKV) against the same model with bf16
    dgrads: after the gradient states calibrate (step 3), the parameter gradients agree to fp8 accuracy
    (the out-projection / FFN weight gradients run on the fp8 TN kernel from step 2 on)."""
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    cfg = get_config("bert-base-uncased", num_hidden_layers=2, hidden_dropout_prob=0.0,
                     attention_probs_dropout_prob=0.0)
    g = torch.Generator().manual_seed(4)
    ids = torch.randint(1, cfg.vocab_size, (4, 256), generator=g).to(cuda)
    grads = {}
    for dg in (False, True):
        m = BertForQuestionAnswering(cfg, seed=0, precision="fp8").to(cuda).train()
        m.fp8_dgrad = dg
        for _ in range(3):
            m.zero_grad()
            out = m(ids)
            sum((v.float() ** 2).mean() for v in out.values()).backward()
        torch.cuda.synchronize()
        if dg:
            s8 = m.fp8_states(0)
            assert all(s8[k].calibrated for k in ("dffn2", "dffn1", "dout", "dqkv"))
        grads[dg] = m.store.grad.clone()
    assert torch.isfinite(grads[True]).all()
    for e in m.store.entries:
        if e.key.startswith("transformer.encoder") and e.key.endswith("weight") and len(e.shape) == 2:
            a, b = (grads[x][e.offset:e.offset + e.numel] for x in (True, False))
            rel = ((a - b).norm() / b.norm()).item()
            assert rel < 0.1, (e.key, rel)


@pytest.mark.gpu
def test_gemm_fp8_dgrad_resid(cuda, variant):
    """QKV dgrad form: C = bf16(dy8·Wᵀ8·sa·sb) + resid (EPI_RESID, e5m2 A operand)."""
    k = _native.kernels()
    M, N, K = 512, 768, 2304
    g = torch.Generator(device=cuda).manual_seed(31)
    sa = torch.full((1,), 1e-2 * 4 / 57344, device=cuda)
    A8 = _q5(torch.randn(M, K, device=cuda, generator=g) * 1e-2, sa)
    B8, sb = _q((torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16())
    R = (torch.randn(M, N, device=cuda, generator=g) * 1e-3).bfloat16()
    C = k.gemm_fp8(A8, B8, 4, None, sa, sb, resid=R)
    mm = ((A8.float() * sa) @ (B8.float() * sb).t()).bfloat16().float()
    torch.testing.assert_close(C.float(), mm + R.float(), atol=2e-3 * mm.abs().max().item(), rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("p", [0.0, 0.1])
def test_attn_bwd_e5m2_output(cuda, p):
    """Attention backward with the e5m2 copy of dQKV for the fp8 QKV dgrad: dqkv equals the plain call
    bitwise, dqkv8 = e5m2(dqkv / s) under the delayed scale (quantised from the fp32 values, so within one
    code of e5m2(bf16(dqkv) / s)), and the amax of BOTH kernels' outputs (dQ from one, dK/dV from the other)
    lands in the state; an amax beyond the scale's headroom saturates instead of overflowing."""
    k = _native.kernels()
    B, L, nh = 2, 384, 12
    g = torch.Generator(device=cuda).manual_seed(41)
    qkv = torch.randn(B * L, 3 * nh * 64, device=cuda, generator=g).bfloat16()
    kb = torch.zeros(B, L, device=cuda)
    kb[1, 250:] = -10000.0
    ctx, lse, bits = k.attn_fwd(qkv, kb, B, L, nh, p, 5, 9, 0.125)
    dctx = (torch.randn(B * L, nh * 64, device=cuda, generator=g) * 1e-2).bfloat16()
    ref = k.attn_bwd(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False)
    state = torch.zeros(4, device=cuda)
    dqkv, dqkv8 = k.attn_bwd_q8(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False, state, 0)
    assert torch.equal(dqkv, ref)
    assert dqkv8.dtype == torch.float8_e5m2 and state[3].item() == 1.0

    def close_codes(got, exp, frac):
        diff = (got.view(torch.uint8).int() - exp.view(torch.uint8).int()).abs()
        assert diff.max().item() <= 1 and (diff > 0).float().mean().item() < frac
    close_codes(dqkv8, _q5(dqkv, 1.0), 0.05)   # bf16 vs fp32 source: differs only at bf16 rounding ties
    amax = state[:3].view(torch.int32)[0].view(torch.float32).item()
    assert amax == pytest.approx(dqkv.float().abs().max().item(), rel=1e-2)
    _, d8b = k.attn_bwd_q8(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False, state, 1)
    s = state[3].item()
    assert s == pytest.approx(64 * amax / 57344, rel=1e-6)
    close_codes(d8b, _q5(dqkv, s), 0.05)
    # calibrated mode: no bf16 dQKV, the same e5m2 bytes, and the QKV bias-gradient column partials
    st2 = state.clone()
    r2 = k.attn_bwd_q8(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False, st2, 1, write_bf16=False)
    assert r2[0].numel() == 0 and torch.equal(r2[1].view(torch.uint8), d8b.view(torch.uint8))
    bpart = r2[2]
    assert bpart.shape == (B * ((L + 31) // 32), 3 * nh * 64)
    colsum = bpart.sum(0)
    ref_sum = dqkv.float().sum(0)
    torch.testing.assert_close(colsum, ref_sum, rtol=2e-2, atol=2e-2 * ref_sum.abs().max().item())
    # a state whose previous amax is 1000x too small: every |x| / s far beyond 57344 → saturated, never inf
    state[:3] = 0.0
    state[2] = amax * 1e-3
    _, d8c = k.attn_bwd_q8(dctx, qkv, ctx, lse, kb, bits, B, L, nh, p, 0.125, False, state, 0)
    assert torch.isfinite(d8c.float()).all()
    assert d8c.float().abs().max().item() == 57344.0


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,K", [(1024, 768, 768), (1024, 3072, 768), (2048, 768, 3072), (1000, 256, 384)])
def test_gemm_tn8_wgrad(cuda, T, N, K):
    """fp8 weight gradient (ds_read_b64_tr_b8 fragments, mixed e5m2 × e4m3 MFMA): out (+)= (dy8·sa)ᵀ(x8·sb)
    against the fp32 product of the dequantised operands; a token tail (T % 128) stages zero rows."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(T + N + K)
    sa = torch.full((1,), 1e-2 * 4 / 57344, device=cuda)
    dy8 = _q5(torch.randn(T, N, device=cuda, generator=g) * 1e-2, sa)
    x8, sb = _q(torch.randn(T, K, device=cuda, generator=g).bfloat16())
    ref = (dy8.float() * sa).t() @ (x8.float() * sb)
    out = torch.full((N, K), 0.5, device=cuda)
    k.gemm_tn8(dy8, x8, sa, sb, out, True)
    torch.testing.assert_close(out, ref + 0.5, atol=1e-4 * ref.abs().max().item() + 1e-6, rtol=1e-4)
    k.gemm_tn8(dy8, x8, sa, sb, out, False)
    torch.testing.assert_close(out, ref, atol=1e-4 * ref.abs().max().item(), rtol=1e-4)


@pytest.mark.gpu
def test_gemm_tn8_exact(cuda):
    """Small integers (exact in e5m2 / e4m3 / fp32): any slip in the transposed-read lane map or the swizzle
    shows as a wrong integer."""
    k = _native.kernels()
    T, N, K = 512, 256, 512
    t = torch.arange(T, device=cuda)[:, None]
    dy = ((t * 5 + torch.arange(N, device=cuda)[None, :] * 3) % 7 - 3).float()
    x = ((t * 3 + torch.arange(K, device=cuda)[None, :] * 11 + 1) % 5 - 2).float()
    one = torch.ones(1, device=cuda)
    out = torch.zeros(N, K, device=cuda)
    k.gemm_tn8(dy.to(torch.float8_e5m2), x.to(torch.float8_e4m3fn), one, one, out, False)
    assert torch.equal(out, dy.t() @ x)


@pytest.mark.gpu
@pytest.mark.parametrize("epi,q8", [(1, False), (5, True), (5, False), (6, True), (0, False), (4, False)])
def test_gemm_fp8_persistent_matches_per_tile(cuda, epi, q8):
    """The persistent form (one workgroup per CU walking 4.5 tiles each, DMA pipelined across tile seams) against
    the per-tile v2 kernel at M = 24576, N = 3072, K = 768: bitwise equal outputs, gelu', fp8 copies, column
    partials and delayed-scaling state (same K order, same epilogue math per tile)."""
    k = _native.kernels()
    M, N, K = 24576, 3072, 768
    g = torch.Generator(device=cuda).manual_seed(epi * 10 + int(q8))
    grad = epi in (0, 4, 6)
    sa = torch.full((1,), 4e-2 / 57344 if grad else 1.0, device=cuda)
    A8 = _q5(torch.randn(M, K, device=cuda, generator=g) * 1e-2, sa) if grad else \
        torch.randn(M, K, device=cuda, generator=g).clamp(-8, 8).to(torch.float8_e4m3fn)
    B8, sb = _q((torch.randn(N, K, device=cuda, generator=g) * 0.05).bfloat16())
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    aux = (torch.rand(M, N, device=cuda, generator=g) * 1.2 - 0.1).bfloat16()
    code = torch.randint(0, 256, (M, N), device=cuda, dtype=torch.uint8, generator=g)
    outs = []
    for v in (2, 3):
        k.gemm_fp8_set_variant(v)
        kw = {}
        if epi in (5, 6):   # with out8 gelu' travels as the 8-bit code, else as bf16
            if q8:
                kw["pre"] = code.clone() if epi == 6 else torch.empty(M, N, device=cuda, dtype=torch.uint8)
            else:
                kw["pre"] = aux.clone() if epi == 6 else torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
        if epi == 4:
            kw["resid"] = aux
        if epi == 6:
            kw["part"] = torch.empty(M // 256, N, device=cuda)
        if q8:
            kw["out8"] = torch.empty(M, N, device=cuda, dtype=torch.float8_e5m2 if epi == 6 else torch.float8_e4m3fn)
            kw["state"] = torch.tensor([0.0, 0.0, 3.0, 0.0], device=cuda)
            kw["phase"] = 0
        C = k.gemm_fp8(A8, B8, epi, None if grad else bias, sa, sb, **kw)
        torch.cuda.synchronize()
        outs.append((C, kw))
    k.gemm_fp8_set_variant(0)
    (c2, kw2), (c3, kw3) = outs
    assert torch.equal(c2, c3)
    for key in ("pre", "part", "out8", "state"):
        if key in kw2:
            assert torch.equal(kw2[key].view(torch.uint8) if kw2[key].element_size() == 1 else kw2[key],
                               kw3[key].view(torch.uint8) if kw3[key].element_size() == 1 else kw3[key]), key


@pytest.mark.gpu
def test_fp8_deferred_amax_folds_match_immediate(cuda):
    """TrainEngine under --precision fp8 with the sites' amax folds batched at the end of each micro-step
    (gemm_fp8.hip FoldDefer; producers publish their dequant scale themselves) against one fold launch per site:
    bitwise the same losses, weights and delayed-scaling states over steps that cross calibration, with a 2-way
    accumulation (every state produced twice per optimizer step) and nothing left pending afterwards."""
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    k = _native.kernels()
    cfg = get_config("bert-base-uncased", num_hidden_layers=2)
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, w_start=1, w_end=1, w_start_reg=1, w_end_reg=1, w_cls=1)
    batches = [synth_batch_native(8, 256, 64, SpecialIds(), seed=s) for s in range(8)]
    runs = {}
    for defer in (False, True):
        torch.manual_seed(0)
        m = BertForQuestionAnswering(cfg, seed=0, precision="fp8").to(cuda).train()
        opt = FusedAdamW(optimizer_groups(m.named_parameters(), 1e-4), m.store, lr=1e-4, correct_bias=False,
                         zero_grad_fn=m.zero_grad)
        eng = TrainEngine(m, build_loss(lp), opt, batch_split=2)
        eng.fp8_fold_defer = defer
        losses = []
        for i in range(0, 8, 2):
            mb = [(to_device(batches[j][0], cuda), to_device(batches[j][1], cuda)) for j in (i, i + 1)]
            losses.append(eng.step(mb).losses.to_floats()["loss"])
        torch.cuda.synchronize()
        assert k.fp8_fold_pending() == 0
        states = [s.buf.clone() for st in (m.fp8_states(l) for l in range(2)) for s in st.values()]
        runs[defer] = (losses, m.store.master.clone(), states)
    (l0, w0, s0), (l1, w1, s1) = runs[False], runs[True]
    assert l0 == l1
    assert torch.equal(w0, w1)
    assert len(s0) == len(s1) > 0 and all(torch.equal(a, b) for a, b in zip(s0, s1))
    assert any(a[:3].abs().sum().item() > 0 for a in s1)
