"""MFMA NT GEMM (gemm.hip) vs an fp32 torch reference, every epilogue, every kernel variant:
auto (0: 128² tiles for M tails / low CU fill, else the persistent v3 for K <= 2304 and v2 above),
v1 (whole-tile staging), forced v2 (deep LDS-DMA pipeline, also at K <= 2304), forced v3 (persistent,
also at K = 3072) and forced vS (the 128²-tile kernel everywhere)."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native


@pytest.fixture(params=[0, 1, 2, 3, 4], ids=["auto", "v1", "v2", "v3", "vS"], autouse=True)
def variant(request):
    if not torch.cuda.is_available():
        yield request.param
        return
    k = _native.kernels()
    k.gemm_set_variant(request.param)
    yield request.param
    k.gemm_set_variant(0)

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_DGELU, EPI_RESID = range(5)
SHAPES = [(256, 256, 64), (512, 384, 192), (1024, 768, 768), (768, 2304, 128), (512, 128, 3072), (256, 256, 192),
          (2048, 768, 3072), (512, 4096, 256)]


def _ref(A, B):
    return A.float() @ B.float().t()


def _close(got, exp, tol=2e-2):
    err = (got.float() - exp).abs().max().item()
    scale = exp.abs().max().item() + 1e-6
    assert err <= tol * scale, f"max err {err} vs scale {scale}"


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_gemm_nt_plain_and_bias(cuda, M, N, K):
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = torch.randn(M, K, device=cuda, generator=g).bfloat16()
    B = torch.randn(N, K, device=cuda, generator=g).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g)
    assert k.gemm_nt_supported(M, N, K) in (1, 128, 256)
    _close(k.gemm_nt(A, B, EPI_NONE), _ref(A, B))
    _close(k.gemm_nt(A, B, EPI_BIAS, bias=bias), _ref(A, B) + bias)


@pytest.mark.gpu
def test_gemm_nt_asymmetric_layout(cuda):
    """A = I (padded) with an asymmetric B: catches a transposed C write."""
    k = _native.kernels()
    M, N, K = 256, 256, 256
    A = torch.eye(M, K, device=cuda).bfloat16()
    B = (torch.arange(N * K, device=cuda).reshape(N, K) % 251).float().bfloat16()
    C = k.gemm_nt(A, B, EPI_NONE)
    assert torch.equal(C.float(), B.float().t()[:M, :N].contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (256, 3072, 768)])
def test_gemm_nt_gelu_dgelu_resid(cuda, M, N, K):
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(7)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    act = k.gemm_nt(A, B, EPI_GELU, bias=bias, pre=pre)
    ref_pre = _ref(A, B) + bias
    _close(pre, ref_pre)
    _close(act, torch.nn.functional.gelu(pre.float()))
    # dgelu: C = (A·Bᵀ) * gelu'(pre), part = column sums per 256-row block
    part = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=cuda)
    d = k.gemm_nt(A, B, EPI_DGELU, pre=pre, part=part)
    x = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(_ref(A, B).bfloat16().float())
    _close(d, x.grad)
    torch.testing.assert_close(part.sum(0), d.float().sum(0), atol=5e-2 * (1 + d.float().abs().sum(0).max().item() / M), rtol=2e-2)
    resid = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    _close(k.gemm_nt(A, B, EPI_RESID, resid=resid), _ref(A, B) + resid.float())


@pytest.mark.gpu
def test_gemm_nt_rejects_bad_shapes(cuda):
    k = _native.kernels()
    A = torch.randn(100, 64, device=cuda).bfloat16()
    B = torch.randn(100, 64, device=cuda).bfloat16()
    assert k.gemm_nt_supported(100, 100, 64) == 0    # N % 128 != 0
    assert k.gemm_nt_supported(100, 128, 96) == 0    # K % 64 != 0
    with pytest.raises(RuntimeError):
        k.gemm_nt(A, B, EPI_NONE)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(100, 256, 64), (1000, 768, 768), (1152, 768, 3072), (4 * 317, 2304, 768),
                                   (24576, 768, 768)])
def test_gemm_nt_m_tail_and_low_fill_all_epilogues(cuda, M, N, K, variant):
    """M % 256 != 0 (dynamically padded batches: 4 × 317 tokens; the reference micro-batch 2 × 512 = 1024
    is aligned but fills 12 tiles) and the batch-64 low-fill grid (24576 × 768) on the 128²-tile kernel,
    every epilogue; rows past M must stay untouched."""
    if variant not in (0, 4):
        pytest.skip("the 256-row kernels need M % 256 == 0")
    EPI_GELUD, EPI_DMUL = 5, 6
    k = _native.kernels()
    assert k.gemm_nt_supported(M, N, K) == 1 or (M % 256 == 0 and variant == 0)
    g = torch.Generator(device=cuda).manual_seed(M + N)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    ref = _ref(A, B)
    big = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
    out = big[:M]
    k.gemm_nt(A, B, EPI_BIAS, bias=bias, out=out)
    _close(out, ref + bias)
    assert torch.equal(big[M:].float(), torch.full((64, N), 7.0, device=cuda)), "rows past M were written"
    _close(k.gemm_nt(A, B, EPI_NONE), ref)
    resid = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    _close(k.gemm_nt(A, B, EPI_RESID, resid=resid), ref + resid.float())
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    act = k.gemm_nt(A, B, EPI_GELU, bias=bias, pre=pre)
    _close(pre, ref + bias)
    _close(act, torch.nn.functional.gelu(pre.float()))
    rows = k.gemm_nt_part_rows(M, N, K)
    part = torch.empty(rows, N, device=cuda)
    d = k.gemm_nt(A, B, EPI_DGELU, pre=pre, part=part)
    x = pre.float().requires_grad_(True)
    torch.nn.functional.gelu(x).backward(ref.bfloat16().float())
    _close(d, x.grad)
    torch.testing.assert_close(part.sum(0), d.float().sum(0), atol=5e-2 * (1 + d.float().abs().sum(0).max().item() / M),
                               rtol=2e-2)
    gd = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    act2 = k.gemm_nt(A, B, EPI_GELUD, bias=bias, pre=gd)
    _close(act2, act.float())
    dm = k.gemm_nt(A, B, EPI_DMUL, pre=gd, part=part)
    _close(dm, ref.bfloat16().float() * gd.float())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(8192, 2304, 768), (4096, 768, 3072), (4096, 4096, 768)])
def test_gemm_nt_repeatable_large(cuda, M, N, K):
    """Race screen: a full-chip grid run repeatedly must be bitwise identical (the kernel is
    deterministic) and match the fp32 reference — an LDS RAW/WAR slip shows up as rare wrong tiles."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(11)
    A = (torch.rand(M, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    B = (torch.rand(N, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    first = k.gemm_nt(A, B, EPI_NONE)
    _close(first, _ref(A, B))
    for _ in range(8):
        assert torch.equal(k.gemm_nt(A, B, EPI_NONE), first)


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,K", [(128, 256, 256), (1024, 768, 256), (4096, 2304, 768), (2048, 768, 3072),
                                   (24576, 768, 768), (4 * 317, 768, 768), (200, 256, 512), (24576 - 37, 3072, 768)])
def test_gemm_tn_wgrad(cuda, T, N, K, variant):
    """dW = dyᵀ·x (split-K TN kernel, fp32 out) vs fp32 torch, default and forced split counts,
    plain and accumulating; bitwise repeatable; token tails (T % 64 != 0) included."""
    if variant:
        pytest.skip("TN kernel has a single variant")
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(T + N + K)
    dy = (torch.rand(T, N, device=cuda, generator=g) * 2 - 1).bfloat16()
    x = (torch.rand(T, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    ref = dy.float().t() @ x.float()
    out = torch.empty(N, K, device=cuda)
    assert k.gemm_tn_splits(T, N, K) >= 1
    k.gemm_tn(dy, x, out, False)
    torch.testing.assert_close(out, ref, atol=1e-3 * T ** 0.5, rtol=1e-3)
    first = out.clone()
    for _ in range(3):
        k.gemm_tn(dy, x, out, False)
        assert torch.equal(out, first)
    for s in (1, 3):
        if T // 64 // s >= 2:
            k.gemm_tn(dy, x, out, False, s)
            torch.testing.assert_close(out, ref, atol=1e-3 * T ** 0.5, rtol=1e-3)
    base = torch.randn(N, K, device=cuda, generator=g)
    acc = base.clone()
    k.gemm_tn(dy, x, acc, True)
    torch.testing.assert_close(acc, base + ref, atol=1e-3 * T ** 0.5, rtol=1e-3)
    # fused bias gradient (column sums of dy), plain and accumulating
    db_ref = dy.float().sum(0)
    db = torch.full((N,), 7.0, device=cuda)
    k.gemm_tn(dy, x, out, False, 0, db)
    torch.testing.assert_close(out, ref, atol=1e-3 * T ** 0.5, rtol=1e-3)
    torch.testing.assert_close(db, db_ref, atol=1e-3 * T ** 0.5, rtol=1e-3)
    b0 = torch.randn(N, device=cuda, generator=g)
    db = b0.clone()
    k.gemm_tn(dy, x, acc, True, 0, db)
    torch.testing.assert_close(db, b0 + db_ref, atol=1e-3 * T ** 0.5, rtol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("T,N,K", [(128, 256, 256), (4 * 317, 768, 768), (200, 256, 512), (24576 - 37, 3072, 768),
                                   (98304, 2304, 768), (98304, 768, 768), (98304, 3072, 768), (98304, 768, 3072)])
def test_gemm_tn_lockstep_bitwise(cuda, T, N, K, variant):
    """The lockstep weight-gradient kernel (gemm_tn_set_variant(1): both waves of a SIMD on MFMAs, one
    barrier per K-tile) against the alternating-row kernel (5): bitwise equal (same K order per accumulator) at
    every split count tried, token tails included, repeatable over launches; the automatic choice (0) equals both."""
    if variant:
        pytest.skip("TN kernel variants are selected below")
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(T + 3 * N + K)
    dy = (torch.rand(T, N, device=cuda, generator=g) * 2 - 1).bfloat16()
    x = (torch.rand(T, K, device=cuda, generator=g) * 2 - 1).bfloat16()
    base = torch.randn(N, K, device=cuda, generator=g)
    splits = [0] + [s for s in (1, 3) if T // 64 // s >= 2]
    try:
        for s in splits:
            outs = []
            for v in (5, 1, 1, 0):
                k.gemm_tn_set_variant(v)
                out = base.clone()
                k.gemm_tn(dy, x, out, True, s)
                torch.cuda.synchronize()
                outs.append(out)
            assert torch.equal(outs[0], outs[1]), (s, (outs[0] - outs[1]).abs().max().item())
            assert torch.equal(outs[1], outs[2]), s
            assert torch.equal(outs[0], outs[3]), s
    finally:
        k.gemm_tn_set_variant(0)


@pytest.mark.gpu
def test_gemm_tn_asymmetric(cuda, variant):
    """Integer data with an asymmetric pattern: catches transposed / misplaced output tiles exactly."""
    if variant:
        pytest.skip("TN kernel has a single variant")
    k = _native.kernels()
    T, N, K = 256, 512, 256
    t = torch.arange(T, device=cuda)
    dy = ((t[:, None] * 3 + torch.arange(N, device=cuda)[None, :] * 7) % 5 - 2).float().bfloat16()
    x = ((t[:, None] * 5 + torch.arange(K, device=cuda)[None, :] * 11) % 7 - 3).float().bfloat16()
    out = torch.empty(N, K, device=cuda)
    k.gemm_tn(dy, x, out, False)
    assert torch.equal(out, dy.float().t() @ x.float())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(512, 768, 256), (256, 3072, 768)])
def test_gemm_nt_gelu_derivative_epilogues(cuda, M, N, K):
    """EPI_GELUD stores gelu'(pre) next to gelu(pre); EPI_DMUL multiplies the dgrad by it (+ column
    partials) — together the stored-derivative FFN1 forward/backward pair."""
    EPI_GELUD, EPI_DMUL = 5, 6
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(9)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    gd = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    act = k.gemm_nt(A, B, EPI_GELUD, bias=bias, pre=gd)
    pre = (_ref(A, B) + bias).bfloat16().float()          # the kernel rounds pre to bf16 first
    x = pre.clone().requires_grad_(True)
    y = torch.nn.functional.gelu(x)
    y.backward(torch.ones_like(y))
    _close(act, y.detach())
    _close(gd, x.grad, tol=1e-2)
    part = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=cuda)
    d = k.gemm_nt(A, B, EPI_DMUL, pre=gd, part=part)
    exp = _ref(A, B).bfloat16().float() * gd.float()
    _close(d, exp)
    torch.testing.assert_close(part.sum(0), exp.sum(0), atol=5e-2 * (1 + exp.abs().sum(0).max().item() / M), rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(1024, 768, 3072), (1000, 768, 2304), (2048, 768, 1024)])
def test_gemm_nt_split_k_low_fill(cuda, M, N, K, variant):
    """Split-K on the 128²-tile kernel for low-fill grids with a long K (the reference micro-batch's
    FFN2 forward / FFN1 and QKV dgrads: 48 tiles at K = 3072 / 2304): none / bias / resid epilogues
    against the fp32 oracle, rows past M untouched, bitwise repeatable (slabs folded in split order)."""
    if variant not in (0, 4):
        pytest.skip("split-K lives in the 128²-tile kernel")
    k = _native.kernels()
    assert k.gemm_nt_supported(M, N, K) == 1
    g = torch.Generator(device=cuda).manual_seed(M + K)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    ref = _ref(A, B)
    big = torch.full((M + 64, N), 7.0, device=cuda, dtype=torch.bfloat16)
    k.gemm_nt(A, B, EPI_BIAS, bias=bias, out=big[:M])
    _close(big[:M], ref + bias)
    assert torch.equal(big[M:].float(), torch.full((64, N), 7.0, device=cuda)), "rows past M were written"
    c0 = k.gemm_nt(A, B, EPI_NONE)
    _close(c0, ref)
    for _ in range(3):
        assert torch.equal(k.gemm_nt(A, B, EPI_NONE), c0)
    resid = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    _close(k.gemm_nt(A, B, EPI_RESID, resid=resid), ref + resid.float())


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(25600, 768, 768), (25600, 768, 2304), (98304, 768, 768), (25600, 768, 3072),
                                   (98304, 768, 3072)])
def test_gemm_nt_half_tile_tail(cuda, M, N, K, variant):
    """The v3 / v2 half-tile tail (a last wave of tiles at most half full runs as 128-row half tiles): 300 or
    1152 256² tiles on 256 CUs.  Every epilogue must be bitwise equal with the tail split on and off (a half
    tile accumulates its rows in the same order) and match the fp32 reference; DGELU / DMUL never split."""
    if variant not in (0, 2, 3):
        pytest.skip("the half-tile tail is a v2 / v3 schedule")
    EPI_GELUD, EPI_DMUL, EPI_BDR = 5, 6, 7
    HT = 1 << 16
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(M + K)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    resid = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    gd = torch.rand(M, N, device=cuda, generator=g).bfloat16()
    rows = torch.cat([torch.arange(0, 1024), torch.arange(M - 2048, M)]).to(cuda)
    ref = _ref(A[rows], B)

    def run(epi, **kw):
        outs = []
        for w in (0, HT):
            k.gemm_set_stagger(w)
            try:
                kk = {n: (v.clone() if torch.is_tensor(v) and n in ("pre",) and epi in (EPI_GELU, EPI_GELUD) else v)
                      for n, v in kw.items()}
                o = k.gemm_nt(A, B, epi, **kk)
                outs.append((o, kk.get("pre")))
            finally:
                k.gemm_set_stagger(HT)
        assert torch.equal(outs[0][0], outs[1][0]), f"epi {epi}: half-tile tail changed the output"
        if outs[0][1] is not None and epi in (EPI_GELU, EPI_GELUD):
            assert torch.equal(outs[0][1], outs[1][1]), f"epi {epi}: half-tile tail changed P"
        return outs[1]

    _close(run(EPI_NONE)[0][rows], ref)
    _close(run(EPI_BIAS, bias=bias)[0][rows], ref + bias)
    _close(run(EPI_RESID, resid=resid)[0][rows], ref + resid[rows].float())
    o, p = run(EPI_GELU, bias=bias, pre=torch.empty(M, N, device=cuda, dtype=torch.bfloat16))
    _close(p[rows], ref + bias)
    _close(o[rows], torch.nn.functional.gelu(p[rows].float()))
    o, _ = run(EPI_GELUD, bias=bias, pre=torch.empty(M, N, device=cuda, dtype=torch.bfloat16))
    _close(o[rows], torch.nn.functional.gelu(ref + bias))
    part = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=cuda)
    _close(run(EPI_DMUL, pre=gd, part=part)[0][rows], ref.bfloat16().float() * gd[rows].float())
    o, _ = run(EPI_BDR, bias=bias, resid=resid, p=0.0, seed=1, opid=2)
    _close(o[rows], ref + bias + resid[rows].float())
    run(EPI_BDR, bias=bias, resid=resid, p=0.1, seed=3, opid=5)   # dropout keyed by the global index: bitwise


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", [(32768, 768, 768), (8192, 3072, 256), (24576, 2304, 128)])
def test_gemm_nt_persistent_every_epilogue_full_output(cuda, M, N, K, variant):
    """The persistent v3 kernel with several tiles per workgroup (and a half-tile tail): EVERY output element
    of every epilogue against the fp32 product — the epilogue's bias staged through LDS per unit, both rounds'
    operands prefetched, the next tile's bias DMA issued at the seam."""
    if variant not in (0, 3):
        pytest.skip("the persistent kernel")
    EPI_GELUD, EPI_DMUL = 5, 6
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(M + N + K)
    A = (torch.randn(M, K, device=cuda, generator=g) * 0.5).bfloat16()
    B = (torch.randn(N, K, device=cuda, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=cuda, generator=g) * 0.1
    resid = torch.randn(M, N, device=cuda, generator=g).bfloat16()
    gd = torch.rand(M, N, device=cuda, generator=g).bfloat16()
    ref = _ref(A, B)
    _close(k.gemm_nt(A, B, EPI_NONE), ref)
    _close(k.gemm_nt(A, B, EPI_BIAS, bias=bias), ref + bias)
    _close(k.gemm_nt(A, B, EPI_RESID, resid=resid), ref + resid.float())
    pre = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    o = k.gemm_nt(A, B, EPI_GELU, bias=bias, pre=pre)
    _close(pre, ref + bias)
    _close(o, torch.nn.functional.gelu(pre.float()))
    gp = torch.empty(M, N, device=cuda, dtype=torch.bfloat16)
    o = k.gemm_nt(A, B, EPI_GELUD, bias=bias, pre=gp)
    x = (ref + bias).bfloat16().float()
    _close(o, torch.nn.functional.gelu(x))
    cdf = 0.5 * (1 + torch.erf(x / 2 ** 0.5))
    _close(gp, cdf + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5)
    rows = k.gemm_nt_part_rows(M, N, K)
    part = torch.empty(rows, N, device=cuda)
    d = k.gemm_nt(A, B, EPI_DMUL, pre=gd, part=part)
    exp_d = ref.bfloat16().float() * gd.float()
    _close(d, exp_d)
    torch.testing.assert_close(part.sum(0), exp_d.sum(0), rtol=2e-2, atol=2e-2 * float(exp_d.sum(0).abs().max()))
    part2 = torch.empty(rows, N, device=cuda)
    d2 = k.gemm_nt(A, B, EPI_DGELU, pre=pre, part=part2)
    pf = pre.float()
    gelu_grad = 0.5 * (1 + torch.erf(pf / 2 ** 0.5)) + pf * torch.exp(-0.5 * pf * pf) / (2 * torch.pi) ** 0.5
    _close(d2, ref.bfloat16().float() * gelu_grad)
