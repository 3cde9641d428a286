"""Run-to-run bitwise stability of the hot kernels at the headline shapes (BERT-base, B = 256, L = 384).

Every kernel here is deterministic (no atomics; split-K partials are reduced in a fixed order), so repeated
launches on the same inputs must agree bit for bit.  A launch that does not is corrupting data at random —
the signature of round 4's late store-data read (profiles/r4_epi1: a dwordx4 store picked up a VALU result
written 5 instructions after it issued, ~3e-5 of the GELU epilogue's elements, different ones each run),
which tolerance checks against an fp32 oracle only catch when a corrupted value happens to be large."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native

EPI_NONE, EPI_BIAS, EPI_GELU, EPI_DGELU, EPI_RESID, EPI_GELUD, EPI_DMUL = range(7)
T, H, F = 256 * 384, 768, 3072
REPS = 4


def _bf(shape, gen, dev, scale=1.0):
    return (torch.randn(*shape, device=dev, generator=gen) * scale).bfloat16()


def _same(outs, what):
    for i, o in enumerate(outs[1:], 1):
        for a, b in zip(outs[0], o):
            diff = (a.view(torch.int16) != b.view(torch.int16)) if a.dtype == torch.bfloat16 else (a != b)
            n = int(diff.sum())
            assert n == 0, f"{what}: launch {i} differs from launch 0 in {n} of {a.numel()} elements"


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["qkv_bias", "ffn1_gelud", "ffn1_gelu", "ffn2_dmul", "attn_out_resid", "qkv_dgrad"])
def test_gemm_nt_repeatable(cuda, name):
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(7)
    x = _bf((T, H), g, cuda, 0.5)
    n_out = {"qkv_bias": 3 * H, "ffn1_gelud": F, "ffn1_gelu": F, "ffn2_dmul": F, "attn_out_resid": H,
             "qkv_dgrad": H}[name]
    a = x if name != "qkv_dgrad" else _bf((T, 3 * H), g, cuda, 0.5)
    k_dim = a.shape[1]
    w = _bf((n_out, k_dim), g, cuda, 0.05)
    bias = torch.randn(n_out, device=cuda, generator=g) * 0.1
    outs = []
    for _ in range(REPS):
        if name == "qkv_bias":
            outs.append((k.gemm_nt(a, w, EPI_BIAS, bias=bias),))
        elif name in ("ffn1_gelud", "ffn1_gelu"):
            pre = torch.empty(T, n_out, device=cuda, dtype=torch.bfloat16)
            epi = EPI_GELUD if name == "ffn1_gelud" else EPI_GELU
            outs.append((k.gemm_nt(a, w, epi, bias=bias, pre=pre), pre))
        elif name == "ffn2_dmul":
            gd = _bf((T, n_out), torch.Generator(device=cuda).manual_seed(11), cuda)
            part = torch.zeros(k.gemm_nt_part_rows(T, n_out, k_dim) * n_out, device=cuda)
            outs.append((k.gemm_nt(a, w, EPI_DMUL, pre=gd, part=part), part))
        elif name == "attn_out_resid":
            r = _bf((T, n_out), torch.Generator(device=cuda).manual_seed(13), cuda)
            outs.append((k.gemm_nt(a, w, EPI_RESID, resid=r),))
        else:
            outs.append((k.gemm_nt(a, w, EPI_NONE),))
    torch.cuda.synchronize()
    _same(outs, name)


@pytest.mark.gpu
@pytest.mark.parametrize("n_out,k_in", [(F, H), (H, F), (3 * H, H)])
def test_gemm_tn_repeatable(cuda, n_out, k_in):
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(5)
    dy, x = _bf((T, n_out), g, cuda), _bf((T, k_in), g, cuda)
    outs = []
    for _ in range(REPS):
        out, b = torch.zeros(n_out, k_in, device=cuda), torch.zeros(n_out, device=cuda)
        k.gemm_tn(dy, x, out, False, 0, b)
        outs.append((out, b))
    torch.cuda.synchronize()
    _same(outs, f"gemm_tn {n_out}x{k_in}")


@pytest.mark.gpu
def test_attention_repeatable(cuda):
    k = _native.kernels()
    B, L, nh = 256, 384, 12
    g = torch.Generator(device=cuda).manual_seed(3)
    qkv = _bf((B * L, 3 * H), g, cuda)
    kb = torch.zeros(B, L, device=cuda)
    kb[:, 300:] = -10000.0
    dctx = _bf((B * L, H), g, cuda)
    outs = []
    for _ in range(REPS):
        ctx, lse, bits = k.attn_fwd(qkv, kb, B, L, nh, 0.1, 555, 3, 0.125)
        dq = k.attn_bwd(dctx, qkv, ctx, lse, kb, bits, B, L, nh, 0.1, 0.125, False)
        outs.append((ctx, lse, bits, dq))
    torch.cuda.synchronize()
    _same(outs, "attention")


@pytest.mark.gpu
def test_gemm_nt_v2_repeatable(cuda):
    """The K = 3072 FFN2 forward at seq 512 (M = 131072: a whole number of tile waves, no half-tile tail) runs the
    non-persistent v2 kernel, whose LDS-DMA pipeline was reworked in round 4 like the persistent one's."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(17)
    Tm = 256 * 512
    x = _bf((Tm, F), g, cuda, 0.5)
    w = _bf((H, F), g, cuda, 0.05)
    bias = torch.randn(H, device=cuda, generator=g) * 0.1
    outs = [(k.gemm_nt(x, w, EPI_BIAS, bias=bias),) for _ in range(REPS)]
    torch.cuda.synchronize()
    _same(outs, "ffn2 fwd v2 (seq 512)")


@pytest.mark.gpu
def test_gemm_nt_cross_epilogue_exact(cuda):
    """Exact guard against a store that writes the wrong register: the epilogues share the mainloop and its
    accumulation order, so GELU's stored P (pre-activation) must equal BIAS's C bit for bit, and GELUD's C (act,
    packed-FMA GELU) GELU's C (scalar GELU, same operations) bit for bit — at the headline FFN1 shape."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(23)
    x = _bf((T, H), g, cuda, 0.5)
    w = _bf((F, H), g, cuda, 0.05)
    bias = torch.randn(F, device=cuda, generator=g) * 0.1
    c_bias = k.gemm_nt(x, w, EPI_BIAS, bias=bias)
    pre = torch.empty(T, F, device=cuda, dtype=torch.bfloat16)
    c_gelu = k.gemm_nt(x, w, EPI_GELU, bias=bias, pre=pre)
    gd = torch.empty(T, F, device=cuda, dtype=torch.bfloat16)
    c_gelud = k.gemm_nt(x, w, EPI_GELUD, bias=bias, pre=gd)
    torch.cuda.synchronize()
    _same([(c_bias,), (pre,)], "GELU P vs BIAS C")
    _same([(c_gelu,), (c_gelud,)], "GELUD C vs GELU C")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["fwd_bias", "fwd_gelud", "dgrad_none", "dgrad_dmul", "dgrad_resid"])
def test_gemm_fp8_repeatable(cuda, name):
    """The fp8 GEMMs (gemm_fp8.hip: e4m3 forward, e5m2-gradient dgrads) share the LDS-DMA / epilogue structure of
    the bf16 kernels: repeated launches at the headline shapes must agree bit for bit."""
    k = _native.kernels()
    g = torch.Generator(device=cuda).manual_seed(29)
    fwd = name.startswith("fwd")
    n_out, k_in = {"fwd_bias": (3 * H, H), "fwd_gelud": (F, H), "dgrad_none": (H, F), "dgrad_dmul": (F, H),
                   "dgrad_resid": (H, 3 * H)}[name]
    A8 = (torch.randn(T, k_in, device=cuda, generator=g) * 2).to(torch.float8_e4m3fn if fwd else torch.float8_e5m2)
    B8 = (torch.randn(n_out, k_in, device=cuda, generator=g) * 2).to(torch.float8_e4m3fn)
    sa = torch.full((1,), 0.01, device=cuda)
    sb = torch.full((1,), 0.02, device=cuda)
    bias = torch.randn(n_out, device=cuda, generator=g) * 0.1
    aux = _bf((T, n_out), torch.Generator(device=cuda).manual_seed(31), cuda)
    code = torch.randint(0, 256, (T, n_out), device=cuda, dtype=torch.uint8,
                         generator=torch.Generator(device=cuda).manual_seed(37))   # gelu' code for the fp8 DMUL
    outs = []
    for _ in range(REPS):
        if name == "fwd_bias":
            outs.append((k.gemm_fp8(A8, B8, EPI_BIAS, bias, sa, sb),))
        elif name == "fwd_gelud":
            gd = torch.empty(T, n_out, device=cuda, dtype=torch.uint8)   # the 8-bit gelu' code
            act8 = torch.empty(T, n_out, device=cuda, dtype=torch.float8_e4m3fn)
            state = torch.tensor([1.0, 1.0, 1.0, 0.01], device=cuda)
            c = k.gemm_fp8(A8, B8, EPI_GELUD, bias, sa, sb, pre=gd, out8=act8, state=state, phase=0)
            outs.append((c, gd, act8.view(torch.uint8)))
        elif name == "dgrad_none":
            outs.append((k.gemm_fp8(A8, B8, EPI_NONE, None, sa, sb),))
        elif name == "dgrad_dmul":
            part = torch.zeros(T // 256, n_out, device=cuda)
            out8 = torch.empty(T, n_out, device=cuda, dtype=torch.float8_e5m2)
            state = torch.tensor([1.0, 1.0, 1.0, 0.01], device=cuda)
            c = k.gemm_fp8(A8, B8, EPI_DMUL, None, sa, sb, pre=code, out8=out8, state=state, phase=0, part=part)
            outs.append((c, part, out8.view(torch.uint8)))
        else:
            outs.append((k.gemm_fp8(A8, B8, EPI_RESID, None, sa, sb, resid=aux),))
    torch.cuda.synchronize()
    _same(outs, f"gemm_fp8 {name}")


@pytest.mark.gpu
def test_embedding_bwd_repeatable(cuda):
    """The embedding backward sorts rows by id and sums each id's rows in a fixed order (no float atomics at the
    default position ids): word / position / type / γ / β gradients bitwise equal across launches at the headline
    shape (V = 30522, 10 % padding)."""
    k = _native.kernels()
    B, L, V = 256, 384, 30522
    g = torch.Generator(device=cuda).manual_seed(37)
    ids = torch.randint(1, V, (B * L,), device=cuda, generator=g)
    ids[torch.rand(B * L, device=cuda, generator=g) < 0.1] = 0
    pids = torch.arange(L, device=cuda).repeat(B)
    tids = torch.randint(0, 2, (B * L,), device=cuda, generator=g)
    ww, wp, wt = _bf((V, H), g, cuda, 0.05), _bf((512, H), g, cuda, 0.05), _bf((2, H), g, cuda, 0.05)
    gamma, beta = torch.ones(H, device=cuda), torch.zeros(H, device=cuda)
    _, m, rs = k.embed_fwd(ids, pids, tids, ww, wp, wt, gamma, beta, 1e-12, 0.1, 41, 0)
    dy = _bf((B * L, H), g, cuda)
    outs = []
    for _ in range(REPS):
        o = [torch.empty(V, H, device=cuda), torch.empty(512, H, device=cuda), torch.empty(2, H, device=cuda),
             torch.empty(H, device=cuda), torch.empty(H, device=cuda)]
        k.embed_bwd(dy, ids, pids, tids, ww, wp, wt, gamma, m, rs, 0.1, 41, 0, *o, False, 0, -1, L)
        outs.append(tuple(o))
    torch.cuda.synchronize()
    _same(outs, "embed_bwd")
