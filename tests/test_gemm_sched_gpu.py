"""Persistent v3 GEMM tile schedule (gemm.hip, gemm_nt3_kernel): the dynamic per-XCD ticket schedule
must compute exactly what the static round-robin schedule computes — every tile once, same values —
on repeated launches (the kernel re-zeroes its counters on exit), under a concurrent CU-holding kernel
on another stream (tiles then land on other workgroups), and inside a captured HIP graph."""
import pytest
import torch

from ml_recipe_distributed_pytorch_amd import _native
from tools.diag import cu_hog

EPI_BIAS, EPI_RESID, EPI_GELUD, EPI_DMUL = 1, 4, 5, 6
# grids above 2 x 256 workgroups (the dynamic schedule's range): 768, 555 and 1152 tiles of 256² (555 and 1152 end in a
# half-full wave: the half-tile tail, whose units a workgroup may draw back to back under the hog)
SHAPES = [(16384, 3072, 768), (9472, 3840, 256), (65536, 768, 1536), (98304, 768, 768)]


def _operands(dev, M, N, K, epi, seed):
    k = _native.kernels()
    g = torch.Generator(device=dev).manual_seed(seed)
    A = torch.randn(M, K, device=dev, generator=g).bfloat16()
    B = (torch.randn(N, K, device=dev, generator=g) * 0.05).bfloat16()
    kw = {}
    if epi in (EPI_BIAS, EPI_GELUD):
        kw["bias"] = torch.randn(N, device=dev, generator=g)
    if epi == EPI_GELUD:
        kw["pre"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    if epi == EPI_DMUL:
        kw["pre"] = torch.rand(M, N, device=dev, generator=g).bfloat16()
        kw["part"] = torch.empty(k.gemm_nt_part_rows(M, N, K), N, device=dev)
    if epi == EPI_RESID:
        kw["resid"] = torch.randn(M, N, device=dev, generator=g).bfloat16()
    return A, B, kw


def _run(A, B, epi, kw):
    k = _native.kernels()
    C = k.gemm_nt(A, B, epi, **kw)
    outs = [C.clone()]
    if epi == EPI_GELUD:
        outs.append(kw["pre"].clone())
    if epi == EPI_DMUL:
        outs.append(kw["part"].clone())
    return outs


@pytest.fixture
def sched_reset():
    k = _native.kernels()
    k.gemm_set_variant(3)
    yield k
    k.gemm_set_sched(0)
    k.gemm_set_variant(0)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K", SHAPES)
@pytest.mark.parametrize("epi", [EPI_BIAS, EPI_RESID, EPI_GELUD, EPI_DMUL])
def test_dynamic_schedule_bitwise_equals_static(cuda, sched_reset, M, N, K, epi):
    k = sched_reset
    A, B, kw = _operands(cuda, M, N, K, epi, seed=M + N + K + epi)
    k.gemm_set_sched(0)
    ref = _run(A, B, epi, kw)
    k.gemm_set_sched(1)
    side = torch.cuda.Stream(cuda)
    for rep in range(3):   # counters must be re-zeroed by the previous launch
        if rep == 2:       # tiles move to other workgroups while 32 CUs are held on another stream
            with torch.cuda.stream(side):
                cu_hog(32, 150)
        got = _run(A, B, epi, kw)
        torch.cuda.synchronize()
        for r, g in zip(ref, got):
            assert torch.equal(r, g), f"rep {rep}: dynamic schedule differs from static"
    if epi == EPI_BIAS:   # and it is the right product
        exp = A.float() @ B.float().t() + kw["bias"]
        err = (ref[0].float() - exp).abs().max().item()
        assert err <= 2e-2 * exp.abs().max().item()


@pytest.mark.gpu
def test_dynamic_schedule_in_graph(cuda, sched_reset):
    k = sched_reset
    M, N, K = SHAPES[0]
    A, B, kw = _operands(cuda, M, N, K, EPI_BIAS, seed=7)
    k.gemm_set_sched(0)
    ref = _run(A, B, EPI_BIAS, kw)[0]
    k.gemm_set_sched(1)
    C = torch.empty_like(ref)
    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        k.gemm_nt(A, B, EPI_BIAS, out=C, **kw)   # eager first use allocates the schedule slot
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        k.gemm_nt(A, B, EPI_BIAS, out=C, **kw)
    for _ in range(4):
        C.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(C, ref)
