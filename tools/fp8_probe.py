#!/usr/bin/env python
"""Probe fp8 GEMM support (torch._scaled_mm → hipBLASLt, OCP e4m3fn on gfx950) at BERT shapes."""
import json
import torch


def timeit(fn, iters=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e3


dev = torch.device("cuda")
for dt in ("float8_e4m3fn", "float8_e4m3fnuz"):
    print(dt, hasattr(torch, dt))
T = 98304
for N, K in ((2304, 768), (3072, 768), (768, 3072), (768, 768)):
    a = torch.randn(T, K, device=dev)
    b = torch.randn(N, K, device=dev)
    ref = (a.bfloat16() @ b.bfloat16().t()).float()
    out = {"N": N, "K": K}
    try:
        sa = a.abs().max() / 448.0
        sb = b.abs().max() / 448.0
        a8 = (a / sa).to(torch.float8_e4m3fn)
        b8 = (b / sb).to(torch.float8_e4m3fn)
        y = torch._scaled_mm(a8, b8.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)
        out["rel_err"] = ((y.float() - ref).norm() / ref.norm()).item()
        out["fp8_us"] = round(timeit(lambda: torch._scaled_mm(a8, b8.t(), scale_a=sa, scale_b=sb,
                                                               out_dtype=torch.bfloat16)), 1)
    except Exception as e:  # noqa
        out["fp8_error"] = str(e)[:300]
    ab, bb = a.bfloat16(), b.bfloat16()
    out["bf16_us"] = round(timeit(lambda: ab @ bb.t()), 1)
    print(json.dumps(out), flush=True)
