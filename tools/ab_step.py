#!/usr/bin/env python
"""In-process A/B of full training steps (BERT-base, the bench.py step) under runtime toggles, so small
per-step differences are not swamped by box-to-box variance.  Rounds alternate A and B; prints the
median ms/step of each.

    python tools/ab_step.py --toggle gelu_deriv [--batch 256] [--rounds 4] [--steps 8]
toggles: fp8_persist (with --precision fp8), tn_lockstep (weight-gradient kernel: lockstep vs alternating rows), gemm_v1 (NT kernel v2 vs v1), halftail (GEMM half-tile tail on / off),
         input_pipeline (on: bench.py's per-step host synthesis + pinned H2D; off: one resident batch)
"""
import argparse
import json
import os
import statistics
import sys
import time
from types import SimpleNamespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ml_recipe_distributed_pytorch_amd import _native, ops  # noqa: E402
from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native  # noqa: E402
from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering  # noqa: E402
from ml_recipe_distributed_pytorch_amd.models.config import get_config  # noqa: E402
from ml_recipe_distributed_pytorch_amd.models.losses import build_loss  # noqa: E402
from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device  # noqa: E402
from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW  # noqa: E402
from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups  # noqa: E402


_MODEL = {}


def set_toggle(name, on):
    if name == "wgrad_stream":   # weight-gradient GEMMs on a side stream (HQ_WGRAD_STREAM)
        m = _MODEL["m"]
        if on and getattr(m, "_ab_side", None) is None:
            m._ab_side = torch.cuda.Stream(device=torch.device("cuda", 0))
        m.grad_side_stream = m._ab_side if on else None
    elif name == "tn_lockstep":   # on: lockstep weight-gradient kernel everywhere (1); off: alternating rows (5)
        _native.kernels().gemm_tn_set_variant(1 if on else 5)
    elif name == "tn_auto":   # on: automatic choice (0, production); off: alternating rows everywhere (5)
        _native.kernels().gemm_tn_set_variant(0 if on else 5)
    elif name == "gemm_v1":
        _native.kernels().gemm_set_variant(1 if on else 0)
    elif name == "gemm_v2":   # on: per-tile v2 everywhere; off: auto (persistent v3 for K <= 2304)
        _native.kernels().gemm_set_variant(2 if on else 0)
    elif name == "halftail":   # on: v2 / v3 half-tile tail (+ v3 at K = 3072 when it applies); off: neither
        _native.kernels().gemm_set_stagger((1 << 16) if on else 0)
    elif name == "store_nt":   # on: streamed epilogue stores at K <= 768 (production); off: default policy
        _native.kernels().gemm_set_store_policy(1 if on else 0)
    elif name == "store_nt_all":   # on: streamed epilogue stores at every K; off: only at K <= 768 (production)
        _native.kernels().gemm_set_store_policy(2 if on else 1)
    elif name == "fp8_persist":   # on: every fp8 GEMM on the persistent kernel (3); off: auto (0, production)
        _native.kernels().gemm_fp8_set_variant(3 if on else 0)
    elif name == "input_pipeline":
        pass
    else:
        raise SystemExit(f"unknown toggle {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--toggle", required=True)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq", type=int, default=384)
    ap.add_argument("--model", default="bert-base-uncased")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--only", choices=["off", "on"], default=None,
                    help="run one arm only (for a kernel-trace profile of that arm)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = get_config(a.model)
    model = BertForQuestionAnswering(cfg, seed=0, precision=a.precision).to(dev).train()
    _MODEL["m"] = model
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, w_start=1, w_end=1, w_start_reg=1, w_end_reg=1, w_cls=1)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=1e-5, correct_bias=False,
                     zero_grad_fn=model.zero_grad)
    eng = TrainEngine(model, build_loss(lp), opt, max_grad_norm=1.0)
    sp = SpecialIds()
    batch = synth_batch_native(a.batch, a.seq, 64, sp, seed=0)
    inputs, labels = to_device(batch[0], dev), to_device(batch[1], dev)
    from ml_recipe_distributed_pytorch_amd.data.dummy import _refill
    slots = [synth_batch_native(a.batch, a.seq, 64, sp, seed=i) for i in range(2)]
    events = [torch.cuda.Event() for _ in slots]
    for e in events:
        e.record()
    cnt = [0]

    def piped():  # bench.py's next_batch
        i = cnt[0]
        s = i % 2
        events[s].synchronize()
        _refill(slots[s], sp, 64, seed=7919 * (i + 2))
        di = {k: v.to(dev, non_blocking=True) for k, v in slots[s][0].items()}
        dl = {k: v.to(dev, non_blocking=True) for k, v in slots[s][1].items()}
        events[s].record()
        cnt[0] += 1
        return di, dl

    def batch_for(on):
        return piped() if (a.toggle == "input_pipeline" and on) else (inputs, labels)
    res = {False: [], True: []}
    for r in range(a.rounds + 1):
        for on in ((False, True) if a.only is None else ((a.only == "on"),)):
            set_toggle(a.toggle, on)
            eng.step([batch_for(on)])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                eng.step([batch_for(on)])
            torch.cuda.synchronize()
            if r > 0:  # round 0 = warm-up of both arms
                res[on].append((time.perf_counter() - t0) / a.steps * 1e3)
    if a.only is not None:
        print(json.dumps({"toggle": a.toggle, "arm": a.only, "ms": round(statistics.median(res[a.only == "on"]), 3)}))
        return
    out = {"toggle": a.toggle, "batch": a.batch, "off_ms": round(statistics.median(res[False]), 3),
           "on_ms": round(statistics.median(res[True]), 3), "off_all": [round(x, 2) for x in res[False]],
           "on_all": [round(x, 2) for x in res[True]]}
    out["on_speedup"] = round(out["off_ms"] / out["on_ms"], 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
