#!/usr/bin/env python
"""Baseline for ``bench.py``: the reference recipe's training step re-run on MI355X (BASELINE.md
"Baseline to beat": HF ``BertModel`` + the recipe's QA heads/loss, ``torch.autocast(bf16)`` in place
of apex O1, stock AdamW, ``clip_grad_norm_``, linear warmup, DDP over RCCL when launched with
torchrun).  Same synthetic data shape and timing protocol as ``bench.py``.

    python tools/ref_recipe_bench.py --batch 64 --attn eager|sdpa [--steps 20 --warmup 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class RefQA(nn.Module):
    """HF encoder + the recipe's heads (reference ``model.py:13-73`` behaviour)."""

    def __init__(self, attn: str):
        super().__init__()
        from transformers import BertConfig, BertModel
        cfg = BertConfig()
        cfg._attn_implementation = attn
        self.transformer = BertModel(cfg)
        H = cfg.hidden_size
        self.position_outputs = nn.Linear(H, 2)
        self.classifier = nn.Sequential(nn.Dropout(cfg.hidden_dropout_prob), nn.Linear(H, 5))
        self.reg_start = nn.Sequential(nn.Linear(H, 1), nn.Sigmoid())
        self.reg_end = nn.Sequential(nn.Linear(H, 1), nn.Sigmoid())

    def forward(self, input_ids, attention_mask, token_type_ids):
        out = self.transformer(input_ids=input_ids, attention_mask=attention_mask, token_type_ids=token_type_ids)
        seq, pooled = out[0], out[1]
        s, e = self.position_outputs(seq).split(1, dim=-1)
        return {"start_class": s.squeeze(-1), "end_class": e.squeeze(-1), "cls": self.classifier(pooled),
                "start_reg": self.reg_start(pooled).squeeze(-1), "end_reg": self.reg_end(pooled).squeeze(-1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--seq", type=int, default=384)
    ap.add_argument("--attn", default="eager", choices=["eager", "sdpa"])
    a = ap.parse_args()
    import torch.distributed as dist
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    torch.manual_seed(1234)
    model = RefQA(a.attn).to(device).train()
    if world > 1:
        model = nn.parallel.DistributedDataParallel(model, device_ids=[local])
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    loss_fn = build_loss(lp).to(device)
    nd = ("bias", "LayerNorm.weight")
    named = list(model.named_parameters())
    groups = [{"params": [p for n, p in named if not any(x in n for x in nd)], "weight_decay": 1e-4},
              {"params": [p for n, p in named if any(x in n for x in nd)], "weight_decay": 0.0}]
    opt = torch.optim.AdamW(groups, lr=1e-5, eps=1e-6)
    total = a.warmup + a.steps
    warm = max(1, int(0.05 * total))
    sched = torch.optim.lr_scheduler.LambdaLR(
        opt, lambda s: s / warm if s < warm else max(0.0, (total - s) / max(1, total - warm)))
    sp = SpecialIds()
    B, L = a.batch, a.seq
    batch = synth_batch_native(B, L, 64, sp, seed=rank)
    inputs = {k: v.to(device) for k, v in batch[0].items()}
    labels = {k: v.to(device) for k, v in batch[1].items()}

    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            preds = model(**inputs)
        loss = loss_fn({k: v.float() for k, v in preds.items()}, labels)
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        opt.step()
        sched.step()
        opt.zero_grad(set_to_none=True)
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": "reference-recipe samples/s (HF BertModel + autocast bf16 + AdamW)",
                          "value": round(world * B * a.steps / el, 2), "ms_per_step": round(el / a.steps * 1e3, 3),
                          "n_gpus": world, "batch_per_gpu": B, "seq_len": L, "attn": a.attn,
                          "final_loss": round(float(loss.item()), 4)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
