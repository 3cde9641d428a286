#!/usr/bin/env python
"""fp8 vs bf16 convergence on a LEARNABLE synthetic QA task (VERDICT r3 "fp8 convergence evidence").

Synthetic Natural-Questions documents (``data/synth_nq.py`` learnable mode: the question names a key word that
marks the answer in the document and a class word that gives the annotation type) go through the real NQ
pipeline (``RawPreprocessor`` → ``SplitDataset`` windows → ``collate_fun``), then BERT-base trains from the same
random init and the same sample order in bf16 and in ``--precision fp8`` (e4m3 forward, e5m2 backward, delayed
scaling) for ``--steps`` optimizer steps.  Recorded per step: the loss terms, the grad norm, and for fp8 the
number of delayed-scaling productions whose fresh amax exceeded the range of the scale in use (a saturating
quantisation: e4m3 448, e5m2 57344).  At the end: the reference's eval metrics on the held-out split (MAP over
the class softmax, start / end / class accuracy; MAPCallback + AccuracyCallback).

    python tools/fp8_convergence.py --precision bf16 --seed 0 --out gpurun_out/r4_fp8_conv
    python tools/fp8_convergence.py --precision fp8  --seed 0 --out gpurun_out/r4_fp8_conv

Two seeds per precision (tools/gpu/r4_fp8_conv.sh) separate fp8's effect from run-to-run divergence: the
seed sets the init and the sample order, identical for both precisions.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time
from collections import defaultdict
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def prepare(d, n_docs, seed):
    from ml_recipe_distributed_pytorch_amd.data.synth_nq import learnable_vocab, write_jsonl
    os.makedirs(d, exist_ok=True)
    vocab = learnable_vocab(os.path.join(d, "vocab.txt"))
    data = os.path.join(d, "nq_learnable.jsonl")
    if not os.path.exists(data):
        write_jsonl(data, n_docs, seed=seed, learnable=True)
    return vocab, data, os.path.join(d, "processed")


def saturation(model, by_site=None):
    """Productions (since the last call) whose amax overflowed the scale in use: state.buf = [amax slots 0-2,
    dequant scale in use]; the slot of the last phase holds the fresh amax of that production.  by_site
    (dict) accumulates the count per quantisation site and the worst overflow factor."""
    import torch
    states = getattr(model, "_fp8_states", {})
    bufs, lims, names = [], [], []
    for mod, st in states.items():
        for k, s in st.items():
            if s.step == 0:
                continue
            bufs.append(s.buf)
            lims.append((57344.0 if s.grad else 448.0, (s.step - 1) % 3))
            names.append(f"{mod}/{k}")
    if not bufs:
        return 0, 0
    b = torch.stack(bufs).cpu()
    n = 0
    for i, (lim, ph) in enumerate(lims):
        amax, scale = float(b[i, ph]), float(b[i, 3])
        if scale > 0 and amax / scale > lim * (1 + 1e-6):
            n += 1
            if by_site is not None:
                c, worst = by_site.get(names[i], (0, 0.0))
                by_site[names[i]] = (c + 1, max(worst, amax / scale / lim))
    return n, len(lims)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--n_docs", type=int, default=8000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--max_seq_len", type=int, default=384)
    ap.add_argument("--out", default="gpurun_out/r4_fp8_conv")
    ap.add_argument("--data_dir", default=os.path.join(tempfile.gettempdir(), "hq_fp8_conv_data"),
                    help="synthetic corpus + preprocessing cache (thousands of files: keep it out of --out)")
    a = ap.parse_args()

    import torch
    from torch.utils.data import DataLoader, RandomSampler
    from ml_recipe_distributed_pytorch_amd import factories
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.train.callbacks import AccuracyCallback, MAPCallback
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine, to_device
    from ml_recipe_distributed_pytorch_amd.train.meters import AverageMeter
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW, get_linear_schedule_with_warmup
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    from ml_recipe_distributed_pytorch_amd.data.items import LABELS

    os.makedirs(a.out, exist_ok=True)
    vocab, data, proc = prepare(a.data_dir, a.n_docs, 1234)
    dev = torch.device("cuda", 0)
    mp = SimpleNamespace(model="bert-base-uncased", hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1,
                         layer_norm_eps=1e-12, vocab_file=vocab, merges_file=None, lowercase=True,
                         handle_chinese_chars=False, pretrained_path=None, random_init=True,
                         legacy_tokenization=False)
    torch.manual_seed(a.seed)
    model, tok = factories.init_model(mp, device=dev, seed=a.seed, precision=a.precision)
    dp = SimpleNamespace(data_path=data, processed_data_path=proc, max_seq_len=a.max_seq_len, max_question_len=64,
                         doc_stride=128, split_by_sentence=False, truncate=False, dummy_dataset=False,
                         train_label_weights=False, train_sampler_weights=False)
    train_ds, test_ds, _ = factories.init_datasets(dp, tokenizer=tok)
    collate = factories.init_collate_fun(tok)
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    loss_fn = build_loss(lp)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=a.lr, eps=1e-6,
                     correct_bias=False, zero_grad_fn=model.zero_grad)
    sched = get_linear_schedule_with_warmup(opt, int(0.1 * a.steps), a.steps)
    eng = TrainEngine(model, loss_fn, opt, scheduler=sched, max_grad_norm=1.0)
    gen = torch.Generator().manual_seed(a.seed)
    loader = DataLoader(train_ds, batch_size=a.batch, sampler=RandomSampler(train_ds, generator=gen),
                        collate_fn=collate, drop_last=True, num_workers=4)
    log = []
    sat_total = prod_total = 0
    sat_sites, sat_steps = {}, []
    t0 = time.time()
    step = 0
    model.train()
    while step < a.steps:
        for inputs, labels in loader:
            res = eng.step([(to_device(inputs, dev), to_device(labels, dev))])
            step += 1
            rec = res.losses.to_floats()
            rec["grad_norm"] = float(res.grad_norm)
            rec["step"] = step
            rec["L"] = int(inputs["input_ids"].shape[1])
            if a.precision == "fp8":
                s, n = saturation(model, sat_sites)
                rec["fp8_saturated"], rec["fp8_productions"] = s, n
                if s:
                    sat_steps.append(step)
                sat_total += s
                prod_total += n
            log.append(rec)
            if step % 25 == 0 or step == 1:
                print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in rec.items()}),
                      flush=True)
            if step >= a.steps:
                break
    train_s = time.time() - t0
    # held-out evaluation: the reference's Trainer.test metrics
    model.eval()
    meters = defaultdict(AverageMeter)
    cbs = [MAPCallback(list(LABELS.values()) if isinstance(LABELS, dict) else list(LABELS)), AccuracyCallback()]
    test_loader = DataLoader(test_ds, batch_size=64, collate_fn=collate, num_workers=4)
    tl = []
    with torch.no_grad():
        for inputs, labels in test_loader:
            inputs, labels = to_device(inputs, dev), to_device(labels, dev)
            preds = model(**inputs)
            tl.append(float(loss_fn(preds, labels)))
            for cb in cbs:
                cb.at_iteration_end(preds, labels, meters)
    # test_loss: the mean over batches with a finite loss (a batch whose span targets are all ignored has an
    # empty mean, NaN by definition); the count of such batches is reported beside it
    for cb in cbs:
        cb.at_epoch_end(meters, None)
    ev = {k: (v() if isinstance(v, AverageMeter) else v) for k, v in meters.items()}
    finite = [x for x in tl if x == x]
    ev["test_loss"] = sum(finite) / max(1, len(finite))
    ev["test_batches_nan_loss"] = len(tl) - len(finite)
    last = log[-20:]
    summary = {"precision": a.precision, "steps": step, "batch": a.batch, "lr": a.lr, "seed": a.seed,
               "train_windows": len(train_ds), "test_windows": len(test_ds), "train_seconds": round(train_s, 1),
               "final_loss_mean_last20": sum(r["loss"] for r in last) / len(last),
               "first_loss": log[0]["loss"], "eval": ev}
    if a.precision == "fp8":
        summary["fp8_saturated_productions"] = sat_total
        summary["fp8_productions_checked"] = prod_total
        summary["fp8_saturated_steps"] = {"first": sat_steps[:10], "count": len(sat_steps),
                                          "after_step_50": sum(1 for x in sat_steps if x > 50)}
        top = sorted(sat_sites.items(), key=lambda kv: -kv[1][0])[:12]
        summary["fp8_saturated_sites_top"] = {k: {"count": c, "worst_overflow": round(w, 2)} for k, (c, w) in top}
    with open(os.path.join(a.out, f"curve_{a.precision}_s{a.seed}.jsonl"), "w") as f:
        for r in log:
            f.write(json.dumps(r) + "\n")
    with open(os.path.join(a.out, f"summary_{a.precision}_s{a.seed}.json"), "w") as f:
        json.dump(summary, f, indent=1, default=float)
    print(json.dumps(summary, default=float), flush=True)


if __name__ == "__main__":
    main()
