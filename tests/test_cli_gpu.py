"""The drop-in CLI on the GPU: ``python modules/train.py -c config/test_bert.cfg --local_rank 0`` (BERT-base, seq 512,
256 per step as the reference's batch_split 128 — merged into exact-objective passes on the GPU), one real epoch
with checkpoints, in bf16, fp8 and fp32; then ``python modules/validate.py`` (BASELINE config #5's eval pass, dummy
chunk dataset) on the written ``last.ch``.  Each run is its own process, as a user launches it
(reference ``modules/train.py:125-167``, ``modules/validate.py:29-63``, ``config/test_bert.cfg:76-77``)."""
import json
import math
import os
import re
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = os.path.join(ROOT, "config", "test_bert.cfg")

pytestmark = pytest.mark.gpu


def _cfg(tmp_path, **over):
    lines = []
    for line in open(BASE).read().splitlines():
        key = line.split("=")[0].strip()
        if key in over:
            line = f"{key} = {over.pop(key)}"
        lines.append(line)
    lines += [f"{k} = {v}" for k, v in over.items()]
    p = tmp_path / "gpu_run.cfg"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _run(cmd, cwd, timeout=400):
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=cwd, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    return r


@pytest.mark.parametrize("precision,extra", [
    ("bf16", []),
    ("fp8", []),
    # fp32 (the reference's Apex-off mode): the row-wise ops run as the fp32 oracle ops, so a smaller step
    ("fp32", ["--train_batch_size", "16", "--batch_split", "2", "--max_seq_len", "128"]),
])
def test_train_then_validate_gpu(cuda, tmp_path, precision, extra):
    dlen = 512 if precision != "fp32" else 64
    cfg = _cfg(tmp_path, debug="False", n_epochs="1", dummy_dataset_len=str(dlen), experiment_name="gpu",
               dump_dir=str(tmp_path), test_batch_size="64")
    r = _run([sys.executable, os.path.join(ROOT, "modules", "train.py"), "-c", cfg, "--local_rank", "0",
              "--precision", precision, "--random_init"] + extra, cwd=str(tmp_path))
    exp = tmp_path / "gpu"
    log = open(next(exp.glob("*.log"))).read()
    assert "Used device: cuda" in log, log[-2000:]
    for f in ("last.ch", "epoch_1.ch"):
        assert (exp / f).exists(), (f, log[-3000:])
    st = torch.load(exp / "last.ch", weights_only=True, map_location="cpu")
    bs = 256 if not extra else 16
    assert st["global_step"] == dlen // bs and st["epoch"] == 1
    assert all(torch.isfinite(v).all() for v in st["model"].values() if v.is_floating_point())
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    ev = list((tmp_path / "board" / "gpu").glob("events.out.tfevents.*"))
    vals = {t: v for _, t, v in read_events(str(ev[0]))}
    assert math.isfinite(vals["train/loss"]) and math.isfinite(vals["test/loss"]) and 0 <= vals["test/map"] <= 1
    # validate.py on that checkpoint (dummy chunk dataset: every document in several windows)
    vcfg = os.path.join(ROOT, "config", "validate.cfg")
    pred = tmp_path / "pred.json"
    v = _run([sys.executable, os.path.join(ROOT, "modules", "validate.py"), "-c", vcfg, "--checkpoint",
              str(exp / "last.ch"), "--dummy_dataset", "--dummy_dataset_len", "24", "--data_path", "x",
              "--processed_data_path", "x", "--gpu", "--precision", precision, "--max_seq_len",
              "512" if not extra else "128", "--dump_predictions", str(pred), "--n_jobs", "0"], cwd=str(tmp_path))
    out = v.stdout + v.stderr
    m = re.search(r"Validation metrics: (.*)", out)
    assert m, out[-3000:]
    nums = [float(x) for x in re.findall(r": (-?[0-9.]+(?:e-?[0-9]+)?)", m.group(1))]
    assert nums and all(math.isfinite(x) for x in nums), m.group(1)
    assert pred.exists() and json.load(open(pred))
