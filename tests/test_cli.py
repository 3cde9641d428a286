"""End-to-end CLI on CPU (BASELINE config #1 shape, tiny model): train (debug + real epochs), resume,
interrupt checkpoint, 2-rank gloo launch, validate (dummy + NQ path), train_metrics (D9 fix)."""
import os
import subprocess
import sys

import pytest
import torch

from conftest import FIXTURES, free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BASE = os.path.join(ROOT, "config", "test_bert.cfg")
VTINY = ["--model", "bert-tiny-test", "--max_seq_len", "48", "--max_question_len", "8", "--n_jobs", "0"]
TINY = VTINY + ["--test_batch_size", "8"]


def _cfg(tmp_path, **over):
    over.setdefault("batch_split", "1")  # the shipped cfg keeps the reference's 128 (micro-batch 2 of 256)
    text = open(BASE).read()
    lines = []
    for line in text.splitlines():
        key = line.split("=")[0].strip()
        if key in over:
            line = f"{key} = {over.pop(key)}"
        lines.append(line)
    lines += [f"{k} = {v}" for k, v in over.items()]
    p = tmp_path / "run.cfg"
    p.write_text("\n".join(lines) + "\n")
    return str(p)


def _train(argv):
    from ml_recipe_distributed_pytorch_amd.cli.train import main
    main(argv)


def test_train_debug_smoke(tmp_path):
    """test_bert.cfg semantics: debug → one step per epoch, 2 epochs, nothing saved, TB + configs written."""
    _train(["-c", BASE, "--dump_dir", str(tmp_path), "--train_batch_size", "8", "--batch_split", "2",
            "--dummy_dataset_len", "32"] + TINY)
    exp = tmp_path / "test"
    assert (exp / "trainer.cfg").exists() and (exp / "model.cfg").exists()
    assert list(exp.glob("*.log"))
    assert not list(exp.glob("*.ch"))
    ev = list((tmp_path / "board" / "test").glob("events.out.tfevents.*"))
    assert ev
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    tags = {t for _, t, _ in read_events(str(ev[0]))}
    assert {"train/loss", "train/lr", "test/loss", "test/map", "test/c_acc"} <= tags


def test_train_resume_and_interrupt(tmp_path, monkeypatch):
    cfg = _cfg(tmp_path, debug="False", n_epochs="1", train_batch_size="8", batch_split="1",
               dummy_dataset_len="32", experiment_name="exp")
    _train(["-c", cfg, "--dump_dir", str(tmp_path)] + TINY)
    exp = tmp_path / "exp"
    for f in ("last.ch", "epoch_1.ch", "best.ch"):
        assert (exp / f).exists(), f
    st = torch.load(exp / "last.ch", weights_only=True)
    assert st["global_step"] == 4 and st["epoch"] == 1
    assert set(st) >= {"model", "optimizer", "scheduler", "global_step"}
    # resume: epoch 2 continues from step 4 with the restored optimizer (no --drop_optimizer)
    cfg2 = _cfg(tmp_path, debug="False", n_epochs="2", train_batch_size="8", batch_split="1",
                dummy_dataset_len="32", experiment_name="exp", drop_optimizer="False")
    _train(["-c", cfg2, "--dump_dir", str(tmp_path), "--last", str(exp / "last.ch")] + TINY)
    st2 = torch.load(exp / "last.ch", weights_only=True)
    assert st2["global_step"] == 8 and st2["epoch"] == 2 and (exp / "epoch_2.ch").exists()
    # the resumed epoch follows the NEW run's schedule (8 steps, warmup 4): the LR never collapses to 0
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    ev = list((tmp_path / "board" / "exp").glob("events.out.tfevents.*"))
    lrs = {step: v for step, t, v in read_events(str(ev[0])) if t == "train/lr"}
    assert sorted(lrs) == [5, 6, 7, 8] and all(v > 0 for s_, v in lrs.items() if s_ < 8), lrs
    # fault injection: KeyboardInterrupt at step 3 → interrupt.ch holds step 3
    monkeypatch.setenv("HQ_FAULT", "0:3:interrupt")
    trace = tmp_path / "samples.jsonl"
    monkeypatch.setenv("HQ_TRACE_SAMPLES", str(trace))
    cfg3 = _cfg(tmp_path, debug="False", n_epochs="1", train_batch_size="8", batch_split="1",
                dummy_dataset_len="32", experiment_name="exp3")
    _train(["-c", cfg3, "--dump_dir", str(tmp_path)] + TINY)
    st3 = torch.load(tmp_path / "exp3" / "interrupt.ch", weights_only=True)
    assert st3["global_step"] == 3 and st3["epoch"] == 1 and st3["epoch_complete"] is False
    # resuming interrupt.ch finishes the interrupted epoch (1 step left) instead of skipping it
    monkeypatch.delenv("HQ_FAULT")
    _train(["-c", cfg3, "--dump_dir", str(tmp_path), "--last", str(tmp_path / "exp3" / "interrupt.ch")] + TINY)
    st4 = torch.load(tmp_path / "exp3" / "last.ch", weights_only=True)
    assert st4["global_step"] == 4 and st4["epoch"] == 1 and st4["epoch_complete"] is True
    # the interrupted run consumed 3 micro-batches, the resumed one the 4th: together exactly one permutation
    # of the 32 samples, none repeated (the sampler order depends on (seed, epoch) only, not the global RNG)
    import json
    rec = [json.loads(x) for x in trace.read_text().splitlines()]
    assert [r["epoch"] for r in rec] == [1, 1, 1, 1]
    idx = [i for r in rec for i in r["idx"]]
    assert sorted(idx) == list(range(32)), idx


def test_profiling_outputs(tmp_path):
    """--profile writes perf/* phase timers (incl. perf/comm_ms) and
    --torch_profile_dir exports a torch.profiler Chrome trace of the chosen optimizer steps."""
    cfg = _cfg(tmp_path, debug="False", n_epochs="1", train_batch_size="8", batch_split="1",
               dummy_dataset_len="48", experiment_name="prof")
    tdir = tmp_path / "trace"
    _train(["-c", cfg, "--dump_dir", str(tmp_path), "--profile", "--torch_profile_dir", str(tdir),
            "--torch_profile_steps", "2:4", "--random_init"] + TINY)
    traces = list(tdir.glob("trace_rank0_steps2-4.json"))
    assert traces and traces[0].stat().st_size > 0
    import json
    assert "traceEvents" in json.load(open(traces[0]))
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    ev = list((tmp_path / "board" / "prof").glob("events.out.tfevents.*"))
    tags = {t for _, t, _ in read_events(str(ev[0]))}
    assert {"perf/samples_per_sec", "perf/step_ms", "perf/fwd_ms", "perf/bwd_ms", "perf/comm_ms"} <= tags


@pytest.mark.slow
def test_train_two_rank_gloo_spawn(tmp_path):
    cfg = _cfg(tmp_path, debug="False", n_epochs="1", train_batch_size="4", batch_split="1",
               dummy_dataset_len="32", experiment_name="dp2")
    cmd = [sys.executable, os.path.join(ROOT, "modules", "train.py"), "-c", cfg, "--dump_dir", str(tmp_path),
           "--local_rank", "0", "--nproc_per_node", "2", "--dist_backend", "gloo",
           "--dist_init_method", f"tcp://127.0.0.1:{free_port()}"] + TINY
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    st = torch.load(tmp_path / "dp2" / "last.ch", weights_only=True)
    assert st["global_step"] == 4  # 32 samples / (4 per rank × 2 ranks)


def test_validate_and_train_metrics(tmp_path, host_lib):
    from ml_recipe_distributed_pytorch_amd.cli import train_metrics, validate
    from ml_recipe_distributed_pytorch_amd.data.synth_nq import write_jsonl
    vocab = os.path.join(FIXTURES, "toy_vocab.txt")
    data = str(tmp_path / "nq.jsonl")
    write_jsonl(data, 40, seed=3, vocab_file=vocab)
    cfg = _cfg(tmp_path, debug="False", n_epochs="1", train_batch_size="8", dummy_dataset="False",
               data_path=data, processed_data_path=str(tmp_path / "proc"), vocab_file=vocab,
               experiment_name="nq", doc_stride="16")
    _train(["-c", cfg, "--dump_dir", str(tmp_path)] + TINY)
    ck = str(tmp_path / "nq" / "best.ch")
    assert os.path.exists(ck)
    vcfg = os.path.join(ROOT, "config", "validate.cfg")
    pred = validate.cli(["-c", vcfg, "--checkpoint", ck, "--data_path", data, "--processed_data_path",
                         str(tmp_path / "proc"), "--vocab_file", vocab, "--dump_predictions",
                         str(tmp_path / "pred.json"), "--limit", "None"] + VTINY)
    m = pred.metrics()
    assert m["chunks"] > 0 and 0.0 <= m.get("label_accuracy", 0.0) <= 1.0
    assert (tmp_path / "pred.json").exists()
    pred2 = validate.cli(["-c", vcfg, "--checkpoint", "None", "--dummy_dataset", "--dummy_dataset_len", "6",
                          "--data_path", "x", "--processed_data_path", "x"] + VTINY)
    assert pred2.n_chunks == 18
    out = train_metrics.cli(["-c", cfg, "--dump_dir", str(tmp_path), "--checkpoint", ck] + TINY)
    assert "map" in out["test"] and "c_acc" in out["train"]


def test_launch_plan_arithmetic(monkeypatch):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.parallel.launch import clamp_jobs, make_plan
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    p = SimpleNamespace(gpu=False, nproc_per_node=4, local_rank=1, dist_world_size=2, dist_backend="nccl",
                        dist_init_method="tcp://127.0.0.1:1")
    plan = make_plan(p)
    assert plan.world_size == 8 and plan.spawn and plan.backend == "gloo"
    assert [plan.global_rank(i) for i in range(4)] == [4, 5, 6, 7]  # node 1 of 2
    p.local_rank = -1
    with pytest.raises(AttributeError):
        make_plan(p)
    p.nproc_per_node, p.dist_world_size = 1, 1
    assert not make_plan(p).distributed  # D5: a single process needs no process group
    monkeypatch.setenv("RANK", "3")
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("LOCAL_RANK", "3")
    plan = make_plan(p)
    assert plan.env and not plan.spawn and plan.world_size == 4 and plan.global_rank(0) == 3  # D4
    assert clamp_jobs(16, 64) == 1  # D20: never 0 workers


def test_reference_config_verbatim_runs(tmp_path):
    """Drop-in contract: the UNMODIFIED reference test_bert.cfg (tests/fixtures, verbatim) runs through the
    reference launch shim ``modules/train.py --local_rank 0`` with batch_split = 128 semantics (micro-batches
    of 2; on CPU auto_batch_split stays off) — only the model size / sequence length are overridden."""
    cfg = os.path.join(ROOT, "tests", "fixtures", "reference_test_bert.cfg")
    cmd = [sys.executable, os.path.join(ROOT, "modules", "train.py"), "-c", cfg, "--dump_dir", str(tmp_path),
           "--local_rank", "0"] + VTINY
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    log = open(next((tmp_path / "test").glob("*.log"))).read()
    # 2 epochs x 10000 samples / micro-batch 2 // batch_split 128 = 78 optimizer steps
    assert "#Training steps: 78." in log and "auto_batch_split: batch_split" not in log
    from ml_recipe_distributed_pytorch_amd.utils.tb import read_events
    ev = list((tmp_path / "board" / "test").glob("events.out.tfevents.*"))
    steps = sorted({s for s, t, _ in read_events(str(ev[0])) if t == "train/loss"})
    assert steps == [1, 2]  # debug: one optimizer step per epoch, two epochs


def test_resume_mid_second_epoch_replays_its_permutation(tmp_path, monkeypatch):
    """Interrupt in epoch 2 (after the first epoch and the dropout seeds have consumed the global RNG): the
    resumed run must finish exactly the rest of epoch 2's permutation (world 1: RandomSampler)."""
    import json
    cfg = _cfg(tmp_path, debug="False", n_epochs="2", train_batch_size="8", batch_split="2",
               dummy_dataset_len="32", experiment_name="ep2")
    trace = tmp_path / "s.jsonl"
    monkeypatch.setenv("HQ_TRACE_SAMPLES", str(trace))
    monkeypatch.setenv("HQ_FAULT", "0:6:interrupt")
    _train(["-c", cfg, "--dump_dir", str(tmp_path)] + TINY)
    st = torch.load(tmp_path / "ep2" / "interrupt.ch", weights_only=True)
    assert st["global_step"] == 6 and st["epoch"] == 2 and st["epoch_complete"] is False
    monkeypatch.delenv("HQ_FAULT")
    _train(["-c", cfg, "--dump_dir", str(tmp_path), "--last", str(tmp_path / "ep2" / "interrupt.ch")] + TINY)
    rec = [json.loads(x) for x in trace.read_text().splitlines()]
    e2 = [i for r in rec if r["epoch"] == 2 for i in r["idx"]]
    assert sorted(e2) == list(range(32)), e2            # 4 micro-batches before, 4 after, no repeats
    e1 = [i for r in rec if r["epoch"] == 1 for i in r["idx"]]
    assert sorted(e1) == list(range(32)) and e1 != e2   # a new permutation each epoch
