"""The native RCCL gradient reducer inside a real BERT-base training step, on one GPU.

With ``force=True`` the reducer keeps a 1-rank RCCL communicator active, so every bucket of the backward
goes through the multi-GPU path (arena slice → fence → ncclAllReduce(avg) on the reducer's comm stream
→ compute-stream wait) — the 8-GPU code path minus the peers.  Averaging over one rank is the identity,
so the weights after each step must be BITWISE equal to a run without a reducer; and with the
weight-gradient GEMMs on a side stream (``HQ_WGRAD_STREAM=1``) the comm-stream checksums taken where the
all-reduce reads each bucket must equal the final gradients (stream-ordering test).

One optimizer step without clipping, so every element is independent: the word / position embedding
gradients are scattered with float atomics (norm.hip embed_bwd, order-nondeterministic), which would
otherwise leak through the global grad norm into every parameter.  Those two tensors are compared with a
tolerance, everything else bitwise."""
import pytest
import torch

pytestmark = pytest.mark.gpu


_ATOMIC = ("word_embeddings", "position_embeddings")


@pytest.fixture(autouse=True)
def _deterministic(monkeypatch):
    """Bitwise comparisons need the deterministic attention backward (ops.deterministic)."""
    monkeypatch.setenv("HQ_DETERMINISTIC", "1")


def _engine(dev, reducer_kw=None, seed=11, clip=0.0):
    from types import SimpleNamespace
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.parallel.reducer import GradReducer
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups
    model = BertForQuestionAnswering(get_config("bert-base-uncased"), seed=seed).to(dev).train()
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    opt = FusedAdamW(optimizer_groups(model.named_parameters(), 1e-4), model.store, lr=1e-4, eps=1e-6,
                     correct_bias=False, zero_grad_fn=model.zero_grad)
    red = GradReducer(model, force=True, **reducer_kw) if reducer_kw is not None else None
    return model, red, TrainEngine(model, build_loss(lp), opt, reducer=red, max_grad_norm=clip)


def _batches(dev, n=2, B=8, L=128):
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.train.engine import to_device
    out = []
    for i in range(n):
        inputs, labels = synth_batch_native(B, L, 32, SpecialIds(), seed=100 + i)
        out.append((to_device(inputs, dev), to_device(labels, dev)))
    return out


def _run(dev, reducer_kw, batches):
    model, red, eng = _engine(dev, reducer_kw)
    torch.manual_seed(1234)  # the model draws each step's dropout seed from the torch CPU generator
    checks, grads = [], []
    for inputs, labels in batches:  # TrainEngine.micro_step, with the gradients captured before the update
        if red is not None:
            red.prepare(sync=True)
        eng.loss_fn(model(**inputs), labels).backward()
        side = getattr(model, "grad_side_stream", None)
        if side is not None:
            torch.cuda.current_stream().wait_stream(side)
        if red is not None:
            red.finalize()
        torch.cuda.synchronize()
        grads.append(model.store.grad.clone())
        if red is not None and red.verify:
            checks.append(red.check_order())
        eng._apply()  # clip (off) + fused AdamW + zero_grad
    master = model.store.master.clone()
    kind, nb = (red.kind, red.n_buckets) if red is not None else ("none", 0)
    if red is not None:
        red.close()
    atomic = torch.zeros(model.store.total, dtype=torch.bool, device=dev)
    for e in model.store.entries:
        if any(a in e.key for a in _ATOMIC):
            atomic[e.offset:e.offset + e.numel] = True
    return (master, grads[0]), kind, nb, checks, atomic


def _assert_same(got, ref, atomic, what):
    det = ~atomic
    assert torch.equal(got[det], ref[det]), f"{what}: max diff {(got[det] - ref[det]).abs().max().item():.3e}"
    torch.testing.assert_close(got[atomic], ref[atomic], atol=1e-5, rtol=1e-4, msg=what + " (atomic-scatter part)")


@pytest.mark.parametrize("bucket_mb", [32.0, 4.0])
def test_forced_native_reducer_bitwise_equals_no_reducer(cuda, bucket_mb):
    batches = _batches(cuda, n=1)
    ref, _, _, _, atomic = _run(cuda, None, batches)
    got, kind, nb, _, _ = _run(cuda, dict(bucket_cap_mb=bucket_mb), batches)
    assert kind == "native-rccl" and nb >= (3 if bucket_mb == 32.0 else 10)
    _assert_same(got[1], ref[1], atomic, "grad")
    _assert_same(got[0], ref[0], atomic, "weights")


def test_reducer_stream_ordering_with_wgrad_side_stream(cuda, monkeypatch):
    monkeypatch.setenv("HQ_WGRAD_STREAM", "1")
    batches = _batches(cuda, n=1)
    ref, _, _, _, atomic = _run(cuda, None, batches)
    got, kind, nb, checks, _ = _run(cuda, dict(bucket_cap_mb=4.0, verify=True), batches)
    assert kind == "native-rccl" and checks and all(len(c) == nb for c in checks)
    for step, c in enumerate(checks):
        bad = {i: v for i, v in c.items() if v != 0.0}
        assert not bad, f"step {step}: comm stream read buckets {sorted(bad)} before their gradients were final"
    _assert_same(got[1], ref[1], atomic, "grad")


def test_reducer_timing_reports_comm_wait(cuda):
    model, red, eng = _engine(cuda, dict(bucket_cap_mb=32.0, timing=True))
    for b in _batches(cuda, n=3):
        eng.step([b])
    t = red.pop_timings()
    red.close()
    assert t["comm_wait_ms"] >= 0.0 and t["comm_span_ms"] > 0.0


def test_torchrun_world1_runs_the_n_rank_path(cuda, tmp_path):
    """`torchrun --nproc-per-node 1 bench.py --force_reducer` executes every line of the 8-GPU bench path:
    RCCL process group (device_id), the reducer's RCCL uid shipped through the TCPStore (rank 0 sets it and
    reads it back, as every rank of an N-rank job does), the native ncclBroadcast of the weights, the dynamic
    GEMM schedule, barrier, all_reduce(MAX) and destroy — and the JSON proves what ran (`uid_via_store`,
    `broadcast_done`, `rccl_comm_ranks`)."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT, free_port
    out = tmp_path / "bench.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "2",
           "--warmup", "1", "--batch", "8", "--seq", "128", "--force_reducer", "--json_out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-4000:]
    rec = json.loads(out.read_text())
    assert rec["reducer"] == "native-rccl", rec
    assert rec["process_group"] == "nccl" and rec["world_size"] == 1 and rec["rccl_comm_ranks"] == 1, rec
    assert rec["gemm_sched"] == "dynamic" and rec["reducer_buckets"] > 1, rec
    assert rec["uid_via_store"] is True and rec["broadcast_done"] is True, rec
    assert "not the headline config" in rec["metric"], rec
    assert rec["value"] > 0 and rec["final_loss"] == rec["final_loss"], rec
    # the N > 1 correctness self-check runs on the same path (a 1-replica gather here)
    assert rec["weights_equal_across_ranks"] is True and rec["grads_equal_across_ranks"] is True, rec
    assert rec["replica_mismatch_parts"] == 0 and rec["rccl_comm_ranks_ok"] is True, rec


def test_fingerprint_kernel_equals_host(cuda):
    """The device fingerprint kernel gives the host (numpy) fingerprint bit for bit, on an odd-sized arena."""
    from ml_recipe_distributed_pytorch_amd.parallel.reducer import fingerprint
    x = torch.randn(3_000_017, generator=torch.Generator().manual_seed(3))
    for parts in (1, 7, 256):
        assert torch.equal(fingerprint(x.to(cuda), parts).cpu(), fingerprint(x, parts)), parts


def test_bench_refuses_more_gpus_than_visible(cuda):
    """`python bench.py --gpus 2` on a one-GPU box must fail loudly instead of reporting a 1-GPU run under a
    2-GPU label (the self-launch checks the visible devices before starting any rank)."""
    import os
    import subprocess
    import sys
    from conftest import ROOT
    n = torch.cuda.device_count()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1",
                        "--warmup", "0"], cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True,
                       timeout=120)
    assert r.returncode != 0 and "GPU(s) are visible" in r.stdout, r.stdout[-2000:]
    assert '"metric"' not in r.stdout


def test_gloo_rehearsal_two_ranks_share_one_gpu(cuda, tmp_path):
    """The one configuration in which ranks share a GPU — the 2-rank gloo rehearsal, both ranks on cuda:0 —
    runs to completion with HIP's default 4 hardware queues per process (`_ranks_share_a_gpu`): round 2 saw this
    setup hang in the gloo all-reduce with 8 queues per process (16 on the device, profiles/r2_reducer).
    Production never shares a GPU (one rank per device; docs/ROUND4.md §7a)."""
    import json
    import os
    import subprocess
    import sys
    from conftest import ROOT, free_port
    out = tmp_path / "bench.json"
    env = dict(os.environ, HQ_BENCH_BACKEND="gloo", HQ_HANG_DUMP_S="200")
    env.pop("GPU_MAX_HW_QUEUES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
           "--warmup", "1", "--batch", "16", "--seq", "128", "--json_out", str(out)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-4000:]
    rec = json.loads(out.read_text())
    assert rec["process_group"] == "gloo" and rec["world_size"] == 2, rec
    assert rec["hw_queues"] == 4, rec   # not raised: the two ranks share cuda:0
    assert rec["value"] > 0, rec
    # the data-parallel replica check ran across the two ranks and found bitwise-equal weights and gradients
    assert rec["weights_equal_across_ranks"] is True and rec["grads_equal_across_ranks"] is True, rec
    assert rec["replica_mismatch_parts"] == 0, rec


@pytest.mark.parametrize("dtype", ["fp32", "emb_bf16"])
def test_comm_stream_norm_partials_equal_full_pass(cuda, dtype):
    """The reducer's comm stream writes each bucket's grad-norm partials right after its all-reduce; folded, they
    must give BITWISE the norm / clip coefficient of the full pass over the same final gradients (the 8-GPU step
    tail then holds one fold instead of a 418 MiB pass).  emb_bf16: the embeddings bucket travels as bf16 — its
    partials are taken after the cast back, i.e. over the gradients the optimizer reads."""
    from ml_recipe_distributed_pytorch_amd._native import kernels
    from ml_recipe_distributed_pytorch_amd.train.optim import grad_norm_and_clip
    model, red, eng = _engine(cuda, dict(bucket_cap_mb=32.0, allreduce_dtype=dtype))
    assert any(b.dtype == ("bf16" if dtype == "emb_bf16" else "fp32") for b in red.buckets)
    if dtype == "emb_bf16":
        assert [b.dtype for b in red.buckets if "embeddings" in b.groups] == ["bf16"]
        assert all(b.dtype == "fp32" for b in red.buckets if "embeddings" not in b.groups)
    inputs, labels = _batches(cuda, n=1)[0]
    red.prepare(sync=True)
    eng.loss_fn(model(**inputs), labels).backward()
    red.finalize()
    parts = red.norm_partials()
    assert parts is not None
    n1, c1 = grad_norm_and_clip(model.store, 1.0, partials=parts)
    n2, c2 = grad_norm_and_clip(model.store, 1.0)
    torch.cuda.synchronize()
    assert torch.equal(n1, n2) and torch.equal(c1, c2), (n1.item(), n2.item())
    ref = float(model.store.grad.double().norm())
    assert abs(n1.item() - ref) <= 1e-5 * ref
    red.prepare(sync=False)          # an accumulation micro-step: no partials, the engine takes the full pass
    assert red.norm_partials() is None
    red.close()
