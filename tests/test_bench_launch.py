"""bench.py's launch contract on the CPU: ``--gpus N`` without a launcher starts its own N-rank job with the
driver's torch.distributed.run command line, and refuses (non-zero, clear message) when fewer GPUs are
visible than requested — a 1-GPU number must never be reported under an N-GPU label."""
import os
import subprocess
import sys

import torch

from conftest import ROOT, free_port


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("hq_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_selflaunch_command_is_the_drivers_torchrun_line():
    b = _bench_module()
    argv = ["--gpus", "8", "--steps", "20", "--warmup", "5"]
    cmd = b.selflaunch_cmd(argv, 8, 29512)
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert cmd[3:11] == ["--nnodes=1", "--nproc-per-node", "8", "--master-addr", "127.0.0.1", "--master-port",
                         "29512", os.path.join(ROOT, "bench.py")]
    assert cmd[11:] == argv


def test_selflaunch_skipped_inside_a_rank(monkeypatch):
    b = _bench_module()
    monkeypatch.setenv("RANK", "0")
    from types import SimpleNamespace
    assert b.self_launch(SimpleNamespace(gpus=8), []) is None
    monkeypatch.delenv("RANK")
    assert b.self_launch(SimpleNamespace(gpus=1), []) is None


def test_bench_refuses_more_gpus_than_visible_on_cpu():
    n = max(torch.cuda.device_count(), 1)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--steps", "1"],
                       cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")})
    assert r.returncode == 2 and f"--gpus {n + 1} requested" in r.stdout, r.stdout[-2000:]
    assert '"metric"' not in r.stdout


def _bcast_worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    from ml_recipe_distributed_pytorch_amd.parallel import dist as hqdist
    from ml_recipe_distributed_pytorch_amd.parallel.reducer import GradReducer
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    hqdist.init_distributed("gloo", init_method=f"tcp://127.0.0.1:{port}", world_size=world, rank=rank,
                            use_gpu=False, timeout_s=60)
    model = BertForQuestionAnswering(get_config("bert-tiny-test"), precision="fp32", seed=rank).train()
    red = GradReducer(model, force=True)
    torch.save({"broadcast_done": red.broadcast_done, "uid_via_store": red.uid_via_store,
                "master": model.store.master.clone()}, os.path.join(out, f"r{rank}.pt"))
    red.close()
    hqdist.destroy()


def test_forced_reducer_broadcasts_whenever_a_group_exists(tmp_path):
    """A process group of one rank (the torchrun --nproc-per-node 1 rehearsal) still runs the DDP-constructor
    broadcast; at two ranks rank 1 ends up with rank 0's weights."""
    import torch.multiprocessing as mp
    for world in (1, 2):
        d = tmp_path / f"w{world}"
        d.mkdir()
        mp.spawn(_bcast_worker, args=(world, free_port(), str(d)), nprocs=world, join=True)
        recs = [torch.load(d / f"r{r}.pt", weights_only=True) for r in range(world)]
        assert all(r["broadcast_done"] for r in recs)
        assert not any(r["uid_via_store"] for r in recs)   # gloo on CPU: no RCCL communicator to set up
        for r in recs[1:]:
            assert torch.equal(r["master"], recs[0]["master"])
