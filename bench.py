#!/usr/bin/env python
"""Headline benchmark: whole-node training samples/s, BERT-base QA fine-tuning at seq=384, bf16.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 it is launched by
``torch.distributed.run`` (one rank per GPU, RCCL over xGMI) — and if it is not, it launches that N-rank job
itself as a child process (``self_launch``); a job whose size differs from ``--gpus`` exits non-zero.  Each timed step is a complete
optimizer step of the recipe's training loop (``config/test_bert.cfg`` loss/optimizer settings):
host batch synthesis (native dummy-QA generator, pinned) → H2D → fused BERT-base forward →
5-way QA loss → backward with bucketed RCCL all-reduce overlapped → on-device grad-norm clip →
fused AdamW → LR schedule.  Weak scaling: ``--batch`` samples per GPU per step.
Rank 0 prints ONE JSON line; ``value`` is the whole-job aggregate (max elapsed over ranks).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from types import SimpleNamespace


def _gemm_sched_label() -> str:
    """'dynamic' / 'static': the persistent GEMM's tile schedule actually in effect in the kernel library."""
    from ml_recipe_distributed_pytorch_amd._native import kernels
    return "dynamic" if kernels().gemm_get_sched() else "static"

METRIC = "samples/sec (whole node) BERT-base QA fine-tune seq=384 at 1/2/4/8 MI355X"   # BASELINE.json


def metric_name(model: str, seq: int, batch: int, precision: str, split: int = 1, passes: int = 0) -> str:
    """BASELINE.json's metric string for the headline config (BERT-base, seq 384, 256 samples per GPU in one
    micro-batch, bf16); any other --model / --seq / --batch / --batch_split / --precision gets a label that
    names what was measured."""
    if model == "bert-base-uncased" and seq == 384 and batch == 256 and precision == "bf16" and split == 1:
        return METRIC
    mb = f" as {split}x{batch // split}" if split > 1 else ""
    if split > 1 and 0 < passes < split:
        mb += f" in {passes} merged pass{'es' if passes > 1 else ''} (per-micro-batch loss segments)"
    return (f"samples/sec (whole node) {model} QA fine-tune seq={seq} batch={batch}/GPU{mb} {precision} "
            "(not the headline config)")
# The reference publishes no numbers; BASELINE.md's "baseline to beat" is the reference recipe re-run
# on the same MI355X (HF BertModel + its QA heads/loss, autocast bf16 for apex O1, AdamW, clip):
# tools/ref_recipe_bench.py --batch 256 --attn sdpa (the faster of its two attention paths) = 1611.65.
BASELINE_VALUE = 1611.65  # per GPU; for N GPUs the baseline is taken as N x this (ideal reference scaling)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256,
                    help="samples per GPU per optimizer step (config/test_bert.cfg train_batch_size=256 per "
                         "process; one micro-batch — 288 GB HBM3E holds it, the reference split it 128 ways)")
    ap.add_argument("--seq", type=int, default=384)
    ap.add_argument("--model", default="bert-base-uncased")
    ap.add_argument("--allreduce_dtype", default="fp32", choices=["fp32", "bf16", "emb_bf16"],
                    help="gradient all-reduce wire dtype: every bucket fp32 / bf16, or only the embeddings bucket (the "
                         "step's exposed comm tail) in bf16")
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp8", "fp32"],
                    help="compute precision; fp8 = OCP e4m3 forward projections and e5m2-gradient dgrads "
                         "(BASELINE config #5); fp32 = the reference's Apex-off mode (exact-f32 MFMA GEMMs, fp32 "
                         "flash attention and row kernels)")
    ap.add_argument("--fp8_dgrad", type=int, default=1, choices=[0, 1],
                    help="with --precision fp8: 0 keeps the backward dgrads in bf16 (A/B of the fp8 backward)")
    ap.add_argument("--bucket_cap_mb", type=float, default=32.0)
    ap.add_argument("--profile", action="store_true", help="per-phase timers (adds syncs; not for the headline)")
    ap.add_argument("--graph", action="store_true",
                    help="replay every micro-step (forward + backward, and the bucket all-reduces on the "
                         "accumulation boundary) from captured HIP graphs")
    ap.add_argument("--batch_split", type=int, default=1,
                    help="micro-batches per optimizer step (reference --batch_split): micro-batch = batch / "
                         "batch_split, gradients accumulated, all-reduce + optimizer once per step")
    ap.add_argument("--merge", default="auto", choices=["auto", "off"],
                    help="with --batch_split S > 1: 'auto' (the trainer's GPU default) runs the S micro-batches in as "
                         "few merged passes as fit HBM, each micro-batch a loss segment — the reference objective "
                         "(mean of per-micro-batch means) at merged speed; 'off' runs one pass per micro-batch")
    ap.add_argument("--force_reducer", action="store_true",
                    help="keep the gradient reducer active at 1 GPU (1-rank RCCL communicator): rehearses the "
                         "multi-GPU fence → ncclAllReduce → wait path on every bucket of the real backward")
    ap.add_argument("--rccl_channels", type=int, default=0,
                    help=">0: NCCL_MIN_NCHANNELS = NCCL_MAX_NCHANNELS = this (RCCL honours both) before the "
                         "communicators are created; 0 leaves RCCL's own topology tuning")
    ap.add_argument("--json_out", default=None)
    return ap.parse_args()


def selflaunch_cmd(argv, nproc: int, port: int):
    """The N-rank job ``python bench.py --gpus N`` starts for itself when no launcher set RANK: the driver's
    own form, ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
    --master-port P bench.py <same args>``, one rank per GPU over RCCL."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv):
    """``--gpus N`` (N > 1) without a launcher: check that N GPUs are visible, then run the N-rank job as a
    CHILD process (no exec: nothing here has touched the GPU — ``device_count`` does not initialise HIP) and
    return its exit status.  None when this process is a rank (RANK set) or N == 1."""
    if args.gpus <= 1 or "RANK" in os.environ:
        return None
    import subprocess
    import torch
    visible = torch.cuda.device_count()
    if visible < args.gpus:
        print(f"[bench] error: --gpus {args.gpus} requested but only {visible} GPU(s) are visible; refusing to "
              "report a smaller job under that label", file=sys.stderr, flush=True)
        return 2
    cmd = selflaunch_cmd(argv, args.gpus, _free_port())
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    args = parse()
    rc = self_launch(args, sys.argv[1:])
    if rc is not None:
        sys.exit(rc)
    if os.environ.get("HQ_HANG_DUMP_S"):   # hang diagnosis: every rank dumps its Python stacks and exits
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["HQ_HANG_DUMP_S"]), exit=True)
    import torch
    import torch.distributed as dist

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from ml_recipe_distributed_pytorch_amd.data.dummy import SpecialIds, synth_batch_native
    from ml_recipe_distributed_pytorch_amd.models.bert import BertForQuestionAnswering
    from ml_recipe_distributed_pytorch_amd.models.config import get_config
    from ml_recipe_distributed_pytorch_amd.models.losses import build_loss
    from ml_recipe_distributed_pytorch_amd.parallel import dist as hqdist
    from ml_recipe_distributed_pytorch_amd.parallel.reducer import GradReducer
    from ml_recipe_distributed_pytorch_amd.train.engine import TrainEngine
    from ml_recipe_distributed_pytorch_amd.train.optim import FusedAdamW, get_linear_schedule_with_warmup
    from ml_recipe_distributed_pytorch_amd.train.trainer import optimizer_groups

    if args.rccl_channels > 0:
        os.environ.setdefault("NCCL_MIN_NCHANNELS", str(args.rccl_channels))
        os.environ.setdefault("NCCL_MAX_NCHANNELS", str(args.rccl_channels))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # Launched by torchrun / torch.distributed.run (RANK in the env): the process group is initialised at ANY
    # world size, so `torchrun --nproc-per-node 1 bench.py --force_reducer` runs every line an 8-GPU run does
    # (RCCL init with device_id, the reducer's TCPStore uid exchange and native broadcast, the dynamic GEMM
    # schedule, barrier, all_reduce(MAX), destroy).  Plain `python bench.py` (the driver's N=1 run) has none.
    launched = hqdist.env_launched()
    backend = None
    if launched and os.environ.get("HQ_BENCH_BACKEND", "nccl") == "nccl":
        local = int(os.environ.get("LOCAL_WORLD_SIZE", world))
        if torch.cuda.device_count() < local:
            raise SystemExit(f"[bench] error: {local} ranks on this node but only {torch.cuda.device_count()} "
                             "GPU(s) visible (RCCL needs one GPU per rank)")
    if launched:
        # HQ_BENCH_BACKEND=gloo: rehearsal of the multi-rank path with every rank on cuda:0 (one-GPU box; gloo
        # all-reduces the CUDA buckets through host memory) — never for a measurement
        backend = os.environ.get("HQ_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            os.environ["LOCAL_RANK"] = "0"
        info = hqdist.init_distributed(backend)
        rank, device, world = info.rank, info.device, dist.get_world_size()
    else:
        rank, device = 0, torch.device("cuda", 0)
        torch.cuda.set_device(device)
    if world != args.gpus:   # never report an N-GPU label for a different job size
        raise SystemExit(f"[bench] error: --gpus {args.gpus} but the job has {world} rank(s)")

    cfg = get_config(args.model)
    model = BertForQuestionAnswering(cfg, seed=1234, precision=args.precision).to(device).train()
    model.fp8_dgrad = bool(args.fp8_dgrad)
    # config/test_bert.cfg: loss=smooth(0.01), all five loss weights 1, lr 1e-5, wd 1e-4, clip 1
    lp = SimpleNamespace(loss="smooth", smooth_alpha=0.01, focal_alpha=1, focal_gamma=2, w_start=1, w_end=1,
                         w_start_reg=1, w_end_reg=1, w_cls=1)
    loss_fn = build_loss(lp)
    groups = optimizer_groups(model.named_parameters(), 1e-4)
    opt = FusedAdamW(groups, model.store, lr=1e-5, eps=1e-6, correct_bias=False, zero_grad_fn=model.zero_grad)
    total = args.warmup + args.steps
    sched = get_linear_schedule_with_warmup(opt, int(0.05 * total), total)
    reducer = None
    if world > 1 or args.force_reducer:
        # world > 1 or --force_reducer (1-rank communicator): every bucket goes through the native RCCL reducer
        # comm timing records HIP timing events around the collectives: not capturable, so off under --graph
        timing = os.environ.get("HQ_BENCH_COMM_TIMING", "0" if args.graph else "1") == "1"
        reducer = GradReducer(model, bucket_cap_mb=args.bucket_cap_mb, allreduce_dtype=args.allreduce_dtype,
                              force=args.force_reducer, timing=timing)
    # HQ_BENCH_REDUCER_IDLE=1 (diagnostic): the reducer and its RCCL communicator exist but the engine never
    # uses them — separates the cost of the communicator's presence from that of its all-reduces
    idle = os.environ.get("HQ_BENCH_REDUCER_IDLE", "0") == "1"
    S = max(1, args.batch_split)
    if args.batch % S:
        raise SystemExit(f"--batch {args.batch} is not a multiple of --batch_split {S}")
    G = 1
    if S > 1 and args.merge == "auto":
        from ml_recipe_distributed_pytorch_amd.train.memory import device_hbm_bytes, plan_exact_merge
        S_plan, G = plan_exact_merge(cfg, args.seq, args.batch, device_hbm_bytes(device), S)
        if S_plan != S:
            raise SystemExit(f"--batch_split {S}: a micro-batch of {args.batch // S} does not fit the memory model")
    engine = TrainEngine(model, loss_fn, opt, scheduler=sched, reducer=None if idle else reducer, max_grad_norm=1.0,
                         batch_split=S // G, profile=args.profile, graph=args.graph, merge_segments=G)

    sp = SpecialIds(cfg.vocab_size, cfg.pad_token_id, cfg.unk_token_id, cfg.cls_token_id, cfg.sep_token_id,
                    "bert" if cfg.family == "bert" else "roberta")
    B, L, Q = args.batch, args.seq, 64
    slots = [synth_batch_native(B, L, Q, sp, seed=rank * 1_000_003 + i) for i in range(2)]
    from ml_recipe_distributed_pytorch_amd.data.dummy import _refill
    from ml_recipe_distributed_pytorch_amd.train.engine import DevicePrefetcher, to_device
    # batch i+1 is synthesised into its pinned slot and copied to the GPU on a copy stream while step i runs
    # (DevicePrefetcher: a copy issued on the compute stream left the GPU idle at every step boundary)
    prefetcher = DevicePrefetcher(device)
    copy_done = [None, None]   # per pinned slot: the event of the last copy out of it
    events = [torch.cuda.Event() for _ in slots]   # compute stream, per slot: keeps the host <= 2 steps ahead
    for e in events:
        e.record()
    step_no = [0]
    pending = [None]
    host_wait = [0.0]   # host time blocked on the slot events: ~0 means the host, not the GPU, paces the loop

    # HQ_BENCH_PREFETCH=0 (A/B only): each batch copied on the compute stream at its own step, the pre-prefetch form
    early = os.environ.get("HQ_BENCH_PREFETCH", "1") == "1"

    def issue(i):
        s = i % 2
        if copy_done[s] is not None:
            copy_done[s].synchronize()       # the copy of batch i-2 out of this slot has finished
        inputs, labels = slots[s]
        _refill(slots[s], sp, Q, seed=rank * 1_000_003 + 7919 * (i + 2))
        if not early:
            dev = to_device((inputs, labels), device)
            ev = torch.cuda.Event()
            ev.record()
            copy_done[s] = ev
            return dev, None
        item = prefetcher.issue((inputs, labels))
        copy_done[s] = item[1]
        return item

    def next_batch():
        i = step_no[0]
        s = i % 2
        t_w = time.perf_counter()
        events[s].synchronize()              # the compute stream has reached step i-2
        host_wait[0] += time.perf_counter() - t_w
        if pending[0] is None or not early:
            pending[0] = issue(i)
        dev_in, dev_lb = prefetcher.claim(pending[0])
        events[s].record()
        pending[0] = issue(i + 1) if early else None   # overlaps step i on the copy stream
        step_no[0] += 1
        return dev_in, dev_lb

    def one_step():
        inputs, labels = next_batch()
        if S == 1:
            return engine.step([(inputs, labels)])
        b = B // S   # the reference's micro-batches: contiguous slices of the step's batch
        return engine.step([({k: v[i * b:(i + 1) * b] for k, v in inputs.items()},
                             {k: v[i * b:(i + 1) * b] for k, v in labels.items()}) for i in range(S)])

    for _ in range(args.warmup):
        res = one_step()
    torch.cuda.synchronize()
    if reducer is not None:
        reducer.pop_timings()  # drop the warmup steps' comm events
    if launched:
        hqdist.barrier()
    torch.cuda.synchronize()
    bytes0 = reducer.stats["bytes"] if reducer is not None else 0
    host_wait[0] = 0.0
    t0 = time.perf_counter()
    phase = {}
    for _ in range(args.steps):
        res = one_step()
        for k, v in res.timings.items():
            phase[k] = phase.get(k, 0.0) + v
    t_host = time.perf_counter() - t0        # the host's own time to issue the K steps (before the final drain)
    torch.cuda.synchronize()
    if launched:
        hqdist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rank_ms = None
    if launched:   # the slowest rank's clock (a 1-rank gather at world 1) + every rank's, for the spread
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        every = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(every, t)
        rank_ms = [float(x.item()) / args.steps * 1e3 for x in every]
        elapsed = max(float(x.item()) for x in every)
    ar_bytes = ((reducer.stats["bytes"] - bytes0) / args.steps) if reducer is not None else 0
    final_loss = res.losses.to_floats().get("loss", float("nan"))
    comm = reducer.pop_timings() if reducer is not None else {}
    # data-parallel self-check, AFTER the clock: one more (untimed) step fingerprints its reduced gradient arena,
    # then every rank's fp32 master weights and that gradient are all-gathered and compared with rank 0's — a
    # reducer bug must fail the run, not be reported as a fast number
    replica = None
    if reducer is not None:
        reducer.snapshot_grads = True
        one_step()
        torch.cuda.synchronize()
        replica = reducer.replica_check()
    ms = elapsed / args.steps * 1e3
    value = world * B * args.steps / elapsed
    H, F, NL = cfg.hidden_size, cfg.intermediate_size, cfg.num_hidden_layers
    enc_linear = NL * (4 * H * H + 2 * H * F)  # 85.0 M (base), 302 M (large)
    flops_per_sample = 6 * enc_linear * L + 12 * L * L * H * NL  # SURVEY §6.2 model
    from ml_recipe_distributed_pytorch_amd import hw_queue_info
    out = {"metric": metric_name(args.model, L, B, args.precision, S, S // G), "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": (round(value / (BASELINE_VALUE * world), 4) if BASELINE_VALUE else None), "dtype": args.precision,
           "data": "synthetic (dummy-QA generator, random-init weights)",
           "config": {"model": args.model, "global_batch": B * world, "per_gpu_batch": B, "seq_len": L,
                      "batch_split": S, "micro_batch": B // S, "merged_passes": S // G,
                      "segments_per_pass": G,
                      "parallelism": f"dp{world}", "allreduce_dtype": args.allreduce_dtype,
                      "bucket_cap_mb": args.bucket_cap_mb,
                      "rccl_channels": os.environ.get("NCCL_MIN_NCHANNELS"),
                      "fp8_dgrad": bool(args.fp8_dgrad) if args.precision == "fp8" else None},
           "world_size": dist.get_world_size() if dist.is_initialized() else 1,
           "process_group": backend or "none",
           "rccl_comm_ranks": reducer.comm_ranks if reducer is not None else None,
           "hw_queues": hw_queue_info()["live"],
           "graph_replays": engine.graph_replays,
           "reducer": reducer.kind if reducer is not None else "none",
           "reducer_buckets": reducer.n_buckets if reducer is not None else 0,
           "uid_via_store": reducer.uid_via_store if reducer is not None else None,
           "broadcast_done": reducer.broadcast_done if reducer is not None else None,
           # the kernel library's setting in effect (HQ_GEMM_SCHED at load, or the reducer's choice)
           "gemm_sched": _gemm_sched_label(),
           "comm_wait_ms": round(comm["comm_wait_ms"], 3) if "comm_wait_ms" in comm else None,
           "comm_span_ms": round(comm["comm_span_ms"], 3) if "comm_span_ms" in comm else None,
           # multi-GPU diagnosis: per-rank step-time spread, bytes all-reduced per step (wire dtype), and the
           # algorithm bandwidth those bytes achieved over the comm span (bytes / span; busbw = algbw·2(N-1)/N)
           "rank_ms_min": round(min(rank_ms), 3) if rank_ms else None,
           "rank_ms_max": round(max(rank_ms), 3) if rank_ms else None,
           "allreduce_bytes_per_step": int(ar_bytes) if reducer is not None else None,
           "algbw_GBps": (round(ar_bytes / (comm["comm_span_ms"] * 1e-3) / 1e9, 1)
                          if reducer is not None and comm.get("comm_span_ms") else None),
           "mfu_bf16_dense": round(value * flops_per_sample / (world * 2.5e15), 4),
           "max_mem_gb": round(torch.cuda.max_memory_allocated(device) / 1e9, 2),
           # host pacing diagnostic (rank 0): per step, the host's issue time and its time blocked on the input slots'
           # events; a blocked time near 0 means the host, not the GPU, sets the step time
           "host_issue_ms": round(t_host / args.steps * 1e3, 3),
           "host_blocked_ms": round(host_wait[0] / args.steps * 1e3, 3),
           "final_loss": round(final_loss, 4),
           # cross-rank replica check (null without a reducer): exact fingerprints of the fp32 master arena and of
           # an untimed extra step's reduced gradients, every rank vs rank 0
           "weights_equal_across_ranks": replica["weights_equal_across_ranks"] if replica else None,
           "grads_equal_across_ranks": replica["grads_equal_across_ranks"] if replica else None,
           "replica_mismatch_parts": replica["replica_mismatch_parts"] if replica else None,
           "max_weight_partial_mismatch": replica["max_weight_partial_mismatch"] if replica else None,
           "rccl_comm_ranks_ok": replica["rccl_comm_ranks_ok"] if replica else None}
    if args.profile:
        out["phase_ms"] = {k: round(v / args.steps, 3) for k, v in phase.items()}
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if reducer is not None:
        reducer.close()
    if launched:
        hqdist.destroy()
    if replica is not None and not replica["ok"]:
        print(f"[bench] error: data-parallel replica check failed on rank {rank}: {replica}", file=sys.stderr,
              flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
