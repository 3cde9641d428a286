"""Training entry point (reference ``modules/train.py:18-167``).

    python -m ml_recipe_distributed_pytorch_amd.cli.train -c config/test_bert.cfg [--flags]
    python modules/train.py -c config/test_bert.cfg                       # drop-in shim
    torchrun --nproc-per-node 8 -m ml_recipe_distributed_pytorch_amd.cli.train -c …   # env contract

Artefacts (reference layout): ``dump_dir/experiment_name/{trainer.cfg, model.cfg, <date>.log,
last.ch, epoch_<i>.ch, best.ch, interrupt.ch}`` and TensorBoard scalars under
``dump_dir/board/experiment_name``.  Ctrl-C **and SIGTERM** (preemption) write ``interrupt.ch``.
"""
from __future__ import annotations

import logging
import os
import signal
from datetime import datetime

import torch

from .. import factories
from ..data.items import LABELS
from ..parallel import dist as hqdist
from ..parallel.launch import clamp_jobs, device_for, launch, make_plan
from ..train.callbacks import AccuracyCallback, MAPCallback, SaveBestCallback
from ..train.trainer import Trainer
from ..utils.flags import get_model_parser, get_params, get_trainer_parser, write_config_file
from ..utils.logging import get_logger, set_seed, show_params


def _raise_interrupt(signum, frame):
    raise KeyboardInterrupt(f"signal {signum}")


def build_trainer(params, model_params, device, *, rank: int, local_idx: int, use_gpu: bool) -> Trainer:
    model, tokenizer = factories.init_model(model_params, device=device, bpe_dropout=params.bpe_dropout,
                                            seed=params.seed, precision=params.precision)
    optimizer = factories.init_optimizer(params, model)
    auto = getattr(params, "auto_batch_split", None)
    merge_segments = 1
    if device.type == "cuda" and auto in (None, True):   # GPU default: exact-objective merge
        from ..train.memory import device_hbm_bytes, estimate, plan_exact_merge
        hbm = device_hbm_bytes(device)
        split, merge_segments = plan_exact_merge(model.config, params.max_seq_len, params.train_batch_size, hbm,
                                                 params.batch_split)
        log = logging.getLogger(__name__)
        if split != params.batch_split:
            log.info(f"auto_batch_split: batch_split {params.batch_split} -> {split} (the micro-batch does not fit "
                     f"the HBM memory model; --auto_batch_split False keeps the configured split)")
        if merge_segments > 1:
            log.info(f"auto_batch_split: {split} micro-batches of {params.train_batch_size // split} run as "
                     f"{split // merge_segments} merged pass(es) of {merge_segments} loss segments each (the "
                     f"reference's mean of per-micro-batch means; --auto_batch_split raise keeps one pass per "
                     f"micro-batch)")
        params.batch_split = split
    elif device.type == "cuda" and auto in ("raise", "merge"):
        from ..train.memory import device_hbm_bytes, estimate, plan_batch_split
        hbm = device_hbm_bytes(device)
        merge = auto == "merge"
        split = plan_batch_split(model.config, params.max_seq_len, params.train_batch_size, hbm, params.batch_split,
                                 merge=merge)
        micro = params.train_batch_size // split
        log = logging.getLogger(__name__)
        if split != params.batch_split:
            log.info(f"auto_batch_split: batch_split {params.batch_split} -> {split} (micro-batch "
                     f"{params.train_batch_size // params.batch_split} -> {micro}, modelled "
                     f"{estimate(model.config, params.max_seq_len).total(micro) / 1e9:.1f} GB of {hbm / 1e9:.0f} GB HBM; "
                     f"--auto_batch_split False keeps the configured split)")
        if split < params.batch_split:
            log.warning("auto_batch_split=merge: micro-batches merged, so the loss is no longer the reference's mean of "
                        "per-micro-batch means (span CE over valid spans, weighted class CE, batchmean KL are "
                        "normalised over the merged batch) — drop 'merge' for the reference objective")
        params.batch_split = split
    dist_rank = rank if hqdist.info().distributed else -1
    if dist_rank in (-1, 0):  # prepare (and cache) the dataset in the main process first
        train_ds, test_ds, weights = factories.init_datasets(params, tokenizer=tokenizer,
                                                             clear=params.clear_processed, rank=dist_rank)
    if dist_rank != -1:
        hqdist.barrier()
    if dist_rank not in (-1, 0):
        train_ds, test_ds, weights = factories.init_datasets(params, tokenizer=tokenizer, clear=False, rank=dist_rank)
    loss = factories.init_loss(params, weights)
    return Trainer(model=model, loss=loss, collate_fun=factories.init_collate_fun(tokenizer), optimizer=optimizer,
                   train_dataset=train_ds, test_dataset=test_ds,
                   writer_dir=params.dump_dir / f"board/{params.experiment_name}", device=device,
                   local_rank=dist_rank, gpu_id=local_idx if use_gpu else None, sync_bn=params.sync_bn,
                   n_epochs=params.n_epochs, train_batch_size=params.train_batch_size,
                   test_batch_size=params.test_batch_size, batch_split=params.batch_split, n_jobs=params.n_jobs,
                   warmup_coef=params.warmup_coef, max_grad_norm=params.max_grad_norm, apex_level=params.apex_level,
                   apex_verbosity=params.apex_verbosity, apex_loss_scale=params.apex_loss_scale,
                   train_weights=weights, drop_optimizer=params.drop_optimizer, debug=params.debug,
                   bucket_cap_mb=params.bucket_cap_mb, allreduce_dtype=params.allreduce_dtype,
                   no_sync_accum=bool(params.no_sync_accum), log_every=params.log_every, profile=params.profile,
                   cuda_graph=bool(getattr(params, "cuda_graph", False)),
                   eval_shard=params.eval_shard, precision=params.precision,
                   torch_profile_dir=params.torch_profile_dir, torch_profile_steps=params.torch_profile_steps,
                   sampler_seed=params.seed if params.seed is not None else 0, merge_segments=merge_segments)


def run_worker(local_idx, plan, params, model_params):
    rank = plan.global_rank(local_idx)
    device = device_for(plan, local_idx)
    if plan.distributed:
        hqdist.init_distributed(plan.backend, init_method=plan.init_method, world_size=plan.world_size, rank=rank,
                                local_rank=local_idx, timeout_s=params.dist_timeout, use_gpu=plan.use_gpu)
    elif device.type == "cuda":
        torch.cuda.set_device(device)
    if device.type == "cpu" and plan.nproc_per_node > 1:  # CPU ranks share the host: no oversubscription
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // plan.nproc_per_node))
    params.n_jobs = clamp_jobs(params.n_jobs, plan.nproc_per_node)
    main_rank = rank == 0
    log_file = params.log_file if main_rank else None
    logger = get_logger(level=logging.INFO if main_rank else logging.WARN, filename=log_file, filemode="a",
                        logger_name="train", debug=params.debug)
    logger.warning(f"Process with rank: {rank}. Used device: {device}. Local index: {local_idx}.")
    if plan.distributed:
        logger.warning(f"Batch size will be increased by {plan.world_size} times because of distributed training. "
                       f"Correct your learning rate in the proper way.")
    set_seed(params.seed)
    trainer = build_trainer(params, model_params, device, rank=rank, local_idx=local_idx, use_gpu=plan.use_gpu)
    if params.last is not None:
        trainer.load_state_dict(params.last)
    out_dir = params.dump_dir / params.experiment_name

    def save_last(*_):
        trainer.save_state_dict(out_dir / "last.ch")

    def save_each(epoch_i):
        trainer.save_state_dict(out_dir / f"epoch_{epoch_i}.ch")

    save_best = SaveBestCallback(params)

    def test_fun(epoch_i):
        trainer.test(epoch_i, callbacks=[MAPCallback(LABELS), AccuracyCallback(), save_best])

    prev = signal.signal(signal.SIGTERM, _raise_interrupt)
    try:
        trainer.train(after_epoch_funcs=[save_last, save_each, test_fun])
    except KeyboardInterrupt:
        logger.error("Training process was interrupted.")
        trainer.save_state_dict(out_dir / "interrupt.ch")
    finally:
        signal.signal(signal.SIGTERM, prev)
        if trainer.reducer is not None:
            trainer.reducer.close()
        if trainer.writer is not None:
            trainer.writer.close()
        hqdist.destroy()
    return trainer


def main(argv=None):
    (parser, model_parser), (params, model_params) = get_params((get_trainer_parser, get_model_parser), argv)
    out_dir = params.dump_dir / params.experiment_name
    os.makedirs(out_dir, exist_ok=True)
    env_rank = int(os.environ.get("RANK", "0"))
    is_main = params.local_rank in (-1, 0) and env_rank == 0
    params.log_file = str(out_dir / f"{datetime.now().strftime('%d-%m-%Y_%H-%M-%S')}.log") if is_main else None
    logger = get_logger(filename=params.log_file, filemode="w", logger_name="train", debug=params.debug)
    if is_main:
        write_config_file(parser, params, out_dir / "trainer.cfg")
        write_config_file(model_parser, model_params, out_dir / "model.cfg")
    show_params(model_params, "model")
    show_params(params, "trainer")
    plan = make_plan(params)
    logger.info(f"Distributed: {plan.distributed}. Spawned workers: {plan.spawn}. World size: {plan.world_size}, "
                f"processes per node: {plan.nproc_per_node}, backend: {plan.backend}.")
    launch(run_worker, plan, params, model_params)


if __name__ == "__main__":
    main()
