"""CLI / config surface of the recipe (drop-in for ``modules/model/utils/parser.py``).

Every reference flag keeps its name, type and default (``parser.py:60-207``).
New flags are additive and default to reference behaviour; they are grouped at the end of each
parser under "MI355X" comments.
"""
from __future__ import annotations

import logging
from pathlib import Path
from typing import Callable, Iterable, List, Sequence, Tuple

from .cfgparse import ArgumentParser

logger = logging.getLogger(__name__)

MODEL_CHOICES = ["bert-base-uncased", "bert-base-cased", "bert-large-uncased", "bert-large-cased",
                 "roberta-base", "roberta-large", "bert-tiny-test"]


def cast2(type_):
    """``'None'`` → ``None``, anything else → ``type_(x)`` (reference ``parser.py:34-35``)."""
    return lambda x: type_(x) if x != "None" else None


def get_params(parser_getters: Sequence[Callable[[], ArgumentParser]], args=None):
    """Parse the same argv with several parsers; abort on args unknown to all (``parser.py:9-31``)."""
    unused = None
    parsers: List[ArgumentParser] = []
    params = []
    for getter in parser_getters:
        parser = getter()
        parsed, unused_params = parser.parse_known_args(args)
        parsers.append(parser)
        params.append(parsed)
        unused_params = set(unused_params)
        unused = unused_params if unused is None else unused.intersection(unused_params)
    if unused:
        for parser in parsers:
            parser.print_help()
        print(f"Incorrect command line parameters: {unused}.")
        raise SystemExit(2)
    return parsers, params


def write_config_file(parser: ArgumentParser, parsed_namespace, output_path) -> None:
    """Serialise every attribute whose name lacks ``config`` (``parser.py:38-50``)."""
    items = {k: getattr(parsed_namespace, k) for k in sorted(parsed_namespace.__dict__.keys()) if "config" not in k}
    contents = parser.serialize(items)
    with open(output_path, "w") as f:
        f.write(contents)
    logger.info(f"Config was saved to {output_path}.")


def load_config_file(parser_getter, config_path):
    parser = parser_getter()
    return parser, parser.parse_args(f"-c {config_path}")


def get_model_parser() -> ArgumentParser:
    parser = ArgumentParser(description="Model config parser.")
    parser.add_argument("-c", "--config_file", required=False, is_config_file=True, help="Config file path.")
    parser.add_argument("--model_config_file", required=False, is_config_file=True, help="Model config file path.")
    parser.add_argument("--model", type=str, default="bert-base-uncased", choices=MODEL_CHOICES,
                        help="Transformer model name.")
    parser.add_argument("--hidden_dropout_prob", type=float, default=0.1, help="Model dropout probability.")
    parser.add_argument("--attention_probs_dropout_prob", type=float, default=0.1,
                        help="Attention dropout probability.")
    parser.add_argument("--layer_norm_eps", type=float, default=1e-12, help="Layer norm eps.")
    parser.add_argument("--vocab_file", type=cast2(str), default=None, help="Path to WordPiece/BPE vocab.")
    parser.add_argument("--merges_file", type=cast2(str), default=None, help="BPE merge table path.")
    parser.add_argument("--lowercase", action="store_true", help="Tokenize lowercase strings.")
    parser.add_argument("--handle_chinese_chars", action="store_true",
                        help="Do not replace chinese symbols with UNK tokens.")
    # --- MI355X additions -------------------------------------------------------------------
    parser.add_argument("--random_init", action="store_true",
                        help="Ignore --pretrained_path and start from random weights (what happens anyway without it).")
    parser.add_argument("--pretrained_path", type=cast2(str), default=None,
                        help="Local dir/file with HF-named weights (safetensors or weights-only torch). "
                             "Random init when absent (no network in this environment).")
    parser.add_argument("--legacy_tokenization", action="store_true",
                        help="Reproduce reference quirk D11: wrap every encoded word in [CLS] ... [SEP].")
    return parser


def init_base_arguments(parser: ArgumentParser) -> None:
    parser.add_argument("-c", "--config_file", required=False, is_config_file=True, help="Config file path.")
    parser.add_argument("--data_path", type=str, required=True, help="Path to JSON with documents.")
    parser.add_argument("--processed_data_path", type=str, required=True,
                        help="Path where processed dataset will be saved.")
    parser.add_argument("--gpu", action="store_true", help="Use gpu to train or validate models.")
    parser.add_argument("--max_seq_len", type=int, default=384, help="Max input seq length.")
    parser.add_argument("--max_question_len", type=int, default=64, help="Max question length.")
    parser.add_argument("--doc_stride", type=int, default=128, help="Step size during doc splitting.")
    parser.add_argument("--split_by_sentence", action="store_true", help="Split document by sentence instead.")
    parser.add_argument("--truncate", action="store_true", help="Cut off long sentences during splitting by sentence.")
    parser.add_argument("--n_jobs", type=int, default=16, help="Number of threads used in dataloader.")
    # --- MI355X additions (shared) ----------------------------------------------------------
    parser.add_argument("--precision", type=cast2(str), default=None, choices=[None, "fp32", "bf16", "fp8"],
                        help="Compute precision. Default: bf16 on GPU (apex O1/O2 map to bf16), fp32 on CPU.")
    parser.add_argument("--dummy_dataset_len", type=int, default=10000, help="Length of the dummy dataset.")


def get_trainer_parser() -> ArgumentParser:
    parser = ArgumentParser(description="Trainer config parser.")
    init_base_arguments(parser)
    parser.add_argument("--trainer_config_file", required=False, is_config_file=True, help="Trainer config file path.")
    parser.add_argument("--dump_dir", type=Path, default="../results", help="Dump path.")
    parser.add_argument("--experiment_name", type=str, required=True, help="Experiment name.")
    parser.add_argument("--last", type=cast2(str), default=None, help="Restored checkpoint.")
    parser.add_argument("--seed", type=cast2(int), default=None, help="Seed for random state.")
    parser.add_argument("--n_epochs", type=int, default=10, help="Number of epochs.")
    parser.add_argument("--train_batch_size", type=int, default=128, help="Number of items in batch.")
    parser.add_argument("--test_batch_size", type=int, default=16, help="Number of items in batch.")
    parser.add_argument("--batch_split", type=int, default=1,
                        help="Batch will be split into this number of chunks during training.")
    parser.add_argument("--lr", type=float, default=1e-5, help="Learning rate for optimizer.")
    parser.add_argument("--weight_decay", type=float, default=0.01, help="Weight decay for optimizer.")
    parser.add_argument("--clear_processed", action="store_true", help="Clear previous processed dataset.")
    parser.add_argument("--w_start", type=float, default=1, help="Weight of start position classification.")
    parser.add_argument("--w_end", type=float, default=1, help="Weight of end position classification.")
    parser.add_argument("--w_start_reg", type=float, default=0, help="Weight of start position regression loss.")
    parser.add_argument("--w_end_reg", type=float, default=0, help="Weight of end position regression loss.")
    parser.add_argument("--w_cls", type=float, default=1, help="Weight of doc label classification.")
    parser.add_argument("--loss", type=str, default="ce", choices=["ce", "focal", "smooth"],
                        help="Type of doc label classification loss")
    parser.add_argument("--smooth_alpha", type=float, default=0.01, help="Smooth CE loss parameter.")
    parser.add_argument("--focal_alpha", type=float, default=1, help="Focal loss parameter.")
    parser.add_argument("--focal_gamma", type=float, default=2, help="Focal loss parameter.")
    parser.add_argument("--max_grad_norm", type=float, default=1, help="Max norm of the gradients")
    parser.add_argument("--sync_bn", action="store_true",
                        help="Synchronize batch norm parameters during distributed training.")
    parser.add_argument("--warmup_coef", type=float, default=0.05, help="Warmup coefficient.")
    parser.add_argument("--apex_level", type=cast2(str), choices=[None, "O0", "O1", "O2", "O3"], default=None,
                        help="Apex optimization level (mapped to native bf16 mixed precision).")
    parser.add_argument("--apex_verbosity", type=int, default=1, help="Apex output verbosity.")
    parser.add_argument("--apex_loss_scale", type=cast2(float), default=None, help="Apex loss scale coef.")
    parser.add_argument("--drop_optimizer", action="store_true",
                        help="Not restore optimizer and scheduler from checkpoint.")
    parser.add_argument("--debug", action="store_true", help="Debug mode.")
    parser.add_argument("--dummy_dataset", action="store_true", help="Use generated dataset instead real data.")
    parser.add_argument("--local_rank", type=int, default=-1,
                        help="Local rank of process during distributed training. "
                             "To run distributed training on single node, set this parameter equals to 0.")
    parser.add_argument("--dist_backend", type=str, default="nccl", choices=["nccl", "gloo"],
                        help="Distributed backend: nccl (= RCCL over xGMI on ROCm) or gloo (CPU).")
    parser.add_argument("--dist_init_method", type=str, default="tcp://127.0.0.1:9080",
                        help="Distributed training init method. Set master process host name.")
    parser.add_argument("--dist_world_size", type=int, default=1,
                        help="Number of machines are used during training. Can be changed during training.")
    parser.add_argument("--best_metric", choices=["map"], type=str, default="map", help="Best metric name.")
    parser.add_argument("--best_order", choices=[">", "<"], type=str, default=">", help="Best metric order.")
    parser.add_argument("--finetune", action="store_true", help="Turn on finetune mode.")
    parser.add_argument("--finetune_transformer", action="store_true", help="Finetune transformer module.")
    parser.add_argument("--finetune_position", action="store_true", help="Finetune classification head.")
    parser.add_argument("--finetune_position_reg", action="store_true", help="Finetune regression head.")
    parser.add_argument("--finetune_class", action="store_true", help="Finetune doc label classification head.")
    parser.add_argument("--bpe_dropout", type=cast2(float), default=None, help="Use BPE dropout.")
    parser.add_argument("--optimizer", type=str, default="adam", choices=["adam", "adamod"], help="Optimizer name.")
    parser.add_argument("--train_label_weights", action="store_true", help="Use label weights in CE loss.")
    parser.add_argument("--train_sampler_weights", action="store_true", help="Use oversampling.")
    parser.add_argument("--log_file", type=str, default=None,
                        help="This parameter is ignored. After dump will consist path to log file.")
    # --- MI355X additions -------------------------------------------------------------------
    parser.add_argument("--bucket_cap_mb", type=float, default=32.0,
                        help="Gradient bucket size (MiB of reduced dtype); sized for 7 xGMI links per GPU.")
    parser.add_argument("--allreduce_dtype", type=str, default="fp32", choices=["fp32", "bf16", "emb_bf16"],
                        help="Dtype of the gradient all-reduce payload: fp32, bf16 (every bucket), or emb_bf16 (only "
                             "the embeddings bucket, the exposed tail of the step, in bf16).")
    parser.add_argument("--no_sync_accum", type=cast2(int), default=1,
                        help="1: all-reduce only at the accumulation boundary (fix of D1); 0: every micro-batch.")
    parser.add_argument("--dist_timeout", type=float, default=1800.0, help="Process-group timeout in seconds.")
    parser.add_argument("--auto_batch_split", type=_auto_split, default=None, nargs="?", const=True,
                        help="GPU only.  Default (unset / True): exact-objective merge — the micro-batches "
                             "train_batch_size // batch_split are collated one by one as the reference does, then run "
                             "in as few merged forward/backward passes as fit the HBM memory model (train/memory.py), "
                             "the loss scoring each micro-batch as its own segment (its span length, its valid-span "
                             "count, its class normaliser) and averaging them: the reference's mean of per-micro-batch "
                             "means at merged speed (128 x 2 -> one pass of 256 on a 288 GB MI355X).  A micro-batch "
                             "that does not fit raises the split.  'raise': one pass per micro-batch (only raises the "
                             "split).  'merge': LOWER the split to the smallest that fits and collate merged batches "
                             "— the losses are then normalised over the merged batch, not per micro-batch.  False: "
                             "off.")
    parser.add_argument("--profile", action="store_true", help="Per-phase step timers + perf/* TB scalars.")
    parser.add_argument("--cuda_graph", type=_opt_bool, default=False, nargs="?", const=True,
                        help="GPU, bf16: capture each kind of micro-step (forward + backward; first / middle / last "
                             "micro-batch of an accumulation cycle, the last one with the gradient all-reduces) into "
                             "a HIP graph after two eager warm-up micro-steps and replay them (launch-bound small "
                             "micro-batches, e.g. the reference's 128 x 2).  Graphs exist for the first two input "
                             "shapes only (one shared mempool); batches of other padded lengths run eagerly.")
    parser.add_argument("--torch_profile_dir", type=cast2(str), default=None,
                        help="Export a torch.profiler Chrome trace of optimizer steps --torch_profile_steps here.")
    parser.add_argument("--torch_profile_steps", type=str, default="3:5",
                        help="first:last optimizer steps (1-based, inclusive) captured by --torch_profile_dir.")
    parser.add_argument("--log_every", type=int, default=1, help="Device→host loss sync cadence (steps).")
    parser.add_argument("--checkpoint", type=cast2(str), default=None,
                        help="Checkpoint for train_metrics evaluation (fix of D9).")
    parser.add_argument("--eval_shard", action="store_true",
                        help="Shard evaluation across ranks and all-reduce the metrics (default: rank-0 eval).")
    parser.add_argument("--nproc_per_node", type=cast2(int), default=None,
                        help="Processes per node (default: #visible GPUs, or 1 on CPU). On CPU >1 spawns gloo ranks.")
    return parser


def _auto_split(v):
    """--auto_batch_split: None / True (exact-objective merge), 'raise' (one pass per micro-batch, only raises the
    split), 'merge' (lower the split, merged objective), False (off)."""
    if isinstance(v, str) and v.strip().lower() in ("merge", "raise"):
        return v.strip().lower()
    return _opt_bool(v)


def _opt_bool(v):
    """Tri-state flag value: None (unset → per-device default), True or False (cfg ``key = True``)."""
    if v is None or isinstance(v, bool):
        return v
    t = str(v).strip().lower()
    if t in ("none", ""):
        return None
    if t in ("1", "true", "yes", "on"):
        return True
    if t in ("0", "false", "no", "off"):
        return False
    raise ValueError(f"expected True/False/None, got {v!r}")


def get_predictor_parser() -> ArgumentParser:
    parser = ArgumentParser(description="Validation config parser.")
    init_base_arguments(parser)
    parser.add_argument("--predictor_config_file", required=False, is_config_file=True,
                        help="Trainer config file path.")
    parser.add_argument("--checkpoint", required=True, type=cast2(str), help="Restored checkpoint path.")
    parser.add_argument("--batch_size", type=int, default=16, help="Batch size.")
    parser.add_argument("--buffer_size", type=int, default=4096, help="Buffer queue size.")
    parser.add_argument("--limit", type=cast2(int), default=None, help="Process only specified number of documents.")
    # --- MI355X additions -------------------------------------------------------------------
    parser.add_argument("--dummy_dataset", action="store_true", help="Validate on generated chunks (no NQ data).")
    parser.add_argument("--dump_predictions", type=cast2(str), default=None, help="Write predictions JSON here.")
    return parser
