"""Chunked-inference validation entry (reference ``modules/validate.py:15-63``).

    python -m ml_recipe_distributed_pytorch_amd.cli.validate -c config/validate.cfg [--dummy_dataset]

Fixes D12: ``max_seq_len`` / ``max_question_len`` / ``doc_stride`` / ``split_by_sentence`` /
``truncate`` from the config are honoured (the reference hard-coded the ChunkDataset defaults),
``--dummy_dataset`` validates without NQ data, and metrics (label accuracy, span EM/F1) are
reported.  The native tokenizer is picklable, so the reference's swap to the slow HF tokenizer for
the worker pool is unnecessary.
"""
from __future__ import annotations

import logging
import os

import torch

from .. import factories
from ..data.dummy import DummyChunkDataset
from ..infer.predictor import Predictor
from ..utils.flags import get_model_parser, get_params, get_predictor_parser
from ..utils.logging import get_logger, show_params

logger = logging.getLogger("validate")


def get_validation_dataset(params, *, tokenizer=None, clear=False):
    common = dict(max_seq_len=params.max_seq_len, max_question_len=params.max_question_len)
    if getattr(params, "dummy_dataset", False):
        return DummyChunkDataset(tokenizer, dataset_len=getattr(params, "dummy_dataset_len", 1000), **common)
    from ..data.nq import ChunkDataset, RawPreprocessor
    pre = RawPreprocessor(raw_json=params.data_path, out_dir=params.processed_data_path, clear=clear)
    _, _, (_, _, val_idx, _) = pre()
    return ChunkDataset(params.processed_data_path, tokenizer, val_idx, doc_stride=params.doc_stride, test=False,
                        split_by_sentence=params.split_by_sentence, truncate=params.truncate, **common)


def main(params, model_params) -> Predictor:
    show_params(model_params, "model")
    show_params(params, "predictor")
    device = torch.device("cuda") if torch.cuda.is_available() and params.gpu else torch.device("cpu")
    if params.checkpoint is not None and not os.path.exists(params.checkpoint):
        raise FileNotFoundError(f"Checkpoint {params.checkpoint} does not exist.")
    model, tokenizer = factories.init_model(model_params, checkpoint=params.checkpoint, device=device,
                                            precision=params.precision)
    dataset = get_validation_dataset(params, tokenizer=tokenizer)
    predictor = Predictor(model, device, collate_fun=factories.init_collate_fun(tokenizer, return_items=True),
                          batch_size=params.batch_size, n_jobs=params.n_jobs, buffer_size=params.buffer_size,
                          limit=params.limit)
    predictor(dataset)
    m = predictor.metrics()
    logger.info("Validation metrics: " + ", ".join(f"{k}: {v:.4f}" if isinstance(v, float) else f"{k}: {v}"
                                                   for k, v in m.items()))
    if getattr(params, "dump_predictions", None):
        predictor.save_predictions(params.dump_predictions)
        logger.info(f"Predictions were dumped to {params.dump_predictions}.")
    return predictor


def cli(argv=None):
    _, (params, model_params) = get_params((get_predictor_parser, get_model_parser), argv)
    get_logger(logger_name="validate")
    params.n_jobs = min(params.n_jobs, max(1, (os.cpu_count() or 2) // 2))
    return main(params, model_params)


if __name__ == "__main__":
    cli()
