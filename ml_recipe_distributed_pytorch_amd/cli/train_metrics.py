"""Re-evaluate a checkpoint on the train and test splits (reference ``modules/train_metrics.py:13-66``).

Fix of D9: the reference parsed with the predictor parser, which lacks ``dummy_dataset``/``loss``/
``w_*`` and crashed in ``init_datasets``/``init_loss``; here the trainer parser (+ ``--checkpoint``)
is used, so the same ``-c`` config that trained the model re-evaluates it.

    python -m ml_recipe_distributed_pytorch_amd.cli.train_metrics -c config/test_bert.cfg --checkpoint best.ch
"""
from __future__ import annotations

import logging
import os

import torch

from .. import factories
from ..data.items import LABELS
from ..train.callbacks import AccuracyCallback, MAPCallback
from ..train.trainer import Trainer
from ..utils.flags import get_model_parser, get_params, get_trainer_parser
from ..utils.logging import get_logger, show_params

logger = logging.getLogger("train_metrics")


def run_test(params, model, loss, collate_fun, dataset, device):
    trainer = Trainer(model=model, loss=loss, collate_fun=collate_fun, test_dataset=dataset, device=device,
                      test_batch_size=params.test_batch_size, n_jobs=params.n_jobs, precision=params.precision,
                      debug=params.debug)
    trainer.test(-1, callbacks=[MAPCallback(LABELS), AccuracyCallback()])
    return trainer.last_metrics


def main(params, model_params):
    show_params(model_params, "model")
    show_params(params, "test")
    device = torch.device("cuda") if torch.cuda.is_available() and params.gpu else torch.device("cpu")
    model, tokenizer = factories.init_model(model_params, checkpoint=params.checkpoint, device=device,
                                            precision=params.precision)
    train_ds, test_ds, weights = factories.init_datasets(params, tokenizer=tokenizer, clear=False)
    loss = factories.init_loss(params, weights)
    collate = factories.init_collate_fun(tokenizer)
    out = {}
    logger.info("Train dataset validation..")
    out["train"] = run_test(params, model, loss, collate, train_ds, device)
    logger.info("Test dataset validation..")
    out["test"] = run_test(params, model, loss, collate, test_ds, device)
    return out


def cli(argv=None):
    _, (params, model_params) = get_params((get_trainer_parser, get_model_parser), argv)
    params.n_jobs = min(params.n_jobs, max(1, (os.cpu_count() or 2) // 2))
    get_logger(logger_name="train_metrics")
    return main(params, model_params)


if __name__ == "__main__":
    cli()
