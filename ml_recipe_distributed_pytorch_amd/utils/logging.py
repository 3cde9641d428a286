"""Logging, seeding and parameter dump — the L9 utilities (reference ``modules/utils.py:10-51``).

Contract kept from the reference: the record layout
``<date> - <LEVEL> - <logger name | path:func:line> -   <message>`` (so existing log parsers keep
working), console + optional file output at ``dump_dir/<exp>/<date>.log``, and a silenced
``transformers`` logger.  Everything else is our own:

* handlers are owned by this module (``_OWNED``) and swapped atomically on reconfiguration, so a
  spawned worker re-opening the run's log in append mode never duplicates console output;
* ``set_seed`` seeds every generator the framework draws from (python, numpy, torch CPU and every
  HIP device) and returns the seed actually used;
* ``show_params`` writes one aligned block instead of a record per key.
"""
from __future__ import annotations

import logging
import os
import random
import sys
from typing import Optional

import numpy as np
import torch

logger = logging.getLogger(__name__)

_DATEFMT = "%m/%d/%Y %H:%M:%S"
_OWNED: list = []  # handlers installed by configure()


def _formatter(debug: bool) -> logging.Formatter:
    origin = "%(pathname)s:%(funcName)s:%(lineno)d" if debug else "%(name)s"
    return logging.Formatter("%(asctime)s - %(levelname)s - " + origin + " -   %(message)s", datefmt=_DATEFMT)


def configure(level: int = logging.INFO, filename: Optional[str] = None, filemode: str = "w",
              debug: bool = False) -> None:
    """(Re)install the root handlers: stderr always, plus ``filename`` when given."""
    root = logging.getLogger()
    for h in list(root.handlers):  # the reference also drops foreign handlers (basicConfig leftovers)
        root.removeHandler(h)
        if h in _OWNED:
            h.close()
    _OWNED.clear()
    fmt = _formatter(debug)
    targets = [logging.StreamHandler(sys.stderr)]
    if filename is not None:
        targets.append(logging.FileHandler(filename, mode=filemode))
    for h in targets:
        h.setFormatter(fmt)
        root.addHandler(h)
        _OWNED.append(h)
    root.setLevel(level)
    logging.getLogger("transformers").setLevel(logging.CRITICAL)


def get_logger(*, level=logging.INFO, filename=None, filemode="w", logger_name=None, debug=False):
    """Configure logging for this process and return the named entry-point logger."""
    configure(level=level, filename=filename, filemode=filemode, debug=debug)
    named = logging.getLogger(logger_name or __name__)
    if filename is not None and filemode == "w":
        named.info(f"All logs will be dumped to {filename}.")
    return named


def set_seed(seed=None) -> Optional[int]:
    """Seed python / numpy / torch (CPU and all HIP devices).  ``None`` leaves every generator alone.

    Like the reference (modules/utils.py:34-43, ``cudnn.deterministic = True``) a seed also selects the
    run-to-run reproducible kernels: ``HQ_DETERMINISTIC=1`` routes the attention backward to its
    two-kernel path instead of the single-kernel one with LDS-atomic dQ (ops.deterministic)."""
    if seed is None:
        return None
    seed = int(seed)
    for fn in (random.seed, np.random.seed, torch.manual_seed):
        fn(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    os.environ["HQ_DETERMINISTIC"] = "1"
    logger.info(f"Random seed was set to {seed}. It can affect speed of training and performance of result model.")
    return seed


def show_params(params, name) -> None:
    """Log every attribute of a parsed namespace as one aligned block."""
    items = sorted(vars(params).items())
    width = max((len(k) for k, _ in items), default=0)
    body = "\n".join(f"\t\t{k.ljust(width)}: {v}" for k, v in items)
    logger.info(f"Input {name} parameters:\n{body}")
