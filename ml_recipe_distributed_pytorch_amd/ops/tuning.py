"""hipBLASLt algorithm selection for the plain library GEMMs (PyTorch TunableOp).

The projection / FFN GEMMs go through ``torch.addmm``/``mm``/``bmm`` → hipBLASLt.  Its default
heuristic pick is measurably slower than the best kernel for several BERT shapes on gfx950 (e.g.
the QKV ``24576×2304×768`` GEMM), so we ship TunableOp results measured on MI355X
(``tuning/tunableop_mi355x.csv``) and load them read-only at start-up.

``HQ_TUNABLEOP``: ``read`` (default) — use shipped results, heuristics elsewhere; ``tune`` — also
tune unseen shapes online (results written to ``HQ_TUNABLEOP_FILE``); ``off`` — plain heuristics.
Results carry validators (torch / HIP / hipBLASLt versions, gfx arch); a mismatching file is
rejected by torch and the heuristics are used.
"""
from __future__ import annotations

import logging
import os

import torch

logger = logging.getLogger(__name__)

SHIPPED = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning", "tunableop_mi355x.csv")
_DONE = False


def _dump_results(path: str):
    """Backup of the tuned table in TunableOp's CSV format (torch also writes its own file at exit)."""
    from torch.cuda import tunable
    try:
        with open(path, "w") as f:
            for k, v in tunable.get_validators():
                f.write(f"Validator,{k},{v}\n")
            for row in tunable.get_results():
                f.write(",".join(str(x) for x in row) + "\n")
    except Exception as e:  # pragma: no cover
        logger.warning(f"could not dump TunableOp results: {e}")


def enable_tuned_gemms(mode: str | None = None) -> bool:
    """Idempotently switch TunableOp on for this process. Returns True if shipped results were loaded."""
    global _DONE
    if _DONE or not torch.cuda.is_available() or torch.version.hip is None:
        return False
    _DONE = True
    mode = (mode or os.environ.get("HQ_TUNABLEOP", "read")).lower()
    if mode == "off" or os.environ.get("PYTORCH_TUNABLEOP_ENABLED") is not None:
        return False  # explicit user env wins
    from torch.cuda import tunable
    tunable.enable(True)
    tunable.tuning_enable(mode == "tune")
    if mode == "tune":
        tunable.set_max_tuning_duration(30)
        out = os.environ.get("HQ_TUNABLEOP_FILE")
        if out:
            tunable.set_filename(out)
            import atexit
            atexit.register(_dump_results, out + ".dump.csv")
    ok = False
    if os.path.exists(SHIPPED):
        try:
            ok = bool(tunable.read_file(SHIPPED))
        except Exception as e:  # pragma: no cover - depends on the box
            logger.warning(f"TunableOp results not loaded ({e}); using hipBLASLt heuristics.")
    logger.info(f"TunableOp {mode}: shipped MI355X GEMM results loaded={ok}.")
    return ok
