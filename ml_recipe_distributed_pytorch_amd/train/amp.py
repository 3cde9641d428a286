"""Mixed-precision policy (replaces the reference's Apex probe and AMP integration,
``modules/model/trainer/utils.py:7-12`` and ``trainer.py:23-32,128-133,200-204``).

NVIDIA Apex does not exist on ROCm, and the design does not need it: master weights are always fp32
(the ParamStore arena), the compute copy is bf16, and bf16 has fp32's exponent range, so there is no
loss scaling, no overflow check and no optimizer wrapping.  The reference's ``--apex_level`` keeps
its meaning as a precision request:

    None / O1 / O2 / O3 → bf16 compute (O1's "fp16 GEMMs, fp32 softmax/LN" is what the fused
                          kernels do in bf16: statistics, softmax and the optimizer stay fp32)
    O0                  → fp32 compute
    --precision fp8     → bf16 + OCP e4m3 forward projections (overrides apex_level)

``--apex_loss_scale`` / ``--apex_verbosity`` are accepted and ignored (logged).
"""
from __future__ import annotations

import importlib.util
import logging
from typing import Optional

import torch

logger = logging.getLogger(__name__)

APEX_AVAILABLE = importlib.util.find_spec("apex") is not None


def apex_to_precision(apex_level: Optional[str], device) -> str:
    if torch.device(device).type != "cuda":
        return "fp32"
    return "fp32" if apex_level == "O0" else "bf16"


def resolve_precision(precision: Optional[str], apex_level: Optional[str], device, apex_loss_scale=None) -> str:
    prec = precision or apex_to_precision(apex_level, device)
    if torch.device(device).type != "cuda" and prec != "fp32":
        logger.warning(f"precision {prec} needs the GPU path; using fp32 on {device}.")
        prec = "fp32"
    if apex_level is not None:
        logger.info(f"apex_level {apex_level} → native {prec} mixed precision (fp32 master weights; Apex "
                    f"{'present but unused' if APEX_AVAILABLE else 'not installed'}).")
    if apex_loss_scale is not None:
        logger.info("apex_loss_scale ignored: bf16 needs no loss scaling.")
    return prec
