"""ml-recipe-distributed-pytorch, rebuilt MI355X-first (PyTorch-ROCm + hand-written gfx950 HIP kernels + RCCL).

Capability parity with neuro-inc/ml-recipe-distributed-pytorch: distributed BERT/RoBERTa QA fine-tuning
(train.py / validate.py CLI, .cfg configs, checkpoints, dummy + Natural Questions data paths).
"""
import os as _os

__version__ = "0.1.0"


def _visible_gpus() -> int:
    """GPUs this process may see, without initialising HIP (the queue count must be set before that)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = _os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    n = 0
    try:
        base = "/sys/class/kfd/kfd/topology/nodes"
        for node in _os.listdir(base):
            try:
                with open(f"{base}/{node}/gpu_id") as f:
                    n += int(f.read().strip() or 0) != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    return n


def _ranks_share_a_gpu() -> bool:
    """Several ranks of this node on one GPU (HQ_BENCH_BACKEND=gloo rehearsal, or more local ranks than
    GPUs): then 8 queues per process oversubscribe the GPU's hardware queue slots — two ranks on cuda:0
    with 8 each hung in a gloo all-reduce, with HIP's default 4 each they ran (profiles/r2_reducer)."""
    if _os.environ.get("HQ_BENCH_BACKEND", "nccl") != "nccl":
        return True
    try:
        lws = int(_os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    except ValueError:
        return False
    if lws <= 1:
        return False
    n = _visible_gpus()
    return 0 < n < lws


def _reserve_hw_queues(minimum: int = 8):
    """Give every HIP stream of the process its own hardware queue (set before HIP initialises).

    The training step uses up to 5 streams (compute, weight-gradient side stream, the reducer's comm
    stream and RCCL's internal streams).  With HIP's default of 4 hardware queues two of them share one
    in-order AQL queue, so the compute stream's kernels queue up behind the all-reduce's cross-stream
    waits: measured on MI355X with the RCCL reducer active, 80.8 ms/step with 4 queues vs 69.6 ms with 8
    (69.1 ms without a reducer; profiles/r2_reducer/).  HQ_KEEP_HW_QUEUES=1 leaves the setting alone."""
    if _os.environ.get("HQ_KEEP_HW_QUEUES") == "1" or _ranks_share_a_gpu():
        return
    try:
        cur = int(_os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        cur = 4
    if cur < minimum:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(minimum)


_reserve_hw_queues()
