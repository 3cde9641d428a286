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


def _hip_already_initialised() -> bool:
    """True when this process has already initialised HIP through torch (HIP then ignores a later change
    of GPU_MAX_HW_QUEUES).  Never initialises HIP itself."""
    import sys as _sys
    t = _sys.modules.get("torch")
    if t is None:
        return False
    try:
        return bool(t.cuda.is_initialized())
    except Exception:  # pragma: no cover
        return False


# What this process runs with: HIP reads GPU_MAX_HW_QUEUES once, when it initialises.
#   requested     the count the package wants (None: left alone — HQ_KEEP_HW_QUEUES=1 or ranks share a GPU)
#   env_at_import the value before the package touched it (None: unset → HIP's default, 4)
#   live          the count HIP uses (known exactly unless HIP had been initialised before the import)
#   set_before_hip_init  False when HIP was already up at import time: a raise would be silently ignored
HW_QUEUES = {"requested": None, "env_at_import": None, "live": None, "set_before_hip_init": True}


def _reserve_hw_queues(minimum: int = 8):
    """Give every HIP stream of the process its own hardware queue (set before HIP initialises).

    The training step uses up to 5 streams (compute, weight-gradient side stream, the reducer's comm
    stream and RCCL's internal streams).  With HIP's default of 4 hardware queues two of them share one
    in-order AQL queue, so the compute stream's kernels queue up behind the all-reduce's cross-stream
    waits: measured on MI355X with the RCCL reducer active, 80.8 ms/step with 4 queues vs 69.6 ms with 8
    (69.1 ms without a reducer; profiles/r2_reducer/).  Never more than 8: eight ranks of a node each hold
    their own GPU, so 8 per process is 8 per GPU.  HQ_KEEP_HW_QUEUES=1 leaves the setting alone, and so do
    runs whose ranks share one GPU (_ranks_share_a_gpu).

    If HIP is already initialised when the package is imported (the caller touched torch.cuda first), the
    new value cannot take effect: the package warns once and records the count HIP actually read."""
    env = _os.environ.get("GPU_MAX_HW_QUEUES")
    HW_QUEUES["env_at_import"] = env
    try:
        cur = int(env) if env else 4
    except ValueError:
        cur = 4
    HW_QUEUES["live"] = cur
    if _os.environ.get("HQ_KEEP_HW_QUEUES") == "1" or _ranks_share_a_gpu():
        return
    want = max(cur, minimum)
    HW_QUEUES["requested"] = want
    if cur >= want:
        return
    if _hip_already_initialised():
        HW_QUEUES["set_before_hip_init"] = False
        import warnings
        warnings.warn(f"ml_recipe_distributed_pytorch_amd imported after HIP was initialised: the process keeps "
                      f"{cur} hardware queues instead of {want} (import the package before touching torch.cuda, "
                      "or export GPU_MAX_HW_QUEUES=8); multi-stream steps run slower", RuntimeWarning)
        return
    _os.environ["GPU_MAX_HW_QUEUES"] = str(want)
    HW_QUEUES["live"] = want


def hw_queue_info() -> dict:
    """Hardware-queue state of this process (see ``HW_QUEUES``); bench.py reports it."""
    return dict(HW_QUEUES)


_reserve_hw_queues()
