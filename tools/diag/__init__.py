"""ctypes handle on the diagnostic kernels in ``_hq_diag.so`` (built by ``csrc/build.py build_diag``)."""
import ctypes
import os

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_hq_diag.so")
        if not os.path.exists(path):
            from ml_recipe_distributed_pytorch_amd.csrc.build import build_diag
            build_diag()
        _LIB = ctypes.CDLL(path)
        _LIB.hq_cu_hog.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        _LIB.hq_cu_hog.restype = ctypes.c_int
    return _LIB


def cu_hog(blocks: int, usec: int):
    """Occupy ``blocks`` CUs (one 96 KiB-LDS workgroup each) for ``usec`` µs on torch's current stream."""
    import torch
    rc = lib().hq_cu_hog(int(blocks), int(usec), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    if rc != 0:
        raise RuntimeError(f"cu_hog launch failed: hip error {rc}")
