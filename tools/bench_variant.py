#!/usr/bin/env python
"""bench.py with kernel-library lab variants set first (for kernel traces of A/B arms in one process tree):
    python tools/bench_variant.py --tn 1 -- [bench.py args]"""
import os
import runpy
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    rest = argv[argv.index("--") + 1:] if "--" in argv else []
    own = argv[:argv.index("--")] if "--" in argv else argv
    from ml_recipe_distributed_pytorch_amd import _native
    k = _native.kernels()
    for flag, val in zip(own[::2], own[1::2]):
        if flag == "--tn":
            k.gemm_tn_set_variant(int(val))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.argv = [os.path.join(root, "bench.py")] + rest
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
