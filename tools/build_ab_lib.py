#!/usr/bin/env python
"""Build a second kernel library for same-box A/B: the in-tree sources, except the listed kernel files taken
from git revision REV, linked into tools/ab_so/_hq_kernels<ext> (load it with HQ_KERNELS_DIR=tools/ab_so;
AB_DIR=tools/<name> picks another directory; HQ_KERNEL_CFLAGS="-DHQ_EPI_DIAG=1 ..." adds lab defines to THIS build
only — the production build never reads it).

    python tools/build_ab_lib.py HEAD ml_recipe_distributed_pytorch_amd/csrc/kernels/gemm.hip
"""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rev, files = sys.argv[1], sys.argv[2:]
    from ml_recipe_distributed_pytorch_amd.csrc import build as b
    out_dir = os.path.join(ROOT, os.environ.get("AB_DIR", os.path.join("tools", "ab_so")))
    tmp = os.path.join(out_dir, "src")
    if os.path.exists(tmp):
        shutil.rmtree(tmp)
    shutil.copytree(b.HERE, tmp, ignore=shutil.ignore_patterns("build"))
    for f in files:
        rel = os.path.relpath(os.path.join(ROOT, f), b.HERE)
        with open(os.path.join(tmp, rel), "wb") as fh:
            fh.write(subprocess.check_output(["git", "show", f"{rev}:{f}"], cwd=ROOT))
    here, pkg = b.HERE, b.PKG
    try:
        b.HERE, b.PKG = tmp, out_dir
        lab = [f for f in os.environ.get("HQ_KERNEL_CFLAGS", "").split() if f.startswith("-D")]
        out = b.build_kernels(8, lab_defines=lab)
    finally:
        b.HERE, b.PKG = here, pkg
    print(out)


if __name__ == "__main__":
    main()
