#!/usr/bin/env python
"""Print the per-step losses of the eager and graph-replay runs of tests/test_graph_gpu.py::_run (diagnostic for
library variants: HQ_KERNELS_DEBUG / HQ_KERNELS_DIR / HQ_DEBUG_NOSYNC)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_graph_gpu import _run  # noqa: E402

cuda = torch.device("cuda", 0)
le, me, _, _, _ = _run(cuda, graph=False)
lg, mg, _, _, _ = _run(cuda, graph=True)
print(json.dumps({"eager": le, "graph": lg, "master_diff": int((mg != me).sum())}))
