"""Drop-in shim for the reference ``modules/init.py`` factories (notebooks import from here)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ml_recipe_distributed_pytorch_amd.factories import (  # noqa: E402,F401
    init_collate_fun, init_datasets, init_loss, init_model, init_optimizer)
