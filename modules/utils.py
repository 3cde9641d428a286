"""Drop-in shim for the reference ``modules/utils.py`` helpers."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ml_recipe_distributed_pytorch_amd.utils.logging import get_logger, set_seed, show_params  # noqa: E402,F401
