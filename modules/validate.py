"""Drop-in shim for the reference CLI (`python modules/validate.py -c <cfg> [--flags]`)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ml_recipe_distributed_pytorch_amd.cli.validate import cli  # noqa: E402

if __name__ == "__main__":
    cli()
