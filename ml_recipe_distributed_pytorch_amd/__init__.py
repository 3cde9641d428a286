"""ml-recipe-distributed-pytorch, rebuilt MI355X-first (PyTorch-ROCm + hand-written gfx950 HIP kernels + RCCL).

Capability parity with neuro-inc/ml-recipe-distributed-pytorch: distributed BERT/RoBERTa QA fine-tuning
(train.py / validate.py CLI, .cfg configs, checkpoints, dummy + Natural Questions data paths).
"""
__version__ = "0.1.0"
