"""Seeding and the ``deterministic`` execution mode.

The fused GPU path with a frozen word table (the reference default) is deterministic by construction
(ordered reductions, no float atomics: eager and hipGraph steps are bit-identical,
tests/test_kernels_gpu.py).  A TRAINED word table is the exception: lstm_bwd adds the non-padding
word-row gradients with global float atomics, so those runs are not bitwise reproducible
(``make_deterministic`` warns about it).  ``Config.deterministic`` extends determinism to everything else
a run touches: Python / NumPy / torch seeds, torch's deterministic-algorithm mode (errors, not warnings,
on a non-deterministic library op of the wide / BERT paths) and a fixed hipBLAS(Lt) workspace, set before
any BLAS handle exists (the trainer calls this before building the model).
"""
import os
import random

import numpy as np
import torch


def seed_everything(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed & 0xFFFFFFFF)
    torch.manual_seed(seed)


def make_deterministic(seed: int, trained_word_table: bool = False) -> None:
    seed_everything(seed)
    # the workspace config is read when a BLAS handle is created: set it unconditionally, before any GEMM
    os.environ["CUBLAS_WORKSPACE_CONFIG"] = ":4096:8"
    torch.use_deterministic_algorithms(True, warn_only=False)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
    if trained_word_table:
        import warnings
        warnings.warn("deterministic=True with a trained word table: the word-row gradients use float atomics "
                      "(csrc/kernels/lstm.hip lstm_bwd WG path), so runs are not bitwise reproducible")
