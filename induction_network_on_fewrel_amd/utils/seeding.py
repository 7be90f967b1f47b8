"""Seeding and the ``deterministic`` execution mode.

The fused GPU path is deterministic by construction (ordered reductions, no float atomics: eager and
hipGraph steps are bit-identical, tests/test_kernels_gpu.py).  ``Config.deterministic`` extends that to
everything else a run touches: Python / NumPy / torch seeds, torch's deterministic-algorithm mode for
the library ops of the wide / BERT paths (index backward, scatter), and a fixed hipBLAS(Lt) workspace.
"""
import os
import random

import numpy as np
import torch


def seed_everything(seed: int) -> None:
    random.seed(seed)
    np.random.seed(seed & 0xFFFFFFFF)
    torch.manual_seed(seed)


def make_deterministic(seed: int) -> None:
    seed_everything(seed)
    os.environ.setdefault("CUBLAS_WORKSPACE_CONFIG", ":4096:8")
    torch.use_deterministic_algorithms(True, warn_only=True)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True
