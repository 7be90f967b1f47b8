"""MI355X-native Induction Network for few-shot relation classification on FewRel.

Capabilities of wws0815/Induction-Network-on-FewRel (TF1 reference) re-designed for gfx950:
BiLSTM + word-level self-attention encoder, dynamic-routing induction, neural-tensor relation
scorer, MSE + Adam episodic training -- as hand-written HIP kernels (MFMA / LDS), with episode
batching, a device-resident sampler, RCCL data parallelism and TF-name-compatible checkpoints.
"""
from .config import Config

__version__ = "0.1.0"
__all__ = ["Config", "__version__"]
