"""gfx950 HIP kernel ops (torch.ops.ina) and their autograd / packing wrappers."""
from ._ext import available, library_path, load, ops

__all__ = ["available", "library_path", "load", "ops"]
