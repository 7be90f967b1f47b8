from . import checkpoint, metrics

__all__ = ["checkpoint", "metrics"]
