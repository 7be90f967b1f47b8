from .dp import DistContext

__all__ = ["DistContext"]
