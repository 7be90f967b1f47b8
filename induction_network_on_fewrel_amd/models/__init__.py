from .params import InductionParams, TF_NAMES
from .induction import InductionNetwork
from . import reference

__all__ = ["InductionParams", "TF_NAMES", "InductionNetwork", "reference"]
