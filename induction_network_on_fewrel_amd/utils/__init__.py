from .timing import GpuTimer, PhaseTimer
from .seeding import seed_everything

__all__ = ["GpuTimer", "PhaseTimer", "seed_everything"]
