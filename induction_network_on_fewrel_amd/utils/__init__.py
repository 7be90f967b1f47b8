from .seeding import make_deterministic, seed_everything

__all__ = ["make_deterministic", "seed_everything"]
