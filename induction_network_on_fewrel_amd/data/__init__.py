from .fewrel import FewRelDataset, truncate_word_vectors, vocab_from_fewrel
from .synthetic import make_synthetic, random_word_vectors
from .sampler import EpisodeSampler

__all__ = ["FewRelDataset", "truncate_word_vectors", "vocab_from_fewrel", "make_synthetic",
           "random_word_vectors", "EpisodeSampler"]
