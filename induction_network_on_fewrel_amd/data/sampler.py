"""Host-side episode sampler (the reference layout, bit-compatible contract).

Reference: ``util/data_loader.py:213-309`` (``next_one``, ``next_one_tf``) and the
abstract ``next_batch(B, N, K, Q)`` (``:8-17``), which is implemented here.

Layout contract:
* support rows first, class-major (``class0 x K, class1 x K, ...``), unshuffled;
* query rows follow, randomly permuted; ``query_label[q]`` is the class index in
  sampled order.

The engine works on *instance indices* (rows of the device-resident arrays) rather than
on copied token arrays; ``gather`` reproduces the reference's dict-of-arrays output.

FewRel 2.0 none-of-the-above (north star): with probability ``nota_rate`` a query is
drawn from a relation outside the episode and labelled ``N``.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np

from .fewrel import FewRelDataset


class EpisodeSampler:
    def __init__(self, data: FewRelDataset, seed: Optional[int] = None, nota_rate: float = 0.0):
        self.data = data
        self.rng = np.random.default_rng(seed)
        self.scopes = data.scope_array()
        self.nota_rate = float(nota_rate)

    # ------------------------------------------------------------ indices
    def sample_indices(self, N: int, K: int, Q: int) -> Tuple[np.ndarray, np.ndarray]:
        """One episode -> (instance indices [N*K + N*Q], query labels [N*Q])."""
        R = self.scopes.shape[0]
        if N > R:
            raise ValueError(f"N={N} > number of relations {R}")
        classes = self.rng.choice(R, N, replace=False)
        sup = np.empty((N, K), dtype=np.int64)
        qry = np.empty((N, Q), dtype=np.int64)
        for i, c in enumerate(classes):
            b, e = self.scopes[c]
            idx = self.rng.choice(np.arange(b, e), K + Q, replace=False)
            sup[i] = idx[:K]
            qry[i] = idx[K:]
        labels = np.repeat(np.arange(N, dtype=np.int64), Q)
        qry = qry.reshape(-1)
        if self.nota_rate > 0.0 and R > N:
            others = np.setdiff1d(np.arange(R), classes)
            for q in range(N * Q):
                if self.rng.random() < self.nota_rate:
                    c = self.rng.choice(others)
                    b, e = self.scopes[c]
                    qry[q] = self.rng.integers(b, e)
                    labels[q] = N
        perm = self.rng.permutation(N * Q)
        return np.concatenate([sup.reshape(-1), qry[perm]]), labels[perm]

    def next_batch_indices(self, B: int, N: int, K: int, Q: int) -> Tuple[np.ndarray, np.ndarray]:
        """B episodes -> (indices [B, N*(K+Q)], labels [B, N*Q])."""
        out = [self.sample_indices(N, K, Q) for _ in range(B)]
        return np.stack([o[0] for o in out]), np.stack([o[1] for o in out])

    # ------------------------------------------------- reference-style outputs
    def gather(self, idx: np.ndarray) -> Dict[str, np.ndarray]:
        d = self.data
        return {"word": d.data_word[idx], "pos1": d.data_pos1[idx], "pos2": d.data_pos2[idx],
                "mask": d.data_mask[idx]}

    def next_one_tf(self, N: int, K: int, Q: int):
        """Reference ``next_one_tf`` (data_loader.py:259): inputs [N*K+N*Q, L] + labels."""
        idx, labels = self.sample_indices(N, K, Q)
        return self.gather(idx), labels

    def next_one(self, N: int, K: int, Q: int):
        """Reference ``next_one`` (data_loader.py:213): support stacked [N, K, L]."""
        idx, labels = self.sample_indices(N, K, Q)
        g = self.gather(idx)
        L = self.data.max_length
        support = {k: v[: N * K].reshape(N, K, L) for k, v in g.items()}
        query = {k: v[N * K:] for k, v in g.items()}
        return support, query, labels

    def next_batch(self, B: int, N: int, K: int, Q: int):
        """Implements the reference's abstract ``next_batch`` (data_loader.py:9-17)."""
        idx, labels = self.next_batch_indices(B, N, K, Q)
        return self.gather(idx), labels
