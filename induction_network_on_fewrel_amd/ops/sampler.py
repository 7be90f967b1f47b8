"""Device-resident episode sampling (HIP kernel ``ina.sample_episodes``).

The dataset's id arrays live on the GPU (``DeviceDataset``); each step samples B episodes
on-device and the encoder gathers tokens by instance index -- no per-step host sampling, no H2D
copies (the reference samples on the host and feeds 5 numpy arrays per ``sess.run``,
util/data_loader.py:259-309, model/base.py:143-152).
"""
from __future__ import annotations

import numpy as np
import torch

from ..data.fewrel import FewRelDataset
from ._ext import ops


class DeviceArrays(tuple):
    """(word, pos1, pos2, mask) device arrays; ``pos_shift`` = every sequence's position ids are a
    shifted arange (pos[s][t] = pos[s][0] + t, 0 <= pos[s][0] <= L: FewRel's ``j - p + L``), which
    lets the backward reduce the position-table gradients as a per-sequence one-hot GEMM.
    ``lengths`` = int32 [NI]: 1 + each instance's last position with mask > 0 (ragged tiles)."""
    pos_shift = False
    lengths = None


def valid_lengths_np(mask: np.ndarray) -> np.ndarray:
    L = mask.shape[1]
    pos = np.where(mask > 0, np.arange(1, L + 1, dtype=np.int32)[None], 0)
    return pos.max(1).astype(np.int32) if mask.size else np.zeros(mask.shape[0], np.int32)


def positions_are_shifted(pos: np.ndarray) -> bool:
    if pos.ndim != 2 or pos.size == 0:
        return False
    L = pos.shape[1]
    return bool((pos - pos[:, :1] == np.arange(L, dtype=pos.dtype)[None]).all() and (pos[:, 0] >= 0).all()
                and (pos[:, 0] <= L).all())


class DeviceDataset:
    def __init__(self, data: FewRelDataset, device):
        self.data = data
        self.device = torch.device(device)
        t = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.int32), device=self.device)
        self.word = t(data.data_word)
        self.pos1 = t(data.data_pos1)
        self.pos2 = t(data.data_pos2)
        self.mask = t(data.data_mask)
        self.lengths = t(valid_lengths_np(np.asarray(data.data_mask)))
        sc = data.scope_array()
        self.scopes = t(sc)
        self.min_span = int((sc[:, 1] - sc[:, 0]).min()) if len(sc) else 0
        self.num_relations = int(len(sc))
        self.L = data.max_length
        self.pos_shift = positions_are_shifted(data.data_pos1) and positions_are_shifted(data.data_pos2)
        self.bert = ({k: t(data.bert[k]) for k in ("ids", "mask", "e1", "e2")} if data.bert is not None else None)

    def arrays(self, encoder: str = "bilstm"):
        if encoder == "bert":
            if self.bert is None:
                raise ValueError("dataset has no BERT features (data/bert_tokenize.py)")
            return self.bert["ids"], self.bert["mask"], self.bert["e1"], self.bert["e2"]
        out = DeviceArrays((self.word, self.pos1, self.pos2, self.mask))
        out.pos_shift = self.pos_shift
        out.lengths = self.lengths
        return out


class DeviceEpisodeSampler:
    def __init__(self, dd: DeviceDataset, seed: int = 0, nota_rate: float = 0.0):
        self.dd = dd
        self.seed = int(seed) & 0x7FFFFFFF
        self.nota_rate = float(nota_rate)
        self.calls = 0
        # set by the kernel when a rejection loop runs out of rounds (possible duplicate classes / instances)
        self.fail = torch.zeros(1, dtype=torch.int32, device=dd.device)

    def sample(self, B: int, N: int, K: int, Q: int, seed_dev=None):
        """-> (idx int32 [B, N*K+N*Q], labels int32 [B, N*Q]) on the device.  ``seed_dev`` (int32
        device scalar) replaces the host seed (HIP-graph replay; runtime/graph.py)."""
        if K + Q > self.dd.min_span or N > self.dd.num_relations:
            # the kernel's rejection loops need K + Q distinct instances per relation and N relations
            raise ValueError(f"episode {N}-way K+Q={K + Q} needs >= {N} relations with >= {K + Q} instances "
                             f"each (have {self.dd.num_relations}, smallest {self.dd.min_span})")
        s = (self.seed * 1000003 + self.calls * 7919) & 0x7FFFFFFF
        self.calls += 1
        return ops().sample_episodes(self.dd.scopes, B, N, K, Q, s, self.nota_rate, seed_dev, self.fail)

    def check(self) -> None:
        """Raise if any sampled episode hit the rejection-round limit (reads the flag: synchronises)."""
        if int(self.fail.item()) != 0:
            raise RuntimeError("device episode sampler: a rejection loop ran out of rounds (duplicate classes or "
                               "instances possible); the relations' instance spans are too small for N / K + Q")

    def seed_base(self) -> int:
        """seed(calls) = (seed_base + calls * 7919) mod 2^31 (the device step-control formula)."""
        return (self.seed * 1000003) & 0x7FFFFFFF

    def state_dict(self):
        return {"seed": self.seed, "calls": self.calls}

    def load_state_dict(self, d):
        self.seed = int(d["seed"])
        self.calls = int(d["calls"])
