"""FewRel 2.0-style evaluation (north star): none-of-the-above (NOTA) episodes, NOTA
threshold selection, domain-adaptation evaluation on another dataset, large eval batches.

The reference only evaluates plain N-way K-shot accuracy on its val loader (``Base.eval``,
model/base.py:186-208).  Additions here:

* ``EvalReport`` -- accuracy over all queries plus the split into in-class accuracy and NOTA
  precision / recall (FewRel 2.0 reports the overall accuracy at a NOTA rate, e.g. 0.15 / 0.5).
* NOTA decision: the model's relation scores are sigmoids (MSE on one-hot targets), so a query whose
  best score is below a threshold is predicted as NOTA (label N; ``models/reference.py::predict``).
  ``select_nota_threshold`` picks the threshold that maximises accuracy on validation episodes.
* ``evaluate_dataset`` -- any FewRelDataset (e.g. a different-domain file tensorised with the
  training vocabulary) is evaluated with a fresh sampler (domain adaptation = train on one
  distribution, test on another; the model itself is unchanged).
* Large batches: ``batch`` episodes per forward (sized for HBM, not for the reference's one
  episode per ``sess.run``).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import Iterable, List, Optional, Sequence

import torch

from ..data.fewrel import FewRelDataset
from ..models import reference as ref


@dataclass
class EvalReport:
    episodes: int
    N: int
    K: int
    Q: int
    nota_rate: float
    threshold: Optional[float]
    accuracy: float              # over all queries (FewRel 2.0 "accuracy")
    in_class_accuracy: float     # queries whose label is one of the N classes
    nota_precision: float        # predicted NOTA that are NOTA
    nota_recall: float           # NOTA queries predicted NOTA
    nota_fraction: float         # share of NOTA queries actually sampled

    def to_dict(self) -> dict:
        return asdict(self)


def make_sampler(trainer, data: FewRelDataset, seed: int, nota_rate: float):
    """A fresh episode sampler over ``data`` on the trainer's device (device-resident on GPU)."""
    return trainer._make_sampler(data, seed, nota_rate)


@torch.no_grad()
def collect_probs(trainer, sampler, iters: int, N: int, K: int, Q: int, batch: Optional[int] = None):
    """Run ``iters`` episodes; returns (probs [E, N*Q, N], labels [E, N*Q]) on the host."""
    cfg = trainer.cfg
    B = batch or max(1, min(cfg.episodes_per_step, iters))
    probs_all, lab_all = [], []
    done = 0
    while done < iters:
        b = min(B, iters - done)
        idx, labels = sampler.sample(b, N, K, Q)
        probs, _ = trainer.model(idx.view(-1), sampler.arrays, b, N, K, Q, training=False)
        probs_all.append(probs.float().cpu())
        lab_all.append(labels.long().cpu())
        done += b
    return torch.cat(probs_all), torch.cat(lab_all)


def report(probs: torch.Tensor, labels: torch.Tensor, N: int, K: int, Q: int, nota_rate: float,
           threshold: Optional[float]) -> EvalReport:
    pred = ref.predict(probs, threshold)
    hit = (pred == labels)
    is_nota = labels == N
    pred_nota = pred == N
    acc = float(hit.float().mean())
    in_cls = float(hit[~is_nota].float().mean()) if bool((~is_nota).any()) else float("nan")
    prec = float((pred_nota & is_nota).sum()) / max(1, int(pred_nota.sum()))
    rec = float((pred_nota & is_nota).sum()) / max(1, int(is_nota.sum()))
    return EvalReport(int(probs.shape[0]), N, K, Q, nota_rate, threshold, acc, in_cls, prec, rec,
                      float(is_nota.float().mean()))


def select_nota_threshold(probs: torch.Tensor, labels: torch.Tensor, N: int,
                          grid: Optional[Sequence[float]] = None) -> float:
    """Threshold on the best relation score that maximises episode accuracy (ties -> lower)."""
    grid = list(grid) if grid is not None else [i / 100.0 for i in range(1, 100)]
    best_t, best_a = grid[0], -1.0
    for t in grid:
        a = float((ref.predict(probs, t) == labels).float().mean())
        if a > best_a + 1e-12:
            best_t, best_a = t, a
    return best_t


def evaluate_dataset(trainer, data: FewRelDataset, iters: int, N: int, K: int, Q: int, nota_rate: float = 0.0,
                     threshold: Optional[float] = None, batch: Optional[int] = None, seed: int = 4242,
                     tune_on: Optional[FewRelDataset] = None, tune_iters: int = 500) -> EvalReport:
    """Evaluate on ``data`` (any domain).  With ``nota_rate > 0`` and ``threshold is None`` the NOTA
    threshold is tuned on ``tune_on`` (default: the trainer's validation data) first."""
    if nota_rate > 0.0 and threshold is None:
        tsamp = make_sampler(trainer, tune_on if tune_on is not None else trainer.val_data, seed + 1, nota_rate)
        tp, tl = collect_probs(trainer, tsamp, tune_iters, N, K, Q, batch)
        threshold = select_nota_threshold(tp, tl, N)
    s = make_sampler(trainer, data, seed, nota_rate)
    probs, labels = collect_probs(trainer, s, iters, N, K, Q, batch)
    r = report(probs, labels, N, K, Q, nota_rate, threshold)
    if trainer.dist.world > 1:   # mean over ranks (each rank sampled its own episodes)
        vals = trainer.dist.mean_scalars([r.accuracy, r.in_class_accuracy, r.nota_precision, r.nota_recall])
        r.accuracy, r.in_class_accuracy, r.nota_precision, r.nota_recall = vals
    return r


def evaluate_grid(trainer, data: FewRelDataset, settings: Iterable[tuple], iters: int, nota_rates=(0.0,),
                  batch: Optional[int] = None) -> List[EvalReport]:
    """FewRel-style table: every (N, K) in ``settings`` x every NOTA rate."""
    out = []
    for (N, K) in settings:
        for nr in nota_rates:
            out.append(evaluate_dataset(trainer, data, iters, N, K, trainer.cfg.eQ, nr, batch=batch))
    return out
