"""Checkpoint save / restore with the reference's layout and TF variable names.

Reference (model/base.py:124,171-178): ``tf.train.Saver()`` (max_to_keep=5) saving to
``<model_dir>/checkpoint/inductionNetwork-<global_step>`` plus the ``checkpoint`` state file, on best
val accuracy; there is NO restore path in the reference (``curr_iter = 0``, :130). This module keeps
the directory layout, the file stem and the state file, and the variable names/shapes of SURVEY 2.4
as tensor keys (params, ``<var>/Adam``, ``<var>/Adam_1``, ``beta1_power``, ``beta2_power``,
``global_step``).  Every checkpoint is written twice under the same stem: as TF's V2 tensor bundle
(``<stem>.index`` + ``<stem>.data-00000-of-00001``, the files ``tf.train.Saver`` writes; runtime/tf_bundle.py
produces them without TF) and as safetensors (``<stem>.safetensors``) + a JSON index (``<stem>.index.json``:
resume metadata -- config, sampler states, best accuracy, optimizer counters).  ``load`` reads either
(safetensors first; a bare TF bundle, e.g. written elsewhere, loads with its metadata if present).
Rank 0 writes; other ranks receive state by broadcast (parallel/dp.py).
"""
from __future__ import annotations

import json
import os
import re
from collections import OrderedDict
from typing import Dict, Optional, Tuple

import torch
from safetensors.torch import load_file, save_file

from . import tf_bundle

FORMAT = "ina-ckpt-v1"


def ckpt_dir(model_dir: str) -> str:
    return os.path.join(model_dir, "checkpoint")


def _state_file(model_dir: str) -> str:
    return os.path.join(ckpt_dir(model_dir), "checkpoint")


def read_state(model_dir: str):
    f = _state_file(model_dir)
    if not os.path.exists(f):
        return None, []
    latest, allp = None, []
    with open(f) as fh:
        for line in fh:
            m = re.match(r'\s*(\w+):\s*"(.*)"', line)
            if not m:
                continue
            if m.group(1) == "model_checkpoint_path":
                latest = m.group(2)
            elif m.group(1) == "all_model_checkpoint_paths":
                allp.append(m.group(2))
    return latest, allp


def _write_state(model_dir: str, latest: str, allp) -> None:
    with open(_state_file(model_dir), "w") as fh:
        fh.write(f'model_checkpoint_path: "{latest}"\n')
        for p in allp:
            fh.write(f'all_model_checkpoint_paths: "{p}"\n')


def _best_file(model_dir: str) -> str:
    return os.path.join(ckpt_dir(model_dir), "best_checkpoint")


def best_stem(model_dir: str) -> Optional[str]:
    """Stem recorded by the last ``save(..., best=True)`` (kept out of the max_to_keep rotation)."""
    f = _best_file(model_dir)
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        m = re.match(r'\s*model_checkpoint_path:\s*"(.*)"', fh.read())
    return m.group(1) if m else None


def save(model_dir: str, name: str, step: int, tensors: "OrderedDict[str, torch.Tensor]", meta: dict,
         max_to_keep: int = 5, best: bool = False, tf_format: bool = True, meta_graph: Optional[bytes] = None) -> str:
    """Write ``<model_dir>/checkpoint/<name>-<step>`` and rotate to ``max_to_keep``.  ``best=True`` also
    points ``best_checkpoint`` at it; the best checkpoint is never rotated away (a periodic or resumed
    checkpoint can be newer, so "latest" is not "best")."""
    d = ckpt_dir(model_dir)
    os.makedirs(d, exist_ok=True)
    stem = f"{name}-{step}"
    cpu = OrderedDict((k, v.detach().to("cpu").contiguous()) for k, v in tensors.items())
    tmp = os.path.join(d, stem + ".safetensors.tmp")
    save_file(cpu, tmp)
    os.replace(tmp, os.path.join(d, stem + ".safetensors"))
    if tf_format:
        tf_bundle.save_bundle(os.path.join(d, stem), cpu)   # <stem>.index + <stem>.data-00000-of-00001
        if meta_graph is not None:   # <stem>.meta: the serialized MetaGraphDef (runtime/tb_graph.py::meta_graph)
            with open(os.path.join(d, stem + ".meta.tmp"), "wb") as fh:
                fh.write(meta_graph)
            os.replace(os.path.join(d, stem + ".meta.tmp"), os.path.join(d, stem + ".meta"))
    index = dict(meta, format=FORMAT, global_step=int(step),
                 variables={k: {"shape": list(v.shape), "dtype": str(v.dtype).replace("torch.", "")}
                            for k, v in cpu.items()})
    with open(os.path.join(d, stem + ".index.json"), "w") as fh:
        json.dump(index, fh, indent=1, sort_keys=True)
    prev_best = best_stem(model_dir)
    if best:
        with open(_best_file(model_dir) + ".tmp", "w") as fh:
            fh.write(f'model_checkpoint_path: "{stem}"\n')
        os.replace(_best_file(model_dir) + ".tmp", _best_file(model_dir))
    keep = best_stem(model_dir)
    _, allp = read_state(model_dir)
    allp = [p for p in allp if p != stem] + [stem]
    while len(allp) > max_to_keep:
        old = allp.pop(0)
        if old != keep:   # the best checkpoint leaves the rotation list but its files stay
            _remove(d, old)
    # a superseded best that already left the rotation is referenced by nothing any more: delete it
    # (otherwise every best that outlives max_to_keep periodic saves and is then beaten leaks a file)
    if best and prev_best is not None and prev_best != stem and prev_best not in allp:
        _remove(d, prev_best)
    _write_state(model_dir, stem, allp)
    return os.path.join(d, stem)


def _remove(d: str, stem: str) -> None:
    for ext in (".safetensors", ".index.json", ".index", ".meta", tf_bundle.DATA_SUFFIX):
        try:
            os.remove(os.path.join(d, stem + ext))
        except FileNotFoundError:
            pass


def latest(model_dir: str) -> Optional[str]:
    stem, _ = read_state(model_dir)
    if stem is None:
        return None
    p = os.path.join(ckpt_dir(model_dir), stem)
    return p if _exists(p) else None


def _exists(p: str) -> bool:
    return os.path.exists(p + ".safetensors") or tf_bundle.exists(p)


def best(model_dir: str) -> Optional[str]:
    """Path stem of the best-val checkpoint, if one was recorded and still exists."""
    stem = best_stem(model_dir)
    if stem is None:
        return None
    p = os.path.join(ckpt_dir(model_dir), stem)
    return p if _exists(p) else None


def load(path_stem: str, prefer: str = "safetensors") -> Tuple[Dict[str, torch.Tensor], dict]:
    """(tensors by TF variable name, metadata).  ``prefer="tf"`` reads the TF bundle even when the
    safetensors copy exists; a bundle without our JSON index gets ``{"format": "tf-bundle"}`` metadata."""
    use_tf = not os.path.exists(path_stem + ".safetensors") or (prefer == "tf" and tf_bundle.exists(path_stem))
    tensors = dict(tf_bundle.load_bundle(path_stem)) if use_tf else load_file(path_stem + ".safetensors")
    if os.path.exists(path_stem + ".index.json"):
        with open(path_stem + ".index.json") as fh:
            meta = json.load(fh)
        if meta.get("format") != FORMAT:
            raise ValueError(f"unknown checkpoint format {meta.get('format')}")
    elif use_tf:
        meta = {"format": "tf-bundle", "global_step": int(tensors["global_step"]) if "global_step" in tensors else 0}
    else:
        raise FileNotFoundError(path_stem + ".index.json")
    return tensors, meta
