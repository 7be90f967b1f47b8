"""Every per-step weight pack of the wide path (ops/packing.py::pack_lstm_wide / pack_attn_wide) in ONE
launch: ``ina.gather_pack_affine`` gathers the elements from the flat parameter buffer with a
precomputed int32 index and applies a per-element affine map (the exp2 gate pre-scales, the TF forget
bias), writing the bf16 packs and the fp32 bias vectors in one pass.  The pack functions themselves ran
as ~65 small PyTorch launches per step at the paper configuration (pads, permutation gathers, scale
multiplies, casts, concatenations: ~0.6 ms of a 9.9 ms step, profiles/r3_head_wide/seq_paper.txt).

The plan is derived from the pack functions, so it cannot drift from them: they are evaluated once on
(1) float tensors holding each element's flat index + 1 with the scales off (-> the gather index, 0 = a
padding element), (2) all-zero and (3) all-one parameters with the scales on (-> add = pack(0) and
mul = pack(1) - pack(0)).  Requires every parameter to be an fp32 contiguous view of one flat buffer
(the trainer's FlatParams) and indices < 2^24 (exact in fp32); otherwise callers use the pack functions.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from ._ext import ops
from .packing import pack_attn_wide, pack_lstm_wide

_LSTM = ("Kf", "bf", "Kb", "bb")
_ATTN = ("W1", "b1", "w2")
_BF16 = ("wxc", "wxcT", "wxtc", "apk", "a2pk", "w1t", "w1")     # output order, bf16 region
_F32 = ("bx", "b1", "w2")                               # fp32 region
_PLANS: Dict[tuple, tuple] = {}


def _flat_of(ts) -> Optional[Tuple[torch.Tensor, Tuple[int, ...]]]:
    base = ts[0]
    st = base.untyped_storage()
    for t in ts:
        if (t.dtype != torch.float32 or not t.is_contiguous() or t.untyped_storage().data_ptr() != st.data_ptr()):
            return None
    n = st.nbytes() // 4
    if n >= (1 << 24):
        return None
    flat = torch.as_strided(base.detach(), (n,), (1,), 0)
    return flat, tuple(int(t.storage_offset()) for t in ts)


def _packs(vals, U: int, D: int, scaled: bool):
    lw = pack_lstm_wide(*vals[:4], U, D, scaled=scaled, cast=False)
    aw = pack_attn_wide(*vals[4:], cast=False)
    out = {k: lw[k] for k in ("wxc", "wxcT", "wxtc", "apk", "a2pk", "bx")}
    out.update({k: aw[k] for k in ("w1t", "w1", "b1", "w2")})
    return out


def _build(ts, offs, U: int, D: int, dev):
    sym = [(torch.arange(t.numel(), dtype=torch.float32, device=dev) + (o + 1)).view(t.shape) for t, o in zip(ts, offs)]
    zero = [torch.zeros_like(t, dtype=torch.float32) for t in ts]
    one = [torch.ones_like(t, dtype=torch.float32) for t in ts]
    pi, p0, p1 = _packs(sym, U, D, False), _packs(zero, U, D, True), _packs(one, U, D, True)
    layout, idx, mul, add = [], [], [], []
    nb = 0
    for region in (_BF16, _F32):
        for k in region:
            v = pi[k].reshape(-1)
            idx.append(torch.round(v).to(torch.int64) - 1)
            add.append(p0[k].reshape(-1).float())
            mul.append((p1[k] - p0[k]).reshape(-1).float())
            layout.append((k, tuple(pi[k].shape), v.numel()))
        if region is _BF16:
            nb = sum(x.numel() for x in idx)
    idx = torch.cat(idx)
    imax = int(idx.max()) if idx.numel() else 0
    return (idx.to(torch.int32).contiguous(), torch.stack([torch.cat(mul), torch.cat(add)]).contiguous(), layout,
            nb, imax)


def wide_packs(Kf, bf, Kb, bb, W1, b1, w2, U: int, D: int) -> Optional[Dict[str, torch.Tensor]]:
    """All wide-path packs from one ``ina.gather_pack_affine`` launch, or None when the parameters are not
    views of one flat fp32 buffer (then the caller runs the pack functions)."""
    ts = (Kf, bf, Kb, bb, W1, b1, w2)
    fo = _flat_of(ts)
    if fo is None:
        return None
    flat, offs = fo
    dev = flat.device
    key = (U, D, tuple(tuple(t.shape) for t in ts), offs, flat.untyped_storage().data_ptr(), flat.numel(), str(dev))
    plan = _PLANS.get(key)
    if plan is None:
        with torch.no_grad():
            plan = _build(ts, offs, U, D, dev)
        if len(_PLANS) > 8:
            _PLANS.pop(next(iter(_PLANS)))
        _PLANS[key] = plan
    idx, ma, layout, nb, imax = plan
    outb = torch.empty(nb, dtype=torch.bfloat16, device=dev)
    outf = torch.empty(idx.numel() - nb, dtype=torch.float32, device=dev)
    ops().gather_pack_affine(flat, idx, nb, outb, outf, ma, imax)
    res, ob, of = {}, 0, 0
    for k, shape, n in layout:
        if k in _BF16:
            res[k] = outb[ob:ob + n].view(shape)
            ob += n
        else:
            res[k] = outf[of:of + n].view(shape)
            of += n
    G4 = res["wxtc"].shape[1] // 2
    res["wxt"] = res["wxtc"].view(D, 2, G4).transpose(0, 1)
    return res


def plan_check(ts, U: int, D: int) -> float:
    """Max |difference| between the gathered packs and the pack functions (tests)."""
    got = wide_packs(*ts, U, D)
    assert got is not None
    ref_l = pack_lstm_wide(*ts[:4], U, D)
    ref_a = pack_attn_wide(*ts[4:])
    ref = dict(ref_l, **{k: ref_a[k] for k in ("w1t", "w1", "b1", "w2")})
    err = 0.0
    for k in _BF16 + _F32:
        a, b = got[k].float(), ref[k].float()
        assert a.shape == b.shape, (k, a.shape, b.shape)
        err = max(err, float((a - b).abs().max()) if a.numel() else 0.0)
    return err


__all__ = ["wide_packs", "plan_check"]
