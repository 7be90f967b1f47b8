"""Fused step plumbing for the GPU BiLSTM training step (kernels: csrc/kernels/glue.hip).

Without it one optimiser step of the default model is ~100 kernel launches, ~80 of them tiny
PyTorch ops (weight re-packing gathers / casts / cats, the MSE loss and its backward, accuracy,
slab ``sum(0)`` reductions, transposes, adds into the flat gradient) at ~5 us of GPU time each --
about 15% of the step.  ``StepGlue`` replaces them with:

* ``packs()``: ONE ``ina.gather_pack`` launch producing every MFMA weight pack of the step (LSTM
  gate / transpose packs, attention W1 packs, NTN M / w packs, stacked LSTM biases) straight from
  the flat parameter buffer through a cached int32 index (parameters are views of that buffer).
* ``head_loss``: one ``ina.head_loss`` launch for loss + accuracy + the NTN's pre-sigmoid gradient
  (see ``ops/head.py::HeadLossFn``).
* ``add()`` / ``flush()``: backward functions queue their per-block gradient slabs with an int32
  map into the flat gradient (transposes, bias columns and pos-table crops live in the map);
  ``flush()`` reduces and scatter-adds all of them with ONE deterministic ``ina.slab_scatter_add``
  (two kernels: chunked partial sums, then ordered finish + scatter).

Reference behaviour is unchanged (same gradients as the per-op path, tested in
tests/test_kernels_gpu.py::test_step_glue_matches_unfused).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ._ext import ops
from .packing import _attn_idx, _attn_rec_idx, _lstm_idx, _ntn_dw_idx, _ntn_tile_idx, lstm_shape


class StepGlue:
    LOSS_BLOCKS = 64     # workgroups of the loss kernel

    def __init__(self, flat):
        self.flat = flat
        dev = flat.flat.device
        self.device = dev
        self.one = torch.ones((), dtype=torch.float32, device=dev)     # loss.backward(one): no fill launch
        self._idx: Dict[tuple, Tuple[torch.Tensor, list, int, int]] = {}
        self._maps: Dict[tuple, torch.Tensor] = {}
        self._jobs: List[tuple] = []
        self._ws = torch.empty(0, dtype=torch.float32, device=dev)
        self.loss_part = torch.empty(self.LOSS_BLOCKS * 18, dtype=torch.float32, device=dev)

    # ------------------------------------------------------------------ offsets
    def off(self, t: torch.Tensor) -> int:
        """Element offset of a parameter inside the flat buffer (== offset of its gradient)."""
        base = self.flat.flat
        d = t.data_ptr() - base.data_ptr()
        if t.dtype != torch.float32 or not t.is_contiguous() or d < 0 or d % 4 or d // 4 + t.numel() > base.numel():
            raise ValueError("StepGlue: parameter is not a contiguous view of the flat parameter buffer")
        return d // 4

    def _dev_i32(self, a: np.ndarray) -> torch.Tensor:
        return torch.from_numpy(np.ascontiguousarray(a, dtype=np.int32)).to(self.device)

    # ------------------------------------------------------------------ packs
    def packs(self, p: Dict[str, torch.Tensor], U: int, DIN: int, bf16: bool, head: Optional[tuple]):
        """All per-step weight packs in one launch.  head = (H, h, N, paper) or None.
        Returns dict(apack, a2pack, bias2, w1pack, w1tpack[, ntn_tiles])."""
        names = ["lstm_fw_kernel", "lstm_bw_kernel", "lstm_fw_bias", "lstm_bw_bias", "attn_kernel"]
        if head is not None:
            names += ["M", "ntn_w"]
        offs = tuple(self.off(p[n]) for n in names)
        key = (U, DIN, bf16, head, offs)
        ent = self._idx.get(key)
        if ent is None:
            ent = self._build_pack_index(U, DIN, bf16, head, dict(zip(names, offs)))
            self._idx[key] = ent
        idx, layout, nb, nf = ent
        outb = torch.empty(nb, dtype=torch.bfloat16, device=self.device)
        outf = torch.empty(nf, dtype=torch.float32, device=self.device)
        ops().gather_pack(self.flat.flat, idx, nb, outb, outf)
        res = {}
        for name, region, start, shape in layout:
            buf = outb if region == "b" else outf
            n = int(np.prod(shape))
            res[name] = buf[start:start + n].view(shape)
        return res

    def _build_pack_index(self, U, DIN, bf16, head, off):
        parts_b, parts_f, layout = [], [], []
        nb = nf = 0

        def put(name, flat_idx: np.ndarray, dtype_bf16: bool):
            nonlocal nb, nf
            if dtype_bf16:
                layout.append((name, "b", nb, flat_idx.shape))
                parts_b.append(flat_idx.reshape(-1))
                nb += flat_idx.size
            else:
                layout.append((name, "f", nf, flat_idx.shape))
                parts_f.append(flat_idx.reshape(-1))
                nf += flat_idx.size

        # LSTM packs: indices into W_ext = pad(W [DIN+U, 4U]) -> [DIN+U+1, 4U+1]
        fi, bi = (t.numpy() for t in _lstm_idx(U, DIN, bf16))
        W = 4 * U + 1

        def lstm_map(ext, base):
            f, g = ext // W, ext % W
            return np.where((f < DIN + U) & (g < 4 * U), base + f * 4 * U + g, -1)

        put("apack", np.stack([lstm_map(fi, off["lstm_fw_kernel"]), lstm_map(fi, off["lstm_bw_kernel"])]), bf16)
        put("a2pack", np.stack([lstm_map(bi, off["lstm_fw_kernel"]), lstm_map(bi, off["lstm_bw_kernel"])]), bf16)
        put("bias2", np.stack([off["lstm_fw_bias"] + np.arange(4 * U), off["lstm_bw_bias"] + np.arange(4 * U)]), False)
        H2 = 2 * U
        pi, ti = (t.numpy() for t in _attn_idx(H2, bf16))
        Z = H2 * H2
        put("w1pack", np.where(pi < Z, off["attn_kernel"] + pi, -1), bf16)
        put("w1tpack", np.where(ti < Z, off["attn_kernel"] + ti, -1), bf16)
        if bf16 and U in (8, 20, 32):   # record-layout attention kernels (ops/packing.py::_attn_rec_idx)
            ri, rti = (t.numpy() for t in _attn_rec_idx(U))
            put("w1rpack", np.where(ri < Z, off["attn_kernel"] + ri, -1), True)
            put("w1rtpack", np.where(rti < Z, off["attn_kernel"] + rti, -1), True)
        if head is not None:
            H, h, N, paper = head
            mi, wi = (t.numpy() for t in _ntn_tile_idx(H, h, N, bool(paper)))
            put("ntn_tiles", np.where(mi >= 0, off["M"] + mi, np.where(wi >= 0, off["ntn_w"] + wi, -1)), True)
        allidx = np.concatenate(parts_b + parts_f) if (parts_b or parts_f) else np.zeros(0)
        return self._dev_i32(allidx), layout, nb, nf

    # ------------------------------------------------------------------ slab maps
    def map_identity(self, t: torch.Tensor) -> torch.Tensor:
        key = ("id", self.off(t), t.numel())
        m = self._maps.get(key)
        if m is None:
            m = self._dev_i32(self.off(t) + np.arange(t.numel()))
            self._maps[key] = m
        return m

    def map_lstm_dw(self, p, U: int, DIN: int) -> torch.Tensor:
        """lstm_bwd dW slab row [2 dir][4U][NF = DIN+U+1] -> (kernel^T, bias) of each direction."""
        ks = (self.off(p["lstm_fw_kernel"]), self.off(p["lstm_bw_kernel"]))
        bs = (self.off(p["lstm_fw_bias"]), self.off(p["lstm_bw_bias"]))
        key = ("lstm", U, DIN, ks, bs)
        m = self._maps.get(key)
        if m is None:
            NF = DIN + U + 1
            d, g, f = np.meshgrid(np.arange(2), np.arange(4 * U), np.arange(NF), indexing="ij")
            kb = np.array(ks)[d]
            bb = np.array(bs)[d]
            m = np.where(f < DIN + U, kb + f * 4 * U + g, bb + g)
            m = self._dev_i32(m)
            self._maps[key] = m
        return m

    def map_pos(self, p, L: int, PD: int) -> torch.Tensor:
        """pos-gradient slab row [2 tables][2L][PD] -> pos1/pos2 tables (rows beyond a table dropped)."""
        t1, t2 = p["pos1_embedding"], p["pos2_embedding"]
        key = ("pos", L, PD, self.off(t1), self.off(t2), t1.shape[0], t2.shape[0])
        m = self._maps.get(key)
        if m is None:
            tb, r, c = np.meshgrid(np.arange(2), np.arange(2 * L), np.arange(PD), indexing="ij")
            base = np.where(tb == 0, self.off(t1), self.off(t2))
            rows = np.where(tb == 0, t1.shape[0], t2.shape[0])
            m = self._dev_i32(np.where(r < rows, base + r * PD + c, -1))
            self._maps[key] = m
        return m

    def map_attn(self, p, H2: int) -> torch.Tensor:
        """attention slab row [dW1 (H2*H2) | db1 (H2) | dw2 (H2)]."""
        o = (self.off(p["attn_kernel"]), self.off(p["attn_bias"]), self.off(p["attn_w2"]))
        key = ("attn", H2, o)
        m = self._maps.get(key)
        if m is None:
            m = self._dev_i32(np.concatenate([o[0] + np.arange(H2 * H2), o[1] + np.arange(H2), o[2] + np.arange(H2)]))
            self._maps[key] = m
        return m

    def map_index(self, t: torch.Tensor, idx: np.ndarray, tag) -> torch.Tensor:
        """Slab column j -> element idx[j] of parameter t (-1: dropped), cached under (tag, offset of t)."""
        key = ("ix", tag, self.off(t), t.numel())
        m = self._maps.get(key)
        if m is None:
            idx = np.asarray(idx, dtype=np.int64)
            if idx.size and (idx.max() >= t.numel()):
                raise ValueError("StepGlue.map_index: index past the parameter")
            m = self._dev_i32(np.where(idx >= 0, self.off(t) + idx, -1))
            self._maps[key] = m
        return m

    def map_merged_lstm(self, p, U: int, D: int, DP: int, G4: int) -> torch.Tensor:
        """The wide BiLSTM's merged weight-gradient GEMM output dwall [DP + 2 UP, 2 G4] (ops/packing.py::
        _merged_wgrad_idx) -> both directions' kernel [D + U, 4U] and bias [4U]; the dropped cross-direction
        blocks and padding map to -1."""
        from .packing import _merged_wgrad_idx
        ks = (self.off(p["lstm_fw_kernel"]), self.off(p["lstm_bw_kernel"]))
        bs = (self.off(p["lstm_fw_bias"]), self.off(p["lstm_bw_bias"]))
        key = ("merged", U, D, DP, G4, ks, bs)
        m = self._maps.get(key)
        if m is None:
            src = _merged_wgrad_idx(U, D, DP).numpy().reshape(2, D + U + 1, 4 * U)
            tgt = np.empty_like(src)
            for d in range(2):
                tgt[d, :D + U] = ks[d] + np.arange((D + U) * 4 * U).reshape(D + U, 4 * U)
                tgt[d, D + U] = bs[d] + np.arange(4 * U)
            mm = np.full((DP + 2 * (G4 // 4)) * 2 * G4, -1, dtype=np.int64)
            mm[src.reshape(-1)] = tgt.reshape(-1)
            m = self._dev_i32(mm)
            self._maps[key] = m
        return m

    def map_ntn_M(self, Mt: torch.Tensor) -> torch.Tensor:
        """dM GEMM output [a][s*H + b] -> M [a][b][s]."""
        H, _, h = Mt.shape
        key = ("M", self.off(Mt), H, h)
        m = self._maps.get(key)
        if m is None:
            a, s, b = np.meshgrid(np.arange(H), np.arange(h), np.arange(H), indexing="ij")
            m = self._dev_i32(self.off(Mt) + (a * H + b) * h + s)
            self._maps[key] = m
        return m

    def map_ntn_dw(self, w: torch.Tensor, h: int, N: int, paper: bool) -> torch.Tensor:
        """ntn_bwd dw slab row ([ntile][SG N][N] / [ntile][SG], ops/packing.py::_ntn_dw_idx) -> ntn_w."""
        key = ("ntn_dw", self.off(w), h, N, bool(paper))
        m = self._maps.get(key)
        if m is None:
            di = _ntn_dw_idx(h, N, bool(paper)).numpy()
            m = self._dev_i32(np.where(di >= 0, self.off(w) + di, -1))
            self._maps[key] = m
        return m

    def map_grad(self, gv: torch.Tensor) -> torch.Tensor:
        """Identity map of a gradient view of the flat GRADIENT buffer (the trainer's grad_views)."""
        base = self.flat.grad
        d = gv.data_ptr() - base.data_ptr()
        if gv.dtype != torch.float32 or not gv.is_contiguous() or d < 0 or d % 4:
            raise ValueError("StepGlue.map_grad: not a contiguous view of the flat gradient buffer")
        key = ("g", d // 4, gv.numel())
        m = self._maps.get(key)
        if m is None:
            m = self._dev_i32(d // 4 + np.arange(gv.numel()))
            self._maps[key] = m
        return m

    def map_cat(self, maps) -> torch.Tensor:
        """Concatenation of maps (one slab job over several parameters' columns), cached."""
        key = ("cat",) + tuple(m.data_ptr() for m in maps)
        m = self._maps.get(key)
        if m is None:
            m = torch.cat(list(maps)).contiguous()
            self._maps[key] = m
        return m

    # ------------------------------------------------------------------ slab queue
    def add(self, slab: torch.Tensor, m: torch.Tensor, nblk: int, scale: Optional[torch.Tensor] = None) -> None:
        """Queue sum_b slab[b] (slab viewed as [nblk, m.numel()]) * scale for a scatter-add at map m."""
        s = slab.contiguous().view(nblk, m.numel())
        sc = scale.reshape(-1).float() if scale is not None else self._noscale()
        self._jobs.append((s, m, int(nblk), sc))

    def _noscale(self):
        if not hasattr(self, "_empty"):
            self._empty = torch.empty(0, dtype=torch.float32, device=self.device)
        return self._empty

    def flush(self) -> None:
        """Reduce + scatter-add every queued slab into the flat gradient (one launch per 8 slabs)."""
        jobs, self._jobs = self._jobs, []
        o = ops()
        for k in range(0, len(jobs), 8):
            grp = jobs[k:k + 8]
            args = ([j[0] for j in grp], [j[1] for j in grp], [j[2] for j in grp], [j[3] for j in grp])
            need = o.slab_scatter_add(self.flat.grad, *args, self._ws)
            if need:   # first use of this job shape: size the workspace (kept; graph replays reuse it)
                self._ws = torch.empty(int(need), dtype=torch.float32, device=self.device)
                assert o.slab_scatter_add(self.flat.grad, *args, self._ws) == 0

    def pending(self) -> int:
        return len(self._jobs)


def lstm_din(p) -> int:
    return p["word_embedding"].shape[1] + 2 * p["pos1_embedding"].shape[1]


def encoder_pack_shape(U: int, DIN: int, bf16: bool):
    return lstm_shape(U, DIN, bf16)
