#!/usr/bin/env python3
"""Dump one training step's flat gradient (fixed problem, fixed seeds) for A/B of kernel builds:
INA_KERNEL_LIB=a.so python tools/grad_dump.py out_a.pt; ... out_b.pt; python tools/grad_dump.py --cmp a.pt b.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    if sys.argv[1] == "--cmp":
        a, b = (torch.load(p, weights_only=True) for p in sys.argv[2:4])
        for k in a:
            x, y = a[k].double(), b[k].double()
            print(f"{k:24s} relerr {float((x - y).abs().max() / (y.abs().max() + 1e-30)):.3e}  max {float(y.abs().max()):.3e}")
        return
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    data = make_synthetic(num_relations=12, instances_per_relation=40, vocab=500, seed=0)
    cfg = Config(N=5, K=3, Q=4, episodes_per_step=24, model_dir="/tmp/gd", seed=6, resume=False)
    tr = Trainer(cfg, data, None, device="cuda", log=False)
    tr.opt.step = lambda *a, **k: None   # gradients only
    tr.train_step()
    torch.cuda.synchronize()
    out = {n: tr.flat.view(tr.flat.grad, n).detach().cpu().clone() for n in tr.flat.names}
    torch.save(out, sys.argv[1])


if __name__ == "__main__":
    main()
