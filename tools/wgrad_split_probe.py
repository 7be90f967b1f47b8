"""Split-K count of the BERT weight-gradient GEMMs (dW = dy^T x, K = tokens): hipBLASLt batched split-K
[nc, o, i] fp32 partials.  usage (GPU box): python tools/wgrad_split_probe.py [T]"""
import sys

import torch


def bench(fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000.0


T = int(sys.argv[1]) if len(sys.argv) > 1 else 102400
for o, i in ((2304, 768), (3072, 768), (768, 3072), (768, 768)):
    dy = torch.randn(T, o, device="cuda").bfloat16()
    x = torch.randn(T, i, device="cuda").bfloat16()
    res = []
    for nc in (4, 8, 16, 32, 64):
        us = bench(lambda: torch.bmm(dy.view(nc, T // nc, o).transpose(1, 2), x.view(nc, T // nc, i),
                                     out_dtype=torch.float32))
        res.append(f"nc={nc}: {us:.1f} us ({2 * T * o * i / us / 1e6:.0f} TF/s)")
    print(f"o={o} i={i}: " + "  ".join(res), flush=True)
