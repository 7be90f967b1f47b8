#!/usr/bin/env python3
"""Forward / dgrad GEMM layouts at the BERT-base bench shapes (T = 102400 tokens): hipBLASLt's choice
for y = x W^T with W [out, in] (as stored) vs a pre-transposed [in, out] copy, and dx = dy W."""
import json
import sys

import torch


def timeit(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0   # us


def main():
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 102400
    dev = torch.device("cuda")
    for (o, i) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        x = torch.randn(T, i, device=dev).bfloat16()
        W = torch.randn(o, i, device=dev).bfloat16()
        Wt = W.t().contiguous()
        b = torch.randn(o, device=dev).bfloat16()
        dy = torch.randn(T, o, device=dev).bfloat16()
        fl = 2.0 * T * o * i
        r = {"out": o, "in": i}
        r["fwd_WT_us"] = timeit(lambda: torch.mm(x, W.t()))
        r["fwd_Wt_us"] = timeit(lambda: torch.mm(x, Wt))
        r["fwd_addmm_WT_us"] = timeit(lambda: torch.addmm(b, x, W.t()))
        r["fwd_addmm_Wt_us"] = timeit(lambda: torch.addmm(b, x, Wt))
        r["dgrad_W_us"] = timeit(lambda: torch.mm(dy, W))
        r["dgrad_WtT_us"] = timeit(lambda: torch.mm(dy, Wt.t()))
        for k in list(r):
            if k.endswith("_us"):
                r[k.replace("_us", "_tf")] = round(fl / r[k] / 1e6, 1)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
