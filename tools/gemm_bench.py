#!/usr/bin/env python3
"""Weight-gradient GEMM variants at the BERT-base bench shapes (T = 102400 tokens): hipBLASLt picks few
output tiles for dW = dy^T x (K = T is the long dimension), so compare fp32-output mm, bf16-output mm
and a K-chunked batched GEMM (split-K by hand) + fp32 reduction."""
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
    out = []
    for (o, i) in ((2304, 768), (768, 768), (3072, 768), (768, 3072)):
        dy = torch.randn(T, o, device=dev).bfloat16()
        x = torch.randn(T, i, device=dev).bfloat16()
        fl = 2.0 * T * o * i
        r = {"out": o, "in": i}
        r["mm_f32out_us"] = timeit(lambda: torch.mm(dy.t(), x, out_dtype=torch.float32))
        r["mm_bf16_us"] = timeit(lambda: torch.mm(dy.t(), x))
        for nc in (4, 8, 16):
            def ch():
                a = dy.view(nc, T // nc, o).transpose(1, 2)
                bb = x.view(nc, T // nc, i)
                try:
                    p = torch.bmm(a, bb, out_dtype=torch.float32)
                except Exception:
                    p = torch.bmm(a, bb).float()
                return p.sum(0)
            r[f"bmm{nc}_us"] = timeit(ch)
        ref = torch.mm(dy.t().float(), x.float())
        r["f32out_err"] = float((torch.mm(dy.t(), x, out_dtype=torch.float32) - ref).abs().max() / ref.abs().max())
        r["bf16_err"] = float((torch.mm(dy.t(), x).float() - ref).abs().max() / ref.abs().max())
        r["tflops_f32out"] = fl / r["mm_f32out_us"] / 1e6
        r["tflops_best_bmm"] = fl / min(r[f"bmm{nc}_us"] for nc in (4, 8, 16)) / 1e6
        out.append(r)
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
