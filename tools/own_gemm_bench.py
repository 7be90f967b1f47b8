#!/usr/bin/env python3
"""Own gfx950 GEMM (ina.bert_gemm, csrc/kernels/gemm.hip) vs hipBLASLt (torch.mm / addmm) + the separate
bias+GELU passes at the BERT-base FFN shapes, T = 102,400 tokens (10-way 5-shot Q=5, 8 episodes, L=128).

Prints one JSON line per case: us per call and TFLOP/s (2 M N K / t, random operands).
usage: own_gemm_bench.py [T] [N,K ...]   (other shapes, e.g. the paper configuration's x-projection:
       own_gemm_bench.py 1184000 1024,320)"""
import json
import sys

import torch


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0


def main():
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from induction_network_on_fewrel_amd.ops._ext import ops
    o = ops()
    T = int(sys.argv[1]) if len(sys.argv) > 1 else 102400
    dev = torch.device("cuda")
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[2:]] or [(3072, 768), (768, 3072), (2304, 768), (768, 768)]
    for (N, K) in shapes:
        x = torch.randn(T, K, device=dev).bfloat16()
        w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
        b = torch.randn(N, device=dev)
        fl = 2.0 * T * N * K
        r = {"M": T, "N": N, "K": K}
        r["blaslt_mm_us"] = timeit(lambda: torch.mm(x, w.t()))
        bh = b.bfloat16()
        r["blaslt_addmm_us"] = timeit(lambda: torch.addmm(bh, x, w.t()))
        r["own_plain_us"] = timeit(lambda: o.bert_gemm(x, w, None, None, 0))
        r["own_bias_us"] = timeit(lambda: o.bert_gemm(x, w, b, None, 0))
        if N % 256 == 0 and N >= 3072:
            h = torch.mm(x, w.t())
            r["blaslt_mm+bias_gelu_fwd_us"] = timeit(lambda: o.bert_bias_gelu_fwd(torch.mm(x, w.t()), b))
            r["own_gelu_us"] = timeit(lambda: o.bert_gemm(x, w, b, None, 1))
            aux = h
            r["blaslt_mm+bias_gelu_bwd_us"] = timeit(lambda: o.bert_bias_gelu_bwd(torch.mm(x, w.t()), aux, b, 0))
            r["own_dgelu_us"] = timeit(lambda: o.bert_gemm(x, w, None, aux, 2))
        for k in list(r):
            if k.endswith("_us") and ("plain" in k or k == "blaslt_mm_us"):
                r[k.replace("_us", "_tflops")] = round(fl / (r[k] * 1e-6) / 1e12, 1)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
        del x, w


if __name__ == "__main__":
    main()
