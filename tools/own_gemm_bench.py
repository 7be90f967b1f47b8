#!/usr/bin/env python3
"""Own gfx950 GEMM family (csrc/kernels/gemm.hip) vs hipBLASLt (torch) at the BERT-base and paper-configuration
shapes, random operands.  One JSON line per case: us per call and TFLOP/s (2 M N K / t).

usage: own_gemm_bench.py [suite ...]       suites: nt nn wgrad paper (default: all)
  nt    : forward linears y = x W^T (+ bias), T = 102,400 tokens (10-way 5-shot Q=5, 8 episodes, L=128)
  nn    : dgrads dx = dy W (+ residual in place) vs torch.mm / res.addmm_
  wgrad : dW = dy^T x, fp32, summed into a flat-gradient span: own split-K slabs + slab_reduce vs the
          hipBLASLt 16-chunk bmm + slab_reduce the BERT path used before
  paper : the paper configuration's merged weight gradient ([x | h_fw | h_bw]^T dG, K = 1.18 M) and attention dW1"""
import json
import os
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


def emit(r, fl):
    for k in list(r):
        if k.endswith("_us"):
            r[k.replace("_us", "_tflops")] = round(fl / (r[k] * 1e-6) / 1e12, 1)
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from induction_network_on_fewrel_amd.ops._ext import ops
    o = ops()
    suites = sys.argv[1:] or ["nt", "nn", "wgrad", "paper"]
    dev = torch.device("cuda")
    T = 102400
    bert = [(3072, 768), (768, 3072), (2304, 768), (768, 768)]   # (out, in)
    if "nt" in suites:
        for (N, K) in bert:
            x = torch.randn(T, K, device=dev).bfloat16()
            w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
            b = torch.randn(N, device=dev)
            bh = b.bfloat16()
            r = {"suite": "nt", "M": T, "N": N, "K": K,
                 "blaslt_addmm_us": timeit(lambda: torch.addmm(bh, x, w.t())),
                 "own_bias_us": timeit(lambda: o.bert_gemm(x, w, b, None, 0))}
            emit(r, 2.0 * T * N * K)
    if "nn" in suites:
        for (o_, i_) in bert:   # dx [T, in] = dy [T, out] W [out, in]
            dy = torch.randn(T, o_, device=dev).bfloat16()
            w = (torch.randn(o_, i_, device=dev) / o_ ** 0.5).bfloat16()
            res = torch.randn(T, i_, device=dev).bfloat16()
            r = {"suite": "nn", "M": T, "N": i_, "K": o_,
                 "blaslt_mm_us": timeit(lambda: torch.mm(dy, w)),
                 "own_us": timeit(lambda: o.gemm_nn(dy, w, None, None, 0)),
                 "blaslt_addmm_res_us": timeit(lambda: res.addmm_(dy, w)),
                 "own_res_us": timeit(lambda: o.gemm_nn(dy, w, None, res, 4))}
            emit(r, 2.0 * T * o_ * i_)
    if "wgrad" in suites:
        for (o_, i_) in bert:   # dW [out, in] = dy^T x
            dy = torch.randn(T, o_, device=dev).bfloat16()
            x = torch.randn(T, i_, device=dev).bfloat16()
            g = torch.zeros(o_ * i_, device=dev)

            def blaslt():
                part = torch.bmm(dy.view(16, T // 16, o_).transpose(1, 2), x.view(16, T // 16, i_),
                                 out_dtype=torch.float32)
                o.slab_reduce(part, g, True)

            def own():
                o.slab_reduce(o.gemm_wgrad(dy, x, 0), g, True)
            r = {"suite": "wgrad", "M": o_, "N": i_, "K": T, "splits": int(o.gemm_wgrad(dy, x, 0).shape[0]),
                 "blaslt_bmm16_reduce_us": timeit(blaslt), "own_reduce_us": timeit(own),
                 "own_gemm_only_us": timeit(lambda: o.gemm_wgrad(dy, x, 0))}
            emit(r, 2.0 * T * o_ * i_)
    if "paper" in suites:
        from induction_network_on_fewrel_amd.ops.wide import _wgrad
        Tp = 256 * 125 * 37
        for (m, n, sp) in [(576, 1024, 64), (256, 256, 128)]:
            a = torch.randn(Tp, m, device=dev).bfloat16()
            b = torch.randn(Tp, n, device=dev).bfloat16()
            r = {"suite": "paper", "M": m, "N": n, "K": Tp,
                 "blaslt_split_sum_us": timeit(lambda: _wgrad(a, b, sp), reps=10),
                 "own_slab_sum_us": timeit(lambda: o.gemm_wgrad(a, b, 0).sum(0), reps=10)}
            emit(r, 2.0 * Tp * m * n)


if __name__ == "__main__":
    main()
