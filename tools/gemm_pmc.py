#!/usr/bin/env python3
"""Short driver for rocprofv3 counter passes over the own GEMM family (csrc/kernels/gemm.hip: NT, NN, TN) and
hipBLASLt at one BERT-base shape (T = 102,400 tokens, out x in = N x K).
usage: rocprofv3 --pmc ... -- python3 tools/gemm_pmc.py [N K]"""
import os
import sys

import torch


def main():
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from induction_network_on_fewrel_amd.ops._ext import ops
    o = ops()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 768
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 3072
    T = 102400
    dev = torch.device("cuda")
    x = torch.randn(T, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    dy = torch.randn(T, N, device=dev).bfloat16()
    for _ in range(5):
        o.bert_gemm(x, w, None, None, 0)      # NT  gemm_bf16_kernel<0, 0>
        o.gemm_nn(dy, w, None, None, 0)       # NN  gemm_bf16_kernel<1, 0>
        o.gemm_wgrad(dy, x, 0)                # TN  gemm_bf16_kernel<2, 5>
        torch.mm(x, w.t())                    # hipBLASLt NT
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
