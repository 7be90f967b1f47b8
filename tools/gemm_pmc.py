#!/usr/bin/env python3
"""Short driver for rocprofv3 counter passes over the own GEMM and hipBLASLt at one BERT FFN shape.
usage: rocprofv3 --pmc ... -- python3 tools/gemm_pmc.py [N K epi]"""
import sys

import torch


def main():
    sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
    from induction_network_on_fewrel_amd.ops._ext import ops
    o = ops()
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 3072
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 768
    epi = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    T = 102400
    dev = torch.device("cuda")
    x = torch.randn(T, K, device=dev).bfloat16()
    w = (torch.randn(N, K, device=dev) / K ** 0.5).bfloat16()
    b = torch.randn(N, device=dev)
    aux = torch.randn(T, N, device=dev).bfloat16()
    for _ in range(5):
        o.bert_gemm(x, w, b if epi == 1 else None, aux if epi == 2 else None, epi)
        torch.mm(x, w.t())
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
