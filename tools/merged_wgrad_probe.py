"""Split-K count of the paper configuration's merged weight-gradient GEMM ([x | h_fw | h_bw]^T dG, ops/wide.py).
usage (GPU box): python tools/merged_wgrad_probe.py"""
import torch
T = 32000 * 37
dev = "cuda"
bf = torch.bfloat16
def bench(name, fn, it=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    print(f"{s.elapsed_time(e) / it * 1000:9.1f} us  {name}", flush=True)
XA = torch.randn(T, 576, device=dev, dtype=bf)
G = torch.randn(T, 1024, device=dev, dtype=bf)
for sp in (64, 100, 128, 160, 200, 250):
    if T % sp: continue
    bench(f"merged split{sp} (gemm + sum)", lambda: torch.bmm(XA.view(sp, T // sp, 576).transpose(1, 2), G.view(sp, T // sp, 1024), out_dtype=torch.float32).sum(0))
