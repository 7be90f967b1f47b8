"""The paper configuration head's dM = C^T dP GEMM (ops/wide.py _wide_head_backward): split-K vs one GEMM.
usage (GPU box): python tools/dm_wide_probe.py"""
import torch
def bench(name, fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    print(f"{s.elapsed_time(e) / it * 1000:9.1f} us  {name}", flush=True)
R, H, hH = 1280, 256, 25600
c = torch.randn(R, H, device="cuda").bfloat16()
d = torch.randn(R, hH, device="cuda").bfloat16()
bench("mm fp32 out (no split)", lambda: torch.mm(c.t(), d, out_dtype=torch.float32))
for ns in (2, 4):
    bench(f"split {ns} + sum", lambda: torch.bmm(c.view(ns, R // ns, H).transpose(1, 2), d.view(ns, R // ns, hH), out_dtype=torch.float32).sum(0))
bench("mm bf16 out", lambda: torch.mm(c.t(), d))
Mt = torch.randn(H, hH, device="cuda")
bench("permute-back copy (dM view permute contiguous)", lambda: Mt.view(H, 100, H).permute(0, 2, 1).contiguous())
# dcls = dP M'^T: [E*N, h*H] x [h*H, H] with K = h*H = 25,600 and a [1280, 256] output (few tiles for one GEMM)
P = torch.randn(R, hH, device="cuda").bfloat16()
Mtb = torch.randn(H, hH, device="cuda").bfloat16()
bench("dcls mm fp32 out", lambda: torch.mm(P, Mtb.t(), out_dtype=torch.float32))
for ns in (4, 8, 16, 32):
    c_ = hH // ns
    bench(f"dcls split-K {ns} (strided bmm) + sum", lambda: torch.bmm(P.view(R, ns, c_).transpose(0, 1),
                                                                   Mtb.view(H, ns, c_).permute(1, 2, 0),
                                                                   out_dtype=torch.float32).sum(0))
# dWs = S^T dE_hat (fp32, [6400, 256]^T [6400, 256]): one fp32 GEMM vs split-K fp32
S_ = torch.randn(6400, H, device="cuda")
D_ = torch.randn(6400, H, device="cuda")
bench("dWs mm fp32", lambda: torch.mm(S_.t(), D_))
for ns in (4, 8, 16):
    bench(f"dWs split-K {ns} fp32 + sum", lambda: torch.bmm(S_.view(ns, 6400 // ns, H).transpose(1, 2), D_.view(ns, 6400 // ns, H)).sum(0))
Mf = torch.randn(H, H, 100, device="cuda")
bench("Mt = M.permute(0,2,1).reshape.to(bf16)", lambda: Mf.permute(0, 2, 1).reshape(H, 100 * H).to(torch.bfloat16))
bench("Mt via transpose(1,2).contiguous then cast", lambda: Mf.transpose(1, 2).contiguous().to(torch.bfloat16))
