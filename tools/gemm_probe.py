"""Time the wide path's big GEMM shapes under layout variants (hipBLASLt picks differ by shape/stride).
usage (GPU box): python tools/gemm_probe.py"""
import torch

T = 32000 * 37
dev = "cuda"


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


bf = torch.bfloat16
for K in (310, 312, 320):
    X = torch.randn(T, K, device=dev, dtype=bf)
    W = torch.randn(K, 1024, device=dev, dtype=bf)
    Wt = W.t().contiguous()
    bench(f"gx mm X[T,{K}] W[{K},1024]", lambda: torch.mm(X, W))
    bench(f"gx mm X[T,{K}] Wt.t()", lambda: torch.mm(X, Wt.t()))
    bench(f"gx (W^T X^T)^T: mm(Wt, X.t())", lambda: torch.mm(Wt, X.t()))
    G = torch.randn(T, 1024, device=dev, dtype=bf)
    bench(f"dwx mm(X.t(), G) fp32 K={K}", lambda: torch.mm(X.t(), G, out_dtype=torch.float32))
    for sp in (8, 16, 32, 64):
        bench(f"dwx split{sp} bmm K={K}", lambda: torch.bmm(X.view(sp, T // sp, K).transpose(1, 2), G.view(sp, T // sp, 1024),
                                                            out_dtype=torch.float32).sum(0))
    del X, W, Wt, G
Hp = torch.randn(2, T, 128, device=dev, dtype=bf)
G = torch.randn(T, 1024, device=dev, dtype=bf)
for sp in (16, 64):
    bench(f"dwh strided split{sp}", lambda: torch.bmm(Hp[0].view(sp, T // sp, 128).transpose(1, 2),
                                                      G[:, :512].view(sp, T // sp, 512), out_dtype=torch.float32).sum(0))
bench("dwh both dirs as one [T, 256]^T [T, 1024] (wasteful 2x)", lambda: torch.mm(Hp.permute(1, 0, 2).reshape(T, 256).t(), G, out_dtype=torch.float32))
Wp = torch.randn(1024, 10, device=dev, dtype=bf)
bench("dX pos mm(G, W[1024,10])", lambda: torch.mm(G, Wp, out_dtype=torch.float32))
Wp16 = torch.randn(1024, 16, device=dev, dtype=bf)
bench("dX pos mm(G, W[1024,16])", lambda: torch.mm(G, Wp16, out_dtype=torch.float32))
bench("dX pos mm(G, W16) bf16 out", lambda: torch.mm(G, Wp16))
# round 5: the attention weight gradient dW1 = H^T dZ (H = 2u = 256) and split counts that fill 256 CUs
Hb = torch.randn(T, 256, device=dev, dtype=bf)
dZ = torch.randn(T, 256, device=dev, dtype=bf)
for sp in (16, 32, 50, 64, 100, 128):
    bench(f"dW1 split{sp} bmm [256x256]", lambda: torch.bmm(Hb.view(sp, T // sp, 256).transpose(1, 2),
                                                             dZ.view(sp, T // sp, 256), out_dtype=torch.float32).sum(0))
X = torch.randn(T, 320, device=dev, dtype=bf)
for sp in (16, 20, 25, 32, 40):
    bench(f"dwx split{sp} bmm K=320", lambda: torch.bmm(X.view(sp, T // sp, 320).transpose(1, 2), G.view(sp, T // sp, 1024),
                                                        out_dtype=torch.float32).sum(0))
for sp in (32, 50, 100, 128):
    bench(f"dwh strided split{sp}", lambda: torch.bmm(Hp[0].view(sp, T // sp, 128).transpose(1, 2),
                                                      G[:, :512].view(sp, T // sp, 512), out_dtype=torch.float32).sum(0))
# round 5: dW_x and both directions' dW_h as ONE split-K GEMM over [x | h_prev fw | h_prev bw] rows (reads dG once;
# 12% extra FLOPs for the two cross-direction blocks) vs the current three GEMMs
XA = torch.randn(T, 576, device=dev, dtype=bf)
for sp in (16, 32, 64):
    bench(f"merged [T,576]^T [T,1024] split{sp}", lambda: torch.bmm(XA.view(sp, T // sp, 576).transpose(1, 2),
                                                                   G.view(sp, T // sp, 1024), out_dtype=torch.float32).sum(0))
bench("current dwx split16 + 2 x dwh split64", lambda: (
    torch.bmm(X.view(16, T // 16, 320).transpose(1, 2), G.view(16, T // 16, 1024), out_dtype=torch.float32).sum(0),
    torch.bmm(Hp[0].view(64, T // 64, 128).transpose(1, 2), G[:, :512].view(64, T // 64, 512), out_dtype=torch.float32).sum(0),
    torch.bmm(Hp[1].view(64, T // 64, 128).transpose(1, 2), G[:, 512:].view(64, T // 64, 512), out_dtype=torch.float32).sum(0)))
