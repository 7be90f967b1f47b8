"""Probe: torch reductions / concatenations of the paper configuration's head + attention backward
(profiles/r5_uw/paper_seq.txt: part.sum(0) 20.8 us, torch.cat(dsup, dQ) 19.4 us) vs alternatives."""
import torch

dev = "cuda"


def t(f, n=50):
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for nb in (512, 1024, 4096):
    part = torch.randn(nb, 2, 256, device=dev)
    ones = torch.ones(1, nb, device=dev)
    r0 = part.sum(0)
    r1 = torch.mm(ones, part.view(nb, -1)).view(2, 256)
    print(f"part [{nb},2,256]: sum(0) {t(lambda: part.sum(0)):.1f} us  mm(ones) {t(lambda: torch.mm(ones, part.view(nb, -1))):.1f} us"
          f"  maxdiff {float((r0 - r1).abs().max()):.2e}")

E, NK, NQ, H, Nh = 256, 25, 100, 256, 5 * 30
dT = torch.randn(E, NQ, Nh, device=dev, dtype=torch.bfloat16)
P = torch.randn(E, Nh, H, device=dev, dtype=torch.bfloat16)
dsup = torch.randn(E * NK, H, device=dev)


def cat_path():
    dQ = torch.bmm(dT, P, out_dtype=torch.float32)
    return torch.cat([dsup.view(E, NK, H), dQ], 1)


de = torch.empty(E, NK + NQ, H, device=dev)


def out_path():
    torch.bmm(dT, P, out_dtype=torch.float32, out=de[:, NK:])
    de[:, :NK].copy_(dsup.view(E, NK, H))
    return de


try:
    ok = torch.equal(cat_path(), out_path())
    print(f"cat path {t(cat_path):.1f} us  bmm(out=strided) path {t(out_path):.1f} us  equal {ok}")
except Exception as ex:  # noqa: BLE001
    print("bmm out= strided failed:", repr(ex)[:200])
