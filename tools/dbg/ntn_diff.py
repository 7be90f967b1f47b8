"""Debug: run ntn_bwd twice on fixed inputs, report run-to-run differences, save the outputs for an
element-wise comparison between kernel builds.  usage (GPU): INA_KERNEL_LIB=... python tools/dbg/ntn_diff.py TAG"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from induction_network_on_fewrel_amd.ops import ops  # noqa: E402
from induction_network_on_fewrel_amd.ops.packing import pack_ntn_tiles  # noqa: E402

tag = sys.argv[1]
E, N, K, Q, H, h = int(os.environ.get("E", 4)), 5, 2, 5, 40, 100
g = torch.Generator().manual_seed(0)
cls = (torch.randn(E * N, H, generator=g) * 0.5).cuda()
e = (torch.randn(E * (N * K + N * Q), H, generator=g) * 0.5).cuda()
M = (torch.randn(H, H, h, generator=g) * 0.1).cuda()
w = (torch.randn(h * N, N, generator=g) * 0.1).cuda()
dz = (torch.randn(E * N * Q, N, generator=g) * 0.1).cuda()
tiles = pack_ntn_tiles(M, w, N, False)
o = ops()
outs = []
for r in range(2):
    de = torch.zeros_like(e)
    dcls, dp, dw_slab, cls_bf = o.ntn_bwd(cls, e, tiles, dz, de, E, N, K, Q, h, False, 0, None)
    torch.cuda.synchronize()
    outs.append(dict(dcls=dcls.cpu(), dp=dp.float().cpu(), dw=dw_slab.cpu(), de=de.cpu(), cls_bf=cls_bf.float().cpu()))
for k in outs[0]:
    a, b = outs[0][k], outs[1][k]
    print(tag, k, tuple(a.shape), "run-to-run max diff", float((a - b).abs().max()), flush=True)
os.makedirs("gpurun_out", exist_ok=True)
torch.save(dict(out=outs[0], inp=dict(cls=cls.cpu(), e=e.cpu(), M=M.cpu(), w=w.cpu(), dz=dz.cpu())),
           f"gpurun_out/ntn_{tag}.pt")
