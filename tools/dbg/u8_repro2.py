"""Debug: lstm_fwd (natural) vs lstm_attn_fwd h slots, many rounds, u=8 / u=20 (no u=32)."""
import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_kernels_gpu import _problem
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.ops.packing import lstm_shape, pack_attn, pack_lstm

bad = {}
for u in (8, 20, 32):
    cfg, data, model, dd, inst, _ = _problem(dtype="bf16", u=u)
    p = model.pdict()
    DIN = model.params.input_dim
    apack, _ = pack_lstm(p["lstm_fw_kernel"], p["lstm_bw_kernel"], u, DIN, True)
    bias = torch.stack([p["lstm_fw_bias"], p["lstm_bw_bias"]]).detach().float().contiguous()
    word, pos1, pos2, mask = dd.arrays()
    args = (inst, word, pos1, pos2, p["word_embedding"].detach(), p["pos1_embedding"].detach(),
            p["pos2_embedding"].detach(), apack, bias, u, lstm_shape(u, DIN, True)["NX"])
    w1p, _ = pack_attn(p["attn_kernel"], True)
    b1 = p["attn_bias"].detach().contiguous()
    w2 = p["attn_w2"].detach().reshape(-1).contiguous()
    ref = None
    for rnd in range(12):
        for kp, store in ((1.0, False), (1.0, True), (0.9, True), (0.9, False)):
            hl0, _, hn0, dm0, _ = ops().lstm_fwd(*args, True, store, 77, kp, None, None)
            e0, a0 = ops().attn_fwd(hn0, inst, mask, w1p, b1, w2, u, True, 0)
            hl1, _, hn1, dm1, _, e1, a1 = ops().lstm_attn_fwd(*args, store, 77, kp, None, None, mask, w1p, b1, w2)
            torch.cuda.synchronize()
            h0, h1 = hl0[:, :, :, 0], hl1[:, :, :, 0]
            if ref is None:
                ref = h0.clone()
            k = (u, kp, store)
            nb = int((h0 != ref).sum()) + int((h1 != ref).sum())
            bad[k] = bad.get(k, 0) + (nb > 0)
print({str(k): v for k, v in bad.items()})
