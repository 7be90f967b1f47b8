"""Debug: replicate the first u8_drop sequence for u=8 only, several rounds."""
import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_kernels_gpu import _problem
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.ops.packing import lstm_shape, pack_attn, pack_lstm

for rnd in range(3):
    for kp in (1.0, 0.9):
        u = 8
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
        for store in (True, False):
            hl0, _, hn0, dm0, _ = ops().lstm_fwd(*args, True, store, 77, kp, None, None)
            torch.cuda.synchronize()
            hl0c = hl0[:, :, :, 0].clone()
            e0, a0 = ops().attn_fwd(hn0, inst, mask, w1p, b1, w2, u, True, 0)
            torch.cuda.synchronize()
            ch1 = torch.equal(hl0c, hl0[:, :, :, 0])
            hl1, _, hn1, dm1, _, e1, a1 = ops().lstm_attn_fwd(*args, store, 77, kp, None, None, mask, w1p, b1, w2)
            torch.cuda.synchronize()
            ch2 = torch.equal(hl0c, hl0[:, :, :, 0])
            d = (hl1[:, :, :, 0] != hl0c)
            nz = d.nonzero()
            seqs = sorted(set((int(t) * 16 + int(l) % 16) for t, _, _, _, l in nz.tolist()))
            print(f"rnd{rnd} kp={kp} store={store}: hl0 unchanged {ch1} {ch2}; hl1 vs hl0 diff {int(d.sum())} "
                  f"seqs {seqs[:10]} S={inst.shape[0]} e eq {torch.equal(e0, e1)} nan e0 {int(torch.isnan(e0).sum())} "
                  f"e1 {int(torch.isnan(e1).sum())}", flush=True)
