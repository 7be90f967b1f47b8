"""Debug: where does NaN appear in the bf16 u=8 dropout encoder forward?"""
import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_kernels_gpu import _problem, _split_stash
from induction_network_on_fewrel_amd.ops import ops
from induction_network_on_fewrel_amd.ops.packing import lstm_shape, pack_attn, pack_lstm

for u in (8, 20, 32):
    for kp in (1.0, 0.9):
        cfg, data, model, dd, inst, _ = _problem(dtype="bf16", u=u)
        p = model.pdict()
        U = u
        DIN = model.params.input_dim
        apack, _ = pack_lstm(p["lstm_fw_kernel"], p["lstm_bw_kernel"], U, DIN, True)
        bias = torch.stack([p["lstm_fw_bias"], p["lstm_bw_bias"]]).detach().float().contiguous()
        word, pos1, pos2, mask = dd.arrays()
        args = (inst, word, pos1, pos2, p["word_embedding"].detach(), p["pos1_embedding"].detach(),
                p["pos2_embedding"].detach(), apack, bias, U, lstm_shape(U, DIN, True)["NX"])
        w1p, _ = pack_attn(p["attn_kernel"], True)
        b1 = p["attn_bias"].detach().contiguous()
        w2 = p["attn_w2"].detach().reshape(-1).contiguous()
        for store in (True, False):
            hl0, _, hn0, dm0, _ = ops().lstm_fwd(*args, True, store, 77, kp, None, None)
            e0, a0 = ops().attn_fwd(hn0, inst, mask, w1p, b1, w2, U, True, 0)
            hl1, _, hn1, dm1, _, e1, a1 = ops().lstm_attn_fwd(*args, store, 77, kp, None, None, mask, w1p, b1, w2)
            torch.cuda.synchronize()
            h0 = hl0[:, :, :, 0].float()
            nan = lambda t: int(torch.isnan(t.float()).sum())
            print(f"u={u} kp={kp} store={store}: hslot nan {nan(h0)} hnat0 nan {nan(hn0)} e0 nan {nan(e0)} "
                  f"a0 nan {nan(a0)} | hnat1 nan {nan(hn1) if store else -1} e1 nan {nan(e1)} a1 nan {nan(a1)} "
                  f"dm eq {torch.equal(dm0, dm1)} e eq {torch.equal(e0, e1)} hl eq {torch.equal(hl0[:, :, :, 0], hl1[:, :, :, 0])} "
                  f"maxabs h {float(h0.abs().max()):.3f}", flush=True)
