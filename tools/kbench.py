#!/usr/bin/env python3
"""Per-kernel timing of the encoder ops at the bench shape (hip events, median of reps).

Used to A/B kernel variants: build one with ``INA_BUILD_TAG=v1 INA_VARIANT_FLAGS=-DSOME_KNOB=0
python csrc/build.py`` and run ``INA_KERNEL_LIB=variants/_ina_kernels_v1.so python tools/kbench.py``.
Prints one JSON line {op: ms}.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--episodes", type=int, default=2048)
    ap.add_argument("--way", type=int, default=5)
    ap.add_argument("--shot", type=int, default=5)
    ap.add_argument("--query", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=20)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--tag", default=os.environ.get("INA_KERNEL_LIB", "default"))
    args = ap.parse_args()
    import torch
    from induction_network_on_fewrel_amd.ops._ext import ops
    from induction_network_on_fewrel_amd.ops.packing import lstm_shape, pack_attn, pack_lstm
    o = ops()
    dev = torch.device("cuda")
    g = torch.Generator(device="cpu").manual_seed(0)
    L, U, E, PD, V, NI = 37, args.hidden, 5, 5, 400000, 64 * 700
    S = args.episodes * args.way * (args.shot + args.query)
    word = torch.randint(0, V, (NI, L), generator=g, dtype=torch.int32).to(dev)
    pos1 = torch.randint(3, 2 * L, (NI, L), generator=g, dtype=torch.int32).to(dev)
    pos2 = torch.randint(3, 2 * L, (NI, L), generator=g, dtype=torch.int32).to(dev)
    mask = (torch.rand(NI, L, generator=g) > 0.3).int().to(dev)
    inst = torch.randint(0, NI, (S,), generator=g, dtype=torch.int32).to(dev)
    wemb = torch.nn.functional.normalize(torch.randn(V, E, generator=g), dim=1).to(dev)
    p1 = (torch.randn(2 * L, PD, generator=g) * 0.1).to(dev)
    p2 = (torch.randn(2 * L, PD, generator=g) * 0.1).to(dev)
    DIN = E + 2 * PD
    Kf = (torch.randn(DIN + U, 4 * U, generator=g) * 0.2).to(dev)
    Kb = (torch.randn(DIN + U, 4 * U, generator=g) * 0.2).to(dev)
    bias = torch.zeros(2, 4 * U, device=dev)
    W1 = (torch.randn(2 * U, 2 * U, generator=g) * 0.2).to(dev)
    b1 = torch.zeros(2 * U, device=dev)
    w2 = (torch.randn(2 * U, generator=g) * 0.2).to(dev)
    sh = lstm_shape(U, DIN, True)
    from induction_network_on_fewrel_amd.ops.encoder import word_rows
    wrows = None if os.environ.get("KB_NO_WROWS") else word_rows(word, wemb, True)
    apack, a2pack = pack_lstm(Kf, Kb, U, DIN, True)
    w1pack, w1tpack = pack_attn(W1, True)
    de = (torch.randn(S, 2 * U, generator=g) * 1e-3).to(dev)

    def timed(fn):
        for _ in range(3):
            out = fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = fn()
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        return ts[len(ts) // 2], out

    res = {"tag": args.tag, "S": S}
    t, (hlane, cst, hnat, dmask, xg) = timed(lambda: o.lstm_fwd(inst, word, pos1, pos2, wemb, p1, p2, apack, bias, U, sh["NX"],
                                                       True, True, 7, 0.9, None, wrows))
    res["lstm_fwd"] = t
    t, _ = timed(lambda: o.lstm_fwd(inst, word, pos1, pos2, wemb, p1, p2, apack, bias, U, sh["NX"], True, False, 7,
                                    1.0, None, wrows))
    res["lstm_fwd_infer"] = t
    t, (e, alphas) = timed(lambda: o.attn_fwd(hnat, inst, mask, w1pack, b1, w2, U, True, 0))
    res["attn_fwd"] = t
    t, (dH, aslab) = timed(lambda: o.attn_bwd(hnat, inst, w1pack, w1tpack, b1, w2, de, alphas, U, True, 0))
    res["attn_bwd"] = t
    t, _ = timed(lambda: o.lstm_bwd(inst, word, pos1, pos2, wemb, p1, p2, apack, a2pack, bias, hlane, cst, dH, dmask, xg, U,
                                    sh["NX"], True, False, 0, 7, 0.9, False, None, None, None))
    res["lstm_bwd"] = t
    if hasattr(o, "lstm_attn_fwd"):
        t, _ = timed(lambda: o.lstm_attn_fwd(inst, word, pos1, pos2, wemb, p1, p2, apack, bias, U, sh["NX"], True, 7,
                                             0.9, None, wrows, mask, w1pack, b1, w2, None, None, None, False))
        res["lstm_attn_fwd"] = t
        t, _ = timed(lambda: o.lstm_attn_fwd(inst, word, pos1, pos2, wemb, p1, p2, apack, bias, U, sh["NX"], False, 7,
                                             1.0, None, wrows, mask, w1pack, b1, w2, None, None, None, False))
        res["lstm_attn_fwd_infer"] = t
    res["encoder_total"] = res["lstm_fwd"] + res["attn_fwd"] + res["attn_bwd"] + res["lstm_bwd"]
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
