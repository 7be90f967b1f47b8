"""Wide-layer GPU path (ops/wide.py + lstm_wide.hip): the paper configuration (u=128, 50-d words,
H=256 head) and the wide path forced at u=20 against the fused kernels and the fp32 oracle."""
import pytest
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data import EpisodeSampler, make_synthetic
from induction_network_on_fewrel_amd.models import InductionNetwork
from induction_network_on_fewrel_amd.models import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _relerr(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


def _setup(u, E, impl, kp_train=True, N=5, K=2, Q=3, B=3, L=37, shifted=True):
    cfg = Config(N=N, K=K, Q=Q, max_length=L, hidden_size=u, lstm_impl=impl, relation_head="reference")
    data = make_synthetic(num_relations=10, instances_per_relation=30, max_length=L, vocab=800, word_dim=E, seed=1)
    torch.manual_seed(0)
    model = InductionNetwork(cfg, data.word_vec_mat, seed=3).to(DEV)
    with torch.no_grad():
        for n in ("lstm_fw_bias", "lstm_bw_bias", "attn_bias"):
            getattr(model.params, n).copy_(torch.randn_like(getattr(model.params, n)) * 0.3)
    idx, lab = EpisodeSampler(data, seed=2).next_batch_indices(B, N, K, Q)
    inst = torch.tensor(idx.reshape(-1), dtype=torch.int32, device=DEV)
    from induction_network_on_fewrel_amd.ops.sampler import DeviceDataset
    arrays = DeviceDataset(data, DEV).arrays()   # pos_shift: the wide_pos_grad kernel path
    if not shifted:
        arrays = tuple(arrays)                   # plain tuple: the one-hot GEMM path
    return cfg, model, inst, arrays, torch.tensor(lab, device=DEV), (B, N, K, Q)


@pytest.mark.parametrize("u", [100, 128, 64])
@pytest.mark.parametrize("keep_prob", [1.0, 0.9])
def test_paper_config_forward_backward_vs_oracle(keep_prob, u):
    """u=128 (the paper), u=100 (the reference Base default, model/base.py:16) and u=64 on the persistent
    wide BiLSTM kernels (lstm_wide.hip lstm_wide_seq_*) + the wide head, against the fp32 oracle; the
    position-table gradient by wide_pos_grad (shifted ids) for keep_prob 1, by the one-hot GEMM for 0.9."""
    cfg, model, inst, arrays, lab, (B, N, K, Q) = _setup(u, 50, "auto", shifted=keep_prob == 1.0)
    cfg.keep_prob = keep_prob
    assert not model.use_fused_lstm(37)
    probs, _ = model(inst, arrays, B, N, K, Q, training=True, dropout_seed=5)
    loss = model.loss(probs, lab)
    loss.backward()
    got = {k: v.grad.clone() for k, v in model.pdict().items() if v.grad is not None}
    # fp32 oracle on the same device, same dropout masks (counter hash)
    p = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in model.pdict().items()}
    w, a1, a2, m = (t[inst.long()] for t in arrays)
    pr, _ = ref.forward(p, w.long(), a1.long(), a2.long(), m, B, N, K, Q, 3, "reference", keep_prob, 5, bf16=False)
    model.loss(pr, lab).backward()
    assert _relerr(probs.detach(), pr.detach()) < 3e-2
    for k in ("lstm_fw_kernel", "lstm_bw_bias", "pos1_embedding", "attn_kernel", "W_s", "M"):
        assert _relerr(got[k], p[k].grad) < 8e-2, k


@pytest.mark.parametrize("U", [128, 100, 64])
def test_bwd_fused_position_columns_match_gemm(U):
    """The BPTT kernel's fused dX_pos (dG W_pos^T from each step's LDS dG image, per direction) against the
    GEMM over the dG it writes; dG itself is unchanged by the fusion.  S = 77: a partial 32-sequence tile."""
    from induction_network_on_fewrel_amd.ops._ext import ops
    from induction_network_on_fewrel_amd.ops.packing import pack_lstm_wide, wide_x_cols
    from induction_network_on_fewrel_amd.ops.wide import pos_frags
    o = ops()
    g = torch.Generator().manual_seed(0)
    S, L, E, P = 77, 37, 50, 5
    D = E + 2 * P
    Kf, Kb = (torch.randn(D + U, 4 * U, generator=g) * 0.1 for _ in range(2))
    bf, bb = (torch.randn(4 * U, generator=g) * 0.1 for _ in range(2))
    pk = pack_lstm_wide(Kf.to(DEV), bf.to(DEV), Kb.to(DEV), bb.to(DEV), U, D)
    X = torch.randn(S * L, wide_x_cols(D), generator=g).to(DEV).bfloat16()
    gx = torch.mm(X, pk["wxc"])
    _, _, acts, cst = o.lstm_wide_seq_fwd(gx, pk["bx"], pk["apk"], S, L, U, True, 7, 0.9, X.new_empty(0), 0)
    dH = torch.randn(S, L, 2 * U, generator=g).to(DEV).bfloat16()
    dG0, none = o.lstm_wide_seq_bwd(dH, acts, cst, pk["a2pk"], S, L, U, 7, 0.9, X.new_empty(0), 2 * P)
    dG, dxp = o.lstm_wide_seq_bwd(dH, acts, cst, pk["a2pk"], S, L, U, 7, 0.9, pos_frags(pk["wxtc"], E, D), 2 * P)
    torch.cuda.synchronize()
    assert none.numel() == 0 and dxp.shape == (2, S * L, 2 * P)
    assert torch.equal(dG, dG0)
    G4 = dG.shape[1] // 2
    for d in range(2):
        c = slice(d * G4, (d + 1) * G4)
        want = torch.mm(dG[:, c].float(), pk["wxtc"][E:D, c].float().t())
        assert float((dxp[d] - want).abs().max()) <= 1e-5 * float(want.abs().max()), d


@pytest.mark.parametrize("u", [129, 130])
def test_odd_and_unaligned_width_per_step_loop_vs_oracle(u):
    """Widths above the last kernel instantiation that are odd or not multiples of 4 run the
    per-step GEMM loop (ops/wide.py WideBiLSTM + lstm_wide_fwd_step / _bwd_step) with dropout on: the pair hash
    over the flat (sequence, step, unit) index is the oracle's for any u, odd included."""
    cfg, model, inst, arrays, lab, (B, N, K, Q) = _setup(u, 50, "auto")
    cfg.keep_prob = 0.9
    assert not model.use_fused_lstm(37)
    probs, _ = model(inst, arrays, B, N, K, Q, training=True, dropout_seed=7)
    loss = model.loss(probs, lab)
    loss.backward()
    got = {k: v.grad.clone() for k, v in model.pdict().items() if v.grad is not None}
    p = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in model.pdict().items()}
    w, a1, a2, m = (t[inst.long()] for t in arrays)
    pr, _ = ref.forward(p, w.long(), a1.long(), a2.long(), m, B, N, K, Q, 3, "reference", 0.9, 7, bf16=False)
    model.loss(pr, lab).backward()
    ep = _relerr(probs.detach(), pr.detach())
    print(f"u={u}: probs {ep:.2e}")
    assert ep < 3e-2
    for k in ("lstm_fw_kernel", "lstm_fw_bias", "lstm_bw_kernel", "lstm_bw_bias", "pos1_embedding", "attn_kernel",
              "W_s", "M"):
        err = _relerr(got[k], p[k].grad)
        print(f"  grad {k}: {err:.2e}")
        assert err < 8e-2, k


def test_wide_matches_fused_at_u20(monkeypatch):
    """the per-step GEMM loop of ops/wide.py (padding off) against the fused kernels at u = 20."""
    monkeypatch.setenv("INA_LSTM_PAD", "0")
    outs = []
    for impl in ("fused", "wide"):
        cfg, model, inst, arrays, lab, (B, N, K, Q) = _setup(20, 5, impl)
        probs, _ = model(inst, arrays, B, N, K, Q, training=True, dropout_seed=9)
        model.loss(probs, lab).backward()
        outs.append((probs.detach(), model.params.lstm_fw_kernel.grad.clone(), model.params.attn_kernel.grad.clone()))
    (p0, g0, a0), (p1, g1, a1) = outs
    assert _relerr(p1, p0) < 2e-2
    assert _relerr(g1, g0) < 6e-2
    assert _relerr(a1, a0) < 6e-2


@pytest.mark.parametrize("u,E,path", [(10, 5, "small"), (16, 5, "small"), (50, 50, "wide"), (80, 50, "wide"),
                                      (24, 300, "wide")])
@pytest.mark.parametrize("keep_prob", [1.0, 0.9])
def test_padded_width_vs_oracle(u, E, path, keep_prob):
    """hidden_size between the kernel instantiations (models/padding.py): the encoder runs on the next
    instantiated width with zero-padded parameters.  keep_prob 1: against the fp32 oracle at the model's own
    width (exact semantics); keep_prob 0.9: against the oracle run on the padded parameters (the dropout
    stream is drawn over the padded width), sliced back to the real units."""
    from induction_network_on_fewrel_amd.models.padding import padded_params
    cfg, model, inst, arrays, lab, (B, N, K, Q) = _setup(u, E, "auto", shifted=keep_prob == 1.0)
    cfg.keep_prob = keep_prob
    plan = model.lstm_plan(37)
    assert plan[0] == path and plan[1] > u, plan
    probs, _ = model(inst, arrays, B, N, K, Q, training=True, dropout_seed=5)
    model.loss(probs, lab).backward()
    got = {k: v.grad.clone() for k, v in model.pdict().items() if v.grad is not None}
    p = {k: v.detach().clone().requires_grad_(v.requires_grad) for k, v in model.pdict().items()}
    w, a1, a2, m = (t[inst.long()] for t in arrays)
    if keep_prob == 1.0:
        pr, _ = ref.forward(p, w.long(), a1.long(), a2.long(), m, B, N, K, Q, 3, "reference", 1.0, 5, bf16=False)
    else:
        pp, real = padded_params(p, u, plan[1], model.params.input_dim)
        e, _ = ref.encode(pp, w.long(), a1.long(), a2.long(), m, keep_prob, 5)
        pr = ref.head_forward(p, e[:, real], B, N, K, Q, 3, "reference")
    model.loss(pr, lab).backward()
    assert probs.shape == pr.shape
    assert _relerr(probs.detach(), pr.detach()) < 3e-2
    tol = 8e-2 if path == "wide" else 1.2e-1   # the small kernels keep the BPTT stash / dH in bf16
    for k in ("lstm_fw_kernel", "lstm_bw_bias", "pos1_embedding", "attn_kernel", "W_s", "M"):
        assert got[k].shape == p[k].shape, k
        assert _relerr(got[k], p[k].grad) < tol, k


@pytest.mark.parametrize("H,L,S", [(256, 37, 101), (200, 37, 64), (128, 37, 33), (256, 90, 5)])
def test_fused_attention_vs_fp32(H, L, S):
    """csrc/kernels/attn_wide.hip (ops/wide.py WideAttn) against the fp32 autograd of the reference
    self-attention (model/layer_module.py:49-98) on the same bf16 BiLSTM output: e, alphas and the
    gradients of H, W1, b1, w2.  Odd S covers a partial last block; L=90 the one-sequence-per-block
    geometry; rows with short masks and one fully-padded-but-one sequence check the masking."""
    from induction_network_on_fewrel_amd.ops.wide import WideAttn
    g = torch.Generator(device="cpu").manual_seed(H + L)
    Hb = (torch.randn(S, L, H, generator=g) * 0.7).to(torch.bfloat16).to(DEV)
    lens = torch.randint(1, L + 1, (S,), generator=g)
    lens[0] = 1
    rows = 2 * S + 3
    mask = torch.zeros(rows, L, dtype=torch.int32)
    inst = torch.randperm(rows, generator=g)[:S].to(torch.int32)
    for i in range(S):
        mask[inst[i], :lens[i]] = torch.randint(1, 4, (int(lens[i]),), generator=g).to(torch.int32)
    mask, inst = mask.to(DEV), inst.to(DEV)
    W1 = (torch.randn(H, H, generator=g) / H ** 0.5).to(DEV).requires_grad_()
    b1 = (torch.randn(H, generator=g) * 0.3).to(DEV).requires_grad_()
    w2 = (torch.randn(H, 1, generator=g) * 0.5).to(DEV).requires_grad_()
    Hk = Hb.clone().requires_grad_()
    e, alpha = WideAttn.apply(Hk, inst, mask, W1, b1, w2)
    de = torch.randn(S, H, generator=g).to(DEV)
    (e * de).sum().backward()
    # fp32 oracle on the bf16-rounded weights the kernels use (bf16 MFMA operands, fp32 accumulation)
    Hr = Hb.float().requires_grad_()
    W1r = W1.detach().clone().requires_grad_()
    b1r, w2r = b1.detach().clone().requires_grad_(), w2.detach().clone().requires_grad_()
    proj = torch.tanh(Hr @ W1r.to(torch.bfloat16).float() + b1r)
    score = (proj @ w2r).squeeze(-1)
    valid = mask[inst.long()] > 0
    al = torch.softmax(score.masked_fill(~valid, float("-inf")), dim=1)
    er = (Hr * al.unsqueeze(-1)).sum(1)
    (er * de).sum().backward()
    assert _relerr(e.detach(), er.detach()) < 1e-2
    assert _relerr(alpha, al.detach()) < 1e-2
    assert float(alpha[~valid].abs().max()) == 0.0
    assert _relerr(Hk.grad.float(), Hr.grad) < 2e-2
    assert _relerr(W1.grad, W1r.grad) < 3e-2
    assert _relerr(b1.grad, b1r.grad) < 2e-2
    assert _relerr(w2.grad, w2r.grad) < 2e-2


@pytest.mark.parametrize("U,D", [(128, 310), (100, 60), (64, 30)])
def test_wide_packs_single_gather_matches_pack_functions(U, D):
    """ops/wide_packs.py: every wide-path weight pack from ONE ina.gather_pack_affine launch over the flat
    parameter buffer == the pack functions (gate pre-scales and forget bias via the affine map)."""
    from induction_network_on_fewrel_amd.ops.optim import FlatParams
    from induction_network_on_fewrel_amd.ops.wide_packs import plan_check
    g = torch.Generator().manual_seed(U)
    H = 2 * U
    shapes = dict(Kf=(D + U, 4 * U), bf=(4 * U,), Kb=(D + U, 4 * U), bb=(4 * U,), W1=(H, H), b1=(H,), w2=(H, 1))
    params = {k: torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for k, s in shapes.items()}
    FlatParams(params)   # re-homes the parameters into one flat buffer (the trainer's layout)
    ts = tuple(params[k] for k in shapes)
    err = plan_check(ts, U, D)
    assert err <= 1e-2 * max(float(t.abs().max()) for t in ts) * 2.0, err


@pytest.mark.parametrize("E", [300, 50])
@pytest.mark.parametrize("table_bf16", [False, True])
def test_wide_x_gather_rows(E, table_bf16):
    """ina.wide_x_gather (8 rows in flight per wave; fp32 or cached-bf16 word table) == the torch gather
    of [word row ; pos1 row ; pos2 row ; 1 ; 0 pad] in bf16, incl. a partial last wave."""
    from induction_network_on_fewrel_amd.ops import ops
    g = torch.Generator().manual_seed(E)
    NI, L, V, PD, S = 40, 37, 500, 5, 13
    word = torch.randint(0, V, (NI, L), generator=g, dtype=torch.int32).to(DEV)
    pos1 = torch.randint(0, 2 * L, (NI, L), generator=g, dtype=torch.int32).to(DEV)
    pos2 = torch.randint(0, 2 * L, (NI, L), generator=g, dtype=torch.int32).to(DEV)
    inst = torch.randint(0, NI, (S,), generator=g, dtype=torch.int32).to(DEV)
    wemb = torch.randn(V, E, generator=g).to(DEV)
    p1, p2 = torch.randn(2 * L, PD, generator=g).to(DEV), torch.randn(2 * L, PD, generator=g).to(DEV)
    tab = wemb.to(torch.bfloat16) if table_bf16 else wemb
    xb = ops().wide_x_gather(inst, word, pos1, pos2, tab, p1, p2, 0)
    il = inst.long()
    ref = torch.cat([wemb[word[il].long()], p1[pos1[il].long()], p2[pos2[il].long()],
                     torch.ones(S, L, 1, device=DEV)], -1).reshape(S * L, -1)
    ref = torch.nn.functional.pad(ref, (0, xb.shape[1] - ref.shape[1])).to(torch.bfloat16)
    assert torch.equal(xb, ref)


@pytest.mark.parametrize("bf16", [False, True])
def test_transpose12_matches_permute(bf16):
    """ina.transpose12 (the wide NTN head's M <-> M' layouts, glue.hip): [A, B, C] -> [A, C, B], ragged tiles."""
    from induction_network_on_fewrel_amd.ops._ext import ops
    x = torch.randn(5, 70, 37, device=DEV)
    y = ops().transpose12(x, bf16)
    want = x.permute(0, 2, 1).contiguous()
    if bf16:
        want = want.to(torch.bfloat16)
    assert y.shape == want.shape and torch.equal(y, want)
