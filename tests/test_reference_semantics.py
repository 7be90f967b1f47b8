"""The PyTorch oracle reproduces the reference's TF1 graph semantics.

Each check re-implements the reference layer literally (loop-for-loop, as written in
model/layer_module.py / model/graph.py) and compares with the batched oracle.
"""
import math

import numpy as np
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.models import InductionNetwork, TF_NAMES
from induction_network_on_fewrel_amd.models import reference as ref

torch.manual_seed(0)


def test_basic_lstm_cell_gate_order_and_forget_bias():
    S, L, D, u = 4, 6, 7, 3
    x = torch.randn(S, L, D)
    W = torch.randn(D + u, 4 * u) * 0.5
    b = torch.randn(4 * u) * 0.1
    h_all, _ = ref.lstm_direction(x, W, b, reverse=False)
    h = torch.zeros(S, u)
    c = torch.zeros(S, u)
    sig = torch.sigmoid
    for t in range(L):   # tf.nn.rnn_cell.BasicLSTMCell: concat([x, h]) @ W + b; split i, j, f, o
        g = torch.cat([x[:, t], h], 1) @ W + b
        i, j, f, o = g[:, :u], g[:, u:2 * u], g[:, 2 * u:3 * u], g[:, 3 * u:]
        c = c * sig(f + 1.0) + sig(i) * torch.tanh(j)
        h = torch.tanh(c) * sig(o)
        assert torch.allclose(h_all[:, t], h, atol=1e-6)
    # bidirectional_dynamic_rnn without sequence_length: bw runs over the FULL reversed sequence
    hb, _ = ref.lstm_direction(x, W, b, reverse=True)
    hr, _ = ref.lstm_direction(x.flip(1), W, b, reverse=False)
    assert torch.allclose(hb, hr.flip(1), atol=1e-6)


def test_self_attention_matches_reference_ops():
    S, L, H = 5, 9, 6
    Hin = torch.randn(S, L, H)
    mask = torch.ones(S, L)
    mask[0, 4:] = 0
    mask[1, 2:] = 0
    Wd, bd, w2 = torch.randn(H, H), torch.randn(H), torch.randn(H, 1)
    e, al = ref.self_attention(Hin, mask > 0, Wd, bd, w2)
    x_proj = torch.tanh(torch.tensordot(Hin, Wd, dims=1) + bd)
    x = torch.tensordot(x_proj, w2, dims=1)
    adder = (1.0 - mask.unsqueeze(-1)) * (-2 ** 31)
    alphas = torch.softmax(x + adder, dim=1)
    out = torch.matmul(Hin.transpose(1, 2), alphas).squeeze(-1)
    assert torch.allclose(e, out, atol=1e-6) and torch.allclose(al, alphas)
    assert float(al[0, 4:].abs().max()) == 0.0  # masked positions get exactly zero weight


def test_dynamic_routing_literal_loop():
    C, K, H = 3, 4, 5
    inp = torch.randn(C, K, H)
    W = torch.randn(H, H)
    b_IJ = torch.zeros(C, K)
    c_I = None
    for _ in range(3):
        d_I = torch.softmax(b_IJ.view(C, K, 1), dim=1)
        e_IJ = (inp.view(-1, H) @ W).view(C, K, -1)
        c_I = (d_I * e_IJ).sum(1, keepdim=True).view(C, -1)
        n = (c_I ** 2).sum(1, keepdim=True)
        c_I = n / (1 + n) / torch.sqrt(n + 1e-9) * c_I
        b_IJ = b_IJ + (e_IJ @ c_I.view(C, H, 1)).view(C, K)
    out = ref.dynamic_routing(inp.unsqueeze(0), W, 3)[0]
    assert torch.allclose(out, c_I, atol=1e-5)


def test_neural_tensor_layer_column_order():
    C, NQ, H, h = 4, 6, 5, 7
    cls, q = torch.randn(C, H), torch.randn(NQ, H)
    M = torch.randn(H, H, h)
    W, b = torch.randn(h * C, C), torch.randn(C)
    mid = [(cls @ M[:, :, s]) @ q.t() for s in range(h)]      # layer_module.py:21-34
    V = torch.relu(torch.cat(mid, 0).t())                       # [NQ, h*C], column s*C + c
    probs = torch.sigmoid(V @ W + b)
    out = ref.relation_probs(cls.unsqueeze(0), q.unsqueeze(0), M, W, b, "reference")[0]
    assert torch.allclose(out, probs, atol=1e-5)


def test_mse_mean_onehot_and_nota():
    probs = torch.rand(2, 6, 3)
    labels = torch.tensor([[0, 1, 2, 0, 1, 3], [2, 2, 1, 0, 3, 3]])  # 3 == NOTA (out of range)
    y = torch.zeros(2, 6, 3)
    for bi in range(2):
        for qi in range(6):
            if labels[bi, qi] < 3:
                y[bi, qi, labels[bi, qi]] = 1
    assert torch.allclose(ref.mse_loss(probs, labels), ((y - probs) ** 2).mean())
    pred = ref.predict(torch.tensor([[[0.1, 0.2, 0.3], [0.9, 0.1, 0.0]]]), nota_threshold=0.5)
    assert pred.tolist() == [[3, 0]]


def test_ce_loss_on_presigmoid_scores_and_nota():
    """loss_type='ce': softmax cross-entropy over the pre-sigmoid relation scores; NOTA rows add 0
    (mean over all query rows); gradient wrt the logits = (softmax - onehot) / rows."""
    z = torch.randn(2, 6, 3, dtype=torch.float64, requires_grad=True)
    labels = torch.tensor([[0, 1, 2, 0, 1, 3], [2, 2, 1, 0, 3, 3]])
    loss = ref.ce_loss(torch.sigmoid(z), labels)
    keep = labels < 3
    want = torch.nn.functional.cross_entropy(z[keep], labels[keep], reduction="sum") / labels.numel()
    assert torch.allclose(loss, want)
    loss.backward()
    sm = torch.softmax(z.detach(), -1)
    g = (sm - torch.nn.functional.one_hot(labels.clamp(max=2), 3)) * keep.unsqueeze(-1) / labels.numel()
    assert torch.allclose(z.grad, g, atol=1e-7)
    cfg = Config(loss_type="ce")
    cfg.validate()


def test_ce_nota_loss_extra_class_of_logit_zero():
    """loss_type='ce_nota': softmax over the N pre-sigmoid scores + a NOTA class of logit 0; NOTA rows (label N)
    target that class, in-class rows their class; mean over all query rows.  The gradient of a NOTA row pushes
    every relation logit down."""
    z = torch.randn(2, 6, 3, dtype=torch.float64, requires_grad=True)
    labels = torch.tensor([[0, 1, 2, 0, 1, 3], [2, 2, 1, 0, 3, 3]])
    loss = ref.ce_nota_loss(torch.sigmoid(z), labels)
    zz = torch.cat([z.detach(), torch.zeros(2, 6, 1, dtype=torch.float64)], -1)
    want = torch.nn.functional.cross_entropy(zz.view(-1, 4), labels.view(-1), reduction="sum") / labels.numel()
    assert torch.allclose(loss, want)
    loss.backward()
    sm = torch.softmax(zz, -1)[..., :3]
    g = (sm - torch.nn.functional.one_hot(labels, 4)[..., :3]) / labels.numel()
    assert torch.allclose(z.grad, g, atol=1e-7)
    assert bool((z.grad[labels == 3] > 0).all())   # NOTA rows: d loss / d z_c > 0 -> every logit pushed down
    assert ref.LOSS_MODES["ce_nota"] == 2 and ref.loss_fn("ce_nota") is ref.ce_nota_loss
    Config(loss_type="ce_nota").validate()


def test_param_names_shapes_and_init():
    cfg = Config(N=5, K=2, Q=5, hidden_size=20, max_length=37)
    wv = np.random.randn(1002, 5).astype(np.float32)
    m = InductionNetwork(cfg, wv)
    st = m.params.tf_state()
    exp = {"embedding/Variable": (1002, 5), "pos1_embedding": (74, 5), "pos2_embedding": (74, 5),
           "bidirectional_rnn/fw/basic_lstm_cell/kernel": (35, 80), "bidirectional_rnn/fw/basic_lstm_cell/bias": (80,),
           "bidirectional_rnn/bw/basic_lstm_cell/kernel": (35, 80), "bidirectional_rnn/bw/basic_lstm_cell/bias": (80,),
           "self_attn/dense/kernel": (40, 40), "self_attn/dense/bias": (40,), "self_attn/W_a2": (40, 1),
           "W_s": (40, 40), "M": (40, 40, 100), "w": (500, 5), "b": (5,)}
    assert {k: tuple(v.shape) for k, v in st.items()} == exp
    n_train = sum(p.numel() for p in m.params.trainable().values())
    assert n_train == 172285          # SURVEY 2.4 default-config total
    assert "word_embedding" not in m.params.trainable()   # frozen pretrained table
    # glorot-normal (truncated) std for M: fan_in = 40*40, fan_out = 100*40
    std = math.sqrt(2.0 / (1600 + 4000))
    assert abs(float(m.params.M.std()) / std - 1.0) < 0.05
    assert float(m.params.lstm_fw_bias.abs().max()) == 0.0
    assert abs(float(m.params.pos1_embedding.std()) - 0.1) < 0.02


def test_l2_vars_follow_reference_filter():
    cfg = Config()
    m = InductionNetwork(cfg, np.zeros((12, 5), np.float32))
    names = {m.params.tf_name(a) for a, p in m.params.trainable().items() if any(p is q for q in m.params.l2_vars())}
    assert names == {"bidirectional_rnn/fw/basic_lstm_cell/kernel", "bidirectional_rnn/bw/basic_lstm_cell/kernel",
                     "self_attn/dense/kernel", "self_attn/W_a2", "W_s", "M", "w", "b"}


def test_dropout_mask_rate_and_determinism():
    m1 = ref.dropout_keep_mask(7, 0, 64, 37, 20, 0.9)
    m2 = ref.dropout_keep_mask(7, 0, 64, 37, 20, 0.9)
    m3 = ref.dropout_keep_mask(7, 1, 64, 37, 20, 0.9)
    assert torch.equal(m1, m2) and not torch.equal(m1, m3)
    assert abs(float(m1.mean()) - 0.9) < 0.01
    # the two units of a hash pair (16-bit halves of one mix) are independent draws
    both = float((m1[..., 0::2] * m1[..., 1::2]).mean())
    assert abs(both - 0.81) < 0.01


def test_full_forward_runtime_nkq():
    """N/K/Q are runtime arguments; only the reference head's w is N-dependent."""
    from induction_network_on_fewrel_amd.data import EpisodeSampler, make_synthetic
    data = make_synthetic(num_relations=12, instances_per_relation=20, vocab=200, seed=0)
    for head, N in (("reference", 5), ("paper", 5), ("paper", 10)):
        cfg = Config(N=5, relation_head=head)
        m = InductionNetwork(cfg, data.word_vec_mat)
        idx, lab = EpisodeSampler(data, seed=0).next_batch_indices(2, N, 3, 2)
        arrays = tuple(torch.as_tensor(a) for a in (data.data_word, data.data_pos1, data.data_pos2, data.data_mask))
        probs, alphas = m(torch.as_tensor(idx.reshape(-1)), arrays, 2, N, 3, 2, training=False)
        assert probs.shape == (2, N * 2, N) and alphas.shape == (2 * (N * 3 + N * 2), 37)
