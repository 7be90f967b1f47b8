"""Zero-padded encoder widths (models/padding.py): the padded network is the unpadded one (fp32 oracle,
forward and every parameter gradient), and the GPU width plan picks the next kernel instantiation."""
import pytest
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.models import InductionNetwork
from induction_network_on_fewrel_amd.models import reference as ref
from induction_network_on_fewrel_amd.models.padding import padded_params


@pytest.mark.parametrize("u,up", [(10, 20), (3, 8), (7, 8), (50, 64), (45, 64), (77, 100), (101, 128)])
def test_padded_encoder_is_exact(u, up):
    torch.manual_seed(u)
    E, P, L, S = 6, 5, 13, 5
    D = E + 2 * P
    p = {"word_embedding": torch.randn(40, E), "pos1_embedding": torch.randn(2 * L, P),
         "pos2_embedding": torch.randn(2 * L, P),
         "lstm_fw_kernel": torch.randn(D + u, 4 * u) * 0.3, "lstm_fw_bias": torch.randn(4 * u) * 0.3,
         "lstm_bw_kernel": torch.randn(D + u, 4 * u) * 0.3, "lstm_bw_bias": torch.randn(4 * u) * 0.3,
         "attn_kernel": torch.randn(2 * u, 2 * u) * 0.3, "attn_bias": torch.randn(2 * u) * 0.3,
         "attn_w2": torch.randn(2 * u, 1) * 0.3}
    for t in p.values():
        t.requires_grad_(True)
    w = torch.randint(0, 40, (S, L))
    a1 = torch.randint(0, 2 * L, (S, L))
    a2 = torch.randint(0, 2 * L, (S, L))
    m = torch.ones(S, L, dtype=torch.int32)
    m[:, 9:] = 0
    e0, al0 = ref.encode(p, w, a1, a2, m)
    pp, real = padded_params(p, u, up, D)
    assert pp["lstm_fw_kernel"].shape == (D + up, 4 * up) and pp["attn_kernel"].shape == (2 * up, 2 * up)
    e1, al1 = ref.encode(pp, w, a1, a2, m)
    e1 = e1[:, real]
    torch.testing.assert_close(e1, e0, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(al1, al0, rtol=1e-5, atol=1e-6)
    g = torch.randn_like(e0)
    g0 = torch.autograd.grad((e0 * g).sum(), list(p.values()))
    g1 = torch.autograd.grad((e1 * g).sum(), list(p.values()))
    for a, b, k in zip(g1, g0, p):
        assert a.shape == b.shape, k
        torch.testing.assert_close(a, b, rtol=1e-3, atol=1e-5, msg=k)


@pytest.mark.parametrize("u,E,impl,plan", [(20, 5, "auto", ("small", 20)), (10, 5, "auto", ("small", 20)),
                                           (33, 5, "auto", ("wide", 64)), (24, 300, "auto", ("wide", 64)),
                                           (128, 300, "auto", ("wide", 128)), (90, 50, "auto", ("wide", 100)),
                                           (160, 50, "auto", ("wide", 160)), (20, 5, "wide", ("wide", 64)),
                                           (12, 5, "fused", ("small", 20))])
def test_width_plan(u, E, impl, plan, monkeypatch):
    monkeypatch.delenv("INA_LSTM_PAD", raising=False)
    cfg = Config(hidden_size=u, synthetic_word_dim=E, lstm_impl=impl, max_length=40)
    m = InductionNetwork(cfg, vocab_size=30)
    assert m.lstm_plan(40) == plan
    assert m.use_fused_lstm(40) == (plan == ("small", u))
    monkeypatch.setenv("INA_LSTM_PAD", "0")
    if plan[1] != u:
        if plan[0] == "small" and impl == "fused":
            with pytest.raises(NotImplementedError):
                m.lstm_plan(40)
        else:
            assert m.lstm_plan(40) == ("wide", u)
