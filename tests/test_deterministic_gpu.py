"""Config.deterministic on the GPU encoder paths: torch's deterministic-algorithm mode raises on
a library op without a deterministic implementation, so every encoder path must run under it -- the fused
BiLSTM, the wide (per-step GEMM / wide kernels) path and BERT -- and repeat bitwise (frozen word table)."""
import pytest
import torch

from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data.synthetic import make_synthetic
from induction_network_on_fewrel_amd.runtime.trainer import Trainer

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kind", ["fused", "wide", "bert"])
def test_deterministic_train_steps_repeat_on_gpu(tmp_path, kind):
    kw = dict(fused={}, wide=dict(hidden_size=64, synthetic_word_dim=50),
              bert=dict(encoder="bert", bert_layers=1, bert_hidden=256, bert_heads=4, bert_intermediate=512,
                        bert_max_length=32, bert_out_dim=40))[kind]
    data = make_synthetic(num_relations=8, instances_per_relation=20, vocab=300, word_dim=kw.pop("synthetic_word_dim", 5),
                          seed=0)
    flats = []
    try:
        for i in range(2):
            cfg = Config(N=5, K=2, Q=2, episodes_per_step=4, model_dir=str(tmp_path / f"{kind}{i}"), seed=3,
                         resume=False, deterministic=True, **kw)
            tr = Trainer(cfg, data, None, device="cuda", log=False)
            for _ in range(2):
                tr.train_step()
            torch.cuda.synchronize()
            flats.append(tr.flat.flat.detach().clone())
    finally:
        torch.use_deterministic_algorithms(False)
    assert torch.isfinite(flats[0]).all()
    assert torch.equal(flats[0], flats[1])
