"""Debug: compare eager/eager and eager/graph training trajectories per parameter."""
import sys, os, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from induction_network_on_fewrel_amd.config import Config
from induction_network_on_fewrel_amd.data import make_synthetic
from induction_network_on_fewrel_amd.runtime.trainer import Trainer

data = make_synthetic(num_relations=12, instances_per_relation=40, vocab=500, seed=0)
runs = []
tmp = tempfile.mkdtemp()
for i, graph in enumerate((False, False, True)):
    cfg = Config(N=5, K=2, Q=3, episodes_per_step=16, model_dir=os.path.join(tmp, f"g{i}"), seed=4, resume=False,
                 use_hip_graph=graph, learning_rate=1e-2)
    tr = Trainer(cfg, data, None, device="cuda", log=False)
    losses = [float(tr.train_step()[0]) for _ in range(6)]
    runs.append({k: v.detach().clone() for k, v in tr.model.pdict().items()})
for a, b, name in ((0, 1, "eager/eager"), (0, 2, "eager/graph")):
    for k in runs[a]:
        x, y = runs[a][k].double(), runs[b][k].double()
        d = (x - y).abs()
        if d.max() > 0:
            idx = torch.nonzero(d == d.max())[0].tolist()
            print(name, k, "maxdiff %.3e" % d.max().item(), "at", idx, "rel %.3e" % (d.max() / (y.abs().max() + 1e-12)).item())
