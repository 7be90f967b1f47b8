"""DP gradient ground truth for the fused GPU step (run by tests/test_dp_gpu.py under torch.distributed.run).

Every rank runs ONE eager fused train step (StepGlue slabs, ragged tiles, the relation-head span all-reduced
under the encoder backward) on its own episodes, keep_prob = 1, learning rate 0.  Afterwards the flat
gradient buffer holds the all-reduced SUM.  Each rank then recomputes, without any collective, one fused
forward + backward over the UNION of all ranks' episodes (gathered from the ranks), and checks
sum / world == union gradient (the loss is a mean over episodes) per parameter.  A collective that read a
bucket before the step glue's scatter finished, or a wrong scale, breaks the equality; with a single rank
the in-place all-reduce would write stale values back over the flushed gradient.

Prints one JSON line per rank: {"rank", "world", "comm", "max_rel_err", "per_param": {...}}.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.parallel.dp import DistContext
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer

    B = int(os.environ.get("DPCHK_EPISODES", "384"))   # 384 x 50 rows per rank: ragged tiles on
    device = os.environ.get("DPCHK_DEVICE", "cuda")      # cpu: the oracle path (plumbing check of this script)
    dist = DistContext.from_env(device)
    cuda = device == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    N, K, Q = 5, 5, 5
    cfg = Config(N=N, K=K, Q=Q, max_length=37, hidden_size=20, dtype="bf16", episodes_per_step=B, seed=77,
                 keep_prob=1.0, learning_rate=0.0, lr_schedule="constant", resume=False,
                 model_dir=f"/tmp/ina_dpchk_{dist.rank}", use_hip_graph=False, hip_graph_max_episodes=0)
    data = make_synthetic(num_relations=20, instances_per_relation=120, max_length=37, vocab=2000, word_dim=5,
                          seed=3)
    tr = Trainer(cfg, data, None, device=device, dist_ctx=dist, log=False)
    rec = []
    orig = tr.train_eps.sample

    def sample(*a, **k):
        idx, lab = orig(*a, **k)
        rec.append((idx.detach().cpu().clone(), lab.detach().cpu().clone()))
        return idx, lab

    tr.train_eps.sample = sample
    tr.train_step()
    sync()
    g_dp = tr.flat.grad.detach().clone()
    parts = dist.all_gather_objects(rec[0])
    idx_all = torch.cat([p[0] for p in parts]).to(tr.device)
    lab_all = torch.cat([p[1] for p in parts]).to(tr.device)
    Bt = idx_all.shape[0]
    # the union step on this rank alone: same kernels, same glue, no collective
    tr.flat.zero_grad()
    loss, _, _ = tr.model.forward_train(idx_all.reshape(-1), tr.train_eps.arrays, Bt, N, K, Q, lab_all,
                                        dropout_seed=0, grad_views=tr.grad_views if cuda else None, overlap=None,
                                        glue=tr.glue)
    torch.autograd.backward(loss, tr.glue.one if tr.glue is not None else None)
    if tr.glue is not None:
        tr.glue.flush()
    tr.flat.sync_grads_into_flat()
    sync()
    g_ref = tr.flat.grad.detach().clone()
    per = {}
    for name in tr.flat.names:
        a = tr.flat.view(g_dp, name).double() / dist.world
        b = tr.flat.view(g_ref, name).double()
        den = float(b.abs().max())
        if den == 0.0:
            continue
        per[name] = float((a - b).abs().max()) / den
    out = dict(rank=dist.rank, world=dist.world, comm=dist.comm_name, episodes_union=Bt,
               max_rel_err=max(per.values()), per_param=per, finite=bool(torch.isfinite(g_dp).all()))
    # one write() per line: the ranks share the launcher's stdout, and print()'s separate newline write let
    # two ranks' lines interleave into one
    sys.stdout.write(json.dumps(out) + "\n")
    sys.stdout.flush()
    dist.destroy()


if __name__ == "__main__":
    main()
