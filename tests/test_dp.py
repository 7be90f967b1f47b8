"""Episode data parallelism, multi-process on CPU with the gloo backend (world_size 2, 4 and 8).

Checks:
* the DP step's gradient (all-reduce of the per-rank gradients, then the optimizer's 1/world scale)
  equals the gradient of ONE single-rank step over the union of every rank's episodes;
* parameters stay bitwise identical across ranks after optimizer steps, and rank samplers differ;
* ``python bench.py --gpus 2`` without a launcher starts the ranks itself (gloo on CPU here; the
  one-card GPU form is tests/test_dp_gpu.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.parallel.dp import DistContext
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    dist = DistContext.from_env("cpu")
    data = make_synthetic(num_relations=10, instances_per_relation=30, vocab=300, seed=0)
    cfg = Config(N=5, K=2, Q=2, episodes_per_step=2, model_dir=os.path.join(out_dir, "m"), resume=False, seed=5)
    tr = Trainer(cfg, data, None, device="cpu", dist_ctx=dist, log=False)
    # 1) DP gradient == single-rank gradient over the union of the ranks' episodes.  Dropout off
    #    (training=False) so the union forward sees exactly the rows each rank saw.
    B = 2
    idx, lab = tr.train_eps.sample(B, 5, 2, 2)

    def grad_of(i, l, b):
        tr.flat.zero_grad()
        probs, _ = tr.model(i.reshape(-1), tr.train_eps.arrays, b, 5, 2, 2, training=False)
        tr.model.loss(probs, l).backward()
        tr.flat.sync_grads_into_flat()
        return tr.flat.grad.clone()

    local = grad_of(idx, lab, B)
    tr.flat.grad.copy_(local)
    tr.dist.allreduce_buckets_(tr.flat.grad, bucket_mb=0.05)   # several buckets
    dp_grad = tr.flat.grad.clone() * (1.0 / world)               # the optimizer's grad_scale
    all_idx = [torch.zeros_like(idx) for _ in range(world)]
    all_lab = [torch.zeros_like(lab) for _ in range(world)]
    torch.distributed.all_gather(all_idx, idx)
    torch.distributed.all_gather(all_lab, lab)
    union = grad_of(torch.cat(all_idx), torch.cat(all_lab), B * world)
    ok_sum = bool(torch.allclose(dp_grad, union, rtol=1e-5, atol=1e-8)) and bool(local.abs().sum() > 0) \
        and not torch.equal(local * world, union)   # the ranks' gradients really differ
    # 2) params identical after optimizer steps
    for _ in range(3):
        tr.train_step()
    in_sync = tr.dist.params_in_sync(tr.flat.flat)
    # 3) backward-overlapped bucket all-reduce: buckets launched out of order + the uncovered rest
    buf = torch.arange(20, dtype=torch.float32) * (rank + 1)
    ov = dist.overlap(buf, [(2, 5), (10, 4)])
    ov.ready(1)
    ov.ready(0)
    ov.ready(1)          # idempotent
    ov.finish()
    ok_overlap = torch.equal(buf, torch.arange(20, dtype=torch.float32) * sum(r + 1 for r in range(world)))
    torch.save({"ok_sum": ok_sum, "in_sync": in_sync, "idx": idx, "ok_overlap": ok_overlap},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.destroy()


def _resume_worker(rank, world, port, out_dir):
    """Save (collective) after 2 steps, continue 1 step, then a fresh trainer resumes from the
    checkpoint: every rank must continue ITS OWN episode stream (advisor finding: rank 0's sampler
    state used to be loaded on every rank, collapsing DP to one rank's episodes)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.parallel.dp import DistContext
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer
    dist = DistContext.from_env("cpu")
    data = make_synthetic(num_relations=10, instances_per_relation=30, vocab=300, seed=0)
    cfg = Config(N=5, K=2, Q=2, episodes_per_step=2, model_dir=os.path.join(out_dir, "m"), resume=False, seed=5)
    tr = Trainer(cfg, data, None, device="cpu", dist_ctx=dist, log=False)
    for _ in range(2):
        tr.train_step()
    tr.save()
    cont = tr.train_eps.sample(2, 5, 2, 2)[0]           # what this rank draws next without a restart
    tr2 = Trainer(cfg.replace(resume=True), data, None, device="cpu", dist_ctx=dist, log=False)
    resumed = tr2.train_eps.sample(2, 5, 2, 2)[0]
    torch.save({"cont": cont, "resumed": resumed, "step": tr2.global_step}, os.path.join(out_dir, f"res{rank}.pt"))
    dist.destroy()


@pytest.mark.slow
def test_dp_resume_keeps_per_rank_samplers(tmp_path):
    world = 2
    mp.start_processes(_resume_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [torch.load(tmp_path / f"res{i}.pt", weights_only=True) for i in range(world)]
    assert all(x["step"] == 2 for x in r)
    for x in r:
        assert torch.equal(x["resumed"], x["cont"])          # each rank continues its own stream
    assert not torch.equal(r[0]["resumed"], r[1]["resumed"])  # ranks still draw different episodes


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_dp_gloo_world(tmp_path, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(world)]
    assert all(x["ok_sum"] for x in r)
    assert all(x["in_sync"] for x in r)
    assert all(x["ok_overlap"] for x in r)
    for i in range(1, world):
        assert not torch.equal(r[0]["idx"], r[i]["idx"])   # rank-folded sampling


@pytest.mark.parametrize("world", [2, 8])
def test_bench_self_launch_cpu(world):
    """``bench.py --gpus N`` with no torch.distributed.run: the parent starts the N ranks, rank 0 prints
    one JSON line with the real collective world size; a failing rank fails the whole job.  N = 8 rehearses the
    driver's 8-GPU scaling run (gloo on CPU: the rank bootstrap, the bucketed all-reduce and the MAX-over-ranks
    timing at the world size of one MI355X node)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "INA_FAULT_STEP"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(root, "bench.py"), "--gpus", str(world), "--device", "cpu", "--steps", "2",
           "--warmup", "1", "--episodes-per-gpu", "2", "--launch-timeout", "240"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == world and out["rccl_world"] == world and out["backend"] == "gloo"
    assert out["params_in_sync"] is True and len(out["rank_ms_per_step"]) == world
    assert out["config"]["global_batch"] == 2 * world and out["config"]["parallelism"] == f"dp{world}"
    bad = subprocess.run(cmd, cwd=root, env=dict(env, INA_FAULT_STEP="1", INA_FAULT_RANK=str(world - 1)), capture_output=True,
                         text=True, timeout=300)
    assert bad.returncode != 0
