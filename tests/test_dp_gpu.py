"""Multi-rank GPU training step on ONE card: bench.py under torch.distributed.run, world_size 2.

RCCL refuses two ranks on the same device, so the collective backend here is gloo
(INA_DIST_BACKEND=gloo, CUDA tensors); everything else is the driver's 8-GPU path: one process per
rank, rank-folded device sampling, the fused kernels writing the flat gradient, the bucketed
all-reduce + 1/world scaling inside the timed step, the fused Adam, the MAX-over-ranks timing and
the rank-0 JSON line.  The check is that parameters stay bitwise identical across ranks
(``params_in_sync``) for the eager step and for the HIP-graph step (all-reduce outside the graph), and --
the ground truth -- that the all-reduced fused-step gradient / world equals one step over the union of the
ranks' episodes (tests/dp_grad_check.py).
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("graph", [0, 1])
def test_bench_world2_one_gpu(graph):
    env = dict(os.environ, INA_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "3", "--warmup", "2", "--episodes-per-gpu", "64", "--graph", str(graph)]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 prints exactly one JSON line
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 128
    assert out["params_in_sync"] is True
    assert out["final_loss"] == out["final_loss"] and out["value"] > 0


def test_bench_rccl_world1():
    """The RCCL (backend "nccl") collective path itself on one card: world size 1 with the process
    group forced on, so the timed step's bucketed all-reduce, the barriers with device ids, the MAX
    timing reduction and the params_in_sync broadcast all go through RCCL."""
    env = dict(os.environ, INA_FORCE_DIST="1", OMP_NUM_THREADS="2")
    env.pop("INA_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "2", "--episodes-per-gpu", "64"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 1 and out["params_in_sync"] is True
    assert out["rccl_world"] == 1 and out["backend"] == "nccl"
    assert out["final_loss"] == out["final_loss"] and out["value"] > 0


def test_bench_self_launch_world2_one_gpu():
    """The driver's form, ``python bench.py --gpus 2`` with NO launcher: bench.py starts both ranks
    itself (before touching the GPU), both ranks share the one card (gloo collectives on CUDA
    tensors), and rank 0 reports the real collective world size."""
    env = dict(os.environ, INA_DIST_BACKEND="gloo", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "2",
           "--episodes-per-gpu", "64", "--launch-timeout", "100"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2 and out["backend"] == "gloo"
    assert out["params_in_sync"] is True and len(out["rank_ms_per_step"]) == 2


def test_bench_native_rccl_world1():
    """INA_COMM=native: the gradient all-reduce, params_in_sync broadcast and bucket paths on the C++ RCCL
    communicator (csrc/comm_bindings.cpp, its own HIP stream + events), gloo for the control plane."""
    env = dict(os.environ, INA_FORCE_DIST="1", INA_COMM="native", OMP_NUM_THREADS="2")
    env.pop("INA_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "3", "--warmup", "2", "--episodes-per-gpu", "64"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["comm"] == "rccl-native" and out["backend"] == "gloo" and out["rccl_world"] == 1
    assert out["params_in_sync"] is True and out["final_loss"] == out["final_loss"]


def test_native_comm_collectives_world1():
    """The communicator's ops in-process: all-reduce (sum / max), grouped buckets, broadcast, the
    stream ordering against the compute stream, async-error check."""
    import torch
    import torch.distributed as dist
    from induction_network_on_fewrel_amd.parallel.native_comm import NativeComm
    store = dist.TCPStore("127.0.0.1", _free_port(), 1, True)
    c = NativeComm(0, 1, torch.device("cuda", 0), store, tag="t")
    try:
        assert c.info()["world"] == 1
        x = torch.arange(1000, device="cuda", dtype=torch.float32)
        y = x * 2                       # produced on the compute stream right before the enqueue
        c.allreduce_(y)
        c.wait()
        z = y + 1                       # consumed after wait() on the compute stream
        assert torch.equal(z, x * 2 + 1)
        parts = [torch.full((n,), float(n), device="cuda") for n in (3, 7, 1 << 20)]
        c.allreduce_many_(parts)
        c.broadcast_(parts[0], 0)
        c.wait()
        assert all(bool((p == p.numel()).all()) for p in parts)
        c.allreduce_(y, "max")
        c.sync()
    finally:
        c.destroy()


def _json_objects(text):
    """Every top-level JSON object in the ranks' merged stdout (robust to lines of two ranks run together)."""
    dec, out, i = json.JSONDecoder(), [], text.find("{")
    while i >= 0:
        try:
            obj, end = dec.raw_decode(text, i)
        except json.JSONDecodeError:
            i = text.find("{", i + 1)
            continue
        if isinstance(obj, dict) and "rank" in obj:
            out.append(obj)
        i = text.find("{", end)
    return out


def _dp_check(nproc, extra_env):
    env = dict(os.environ, OMP_NUM_THREADS="2", **extra_env)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "tests", "dp_grad_check.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=140)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    rows = _json_objects(r.stdout)
    assert len(rows) == nproc, r.stdout
    for row in rows:
        print(row["rank"], row["comm"], f"{row['max_rel_err']:.2e}")
        assert row["finite"] and row["world"] == nproc and row["episodes_union"] == nproc * 384
        assert row["max_rel_err"] < 1e-3, row["per_param"]   # fp32 reduction order + bf16 rounding of the loss gradient
    return rows


def test_dp_gradient_equals_union_step_world2_gloo():
    """SURVEY 7.4 on the fused GPU path: two ranks on one card (gloo collectives on CUDA tensors), the
    relation-head span all-reduced under the encoder backward, slabs scattered by the step glue."""
    _dp_check(2, dict(INA_DIST_BACKEND="gloo"))


@pytest.mark.parametrize("comm", ["nccl", "native"])
def test_dp_gradient_equals_union_step_world1(comm):
    """The RCCL data planes (torch "nccl" and the native C++ communicator) at world 1: the in-place
    all-reduce of the overlapped head span must not write a stale bucket back over the flushed gradient."""
    env = dict(INA_FORCE_DIST="1")
    if comm == "native":
        env["INA_COMM"] = "native"
    os.environ.pop("INA_DIST_BACKEND", None)
    rows = _dp_check(1, env)
    assert rows[0]["comm"] == ("rccl-native" if comm == "native" else "nccl")
