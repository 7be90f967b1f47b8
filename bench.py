#!/usr/bin/env python3
"""Headline benchmark: whole-node training episodes/sec of the Induction Network on MI355X.

Metric / config (BASELINE.json): "episodes/sec (whole node)" on FewRel-shaped episodes,
default 5-way 5-shot, Q=5, max_length 37, BiLSTM u=20 + self-attention, 3 routing iterations,
NTN h=100, 5-d word table over a 400k vocabulary (the reference's train.py defaults), bf16 MFMA
compute with fp32 master weights, Adam with the reference's staircase LR.
Data: synthetic token sequences (64 relations x 700 instances, FewRel 1.0 train shape), random-init
weights -- no dataset or checkpoint downloads are possible here.

A timed step is the FULL training step: device episode sampling, forward, backward, RCCL
all-reduce of the flat gradient (N > 1), fused Adam update. Weak scaling: episodes per GPU fixed.

BERT configuration (BASELINE.json "FewRel 10-way 5-shot with BERT-base encoder"):
  python bench.py --encoder bert   (10-way 5-shot Q=5, BERT-base 12x768, L=128, 8 episodes/GPU)

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--episodes-per-gpu B] [--shot K]
Multi-GPU, either form:
  python bench.py --gpus N       (no launcher: this process starts N rank processes itself -- before it
                                  touches the GPU -- and exits non-zero if any rank fails or times out)
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
One process per GPU (LOCAL_RANK -> device), RCCL all-reduce ("nccl" backend) of the flat gradient.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv, timeout_s: float) -> int:
    """Start ``n`` rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set),
    forward rank 0's stdout, return non-zero if any rank fails or exceeds ``timeout_s``.

    Called before anything imports torch's GPU runtime: the parent never initialises HIP, so it
    is safe to fork/spawn the ranks (each rank then owns its device)."""
    import signal
    import subprocess
    import tempfile
    port = _free_port()
    out_file = tempfile.TemporaryFile(mode="w+")   # rank 0's stdout (a file: no pipe to fill up)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), INA_BENCH_CHILD="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env,
                                      stdout=out_file if r == 0 else subprocess.DEVNULL,
                                      start_new_session=True, text=True))
    t_end = time.time() + timeout_s
    rc = 0
    try:   # poll every rank: the first failure (or the deadline) ends the whole job
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            if time.time() > t_end:
                print(f"bench: ranks still running after {timeout_s:.0f}s, killing all", file=sys.stderr)
                rc = 124
                break
            time.sleep(0.2)
        rc = rc or next((p.returncode for p in procs if p.returncode), 0)
    finally:
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except ProcessLookupError:
                    pass
                p.wait()
    out_file.seek(0)
    sys.stdout.write(out_file.read())
    sys.stdout.flush()
    if rc != 0:
        print(f"bench: rank failure (exit codes {[p.returncode for p in procs]})", file=sys.stderr)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--encoder", default="bilstm", choices=["bilstm", "bert"])
    ap.add_argument("--episodes-per-gpu", type=int, default=0, help="default 8192 (bilstm: measured best of 2048..16384, ~3%% over 4096 and 13%% over 2048; peak_mem_gb in the output) / 8 (bert)")
    ap.add_argument("--way", type=int, default=0, help="default 5 (bilstm) / 10 (bert)")
    ap.add_argument("--shot", type=int, default=5)
    ap.add_argument("--query", type=int, default=5)
    ap.add_argument("--bert-layers", type=int, default=12)
    ap.add_argument("--bert-len", type=int, default=128)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--hidden", type=int, default=20)
    ap.add_argument("--word-dim", type=int, default=5, help="5 = reference train.py; paper config: --hidden 128 --word-dim 300")
    ap.add_argument("--profile-json", default="")
    ap.add_argument("--graph", type=int, default=-1,
                    help="capture the BiLSTM train step as a hipGraph: 1 always, 0 never, -1 auto (steps of <= 64 "
                         "episodes, Config.hip_graph_max_episodes)")
    ap.add_argument("--mode", default="train", choices=["train", "eval"],
                    help="eval: forward-only episodic evaluation (FewRel 2.0 style, dropout off, accuracy "
                         "computed); a step = one batch of --episodes-per-gpu episodes (default 16384)")
    ap.add_argument("--nota", type=float, default=0.0, help="eval: none-of-the-above query rate (FewRel 2.0)")
    ap.add_argument("--ragged", type=int, default=1,
                    help="length-sorted ragged tiles (forward direction + attention stop at each tile's longest "
                         "length; exact)")
    ap.add_argument("--skip-padding", type=int, default=0,
                    help="lstm_skip_padding: TF sequence_length semantics (NOT the reference's full-L BiLSTM)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: the oracle path (launcher / plumbing tests only; not a benchmark)")
    ap.add_argument("--launch-timeout", type=float, default=1500.0,
                    help="self-launched multi-rank run: kill every rank after this many seconds")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], args.launch_timeout))

    import torch
    from induction_network_on_fewrel_amd.config import Config
    from induction_network_on_fewrel_amd.data import make_synthetic
    from induction_network_on_fewrel_amd.parallel.dp import DistContext
    from induction_network_on_fewrel_amd.runtime.trainer import Trainer

    dist = DistContext.from_env(args.device)
    world = dist.world
    if world != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}")
    cuda = args.device == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)
    bert = args.encoder == "bert"
    evalm = args.mode == "eval"
    B = args.episodes_per_gpu or (8 if bert else (16384 if evalm else 8192))
    args.way = args.way or (10 if bert else 5)
    cfg = Config(N=args.way, K=args.shot, Q=args.query, max_length=37, hidden_size=args.hidden, dtype=args.dtype,
                 episodes_per_step=B, seed=1234, resume=False, model_dir="/tmp/ina_bench",
                 train_iter=args.steps + args.warmup, use_hip_graph=args.graph == 1 and not bert and not evalm,
                 hip_graph_max_episodes=64 if args.graph == -1 else 0,
                 nota_rate=args.nota, eval_batch=B, ragged_tiles=bool(args.ragged),
                 lstm_skip_padding=bool(args.skip_padding))
    if bert:
        cfg = cfg.replace(encoder="bert", bert_layers=args.bert_layers, bert_max_length=args.bert_len,
                          relation_head="reference")
    data = make_synthetic(num_relations=64, instances_per_relation=700, max_length=37, vocab=400000,
                          word_dim=args.word_dim, seed=0)
    if bert:   # random token ids over the BERT vocabulary, full-length sequences (worst case for L)
        import numpy as np
        from induction_network_on_fewrel_amd.data.bert_tokenize import synthetic_features
        f = synthetic_features(data, cfg.bert_vocab, cfg.bert_max_length)
        rng = np.random.default_rng(0)
        n = f["ids"].shape[0]
        f["ids"][:, 1:-1] = rng.integers(9, cfg.bert_vocab, (n, cfg.bert_max_length - 2), dtype=np.int32)
        f["mask"][:] = 1
        f["ids"][:, -1] = 3
        f["length"][:] = cfg.bert_max_length
        data.bert = f
    tr = Trainer(cfg, data, None, device=args.device, dist_ctx=dist, log=False)
    if evalm:
        tr.nota_threshold = 0.5 if args.nota > 0 else None

        def step():
            return tr.evaluate(B, batch=B), None
    else:
        step = tr.train_step_async
    for _ in range(args.warmup):
        step()
    sync()
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    loss_t = None
    for _ in range(args.steps):
        loss_t, _ = step()
    sync()
    dist.barrier()
    sync()
    dt_rank = time.perf_counter() - t0
    rank_ms = [round(1000 * float(x) / args.steps, 3) for x in dist.all_gather_objects(dt_rank)]
    dt = dist.max_scalar(dt_rank)
    loss = float(loss_t) if loss_t is not None else float("nan")
    # per-phase GPU time (HIP events at the phase boundaries of the eager train step: device sampling,
    # forward + backward (incl. the head-span all-reduce overlapped with it), the EXPOSED all-reduce tail,
    # optimizer), from a few extra steps AFTER the timed region; MAX over ranks per phase
    phase_ms = None
    if cuda and not evalm and not tr.graph_step_enabled:
        tr.cfg = tr.cfg.replace(profile=True)
        n_prof = max(1, min(5, args.steps))
        for _ in range(n_prof):
            tr.train_step_async()
        sync()
        ph = tr.drain_phase_events()
        phase_ms = {k: round(dist.max_scalar(v / n_prof), 3) for k, v in ph.items()}
    in_sync = dist.params_in_sync(tr.flat.flat)
    episodes = args.steps * B * world
    value = episodes / dt
    if dist.is_main:
        out = {
            "metric": "eval episodes/sec (whole node)" if evalm else "episodes/sec (whole node)",
            "value": round(value, 2),
            "unit": "episodes/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype if cuda else "fp32",
            "data": ("synthetic (64 relations x 700 instances, " +
                     (f"L={cfg.bert_max_length} full-length token ids over a {cfg.bert_vocab} vocab"
                      if bert else f"L=37, 400k vocab, {args.word_dim}-d word table") + "); random-init weights"),
            "config": {
                "model": (f"induction-network bert-base({cfg.bert_layers}x{cfg.bert_hidden}, {cfg.bert_heads} heads)"
                          f"+entity-pool->{cfg.bert_out_dim}, routing x3, ntn h=100" if bert else
                          f"induction-network bilstm(u={args.hidden})+self-attn, routing x3, ntn h=100"),
                "episode": f"{args.way}-way {args.shot}-shot Q={args.query}",
                "global_batch": B * world,
                "episodes_per_gpu": B,
                "seq_len": cfg.bert_max_length if bert else 37,
                "sentences_per_step_per_gpu": B * args.way * (args.shot + args.query),
                "parallelism": f"dp{world}",
                "mode": args.mode + (f", nota_rate={args.nota}" if evalm else ""),
                "lstm": ("sequence_length (lstm_skip_padding)" if args.skip_padding else
                         "full-L parity" + (", ragged tiles" if args.ragged else "")),
            },
            ("eval_accuracy" if evalm else "final_loss"): round(loss, 6),
            "params_in_sync": bool(in_sync),
            "rccl_world": (torch.distributed.get_world_size() if dist.initialized else 1),
            "backend": dist.backend or "none",
            "comm": dist.comm_name,
            "rank_ms_per_step": rank_ms,
            "phase_ms": phase_ms,
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2 ** 30, 2) if cuda else 0.0,
        }
        print(json.dumps(out))
        if args.profile_json:
            with open(args.profile_json, "w") as fh:
                json.dump(dict(out, timers=tr.timers), fh, indent=1)
    dist.destroy()


if __name__ == "__main__":
    main()
