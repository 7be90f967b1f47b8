"""Single configuration object for the whole engine.

Every knob of the reference is exposed here with the reference's default:

* episode shape N/K/Q and the CLI defaults    -- ``train.py:10-18,24,31-37``
* model hyper-parameters (``Base.__init__``)  -- ``model/base.py:12-27``
* routing iterations / NTN slices             -- ``model/layer_module.py:8,101``
* train-loop cadence                          -- ``model/base.py:115-116``
* GloVe truncation width                      -- ``util/convert_glove_vec.py:3``

Additions beyond the reference (north star): episode batching, dtype, DP, encoder
choice, relation-head variant, NOTA rate, L2 opt-in, LR-schedule choice.
"""
from __future__ import annotations

import dataclasses
import json
from dataclasses import dataclass, field
from typing import Optional


@dataclass
class Config:
    # ---------------- episode shape (train.py:11-12, :33) ----------------
    model_name: str = "induction"
    N: int = 5                 # ways
    K: int = 2                 # shots
    Q: int = 5                 # queries per class
    # optional eval-time overrides (None -> same as train)
    eval_N: Optional[int] = None
    eval_K: Optional[int] = None
    eval_Q: Optional[int] = None

    # ---------------- data (train.py:24-27) ----------------
    max_length: int = 37
    train_file: str = "./data/train.json"
    val_file: str = "./data/val.json"
    word_vec_file: str = "./data/glove.6B.5d.json"
    case_sensitive: bool = False
    processed_dir: str = "_processed_data"
    synthetic: bool = False            # synthetic tokens / random relations
    synthetic_relations: int = 64
    synthetic_instances: int = 700
    synthetic_vocab: int = 400000
    synthetic_word_dim: int = 5
    synthetic_task: str = "lexical"    # "lexical": per-relation trigger words anywhere (benchmarks); "transfer":
                                       # relation-disjoint train / val / test splits, relations told apart only by
                                       # the span between the entities (data/synthetic.py::make_transfer_splits)
    synthetic_val_relations: int = 8   # transfer task: validation (checkpoint selection) relations
    synthetic_test_relations: int = 8  # transfer task: held-out test relations

    # ---------------- model (model/base.py:12-27, train.py:31-37) ----------------
    hidden_size: int = 20              # LSTM units per direction (u); BiLSTM out = 2u
    pos_embedding_dim: int = 5         # fixed in reference (base.py:24)
    init_std: float = 0.1              # tf.random_normal_initializer(stddev=0.1)
    keep_prob: float = 0.9             # DropoutWrapper output_keep_prob (train)
    routing_iters: int = 3             # dynamic_routing(iter_routing=3)
    ntn_slices: int = 100              # neural_tensor_layer(out_size=100)
    relation_head: str = "reference"   # "reference": W[h*N, N] mixes classes; "paper": per-pair W_r in R^h
    encoder: str = "bilstm"            # "bilstm" | "bert"
    lstm_skip_padding: bool = False    # parity: process all L steps; True: TF sequence_length
                                       # semantics (fw stops at length, bw starts at length - 1)
    ragged_tiles: bool = True          # GPU bf16: length-sorted 16-row tiles; the fw direction and the attention
                                       # stop at each tile's longest length (exact: padding is masked)
    lstm_impl: str = "auto"            # GPU BiLSTM: "fused" (lane-ownership kernel, u<=32) | "wide" (GEMM + cell kernels) | "auto"
    train_word_embedding: bool = False # only used when no pretrained table is given

    # BERT encoder (north star); BERT-base defaults
    bert_layers: int = 12
    bert_hidden: int = 768
    bert_heads: int = 12
    bert_intermediate: int = 3072
    bert_vocab: int = 30522
    bert_max_position: int = 512
    bert_max_length: int = 128         # tokens per sentence incl. [CLS]/[SEP]/entity markers
    bert_pool: str = "entity"          # "entity": concat([E1], [E2]) states | "cls"
    bert_out_dim: int = 64             # sentence-vector width fed to routing / NTN (fused kernels: 16/40/64)
    bert_dropout: float = 0.1          # hidden dropout (embeddings, attention output, FFN output)
    bert_attn_dropout: float = 0.1     # attention-probability dropout
    bert_vocab_file: str = ""          # WordPiece vocab.txt; empty = word-level vocab from the data
    bert_checkpoint: str = ""          # local HF checkpoint dir (model.safetensors / pytorch_model.bin)

    # ---------------- optimisation (model/base.py:94-99) ----------------
    optimizer: str = "adam"            # "adam" (reference) | "adagrad" (paper 4.4)
    learning_rate: float = 1e-3
    decay_steps: int = 100
    decay_rate: float = 0.9
    staircase: bool = True
    lr_schedule: str = "exponential"   # "exponential" (reference) | "constant"
    adam_beta1: float = 0.9
    adam_beta2: float = 0.999
    adam_eps: float = 1e-8
    adagrad_init_acc: float = 0.1
    l2_lambda: float = 1e-5
    use_l2: bool = False               # reference computes then discards it (graph.py:108-109)
    loss_reduction: str = "mean"       # "mean" (reference) | "sum" (paper Eq.12)
    loss_type: str = "mse"             # "mse" on sigmoid scores (reference) | "ce": softmax over the N scores |
                                       # "ce_nota": softmax over the N scores + a NOTA class of logit 0 (train
                                       # with nota_rate > 0: FewRel 2.0)

    # ---------------- loop cadence (model/base.py:115-116) ----------------
    train_iter: int = 30000
    val_iter: int = 1000
    val_step: int = 2000
    test_iter: int = 3000
    log_every: int = 100
    model_dir: str = "checkpoints/inductionNetwork_test"
    ckpt_name: str = "inductionNetwork"
    max_to_keep: int = 5
    tf_checkpoint: bool = True         # also write the TF V2 bundle (.index / .data) + .meta next to safetensors
    resume: bool = True

    # ---------------- execution ----------------
    episodes_per_step: int = 1         # B episodes per optimiser step (per rank)
    dtype: str = "bf16"                # MFMA operand dtype on GPU: "bf16" | "fp32"
    device: str = "auto"               # "auto" | "cuda" | "cpu"
    seed: int = 12345
    deterministic: bool = False        # seeds + torch deterministic algorithms (utils/seeding.py); the fused
                                       # GPU path is deterministic regardless (ordered reductions)
    use_hip_graph: bool = False        # replay the BiLSTM train step as one captured hipGraph (runtime/graph.py)
    hip_graph_max_episodes: int = 64   # ... and by default whenever episodes_per_step <= this (launch-bound small
                                       # steps, e.g. the reference's 1 episode per step); 0 = only use_hip_graph
    step_glue: bool = True             # GPU BiLSTM: one-launch packs / loss / gradient scatter (ops/glue.py)
    nota_rate: float = 0.0             # FewRel 2.0 none-of-the-above probability per query
    eval_nota_rate: float = -1.0       # NOTA rate of val/test episodes (-1: same as nota_rate)
    nota_threshold: float = -1.0       # best-score threshold for predicting NOTA (-1: tuned on val when NOTA > 0)
    eval_batch: int = 0                # episodes per eval forward (0: episodes_per_step); sized for HBM
    test_file: str = ""                # final test set (e.g. another domain for FewRel 2.0 DA); empty = val
    test_best: bool = False            # final test from the best-val checkpoint (reference: the last weights)
    grad_check_finite: bool = True     # NaN/Inf guard on the loss
    profile: bool = False              # per-phase GPU time (HIP events) into metrics.jsonl at log points
    # optimize_loss summaries (model/base.py:98,113; tf.contrib.layers.optimize_loss's default list is
    # loss, learning_rate, global_gradient_norm); add "gradient_norm" for one norm per variable
    summaries: str = "loss,learning_rate,global_gradient_norm"
    watchdog_s: float = 0.0            # abort (traceback + exit) if one train step takes longer (0 = off)
    save_every: int = 0                # periodic checkpoints for restart-resume (reference: best-val only)

    # ------------------------------------------------------------------
    @property
    def H(self) -> int:
        return 2 * self.hidden_size

    @property
    def eN(self) -> int:
        return self.eval_N or self.N

    @property
    def eK(self) -> int:
        return self.eval_K or self.K

    @property
    def eQ(self) -> int:
        return self.eval_Q or self.Q

    def replace(self, **kw) -> "Config":
        return dataclasses.replace(self, **kw)

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    def to_json(self) -> str:
        return json.dumps(self.to_dict(), sort_keys=True)

    @classmethod
    def from_dict(cls, d: dict) -> "Config":
        names = {f.name for f in dataclasses.fields(cls)}
        return cls(**{k: v for k, v in d.items() if k in names})

    def validate(self) -> None:
        if self.N < 1 or self.K < 1 or self.Q < 1:
            raise ValueError("N, K, Q must be >= 1")
        if self.hidden_size < 1:
            raise ValueError("hidden_size must be >= 1 (widths between the kernel instantiations run zero-padded, "
                             "models/padding.py)")
        if self.relation_head not in ("reference", "paper"):
            raise ValueError(f"unknown relation_head {self.relation_head}")
        if self.dtype not in ("bf16", "fp32"):
            raise ValueError(f"unknown dtype {self.dtype}")
        if self.loss_type not in ("mse", "ce", "ce_nota"):
            raise ValueError(f"unknown loss_type {self.loss_type}")
        if self.optimizer not in ("adam", "adagrad"):
            raise ValueError(f"unknown optimizer {self.optimizer}")
        if self.encoder not in ("bilstm", "bert"):
            raise ValueError(f"unknown encoder {self.encoder}")
        if self.synthetic_task not in ("lexical", "transfer"):
            raise ValueError(f"unknown synthetic_task {self.synthetic_task}")
        if self.encoder == "bert":
            if self.bert_hidden % self.bert_heads != 0 or self.bert_hidden // self.bert_heads != 64:
                raise ValueError("BERT heads must be 64 wide (bert_hidden = 64 * bert_heads)")
            if self.bert_pool not in ("entity", "cls"):
                raise ValueError(f"unknown bert_pool {self.bert_pool}")
            if self.bert_max_length > min(128, self.bert_max_position):
                raise ValueError("bert_max_length must be <= 128 (fused attention keeps the sequence in LDS)")


def add_cli_args(p) -> None:
    """Register every Config field as ``--field`` on an argparse parser."""
    for f in dataclasses.fields(Config):
        default = f.default if f.default is not dataclasses.MISSING else None
        flag = "--" + f.name
        if isinstance(default, bool):
            p.add_argument(flag, type=lambda s: s.lower() in ("1", "true", "yes", "y"), default=None,
                           metavar="BOOL")
        elif default is None:
            p.add_argument(flag, type=int if f.name.startswith("eval_") else str, default=None)
        else:
            p.add_argument(flag, type=type(default), default=None)


def config_from_args(args, base: Optional[Config] = None) -> Config:
    cfg = base or Config()
    kw = {}
    for f in dataclasses.fields(Config):
        v = getattr(args, f.name, None)
        if v is not None:
            kw[f.name] = v
    return cfg.replace(**kw)
