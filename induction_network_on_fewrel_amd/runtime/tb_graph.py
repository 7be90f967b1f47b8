"""TensorBoard graph of the model (the reference hands ``sess.graph`` to its FileWriter,
/root/reference/model/base.py:125).

There is no TF graph here, so the GraphDef is written from the model's structure: the reference's
placeholders (input_words / input_pos1 / input_pos2 / mask_padding / query_label / keep_probx,
model/base.py:44-52), every variable under its checkpoint name (``VariableV2`` + ``/read``, dtype and shape
attributes), and the compute nodes under the reference's name scopes (embedding, EncoderModule,
InductionModule, RelationModule, loss; model/graph.py:30-89), each tagged with the kernel that runs it here
(attr ``_ina_kernel``).  TensorBoard's graph dashboard renders it like the reference's graph.

Proto fields (tensorflow/core/framework): GraphDef{node=1, versions=4}; NodeDef{name=1, op=2, input=3,
device=4, attr=5 (map<string, AttrValue>)}; AttrValue{s=2, i=3, type=6, shape=7}; TensorShapeProto{dim=2
{size=1}}; VersionDef{producer=1}; Event{graph_def=4}.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

from .metrics import _key, _ld, _varint

DT_FLOAT, DT_INT32 = 1, 3


def _shape(dims: Sequence[int]) -> bytes:
    return b"".join(_ld(2, _key(1, 0) + _varint(int(d) & ((1 << 64) - 1))) for d in dims)


def _attr(key: str, value: bytes) -> bytes:
    return _ld(5, _ld(1, key.encode()) + _ld(2, value))


def attr_type(t: int) -> bytes:
    return _key(6, 0) + _varint(t)


def attr_shape(dims: Sequence[int]) -> bytes:
    return _ld(7, _shape(dims))


def attr_str(s: str) -> bytes:
    return _ld(2, s.encode())


def attr_int(i: int) -> bytes:
    return _key(3, 0) + _varint(i)


def node(name: str, op: str, inputs: Sequence[str] = (), attrs: Optional[Dict[str, bytes]] = None,
         device: str = "") -> bytes:
    b = _ld(1, name.encode()) + _ld(2, op.encode())
    for i in inputs:
        b += _ld(3, i.encode())
    if device:
        b += _ld(4, device.encode())
    for k, v in (attrs or {}).items():
        b += _attr(k, v)
    return b


def graph_def(nodes: List[bytes], producer: int = 27) -> bytes:
    return b"".join(_ld(1, n) for n in nodes) + _ld(4, _key(1, 0) + _varint(producer))


def model_graph(model, N: int, K: int, Q: int) -> bytes:
    """GraphDef bytes of an InductionNetwork (BiLSTM or BERT encoder) training graph."""
    cfg = model.cfg
    names = model.params.names()
    L = cfg.max_length if cfg.encoder == "bilstm" else cfg.bert_max_length
    nodes: List[bytes] = []
    k = lambda s: {"_ina_kernel": attr_str(s)}  # noqa: E731

    def ph(name, dt, shape):
        nodes.append(node(name, "Placeholder", attrs={"dtype": attr_type(dt), "shape": attr_shape(shape)}))

    ph("input_words", DT_INT32, [-1, L])
    ph("input_pos1", DT_INT32, [-1, L])
    ph("input_pos2", DT_INT32, [-1, L])
    ph("mask_padding", DT_INT32, [-1, L])
    ph("query_label", DT_INT32, [-1])
    ph("keep_probx", DT_FLOAT, [])
    nodes.append(node("global_step", "VariableV2", attrs={"dtype": attr_type(9), "shape": attr_shape([])}))
    var = {}
    for attr, tfname in names.items():
        t = getattr(model.params, attr)
        nodes.append(node(tfname, "VariableV2", attrs={"dtype": attr_type(DT_FLOAT), "shape": attr_shape(t.shape)}))
        nodes.append(node(tfname + "/read", "Identity", [tfname], attrs={"T": attr_type(DT_FLOAT)}))
        var[attr] = tfname + "/read"
    H = int(model.params.head_dim)
    if cfg.encoder == "bilstm":
        nodes.append(node("embedding/embedding_lookup", "GatherV2", [var["word_embedding"], "input_words"],
                          k("x_gather (lstm.hip) / wide_x_gather (lstm_wide.hip)")))
        nodes.append(node("embedding/embedding_lookup_1", "GatherV2", [var["pos1_embedding"], "input_pos1"],
                          k("x_gather")))
        nodes.append(node("embedding/embedding_lookup_2", "GatherV2", [var["pos2_embedding"], "input_pos2"],
                          k("x_gather")))
        nodes.append(node("embedding/concat", "ConcatV2", ["embedding/embedding_lookup", "embedding/embedding_lookup_1",
                                                           "embedding/embedding_lookup_2"], k("x_gather")))
        for d in ("fw", "bw"):
            nodes.append(node(f"EncoderModule/bidirectional_rnn/{d}/{d}/while", "BasicLSTMCell",
                              ["embedding/concat", var[f"lstm_{d}_kernel"], var[f"lstm_{d}_bias"], "keep_probx"],
                              k("lstm_fwd / lstm_bwd (lstm.hip) or lstm_wide_seq_fwd / _bwd (lstm_wide.hip)")))
        nodes.append(node("EncoderModule/concat", "ConcatV2", ["EncoderModule/bidirectional_rnn/fw/fw/while",
                                                               "EncoderModule/bidirectional_rnn/bw/bw/while"]))
        nodes.append(node("EncoderModule/self_attn/attention", "SelfAttention",
                          ["EncoderModule/concat", "mask_padding", var["attn_kernel"], var["attn_bias"],
                           var["attn_w2"]], k("rec_attn_fwd / _bwd (rec_attn.hip) or wide_attn (attn_wide.hip)")))
        enc = "EncoderModule/self_attn/attention"
    else:
        nodes.append(node("EncoderModule/bert", "BertEncoder", ["input_words", "mask_padding"],
                          k("bert.hip (embed / LN / MHA / bias+GELU) + hipBLASLt or gemm.hip GEMMs")))
        proj = [var[a] for a in ("bert__bert_proj__kernel", "bert__bert_proj__bias") if a in var]
        nodes.append(node("EncoderModule/bert_proj", "MatMul", ["EncoderModule/bert"] + proj))
        enc = "EncoderModule/bert_proj"
    shape = {"N": attr_int(N), "K": attr_int(K), "Q": attr_int(Q), "H": attr_int(H)}
    nodes.append(node("EncoderModule/support", "StridedSlice", [enc], shape))
    nodes.append(node("EncoderModule/query", "StridedSlice", [enc], shape))
    prev = "EncoderModule/support"
    for r in range(cfg.routing_iters):
        nm = f"InductionModule/iter_{r}/squash"
        nodes.append(node(nm, "DynamicRouting", [prev, var["W_s"]], k("routing_fwd / _bwd (routing.hip)")))
        prev = nm
    nodes.append(node("RelationModule/ntn", "NeuralTensorLayer", [prev, "EncoderModule/query", var["M"]],
                      k("ntn_fwd / ntn_bwd (ntn.hip)")))
    nodes.append(node("RelationModule/fc", "MatMul", ["RelationModule/ntn", var["ntn_w"]], k("ntn.hip epilogue")))
    nodes.append(node("RelationModule/probs", "Sigmoid", ["RelationModule/fc", var["ntn_b"]], k("ntn.hip epilogue")))
    loss_op = "SoftmaxCrossEntropy" if cfg.loss_type != "mse" else "MeanSquaredError"
    nodes.append(node("loss/loss", loss_op, ["RelationModule/probs", "query_label"], k("head_loss (glue.hip)")))
    nodes.append(node("predictions", "ArgMax", ["RelationModule/probs"]))
    nodes.append(node("accuracy", "Mean", ["predictions", "query_label"]))
    opt = "Adam" if cfg.optimizer == "adam" else "Adagrad"
    nodes.append(node(f"OptimizeLoss/{opt}", "ApplyFused" + opt, ["loss/loss", "global_step"] + list(var.values()),
                      k("adam / adagrad (optim.hip) over the flat parameter buffer")))
    return graph_def(nodes)


# ------------------------------------------------------------------ MetaGraphDef (<stem>.meta)
def _var_def(name: str, trainable: bool) -> bytes:
    """VariableDef{variable_name=1, initializer_name=2, snapshot_name=3, initial_value_name=6, trainable=7}."""
    return (_ld(1, f"{name}:0".encode()) + _ld(2, f"{name}/Assign".encode()) + _ld(3, f"{name}/read:0".encode()) +
            _ld(6, f"{name}/Initializer:0".encode()) + (_key(7, 0) + _varint(1) if trainable else b""))


def _collection(name: str, kind: int, values: Sequence[bytes]) -> bytes:
    """map<string, CollectionDef> entry; CollectionDef{node_list=1 | bytes_list=2 {value=1}}."""
    inner = b"".join(_ld(1, v) for v in values)
    return _ld(4, _ld(1, name.encode()) + _ld(2, _ld(kind, inner)))


def meta_graph(model, N: int, K: int, Q: int, max_to_keep: int = 5) -> bytes:
    """Serialized DESCRIPTIVE MetaGraphDef in the place ``tf.train.Saver.save`` writes one
    (/root/reference/model/base.py:124,177).  It is not importable by ``tf.train.import_meta_graph``: the compute
    nodes carry this framework's op types (BasicLSTMCell, SelfAttention, DynamicRouting, ... -- each tagged with the
    kernel that runs it), the SaveV2 / RestoreV2 nodes lack TF's tensor_names / shape_and_slices inputs and dtypes
    attrs, and the variables collection lists the parameters and global_step only (the bundle also holds the
    optimizer slots <var>/Adam, <var>/Adam_1 or /Adagrad and beta1_power / beta2_power).  Contents:
    meta_info_def {meta_graph_version "v0", tags}, the model's
    GraphDef plus the Saver's nodes (save/Const filename, save/SaveV2, save/control_dependency,
    save/RestoreV2, save/Assign_i, save/restore_all), a V2 SaverDef (tensor / op names as TF1's Saver names
    them, max_to_keep, keep_checkpoint_every_n_hours 10000) and the variables / trainable_variables /
    train_op / global_step collections (VariableDef entries under the checkpoint's variable names).
    Parity with TF's own bytes is unpinned (TF is not installed); tests/test_tf_bundle.py parses it back.

    Fields (tensorflow/core/protobuf/meta_graph.proto, saver.proto): MetaGraphDef{meta_info_def=1,
    graph_def=2, saver_def=3, collection_def=4}; MetaInfoDef{meta_graph_version=1, tags=4,
    tensorflow_version=5}; SaverDef{filename_tensor_name=1, save_tensor_name=2, restore_op_name=3,
    max_to_keep=4, sharded=5, keep_checkpoint_every_n_hours=6 (float), version=7 (V2 = 2)}."""
    import struct
    g = model_graph(model, N, K, Q)
    prm = model.params
    names = [prm.tf_name(a) for a in prm.names()]
    trainable = {prm.tf_name(a) for a in prm.trainable()}
    save_nodes = [node("save/Const", "Const", attrs={"dtype": _key(6, 0) + _varint(7)})]   # DT_STRING
    save_nodes.append(node("save/SaveV2", "SaveV2", ["save/Const"] + [f"{n}" for n in names] + ["global_step"]))
    save_nodes.append(node("save/control_dependency", "Identity", ["save/Const", "^save/SaveV2"]))
    save_nodes.append(node("save/RestoreV2", "RestoreV2", ["save/Const"]))
    for i, n in enumerate(names + ["global_step"]):
        save_nodes.append(node(f"save/Assign_{i}" if i else "save/Assign", "Assign", [n, f"save/RestoreV2:{i}"]))
    save_nodes.append(node("save/restore_all", "NoOp",
                           [f"^save/Assign_{i}" if i else "^save/Assign" for i in range(len(names) + 1)]))
    g = g + b"".join(_ld(1, n) for n in save_nodes)
    info = _ld(1, b"v0") + _ld(4, b"train") + _ld(5, b"ina-mi355x (TF1 layout)")
    saver = (_ld(1, b"save/Const:0") + _ld(2, b"save/control_dependency:0") + _ld(3, b"save/restore_all") +
             _key(4, 0) + _varint(int(max_to_keep)) + _key(6, 5) + struct.pack("<f", 10000.0) + _key(7, 0) + _varint(2))
    var_all = [_var_def(n, n in trainable) for n in names] + [_var_def("global_step", False)]
    var_tr = [_var_def(n, True) for n in names if n in trainable]
    opt = "Adam" if model.cfg.optimizer == "adam" else "Adagrad"
    return (_ld(1, info) + _ld(2, g) + _ld(3, saver) +
            _collection("global_step", 2, [_var_def("global_step", False)]) +
            _collection("train_op", 1, [f"OptimizeLoss/{opt}".encode()]) +
            _collection("trainable_variables", 2, var_tr) +
            _collection("variables", 2, var_all))


def parse_meta_graph(b: bytes) -> dict:
    """Minimal MetaGraphDef reader (tests): -> {meta_info: raw, nodes: parse_graph(...), saver: {field: value},
    collections: {name: (kind, [values])}}."""
    import struct
    from .metrics import _read_varint

    def fields(buf):
        i, out = 0, []
        while i < len(buf):
            key, i = _read_varint(buf, i)
            f, wt = key >> 3, key & 7
            if wt == 0:
                v, i = _read_varint(buf, i)
            elif wt == 5:
                v = struct.unpack_from("<f", buf, i)[0]
                i += 4
            else:
                ln, i = _read_varint(buf, i)
                v = buf[i:i + ln]
                i += ln
            out.append((f, v))
        return out

    res = {"nodes": [], "saver": {}, "collections": {}, "meta_info": b""}
    for f, v in fields(b):
        if f == 1:
            res["meta_info"] = v
        elif f == 2:
            res["nodes"] = parse_graph(v)
        elif f == 3:
            res["saver"] = dict(fields(v))
        elif f == 4:
            ent = dict(fields(v))
            (kind, inner), = fields(ent[2])
            res["collections"][ent[1].decode()] = (kind, [x for _, x in fields(inner)])
    return res


def parse_graph(b: bytes) -> List[dict]:
    """Minimal GraphDef reader (tests): -> [{name, op, inputs, attrs: {key: raw bytes}}]."""
    from .metrics import _read_varint
    out = []
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        ln, i = _read_varint(b, i)
        sub = b[i:i + ln]
        i += ln
        if key >> 3 != 1:
            continue
        nd = {"name": "", "op": "", "inputs": [], "attrs": {}}
        j = 0
        while j < len(sub):
            kk, j = _read_varint(sub, j)
            l2, j = _read_varint(sub, j)
            val = sub[j:j + l2]
            j += l2
            f = kk >> 3
            if f == 1:
                nd["name"] = val.decode()
            elif f == 2:
                nd["op"] = val.decode()
            elif f == 3:
                nd["inputs"].append(val.decode())
            elif f == 5:
                t = 0
                k3, t = _read_varint(val, t)
                l3, t = _read_varint(val, t)
                akey = val[t:t + l3].decode()
                t += l3
                k4, t = _read_varint(val, t)
                l4, t = _read_varint(val, t)
                nd["attrs"][akey] = val[t:t + l4]
        out.append(nd)
    return out


def read_graph(path: str) -> List[dict]:
    """The nodes of the first graph_def event in an event file written by metrics.EventWriter."""
    import struct
    from .metrics import _read_varint
    with open(path, "rb") as fh:
        data = fh.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        ev = data[i + 12:i + 12 + n]
        i += 16 + n
        j = 0
        while j < len(ev):
            key, j = _read_varint(ev, j)
            wt = key & 7
            if wt == 0:
                _, j = _read_varint(ev, j)
            elif wt == 1:
                j += 8
            elif wt == 5:
                j += 4
            else:
                ln, j = _read_varint(ev, j)
                if key >> 3 == 4:
                    return parse_graph(ev[j:j + ln])
                j += ln
    return []
