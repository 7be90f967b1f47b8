"""TensorFlow V2 checkpoint bundle (``tf.train.Saver`` / ``BundleWriter`` format) written and read without TF.

The reference saves with ``tf.train.Saver().save(sess, <dir>/checkpoint/inductionNetwork, global_step)``
(``model/base.py:124,173-177``), which produces

* ``inductionNetwork-<step>.index`` -- an SSTable (LevelDB table format as in TF's ``core/lib/io/table``):
  key ``""`` -> ``BundleHeaderProto`` {num_shards: 1, endianness: LITTLE, version {producer: 1}}, then one
  ``BundleEntryProto`` per tensor name {dtype, shape, shard_id, offset, size, crc32c (masked)}, keys in
  bytewise order; blocks = prefix-compressed entries + restart array + (type byte, masked CRC32C);
  metaindex and index blocks; a 48-byte footer ending in the table magic 0xdb4775248b80fb57;
* ``inductionNetwork-<step>.data-00000-of-00001`` -- the tensors' raw little-endian bytes back to back;
* ``inductionNetwork-<step>.meta`` -- the serialized MetaGraphDef (runtime/tb_graph.py::meta_graph): the
  model's GraphDef (the same one the summary writer puts in the event file) with the Saver's save / restore
  nodes, a V2 SaverDef and the variables / trainable_variables / train_op / global_step collections.

The tensor keys are the reference's TF variable names, so a TF ``CheckpointReader`` sees the
same variables, shapes and dtypes.  Parity with TensorFlow itself is unpinned (TF is not installed and
the reference ships no checkpoint); tests/test_tf_bundle.py checks the format's invariants (footer
magic, handles, block and tensor CRCs, header / entry protos) byte-exactly on a round trip.
"""
from __future__ import annotations

import os
import struct
from collections import OrderedDict
from typing import Dict, List, Tuple

import torch

TABLE_MAGIC = 0xDB4775248B80FB57
FOOTER_LEN = 48           # 2 BlockHandles padded to 2 * 20 bytes + 8-byte magic
BLOCK_SIZE = 262144       # TF table::Options default block_size (TensorBundle keeps it)
RESTART_INTERVAL = 16     # table::Options default block_restart_interval
DATA_SUFFIX = ".data-00000-of-00001"

# tensorflow/core/framework/types.proto
_DT = {torch.float32: 1, torch.float64: 2, torch.int32: 3, torch.uint8: 4, torch.int16: 5, torch.int8: 6,
       torch.int64: 9, torch.bool: 10, torch.bfloat16: 14, torch.float16: 19}
_DT_INV = {v: k for k, v in _DT.items()}


# ------------------------------------------------------------------ CRC32C
_CRC_WARNED = False


def crc32c(data, crc: int = 0) -> int:
    """CRC-32C of a bytes-like object; the host-only native module (csrc/host/ina_host.c, no torch / HIP
    dependency) when it is built, else a table loop."""
    global _CRC_WARNED
    try:
        from .. import _ina_host
        return _ina_host.crc32c(data, crc)
    except ImportError:
        if not _CRC_WARNED:
            _CRC_WARNED = True
            import warnings
            warnings.warn("ina: the host CRC32C extension is not built (python csrc/build.py --host); checkpoint "
                          "CRCs use the per-byte Python loop (slow for large bundles)")
    from .metrics import _TABLE
    c = crc ^ 0xFFFFFFFF
    for b in bytes(data):
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def mask(c: int) -> int:
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def unmask(m: int) -> int:
    r = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((r >> 17) | (r << 15)) & 0xFFFFFFFF


# ------------------------------------------------------------------ protobuf wire format
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _get_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = r = 0
    while True:
        x = b[i]
        i += 1
        r |= (x & 0x7F) << shift
        if not x & 0x80:
            return r, i
        shift += 7


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v) if v else b""   # proto3: defaults are not serialized


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def _parse(b: bytes) -> Dict[int, list]:
    """Generic proto parse -> {field: [values]} (varints as int, length-delimited as bytes, fixed32/64 as int)."""
    out: Dict[int, list] = {}
    i = 0
    while i < len(b):
        tag, i = _get_varint(b, i)
        num, wt = tag >> 3, tag & 7
        if wt == 0:
            v, i = _get_varint(b, i)
        elif wt == 2:
            n, i = _get_varint(b, i)
            v, i = b[i:i + n], i + n
        elif wt == 5:
            v, i = struct.unpack_from("<I", b, i)[0], i + 4
        elif wt == 1:
            v, i = struct.unpack_from("<Q", b, i)[0], i + 8
        else:
            raise ValueError(f"unsupported wire type {wt}")
        out.setdefault(num, []).append(v)
    return out


def header_proto() -> bytes:
    """BundleHeaderProto{num_shards: 1, endianness: LITTLE (0, default), version: VersionDef{producer: 1}}."""
    return _field_varint(1, 1) + _field_bytes(3, _field_varint(1, 1))


def entry_proto(dtype: int, shape, offset: int, size: int, crc_masked: int) -> bytes:
    dims = b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)
    return (_field_varint(1, dtype) + _field_bytes(2, dims) + _field_varint(4, offset) + _field_varint(5, size)
            + _varint((6 << 3) | 5) + struct.pack("<I", crc_masked))


def parse_entry(b: bytes) -> dict:
    f = _parse(b)
    shape = []
    for dim in _parse(f.get(2, [b""])[0]).get(2, []):
        shape.append(_parse(dim).get(1, [0])[0])
    return dict(dtype=f.get(1, [0])[0], shape=shape, shard_id=f.get(3, [0])[0], offset=f.get(4, [0])[0],
                size=f.get(5, [0])[0], crc32c=f.get(6, [0])[0])


# ------------------------------------------------------------------ SSTable
def _block(entries: List[Tuple[bytes, bytes]]) -> bytes:
    """One table block: prefix-compressed entries, restart offsets every RESTART_INTERVAL entries."""
    out = bytearray()
    restarts, last = [], b""
    for k, (key, val) in enumerate(entries):
        if k % RESTART_INTERVAL == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(last), len(key)) and last[shared] == key[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(key) - shared) + _varint(len(val)) + key[shared:] + val
        last = key
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _handle(offset: int, size: int) -> bytes:
    return _varint(offset) + _varint(size)


def _write_block(f, contents: bytes) -> Tuple[int, int]:
    off = f.tell()
    f.write(contents)
    f.write(b"\x00" + struct.pack("<I", mask(crc32c(contents + b"\x00"))))   # kNoCompression + crc
    return off, len(contents)


def write_table(path: str, items: List[Tuple[bytes, bytes]]) -> None:
    items = sorted(items, key=lambda kv: kv[0])
    with open(path, "wb") as f:
        index, cur, cur_bytes = [], [], 0
        for kv in items:
            cur.append(kv)
            cur_bytes += len(kv[0]) + len(kv[1]) + 8
            if cur_bytes >= BLOCK_SIZE:
                off, n = _write_block(f, _block(cur))
                index.append((cur[-1][0], _handle(off, n)))   # separator: the block's last key (>= all its keys)
                cur, cur_bytes = [], 0
        if cur:
            off, n = _write_block(f, _block(cur))
            index.append((cur[-1][0], _handle(off, n)))
        meta_off, meta_n = _write_block(f, _block([]))
        idx_off, idx_n = _write_block(f, _block(index))
        footer = _handle(meta_off, meta_n) + _handle(idx_off, idx_n)
        footer += b"\x00" * (40 - len(footer)) + struct.pack("<Q", TABLE_MAGIC)
        f.write(footer)


def _read_block(buf: bytes, off: int, n: int) -> List[Tuple[bytes, bytes]]:
    contents = buf[off:off + n]
    typ = buf[off + n]
    crc = struct.unpack_from("<I", buf, off + n + 1)[0]
    if typ != 0:
        raise ValueError("compressed table blocks are not supported")
    if unmask(crc) != crc32c(contents + bytes([typ])):
        raise ValueError(f"block CRC mismatch at offset {off}")
    nres = struct.unpack_from("<I", contents, n - 4)[0]
    end = n - 4 - 4 * nres
    out, i, last = [], 0, b""
    while i < end:
        shared, i = _get_varint(contents, i)
        nonshared, i = _get_varint(contents, i)
        vlen, i = _get_varint(contents, i)
        key = last[:shared] + contents[i:i + nonshared]
        i += nonshared
        out.append((key, contents[i:i + vlen]))
        i += vlen
        last = key
    return out


def read_table(path: str) -> "OrderedDict[bytes, bytes]":
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < FOOTER_LEN or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != TABLE_MAGIC:
        raise ValueError(f"{path}: not an SSTable (bad footer magic)")
    foot = buf[len(buf) - FOOTER_LEN:]
    _, i = _get_varint(foot, 0)
    _, i = _get_varint(foot, i)
    idx_off, i = _get_varint(foot, i)
    idx_n, i = _get_varint(foot, i)
    out = OrderedDict()
    for _, h in _read_block(buf, idx_off, idx_n):
        off, j = _get_varint(h, 0)
        n, _ = _get_varint(h, j)
        for k, v in _read_block(buf, off, n):
            out[k] = v
    return out


# ------------------------------------------------------------------ bundle
def save_bundle(prefix: str, tensors: "OrderedDict[str, torch.Tensor]") -> None:
    """Write ``prefix.index`` + ``prefix.data-00000-of-00001`` (names sorted, data in key order)."""
    items, off = [(b"", header_proto())], 0
    tmp_data = prefix + DATA_SUFFIX + ".tmp"
    with open(tmp_data, "wb") as f:
        for name in sorted(tensors):
            t = tensors[name].detach().to("cpu").contiguous()
            if t.dtype not in _DT:
                raise TypeError(f"{name}: dtype {t.dtype} has no TF DataType here")
            raw = t.reshape(-1).view(torch.uint8).numpy() if t.numel() else b""   # no copy (buffer protocol)
            f.write(raw)
            items.append((name.encode(), entry_proto(_DT[t.dtype], list(t.shape), off, len(raw), mask(crc32c(raw)))))
            off += len(raw)
    write_table(prefix + ".index.tmp", items)
    os.replace(tmp_data, prefix + DATA_SUFFIX)
    os.replace(prefix + ".index.tmp", prefix + ".index")


def load_bundle(prefix: str, verify: bool = True) -> "OrderedDict[str, torch.Tensor]":
    table = read_table(prefix + ".index")
    hdr = _parse(table.get(b"", b""))
    if hdr.get(1, [1])[0] != 1:
        raise ValueError("multi-shard bundles are not supported")
    if hdr.get(2, [0])[0] != 0:
        raise ValueError("big-endian bundles are not supported")
    with open(prefix + DATA_SUFFIX, "rb") as f:
        data = f.read()
    out = OrderedDict()
    for k, v in table.items():
        if k == b"":
            continue
        e = parse_entry(v)
        raw = data[e["offset"]:e["offset"] + e["size"]]
        if verify and unmask(e["crc32c"]) != crc32c(raw):
            raise ValueError(f"{k.decode()}: tensor CRC mismatch")
        dt = _DT_INV[e["dtype"]]
        arr = torch.frombuffer(bytearray(raw), dtype=dt) if raw else torch.empty(0, dtype=dt)
        out[k.decode()] = arr.reshape(e["shape"]).clone()
    return out


def exists(prefix: str) -> bool:
    return os.path.exists(prefix + ".index") and os.path.exists(prefix + DATA_SUFFIX)

