"""Structured metrics: JSONL + a dependency-free TensorBoard event-file writer.

Reference (model/base.py:109-113,125,155): scalar summaries ``loss``, ``accuracy``, ``learning_rate``
written every train step to ``<model_dir>/train`` via ``tf.summary.FileWriter``, merged with the
summaries ``optimize_loss`` registers (model/base.py:98,113: ``global_norm/gradient_norm``, and per
variable ``gradient_norm/<var>`` when asked for; Config.summaries). TensorBoard is not
installed here, so the event file is produced directly: TFRecord framing (length, masked CRC32C of
the length, payload, masked CRC32C of the payload) around hand-encoded ``Event`` protos
(wall_time=1:double, step=2:int64, file_version=3:string, summary=5:{value=1:{tag=1, simple_value=2}}).
Only rank 0 writes.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Dict, Optional

# ------------------------------------------------------------------ CRC32C (Castagnoli)
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    try:
        from .. import _ina_host   # host-only native CRC32C (csrc/host/ina_host.c)
        return _ina_host.crc32c(data)
    except ImportError:
        pass
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ------------------------------------------------------------------ protobuf encoding
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


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _ld(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_event(step: int, wall_time: float, scalars: Optional[Dict[str, float]] = None,
                 file_version: Optional[str] = None) -> bytes:
    ev = _key(1, 1) + struct.pack("<d", wall_time) + _key(2, 0) + _varint(int(step))
    if file_version is not None:
        ev += _ld(3, file_version.encode())
    if scalars:
        summ = b""
        for tag, v in scalars.items():
            val = _ld(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(v))
            summ += _ld(1, val)
        ev += _ld(5, summ)
    return ev


def tfrecord(payload: bytes) -> bytes:
    hdr = struct.pack("<Q", len(payload))
    return hdr + struct.pack("<I", masked_crc(hdr)) + payload + struct.pack("<I", masked_crc(payload))


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}")
        self.fh = open(self.path, "ab")
        self.fh.write(tfrecord(encode_event(0, time.time(), file_version="brain.Event:2")))
        self.fh.flush()

    def scalars(self, step: int, values: Dict[str, float]) -> None:
        self.fh.write(tfrecord(encode_event(step, time.time(), values)))

    def graph(self, graph_def: bytes) -> None:
        """Event{graph_def = 4}: the model graph for TensorBoard's graph dashboard (runtime/tb_graph.py)."""
        ev = _key(1, 1) + struct.pack("<d", time.time()) + _key(2, 0) + _varint(0) + _ld(4, graph_def)
        self.fh.write(tfrecord(ev))
        self.fh.flush()

    def flush(self) -> None:
        self.fh.flush()

    def close(self) -> None:
        self.fh.close()


def read_events(path: str):
    """Parse an event file written by EventWriter (used by tests): -> list of (step, {tag: value})."""
    out = []
    with open(path, "rb") as fh:
        data = fh.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (hc,) = struct.unpack_from("<I", data, i + 8)
        assert hc == masked_crc(data[i:i + 8]), "bad length crc"
        payload = data[i + 12:i + 12 + n]
        (pc,) = struct.unpack_from("<I", data, i + 12 + n)
        assert pc == masked_crc(payload), "bad payload crc"
        i += 16 + n
        out.append(_parse_event(payload))
    return out


def _read_varint(b: bytes, i: int):
    shift, n = 0, 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        shift += 7
        if not c & 0x80:
            return n, i


def _parse_event(b: bytes):
    i, step, vals = 0, 0, {}
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
            if f == 2:
                step = v
        elif wt == 1:
            i += 8
        elif wt == 5:
            i += 4
        elif wt == 2:
            ln, i = _read_varint(b, i)
            sub = b[i:i + ln]
            i += ln
            if f == 5:
                j = 0
                while j < len(sub):
                    kk, j = _read_varint(sub, j)
                    ln2, j = _read_varint(sub, j)
                    val = sub[j:j + ln2]
                    j += ln2
                    tag, sv, t = None, None, 0
                    while t < len(val):
                        k3, t = _read_varint(val, t)
                        if k3 >> 3 == 1:
                            l3, t = _read_varint(val, t)
                            tag = val[t:t + l3].decode()
                            t += l3
                        elif k3 >> 3 == 2:
                            (sv,) = struct.unpack_from("<f", val, t)
                            t += 4
                    vals[tag] = sv
    return step, vals


TB_PREFIXES = ("global_norm/", "gradient_norm/")   # optimize_loss's gradient summaries


class MetricsLogger:
    """Rank-0 JSONL (``<model_dir>/train/metrics.jsonl``) + TensorBoard events + stdout."""

    def __init__(self, model_dir: str, enabled: bool = True, tensorboard: bool = True, stdout: bool = True):
        self.enabled = enabled
        self.stdout = stdout
        self.jsonl = None
        self.tb = None
        if enabled:
            d = os.path.join(model_dir, "train")
            os.makedirs(d, exist_ok=True)
            self.jsonl = open(os.path.join(d, "metrics.jsonl"), "a")
            if tensorboard:
                self.tb = EventWriter(d)

    def log(self, step: int, kind: str, **values) -> None:
        if not self.enabled:
            return
        rec = {"ts": time.time(), "step": int(step), "kind": kind}
        rec.update({k: (float(v) if isinstance(v, (int, float)) else v) for k, v in values.items()})
        self.jsonl.write(json.dumps(rec) + "\n")
        if self.tb is not None and kind == "train":
            self.tb.scalars(step, {k: v for k, v in values.items()
                                   if k in ("loss", "accuracy", "learning_rate") or k.startswith(TB_PREFIXES)})

    def graph(self, graph_def: bytes) -> None:
        if self.enabled and self.tb is not None:
            self.tb.graph(graph_def)

    def print(self, msg: str) -> None:
        if self.enabled and self.stdout:
            print(msg, flush=True)

    def flush(self) -> None:
        if self.jsonl:
            self.jsonl.flush()
        if self.tb:
            self.tb.flush()

    def close(self) -> None:
        self.flush()
        if self.jsonl:
            self.jsonl.close()
        if self.tb:
            self.tb.close()
