"""Chief-side event logging (README.md:51: "chief ... generates TensorBoard").

:class:`EventFileWriter` writes TensorBoard-readable ``events.out.tfevents.*`` files: TFRecord
framing (length + masked CRC-32C) around hand-encoded ``tensorflow.Event`` protobufs carrying
scalar summaries.  The ``tensorboard`` package is not needed (nor installed); a JSON-lines mirror
(``metrics.jsonl``) is written next to it for scripts.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Dict, Optional

_CRC_TABLE = None


def _crc32c_py(data: bytes) -> int:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        tab = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (0x82F63B78 ^ (c >> 1)) if (c & 1) else (c >> 1)
            tab.append(c)
        _CRC_TABLE = tab
    crc = 0xFFFFFFFF
    for b in data:
        crc = _CRC_TABLE[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def crc32c(data: bytes) -> int:
    try:
        from .. import ops

        if ops.native_available():
            return ops.native().crc32c(data, 0)
    except Exception:
        pass
    return _crc32c_py(data)


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


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


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_delim(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    val = _len_delim(1, tag.encode()) + _key(2, 5) + struct.pack("<f", float(value))
    summary = _len_delim(1, val)
    return (_key(1, 1) + struct.pack("<d", wall_time if wall_time is not None else time.time()) +
            _key(2, 0) + _varint(int(step)) + _len_delim(5, summary))


def encode_file_version_event(wall_time: Optional[float] = None) -> bytes:
    return (_key(1, 1) + struct.pack("<d", wall_time if wall_time is not None else time.time()) +
            _len_delim(3, b"brain.Event:2"))


def tfrecord(data: bytes) -> bytes:
    ln = struct.pack("<Q", len(data))
    return ln + struct.pack("<I", masked_crc(ln)) + data + struct.pack("<I", masked_crc(data))


def read_tfrecords(path: str):
    """Yield record payloads, verifying both CRCs (used by tests)."""
    with open(path, "rb") as f:
        while True:
            h = f.read(12)
            if not h:
                return
            (n,) = struct.unpack("<Q", h[:8])
            if struct.unpack("<I", h[8:])[0] != masked_crc(h[:8]):
                raise ValueError("corrupt record length")
            d = f.read(n)
            (c,) = struct.unpack("<I", f.read(4))
            if c != masked_crc(d):
                raise ValueError("corrupt record payload")
            yield d


class EventFileWriter:
    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.logdir = logdir
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}{filename_suffix}"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._f.write(tfrecord(encode_file_version_event()))
        self._jsonl = open(os.path.join(logdir, "metrics.jsonl"), "a")

    def scalar(self, tag: str, value: float, step: int):
        self._f.write(tfrecord(encode_scalar_event(tag, value, step)))
        self._jsonl.write(json.dumps({"tag": tag, "value": float(value), "step": int(step), "time": time.time()}) + "\n")

    def scalars(self, values: Dict[str, float], step: int, prefix: str = ""):
        for k, v in values.items():
            self.scalar(prefix + k, v, step)

    def flush(self):
        self._f.flush()
        self._jsonl.flush()

    def close(self):
        self.flush()
        self._f.close()
        self._jsonl.close()
