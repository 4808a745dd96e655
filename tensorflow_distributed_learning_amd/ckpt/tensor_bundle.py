"""TensorFlow's tensor-bundle checkpoint index, written and read without TensorFlow.

``<prefix>.index`` in a TF checkpoint / SavedModel ``variables/`` directory (README.md:51: the chief
saves them) is a LevelDB-format sorted table (TF ``core/lib/io/table``):

* entry ``""`` (sorts first) -> ``BundleHeaderProto{num_shards, endianness, version}``;
* entry ``<tensor name>``    -> ``BundleEntryProto{dtype, shape, shard_id, offset, size, crc32c}``
  pointing into ``<prefix>.data-00000-of-00001`` (raw little-endian bytes; crc32c masked);
* table layout: data block(s) of prefix-compressed ``(shared, unshared, value_len, key, value)``
  records with a restart-point array, an empty metaindex block, an index block mapping each data
  block's last key to its ``BlockHandle``, every block followed by a 5-byte trailer (compression
  type 0 + masked crc32c of block+type), and a 48-byte footer (two varint handles padded to 40
  bytes + magic ``0xdb4775248b80fb57``).

The protobufs are encoded by hand (field numbers of tensorflow/core/protobuf/tensor_bundle.proto and
framework/tensor_shape.proto, types.proto); no protobuf/TensorFlow import.  TF itself is not
installed here, so byte-level parity with a TF-written file is unpinned: the tests check the
structure against the format specification and round-trip every dtype.
"""
from __future__ import annotations

import struct
from typing import Dict, List, Tuple

from ..utils.events import crc32c

MAGIC = 0xDB4775248B80FB57
RESTART_INTERVAL = 16
BLOCK_SIZE = 4096  # target data block size before a new block is started (TF's default)

# tensorflow DataType enum (types.proto)
DT = {"float32": 1, "float64": 2, "int32": 3, "uint8": 4, "int16": 5, "int8": 6, "int64": 9, "bool": 10,
      "bfloat16": 14, "float16": 19}
DT_INV = {v: k for k, v in DT.items()}
# read-only: TF2 checkpoints carry _CHECKPOINTABLE_OBJECT_GRAPH as a DT_STRING tensor (the object
# graph proto); bundles written here hold numeric tensors only (name-based loading: the files work
# with tf.train.load_checkpoint / list_variables, not with a TF2 object-graph restore)
DT_INV[7] = "string"


def dtype_name(code: int) -> str:
    return DT_INV.get(int(code), f"unsupported-dtype-{int(code)}")


def mask_crc(c: int) -> int:
    """LevelDB / TF crc masking (crc32c::Mask)."""
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


def unmask_crc(m: int) -> int:
    rot = (m - 0xA282EAD8) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---------------------------------------------------------------------------- protobuf wire format
def _varint(v: int) -> bytes:
    if v < 0:
        v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, pos: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[pos]
        pos += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, pos
        shift += 7


def _field_varint(num: int, v: int) -> bytes:
    return _varint(num << 3) + _varint(v)


def _field_bytes(num: int, b: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(b)) + b


def _field_fixed32(num: int, v: int) -> bytes:
    return _varint((num << 3) | 5) + struct.pack("<I", v)


def _parse(buf: bytes) -> Dict[int, list]:
    """Generic protobuf message -> {field: [values]} (varint ints, fixed32 ints, bytes)."""
    out: Dict[int, list] = {}
    pos = 0
    while pos < len(buf):
        key, pos = _read_varint(buf, pos)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, pos = _read_varint(buf, pos)
        elif wt == 1:
            v = struct.unpack_from("<Q", buf, pos)[0]
            pos += 8
        elif wt == 2:
            n, pos = _read_varint(buf, pos)
            v = bytes(buf[pos:pos + n])
            pos += n
        elif wt == 5:
            v = struct.unpack_from("<I", buf, pos)[0]
            pos += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        out.setdefault(num, []).append(v)
    return out


def header_proto(num_shards: int = 1) -> bytes:
    # BundleHeaderProto: 1 num_shards, 2 endianness (LITTLE = 0, the default: omitted), 3 version
    version = _field_varint(1, 1)  # VersionDef.producer = 1
    return _field_varint(1, num_shards) + _field_bytes(3, version)


def entry_proto(dtype: str, shape, offset: int, size: int, crc: int, shard_id: int = 0) -> bytes:
    # TensorShapeProto: 2 dim (repeated Dim{1 size}); BundleEntryProto: 1 dtype, 2 shape,
    # 3 shard_id, 4 offset, 5 size, 6 crc32c (fixed32, masked)
    shp = b"".join(_field_bytes(2, _field_varint(1, int(d))) for d in shape)
    out = _field_varint(1, DT[dtype]) + _field_bytes(2, shp)
    if shard_id:
        out += _field_varint(3, shard_id)
    if offset:
        out += _field_varint(4, offset)
    if size:
        out += _field_varint(5, size)
    return out + _field_fixed32(6, mask_crc(crc))


def parse_entry(buf: bytes) -> dict:
    f = _parse(buf)
    shape = []
    for shp in f.get(2, [b""]):
        for dim in _parse(shp).get(2, []):
            shape.append(int(_parse(dim).get(1, [0])[0]))
    return {"dtype": dtype_name(f.get(1, [0])[0]), "shape": shape, "shard_id": f.get(3, [0])[0],
            "offset": f.get(4, [0])[0], "size": f.get(5, [0])[0],
            "crc32c": unmask_crc(f[6][0]) if 6 in f else None}


def parse_header(buf: bytes) -> dict:
    f = _parse(buf)
    ver = _parse(f[3][0]) if 3 in f else {}
    return {"num_shards": f.get(1, [0])[0], "endianness": f.get(2, [0])[0], "producer": ver.get(1, [0])[0]}


# ---------------------------------------------------------------------------- LevelDB table
def _block(entries: List[Tuple[bytes, bytes]]) -> bytes:
    out = bytearray()
    restarts = []
    prev = b""
    for i, (k, v) in enumerate(entries):
        if i % RESTART_INTERVAL == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(prev), len(k)) and prev[shared] == k[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        prev = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack("<I", r)
    out += struct.pack("<I", len(restarts))
    return bytes(out)


def _trailer(block: bytes) -> bytes:
    return b"\x00" + struct.pack("<I", mask_crc(crc32c(block + b"\x00")))


def _handle(offset: int, size: int) -> bytes:
    return _varint(offset) + _varint(size)


def write_table(path: str, entries: List[Tuple[bytes, bytes]]) -> None:
    """A LevelDB-format table of (key, value) pairs (sorted here by key bytes)."""
    entries = sorted(entries, key=lambda kv: kv[0])
    out = bytearray()
    index = []
    cur: List[Tuple[bytes, bytes]] = []
    cur_bytes = 0

    def flush():
        nonlocal cur, cur_bytes
        if not cur:
            return
        blk = _block(cur)
        index.append((cur[-1][0], _handle(len(out), len(blk))))
        out.extend(blk + _trailer(blk))
        cur, cur_bytes = [], 0

    for k, v in entries:
        cur.append((k, v))
        cur_bytes += len(k) + len(v) + 8
        if cur_bytes >= BLOCK_SIZE:
            flush()
    flush()
    meta = _block([])
    meta_handle = _handle(len(out), len(meta))
    out.extend(meta + _trailer(meta))
    idx = _block(index)
    idx_handle = _handle(len(out), len(idx))
    out.extend(idx + _trailer(idx))
    footer = (meta_handle + idx_handle).ljust(40, b"\x00") + struct.pack("<Q", MAGIC)
    out.extend(footer)
    with open(path, "wb") as f:
        f.write(bytes(out))


def _read_block(buf: bytes, offset: int, size: int, verify: bool) -> List[Tuple[bytes, bytes]]:
    blk = buf[offset:offset + size]
    if verify:
        typ, crc = buf[offset + size], struct.unpack_from("<I", buf, offset + size + 1)[0]
        if typ != 0:
            raise ValueError("compressed table blocks are not supported")
        if unmask_crc(crc) != crc32c(bytes(blk) + b"\x00"):
            raise ValueError("table block checksum mismatch")
    n = struct.unpack_from("<I", blk, len(blk) - 4)[0]
    end = len(blk) - 4 - 4 * n
    pos, prev, out = 0, b"", []
    while pos < end:
        shared, pos = _read_varint(blk, pos)
        unshared, pos = _read_varint(blk, pos)
        vlen, pos = _read_varint(blk, pos)
        k = prev[:shared] + bytes(blk[pos:pos + unshared])
        pos += unshared
        out.append((k, bytes(blk[pos:pos + vlen])))
        pos += vlen
        prev = k
    return out


def read_table(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    with open(path, "rb") as f:
        buf = f.read()
    if len(buf) < 48 or struct.unpack_from("<Q", buf, len(buf) - 8)[0] != MAGIC:
        raise ValueError(f"{path} is not a LevelDB-format table")
    foot = buf[len(buf) - 48:len(buf) - 8]
    _, p = _read_varint(foot, 0)
    _, p = _read_varint(foot, p)
    io, p = _read_varint(foot, p)
    isz, p = _read_varint(foot, p)
    out = []
    for _, h in _read_block(buf, io, isz, verify):
        off, q = _read_varint(h, 0)
        sz, _ = _read_varint(h, q)
        out.extend(_read_block(buf, off, sz, verify))
    return out


def is_table(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            f.seek(-8, 2)
            return struct.unpack("<Q", f.read(8))[0] == MAGIC
    except OSError:
        return False


def write_index(path: str, entries: Dict[str, dict]) -> None:
    """``entries``: tensor name -> {dtype, shape, offset, nbytes, crc32c (unmasked)}."""
    kv = [(b"", header_proto(1))]
    for name, e in entries.items():
        kv.append((name.encode(), entry_proto(e["dtype"], e["shape"], e["offset"], e["nbytes"], e["crc32c"])))
    write_table(path, kv)


def read_index(path: str, verify: bool = True) -> Dict[str, dict]:
    """tensor name -> {dtype, shape, offset, nbytes, crc32c}; raises on a bad header."""
    out = {}
    header = None
    for k, v in read_table(path, verify):
        if k == b"":
            header = parse_header(v)
            continue
        e = parse_entry(v)
        if e["shard_id"] != 0:
            raise ValueError("multi-shard bundles are not supported")
        out[k.decode()] = {"dtype": e["dtype"], "shape": e["shape"], "offset": e["offset"], "nbytes": e["size"],
                           "crc32c": e["crc32c"]}
    if header is None or header["num_shards"] != 1 or header["endianness"] != 0:
        raise ValueError(f"{path}: unsupported bundle header {header}")
    return out
