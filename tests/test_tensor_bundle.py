"""TensorFlow tensor-bundle checkpoint index (ckpt/tensor_bundle.py): LevelDB-table structure per
the format specification, protobuf records, and round trips through the checkpoint API.  (TF is
not installed, so byte parity with a TF-written index is unpinned.)"""
import struct

import numpy as np
import pytest
import torch

from tensorflow_distributed_learning_amd.ckpt import checkpoint as ck
from tensorflow_distributed_learning_amd.ckpt import tensor_bundle as TB
from tensorflow_distributed_learning_amd.utils.events import crc32c


def test_table_structure_and_records(tmp_path):
    tensors = {"conv2d/kernel": torch.randn(3, 3, 1, 32), "conv2d/bias": torch.zeros(32),
               "iterations": torch.tensor(7, dtype=torch.int64), "w_bf16": torch.randn(5).bfloat16()}
    prefix = str(tmp_path / "ckpt-1")
    ck.write_bundle(prefix, tensors)
    raw = open(prefix + ".index", "rb").read()
    assert struct.unpack("<Q", raw[-8:])[0] == 0xDB4775248B80FB57  # table magic
    kv = TB.read_table(prefix + ".index")
    keys = [k for k, _ in kv]
    assert keys[0] == b"" and keys == sorted(keys)  # header entry first, keys sorted
    hdr = TB.parse_header(kv[0][1])
    assert hdr == {"num_shards": 1, "endianness": 0, "producer": 1}
    data = open(prefix + ".data-00000-of-00001", "rb").read()
    for k, v in kv[1:]:
        e = TB.parse_entry(v)
        t = tensors[k.decode()]
        assert e["shape"] == list(t.shape)
        assert e["dtype"] == {torch.float32: "float32", torch.int64: "int64", torch.bfloat16: "bfloat16"}[t.dtype]
        blob = data[e["offset"]:e["offset"] + e["size"]]
        assert e["crc32c"] == crc32c(blob)  # stored masked, as TF does
    # the raw entry record of conv2d/bias: dtype DT_FLOAT (1), shape {dim {size: 32}}
    rec = dict(kv)[b"conv2d/bias"]
    assert rec.startswith(bytes([0x08, 0x01, 0x12, 0x04, 0x12, 0x02, 0x08, 0x20]))


def test_round_trip_all_dtypes_and_many_blocks(tmp_path):
    g = torch.Generator().manual_seed(0)
    tensors = {f"layer_{i:04d}/kernel": torch.randn(i % 7 + 1, 3, generator=g) for i in range(400)}
    tensors.update({"i8": torch.tensor([-3, 4], dtype=torch.int8), "u8": torch.tensor([250], dtype=torch.uint8),
                    "b": torch.tensor([True, False]), "f16": torch.randn(4).half(), "f64": torch.randn(2).double(),
                    "i32": torch.arange(5, dtype=torch.int32), "scalar": torch.tensor(1.5)})
    prefix = str(tmp_path / "variables")
    ck.write_bundle(prefix, tensors)
    assert len(TB.read_table(prefix + ".index")) == len(tensors) + 1  # several data blocks
    back = ck.read_bundle(prefix)
    assert set(back) == set(tensors)
    for k, t in tensors.items():
        assert back[k].dtype == t.dtype and torch.equal(back[k], t), k
    assert dict(ck.list_variables(prefix))["scalar"] == ()


def test_corruption_detected_and_json_index_still_read(tmp_path, monkeypatch):
    prefix = str(tmp_path / "c")
    ck.write_bundle(prefix, {"a": torch.ones(8)})
    raw = bytearray(open(prefix + ".index", "rb").read())
    raw[3] ^= 0xFF  # inside the data block
    open(prefix + ".index", "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        ck.read_bundle(prefix)
    monkeypatch.setenv("TDL_CKPT_INDEX", "json")
    ck.write_bundle(prefix, {"a": torch.ones(8)})
    assert not TB.is_table(prefix + ".index")
    assert torch.equal(ck.read_bundle(prefix)["a"], torch.ones(8))


def test_string_entries_listed_and_object_graph_skipped(tmp_path):
    """TF2 bundles carry _CHECKPOINTABLE_OBJECT_GRAPH as a DT_STRING (7) tensor: list_variables
    shows it, read_bundle skips it, and any other string tensor is refused by name."""
    prefix = str(tmp_path / "tf2")
    ck.write_bundle(prefix, {"dense/kernel": torch.ones(2, 3)})
    kv = TB.read_table(prefix + ".index")
    data_len = len(open(prefix + ".data-00000-of-00001", "rb").read())
    blob = b"\x0a\x03obj"

    def string_entry():
        return TB._field_varint(1, 7) + TB._field_varint(4, data_len) + TB._field_varint(5, len(blob)) + \
            TB._field_fixed32(6, TB.mask_crc(crc32c(blob)))
    with open(prefix + ".data-00000-of-00001", "ab") as f:
        f.write(blob)
    TB.write_table(prefix + ".index", kv + [(b"_CHECKPOINTABLE_OBJECT_GRAPH", string_entry())])
    assert dict(ck.list_variables(prefix))["_CHECKPOINTABLE_OBJECT_GRAPH"] == ()
    assert set(ck.read_bundle(prefix)) == {"dense/kernel"}
    TB.write_table(prefix + ".index", kv + [(b"vocab", string_entry())])
    with pytest.raises(ValueError, match="vocab"):
        ck.read_bundle(prefix)
