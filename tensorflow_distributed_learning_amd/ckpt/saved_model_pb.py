"""``saved_model.pb`` of a SavedModel directory, written and read without TensorFlow.

A TF SavedModel directory (README.md:51: the chief saves it) is ``saved_model.pb`` + ``variables/`` +
``assets/``.  This module writes the ``SavedModel`` protobuf header: schema version 1, and one
``MetaGraphDef`` with

* ``meta_info_def``: tags (``serve``), the producer's version strings, and ``stripped_default_attrs``;
* ``signature_def["serving_default"]``: the model's inputs and outputs as ``TensorInfo`` (name, dtype,
  shape with ``-1`` for the batch dimension), method ``tensorflow/serving/predict`` -- the names
  follow Keras's ``serving_default_<input>:0`` / ``StatefulPartitionedCall:<i>`` convention;
* ``saver_def``: V2 checkpoint format pointing at the ``variables/variables`` tensor bundle
  (ckpt/tensor_bundle.py writes TF's own ``.index`` table);
* ``graph_def``: the model's serving graph, variables and V2 saver (``ckpt/graph_def.py``), with the
  ``variables`` / ``trainable_variables`` collections -- a TF1-format SavedModel; ``versions`` only
  (the round-4 header) for a model with a layer that has no TF op mapping there.

The architecture also lives in this framework's ``saved_model.json`` (architecture + compile config),
which ``load_model`` reads.  The protobufs are encoded by hand with the field numbers of
tensorflow/core/protobuf/{saved_model,meta_graph,saver}.proto and
framework/{tensor_shape,types,versions}.proto.  TensorFlow is not installed here, so loading the
file with ``tf.saved_model.load`` is not pinned; the tests check the bytes against descriptors of
those messages built with the ``protobuf`` package, round-trip every field written here, and run
the graph with ``graph_def.run_graph`` against the model's predictions.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import struct

from .tensor_bundle import DT, _field_bytes, _field_fixed32, _field_varint, _parse

SCHEMA_VERSION = 1
PREDICT_METHOD = "tensorflow/serving/predict"
GRAPH_PRODUCER = 1205  # VersionDef.producer of a TF 2.x-era graph (informational)
TAG_SERVE = "serve"

TensorSpec = Tuple[str, Sequence, str]  # (signature key, shape with None for unknown dims, dtype name)


def _str(num: int, s: str) -> bytes:
    return _field_bytes(num, s.encode())


def _shape(shape) -> bytes:
    # TensorShapeProto: 2 repeated Dim {1 size (int64, -1 = unknown)}
    return b"".join(_field_bytes(2, _field_varint(1, -1 if d is None else int(d))) for d in shape)


def _tensor_info(name: str, dtype: str, shape) -> bytes:
    # TensorInfo: 1 name (oneof encoding), 2 dtype, 3 tensor_shape
    return _str(1, name) + _field_varint(2, DT[dtype]) + _field_bytes(3, _shape(shape))


def _map_entry(num: int, key: str, value: bytes) -> bytes:
    return _field_bytes(num, _str(1, key) + _field_bytes(2, value))


def signature_def(inputs: List[TensorSpec], outputs: List[TensorSpec], in_names=None, out_names=None) -> bytes:
    # SignatureDef: 1 inputs map<string, TensorInfo>, 2 outputs map (entries sorted by key), 3 method_name
    ins = {key: _tensor_info(in_names[i] if in_names else f"serving_default_{key}:0", dtype, shape)
           for i, (key, shape, dtype) in enumerate(inputs)}
    outs = {key: _tensor_info(out_names[i] if out_names else f"StatefulPartitionedCall:{i}", dtype, shape)
            for i, (key, shape, dtype) in enumerate(outputs)}
    out = b"".join(_map_entry(1, k, ins[k]) for k in sorted(ins))
    out += b"".join(_map_entry(2, k, outs[k]) for k in sorted(outs))
    return out + _str(3, PREDICT_METHOD)


def encode_saved_model(inputs: List[TensorSpec], outputs: List[TensorSpec], tags: Sequence[str] = (TAG_SERVE,),
                       producer: str = "tensorflow_distributed_learning_amd", graph=None) -> bytes:
    """``graph``: a ``graph_def.GraphSpec`` (serving graph + saver + collections), or None for the
    header-only file (GraphDef with ``versions`` only)."""
    # MetaInfoDef: 1 meta_graph_version, 4 tags, 5 tensorflow_version, 6 tensorflow_git_version,
    # 7 stripped_default_attrs
    meta_info = b"".join(_str(4, t) for t in tags) + _str(5, producer) + _str(6, producer) + _field_varint(7, 1)
    # SaverDef: 1 filename_tensor_name, 2 save_tensor_name, 3 restore_op_name, 4 max_to_keep,
    # 5 sharded, 6 keep_checkpoint_every_n_hours (float), 7 version (V2 = 2)
    if graph is None:
        # GraphDef: 4 versions (VersionDef: 1 producer)
        graph_def = _field_bytes(4, _field_varint(1, GRAPH_PRODUCER))
        saver_def = (_str(1, "saver_filename:0") + _str(2, "StatefulPartitionedCall_1:0")
                     + _str(3, "StatefulPartitionedCall_2") + _field_varint(4, 5) + _field_varint(5, 1)
                     + _field_varint(7, 2))
        collections = b""
        in_names, out_names = None, None
    else:
        graph_def = graph.graph_def
        sv = graph.saver
        saver_def = (_str(1, sv["filename_tensor_name"]) + _str(2, sv["save_tensor_name"])
                     + _str(3, sv["restore_op_name"]) + _field_varint(4, 5)
                     + _field_fixed32(6, struct.unpack("<I", struct.pack("<f", 10000.0))[0]) + _field_varint(7, 2))
        # MetaGraphDef.collection_def (4): map<string, CollectionDef>, entries sorted by key
        collections = b"".join(_field_bytes(4, _str(1, k) + _field_bytes(2, graph.collections[k]))
                               for k in sorted(graph.collections))
        in_names = [n for _, n in graph.inputs]
        out_names = list(graph.outputs)
    # MetaGraphDef: 1 meta_info_def, 2 graph_def, 3 saver_def, 4 collection_def, 5 signature_def map
    meta_graph = (_field_bytes(1, meta_info) + _field_bytes(2, graph_def) + _field_bytes(3, saver_def)
                  + collections + _map_entry(5, "serving_default", signature_def(inputs, outputs, in_names, out_names)))
    # SavedModel: 1 saved_model_schema_version, 2 meta_graphs
    return _field_varint(1, SCHEMA_VERSION) + _field_bytes(2, meta_graph)


_DT_NAME = {v: k for k, v in DT.items()}


def _parse_tensor_info(buf: bytes) -> dict:
    f = _parse(buf)
    shape = []
    for shp in f.get(3, []):
        for dim in _parse(shp).get(2, []):
            v = int(_parse(dim).get(1, [0])[0])
            shape.append(None if v >= (1 << 63) else v)  # varint of -1
    return {"name": f.get(1, [b""])[0].decode(), "dtype": _DT_NAME.get(f.get(2, [0])[0], "unknown"), "shape": shape}


def _parse_map(entries: List[bytes]) -> Dict[str, bytes]:
    out = {}
    for e in entries:
        f = _parse(e)
        out[f.get(1, [b""])[0].decode()] = f.get(2, [b""])[0]
    return out


def parse_saved_model(buf: bytes) -> dict:
    """The fields this module writes, as a dict (any SavedModel's header parses; unknown fields skipped)."""
    f = _parse(buf)
    graphs = []
    for mg in f.get(2, []):
        g = _parse(mg)
        info = _parse(g[1][0]) if 1 in g else {}
        sigs = {}
        for key, sd in _parse_map(g.get(5, [])).items():
            s = _parse(sd)
            sigs[key] = {"inputs": {k: _parse_tensor_info(v) for k, v in _parse_map(s.get(1, [])).items()},
                         "outputs": {k: _parse_tensor_info(v) for k, v in _parse_map(s.get(2, [])).items()},
                         "method_name": s.get(3, [b""])[0].decode()}
        saver = _parse(g[3][0]) if 3 in g else {}
        graphs.append({"tags": [t.decode() for t in info.get(4, [])],
                       "tensorflow_version": info.get(5, [b""])[0].decode(),
                       "signature_def": sigs,
                       "saver_version": saver.get(7, [0])[0],
                       "saver": {"filename_tensor_name": saver.get(1, [b""])[0].decode(),
                                 "save_tensor_name": saver.get(2, [b""])[0].decode(),
                                 "restore_op_name": saver.get(3, [b""])[0].decode()},
                       "graph_def": g[2][0] if 2 in g else b"",
                       "collection_def": _parse_map(g.get(4, []))})
    return {"saved_model_schema_version": f.get(1, [0])[0], "meta_graphs": graphs}


def model_signature(model) -> Tuple[List[TensorSpec], List[TensorSpec]]:
    """(inputs, outputs) of a built Keras-style model for ``signature_def``: the Input layers' names
    (Sequential: ``<first layer>_input``) and the output layers' names, float32, batch dim unknown."""
    from ..keras.layers import _flat

    in_shape = model._built_input_shape
    if in_shape is None:
        raise ValueError("saved_model.pb: the model is not built")
    shapes = in_shape if isinstance(in_shape, list) else [in_shape]
    if getattr(model, "_inputs", None):
        names = [t.name or f"input_{i + 1}" for i, t in enumerate(model._inputs)]
        outs = [(t._node.layer.name, t.shape) for t in _flat(model._outputs)]
    else:  # Sequential
        layers = getattr(model, "_seq", None) or model.layers
        names = [f"{layers[0].name}_input"]
        o = model.compute_output_shape(tuple(in_shape))
        outs = [(layers[-1].name, o)]
    inputs = [(n, (None,) + tuple(s)[1:], "float32") for n, s in zip(names, shapes)]
    outputs = [(n, (None,) + tuple(s)[1:], "float32") for n, s in outs]
    return inputs, outputs
