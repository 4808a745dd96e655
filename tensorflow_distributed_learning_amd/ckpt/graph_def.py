"""TensorFlow ``GraphDef`` of a model's serving function, written without TensorFlow.

``model.save`` (README.md:51: the chief saves the model) puts this graph into ``saved_model.pb``'s
``MetaGraphDef``, which makes the directory a TF1-format SavedModel: what
``tf.compat.v1.saved_model.load`` reads, and what ``tf.saved_model.load`` loads through its v1 path
(restore op fed with ``variables/variables``, variables from the ``variables`` collection, the
``serving_default`` signature pruned out of the graph).  The graph holds

* one ``Placeholder`` per model input (``serving_default_<input>``, batch dimension -1);
* per variable a resource ``VarHandleOp`` (shared name = the Keras variable name), a zeros ``Const``
  initial value, its ``AssignVariableOp`` initializer and a ``ReadVariableOp`` snapshot, listed as
  ``VariableDef``s in the ``variables`` / ``trainable_variables`` collections;
* the inference computation of every layer, NHWC, float32 -- Conv2D (+BiasAdd), Dense (MatMul +
  BiasAdd), Max/AvgPool, Mean/Max (global pools), Reshape (Flatten/Reshape), Pad (ZeroPadding2D),
  FusedBatchNormV3 (``is_training=false``: moving statistics), AddV2/AddN/Sub/Mul/Maximum/ConcatV2
  (merge layers), the activations, Identity for Dropout;
* the outputs as ``StatefulPartitionedCall`` (Identity, or IdentityN for several outputs), the names
  the signature has always used;
* a V2 ``Saver``: ``save/Const`` (PlaceholderWithDefault filename), ``SaveV2`` / ``RestoreV2`` over
  the bundle keys ``model.save`` writes (``ckpt/checkpoint.py``), one ``AssignVariableOp`` per
  restored tensor and the ``save/restore_all`` NoOp.

Encoding: tensorflow/core/framework/{graph,node_def,attr_value,tensor,tensor_shape,types,
versions,variable}.proto and protobuf/{meta_graph,saver}.proto field numbers; map entries are
emitted sorted by key and default-valued proto3 scalars omitted, so the protobuf runtime
re-serialises the bytes identically (tests/test_graph_def_cpu.py).  TensorFlow is not installed
here: whether TF loads the file is parity unpinned; ``run_graph`` below is a small interpreter of
these bytes (numpy/torch CPU) that the tests run against the model's own predictions.

Layers without a TF op mapping here (Lambda, Embedding, LayerNormalization, ...) raise
``UnsupportedLayer``; ``model.save`` then writes the header-only ``saved_model.pb``.
"""
from __future__ import annotations

import math
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .tensor_bundle import DT, _field_bytes, _field_varint, _parse, _varint

DT_STRING, DT_RESOURCE = 7, 20


class UnsupportedLayer(ValueError):
    """A layer this module has no TensorFlow op mapping for."""


# ------------------------------------------------------------------------------------ encoding
def _s(num: int, s) -> bytes:
    return _field_bytes(num, s.encode() if isinstance(s, str) else s)


def _packed_varints(num: int, vals: Sequence[int]) -> bytes:
    return _field_bytes(num, b"".join(_varint(int(v)) for v in vals)) if len(vals) else b""


def _packed_floats(num: int, vals: Sequence[float]) -> bytes:
    return _field_bytes(num, struct.pack(f"<{len(vals)}f", *vals)) if len(vals) else b""


def shape_proto(dims: Optional[Sequence]) -> bytes:
    """TensorShapeProto: 2 dim {1 size}, 3 unknown_rank; None = unknown rank, a None dim = -1."""
    if dims is None:
        return _field_varint(3, 1)
    # (a Dim of size 0 is an empty message: proto3 omits the default)
    return b"".join(_field_bytes(2, _field_varint(1, -1 if d is None else int(d)) if d != 0 else b"") for d in dims)


def tensor_proto(dtype: int, shape: Sequence[int], floats=None, ints=None, strings=None, content: bytes = b"") -> bytes:
    """TensorProto: 1 dtype, 2 tensor_shape, 4 tensor_content, 5 float_val, 7 int_val, 8 string_val."""
    out = _field_varint(1, dtype) + _field_bytes(2, shape_proto(shape))
    if content:
        out += _field_bytes(4, content)
    if floats is not None:
        out += _packed_floats(5, floats)
    if ints is not None:
        out += _packed_varints(7, ints)
    if strings is not None:
        out += b"".join(_s(8, x) for x in strings)
    return out


class Attr:
    """AttrValue constructors (oneof value: 1 list, 2 s, 3 i, 4 f, 5 b, 6 type, 7 shape, 8 tensor)."""

    @staticmethod
    def s(v: str) -> bytes:
        return _s(2, v)

    @staticmethod
    def i(v: int) -> bytes:
        return _field_varint(3, int(v))

    @staticmethod
    def f(v: float) -> bytes:
        return _varint((4 << 3) | 5) + struct.pack("<f", float(v))

    @staticmethod
    def b(v: bool) -> bytes:
        return _field_varint(5, 1 if v else 0)

    @staticmethod
    def type(v: int) -> bytes:
        return _field_varint(6, int(v))

    @staticmethod
    def shape(dims) -> bytes:
        return _field_bytes(7, shape_proto(dims))

    @staticmethod
    def tensor(t: bytes) -> bytes:
        return _field_bytes(8, t)

    # ListValue: 2 s, 3 i (packed), 6 type (packed), 7 shape
    @staticmethod
    def ilist(vals) -> bytes:
        return _field_bytes(1, _packed_varints(3, vals))

    @staticmethod
    def tlist(vals) -> bytes:
        return _field_bytes(1, _packed_varints(6, vals))

    @staticmethod
    def slist(vals) -> bytes:
        return _field_bytes(1, b"".join(_s(2, v) for v in vals))


def node_def(name: str, op: str, inputs: Sequence[str] = (), attrs: Optional[Dict[str, bytes]] = None) -> bytes:
    """NodeDef: 1 name, 2 op, 3 input, 5 attr (map, entries sorted by key)."""
    out = _s(1, name) + _s(2, op) + b"".join(_s(3, x) for x in inputs)
    for k in sorted(attrs or {}):
        out += _field_bytes(5, _s(1, k) + _field_bytes(2, attrs[k]))
    return out


def variable_def(name: str, trainable: bool) -> bytes:
    """VariableDef: 1 variable_name, 2 initializer_name, 3 snapshot_name, 5 is_resource,
    6 initial_value_name, 7 trainable."""
    out = (_s(1, f"{name}:0") + _s(2, f"{name}/Assign") + _s(3, f"{name}/Read/ReadVariableOp:0")
           + _field_varint(5, 1) + _s(6, f"{name}/Initializer/zeros:0"))
    return out + (_field_varint(7, 1) if trainable else b"")


def collection_bytes_list(values: Sequence[bytes]) -> bytes:
    """CollectionDef with a bytes_list (2) {1 value}."""
    return _field_bytes(2, b"".join(_field_bytes(1, v) for v in values))


# ------------------------------------------------------------------------------------ builder
_F32 = DT["float32"]
_I32 = DT["int32"]


class _Graph:
    def __init__(self):
        self.nodes: List[bytes] = []
        self.names: set = set()

    def uniq(self, base: str) -> str:
        name, k = base, 0
        while name in self.names:
            k += 1
            name = f"{base}_{k}"
        return name

    def add(self, name: str, op: str, inputs: Sequence[str] = (), **attrs) -> str:
        name = self.uniq(name)
        self.names.add(name)
        self.nodes.append(node_def(name, op, inputs, attrs))
        return name

    def const_i32(self, name: str, vals, shape) -> str:
        return self.add(name, "Const", dtype=Attr.type(_I32),
                        value=Attr.tensor(tensor_proto(_I32, shape, content=np.asarray(vals, "<i4").tobytes())))

    def const_f32(self, name: str, v: float) -> str:
        return self.add(name, "Const", dtype=Attr.type(_F32), value=Attr.tensor(tensor_proto(_F32, [], floats=[v])))


_ACT_OPS = {"relu": "Relu", "relu6": "Relu6", "sigmoid": "Sigmoid", "tanh": "Tanh", "softmax": "Softmax",
            "log_softmax": "LogSoftmax", "elu": "Elu", "selu": "Selu", "softplus": "Softplus",
            "softsign": "Softsign", "exponential": "Exp"}


def _act_name(fn) -> str:
    from ..keras import activations as _act

    return _act.serialize(fn) if fn is not None else "linear"


def _activation(g: _Graph, scope: str, x: str, act: str) -> str:
    T = Attr.type(_F32)
    if act in ("linear", None):
        return x
    if act == "swish":
        s = g.add(f"{scope}/Sigmoid", "Sigmoid", [x], T=T)
        return g.add(f"{scope}/mul", "Mul", [x, s], T=T)
    op = _ACT_OPS.get(act)
    if op is None:
        raise UnsupportedLayer(f"activation {act!r} has no TF op mapping here")
    return g.add(f"{scope}/{op}", op, [x], T=T)


def _pool_padding(p: str) -> bytes:
    return Attr.s("SAME" if p == "same" else "VALID")


def _var_name(v) -> str:
    n = v.name
    return n[:-2] if n.endswith(":0") else n


class GraphSpec:
    """The encoded graph plus what the MetaGraphDef around it names."""

    def __init__(self, graph_def: bytes, collections: Dict[str, bytes], saver: Dict[str, str],
                 inputs: List[Tuple[str, str]], outputs: List[str]):
        self.graph_def = graph_def
        self.collections = collections
        self.saver = saver
        self.inputs = inputs    # (signature key, tensor name)
        self.outputs = outputs  # tensor names, in output order


def build_graph(model, producer: int) -> GraphSpec:
    """The serving graph + variables + V2 saver of a built Sequential or functional model."""
    from ..keras import layers as L

    g = _Graph()
    T = Attr.type(_F32)
    # ---- variables ----
    var_of: Dict[int, str] = {}
    var_defs, train_defs, bundle_keys, var_shapes = [], [], [], []
    for v in model.weights:
        name = _var_name(v)
        shape = [int(d) for d in v.shape]
        h = g.add(name, "VarHandleOp", allowed_devices=Attr.slist([]), container=Attr.s(""),
                  dtype=T, shape=Attr.shape(shape), shared_name=Attr.s(name))
        if h != name:
            raise UnsupportedLayer(f"variable name {name!r} collides with another graph node")
        z = g.add(f"{name}/Initializer/zeros", "Const", dtype=T,
                  value=Attr.tensor(tensor_proto(_F32, shape, floats=[0.0])))
        g.add(f"{name}/Assign", "AssignVariableOp", [h, z], dtype=T)
        g.add(f"{name}/Read/ReadVariableOp", "ReadVariableOp", [h], dtype=T)
        vd = variable_def(name, bool(getattr(v, "trainable", True)))
        var_defs.append(vd)
        if getattr(v, "trainable", True):
            train_defs.append(vd)
        var_of[id(v)] = h
        bundle_keys.append(v.name)
        var_shapes.append(shape)

    def read(layer, v) -> str:
        return g.add(f"{model.name}/{layer.name}/{_var_name(v).split('/')[-1]}/ReadVariableOp", "ReadVariableOp",
                     [var_of[id(v)]], dtype=T)

    # ---- inputs ----
    if getattr(model, "_nodes", None) is not None and getattr(model, "_inputs", None) and not hasattr(model, "_seq"):
        in_tensors = model._inputs
        in_names = [t.name or f"input_{i + 1}" for i, t in enumerate(in_tensors)]
        in_shapes = [t.shape for t in in_tensors]
        steps = [(n.layer, L._flat(n.inputs), L._flat(n.outputs)) for n in model._nodes]
        out_tensors = L._flat(model._outputs)
    else:
        seq = getattr(model, "_seq", None) or model.layers
        shape = model._built_input_shape
        if shape is None:
            raise ValueError("graph_def: the model is not built")
        in_tensors = [object()]
        in_names = [f"{seq[0].name}_input"]
        in_shapes = [tuple(shape)]
        steps, prev = [], in_tensors[0]
        for layer in seq:
            o = object()
            steps.append((layer, [prev], [o]))
            prev = o
        out_tensors = [prev]
    val: Dict[int, str] = {}
    sig_inputs = []
    shape_of: Dict[int, tuple] = {}
    for t, n, s in zip(in_tensors, in_names, in_shapes):
        ph = g.add(f"serving_default_{n}", "Placeholder", dtype=T, shape=Attr.shape((None,) + tuple(s)[1:]))
        val[id(t)] = ph
        shape_of[id(t)] = (None,) + tuple(s)[1:]
        sig_inputs.append((n, f"{ph}:0"))

    # ---- layers ----
    for layer, ins, outs in steps:
        if isinstance(layer, L.InputLayer):
            continue
        xs = [val[id(t)] for t in ins]
        in_shape = shape_of.get(id(ins[0]))
        sc = f"{model.name}/{layer.name}"
        y = _emit_layer(g, layer, sc, xs, in_shape, read)
        val[id(outs[0])] = y
        if in_shape is not None:
            try:
                shape_of[id(outs[0])] = tuple(layer.compute_output_shape(
                    in_shape if len(ins) == 1 else [shape_of[id(t)] for t in ins]))
            except Exception:
                pass

    # ---- outputs ----
    ys = [val[id(t)] for t in out_tensors]
    if len(ys) == 1:
        out = g.add("StatefulPartitionedCall", "Identity", ys, T=T)
        out_names = [f"{out}:0"]
    else:
        out = g.add("StatefulPartitionedCall", "IdentityN", ys, T=Attr.tlist([_F32] * len(ys)))
        out_names = [f"{out}:{i}" for i in range(len(ys))]

    # ---- V2 saver over the bundle keys model.save writes ----
    S = Attr.type(DT_STRING)
    fin = g.add("save/filename/input", "Const", dtype=S, value=Attr.tensor(tensor_proto(DT_STRING, [], strings=["model"])))
    fn = g.add("save/filename", "PlaceholderWithDefault", [fin], dtype=S, shape=Attr.shape([]))
    fc = g.add("save/Const", "PlaceholderWithDefault", [fn], dtype=S, shape=Attr.shape([]))
    nv = len(bundle_keys)
    names_t = Attr.tensor(tensor_proto(DT_STRING, [nv], strings=bundle_keys))
    slices_t = Attr.tensor(tensor_proto(DT_STRING, [nv], strings=[""] * nv))
    dts = Attr.tlist([_F32] * nv)
    sn = g.add("save/SaveV2/tensor_names", "Const", dtype=S, value=names_t)
    ss = g.add("save/SaveV2/shape_and_slices", "Const", dtype=S, value=slices_t)
    reads = [f"{_var_name(v)}/Read/ReadVariableOp" for v in model.weights]
    sv = g.add("save/SaveV2", "SaveV2", [fc, sn, ss] + reads, dtypes=dts)
    cd = g.add("save/control_dependency", "Identity", [fc, f"^{sv}"], T=S, _class=Attr.slist([f"loc:@{fc}"]))
    rn = g.add("save/RestoreV2/tensor_names", "Const", dtype=S, value=names_t)
    rs = g.add("save/RestoreV2/shape_and_slices", "Const", dtype=S, value=slices_t)
    rv = g.add("save/RestoreV2", "RestoreV2", [fc, rn, rs], dtypes=dts)
    assigns = []
    for k, v in enumerate(model.weights):
        idn = g.add("save/Identity", "Identity", [f"{rv}:{k}" if k else rv], T=T)
        assigns.append(g.add("save/AssignVariableOp", "AssignVariableOp", [var_of[id(v)], idn], dtype=T))
    ra = g.add("save/restore_all", "NoOp", [f"^{a}" for a in assigns])

    # GraphDef: 1 node, 4 versions (VersionDef: 1 producer)
    gd = b"".join(_field_bytes(1, n) for n in g.nodes) + _field_bytes(4, _field_varint(1, producer))
    collections = {"variables": collection_bytes_list(var_defs)}
    if train_defs:
        collections["trainable_variables"] = collection_bytes_list(train_defs)
    saver = {"filename_tensor_name": f"{fc}:0", "save_tensor_name": f"{cd}:0", "restore_op_name": ra}
    return GraphSpec(gd, collections, saver, sig_inputs, out_names)


def _emit_layer(g: _Graph, layer, sc: str, xs: List[str], in_shape, read) -> str:
    from ..keras import layers as L

    T = Attr.type(_F32)
    NHWC = Attr.s("NHWC")
    x = xs[0]
    if isinstance(layer, L.Conv2D):
        if tuple(layer.dilation_rate) != (1, 1) and tuple(layer.strides) != (1, 1):
            raise UnsupportedLayer("Conv2D with both strides and dilations")
        k = read(layer, layer.kernel)
        y = g.add(f"{sc}/Conv2D", "Conv2D", [x, k], T=T, data_format=NHWC,
                  dilations=Attr.ilist([1, *layer.dilation_rate, 1]), explicit_paddings=Attr.ilist([]),
                  padding=Attr.s(layer.padding.upper()), strides=Attr.ilist([1, *layer.strides, 1]),
                  use_cudnn_on_gpu=Attr.b(True))
        if layer.use_bias:
            y = g.add(f"{sc}/BiasAdd", "BiasAdd", [y, read(layer, layer.bias)], T=T, data_format=NHWC)
        return _activation(g, sc, y, _act_name(layer.activation))
    if isinstance(layer, L.Dense):
        if in_shape is not None and len(in_shape) != 2:
            raise UnsupportedLayer("Dense on a rank > 2 input (Tensordot) has no mapping here")
        y = g.add(f"{sc}/MatMul", "MatMul", [x, read(layer, layer.kernel)], T=T, transpose_a=Attr.b(False),
                  transpose_b=Attr.b(False))
        if layer.use_bias:
            y = g.add(f"{sc}/BiasAdd", "BiasAdd", [y, read(layer, layer.bias)], T=T, data_format=NHWC)
        return _activation(g, sc, y, _act_name(layer.activation))
    if isinstance(layer, (L.MaxPooling2D, L.AveragePooling2D)):
        op = "MaxPool" if isinstance(layer, L.MaxPooling2D) else "AvgPool"
        extra = {"explicit_paddings": Attr.ilist([])} if op == "MaxPool" else {}
        return g.add(f"{sc}/{op}", op, [x], T=T, data_format=NHWC, ksize=Attr.ilist([1, *layer.pool_size, 1]),
                     padding=_pool_padding(layer.padding), strides=Attr.ilist([1, *layer.strides, 1]), **extra)
    if isinstance(layer, L.GlobalAveragePooling2D):  # (GlobalMaxPooling2D subclasses it)
        op = "Max" if isinstance(layer, L.GlobalMaxPooling2D) else "Mean"
        ax = g.const_i32(f"{sc}/{op}/reduction_indices", [1, 2], [2])
        return g.add(f"{sc}/{op}", op, [x, ax], T=T, Tidx=Attr.type(_I32), keep_dims=Attr.b(bool(layer.keepdims)))
    if isinstance(layer, (L.Flatten, L.Reshape)):
        if isinstance(layer, L.Flatten):
            if in_shape is None or any(d is None for d in in_shape[1:]):
                raise UnsupportedLayer("Flatten of an input with unknown dimensions")
            tgt = [-1, int(math.prod(in_shape[1:]))]
        else:
            tgt = [-1] + [int(d) for d in layer.target_shape]
        sh = g.const_i32(f"{sc}/Const", tgt, [len(tgt)])
        return g.add(f"{sc}/Reshape", "Reshape", [x, sh], T=T, Tshape=Attr.type(_I32))
    if isinstance(layer, L.Activation):
        return _activation(g, sc, x, _act_name(layer.activation))
    if isinstance(layer, L.ReLU):
        if layer.negative_slope or layer.threshold:
            raise UnsupportedLayer("ReLU with negative_slope / threshold")
        if layer.max_value is None:
            return g.add(f"{sc}/Relu", "Relu", [x], T=T)
        if float(layer.max_value) == 6.0:
            return g.add(f"{sc}/Relu6", "Relu6", [x], T=T)
        r = g.add(f"{sc}/Relu", "Relu", [x], T=T)
        return g.add(f"{sc}/Minimum", "Minimum", [r, g.const_f32(f"{sc}/max_value", float(layer.max_value))], T=T)
    if isinstance(layer, L.Softmax):
        if layer.axis not in (-1, len(in_shape or [0, 0]) - 1):
            raise UnsupportedLayer("Softmax over a non-last axis")
        return g.add(f"{sc}/Softmax", "Softmax", [x], T=T)
    if isinstance(layer, L.Dropout):
        return g.add(f"{sc}/Identity", "Identity", [x], T=T)  # inference: no dropout
    if isinstance(layer, L.Rescaling):
        y = g.add(f"{sc}/mul", "Mul", [x, g.const_f32(f"{sc}/Cast", float(layer.scale))], T=T)
        return g.add(f"{sc}/add", "AddV2", [y, g.const_f32(f"{sc}/Cast_1", float(layer.offset))], T=T)
    if isinstance(layer, L.ZeroPadding2D):
        (t, b), (l, r) = layer.padding
        pads = g.const_i32(f"{sc}/Pad/paddings", [0, 0, t, b, l, r, 0, 0], [4, 2])
        return g.add(f"{sc}/Pad", "Pad", [x, pads], T=T, Tpaddings=Attr.type(_I32))
    if isinstance(layer, L.BatchNormalization):
        ax = layer.axis if isinstance(layer.axis, int) else (layer.axis[0] if len(layer.axis) == 1 else None)
        if ax not in (-1, 3) or (in_shape is not None and len(in_shape) != 4):
            raise UnsupportedLayer("BatchNormalization other than over the channels of an NHWC tensor")
        c = int(layer.moving_mean.shape[0])

        def ones_or(v, val, nm):
            if v is not None:
                return read(layer, v)
            return g.add(f"{sc}/{nm}", "Const", dtype=T, value=Attr.tensor(tensor_proto(_F32, [c], floats=[val])))

        gam, bet = ones_or(layer.gamma, 1.0, "Const"), ones_or(layer.beta, 0.0, "Const_1")
        return g.add(f"{sc}/FusedBatchNormV3", "FusedBatchNormV3",
                     [x, gam, bet, read(layer, layer.moving_mean), read(layer, layer.moving_variance)], T=T,
                     U=T, data_format=NHWC, epsilon=Attr.f(layer.epsilon), exponential_avg_factor=Attr.f(1.0),
                     is_training=Attr.b(False))
    if isinstance(layer, L.Add):
        if len(xs) == 2:
            return g.add(f"{sc}/add", "AddV2", xs, T=T)
        return g.add(f"{sc}/AddN", "AddN", xs, N=Attr.i(len(xs)), T=T)
    if isinstance(layer, L.Subtract):
        return g.add(f"{sc}/sub", "Sub", xs, T=T)
    if isinstance(layer, L.Multiply):
        y = xs[0]
        for k, z in enumerate(xs[1:]):
            y = g.add(f"{sc}/mul" + (f"_{k}" if k else ""), "Mul", [y, z], T=T)
        return y
    if isinstance(layer, L.Average):
        s = g.add(f"{sc}/AddN", "AddN", xs, N=Attr.i(len(xs)), T=T)
        return g.add(f"{sc}/truediv", "Mul", [s, g.const_f32(f"{sc}/inv_n", 1.0 / len(xs))], T=T)
    if isinstance(layer, L.Maximum):
        y = xs[0]
        for k, z in enumerate(xs[1:]):
            y = g.add(f"{sc}/Maximum" + (f"_{k}" if k else ""), "Maximum", [y, z], T=T)
        return y
    if isinstance(layer, L.Concatenate):
        rank = len(in_shape) if in_shape is not None else 4
        ax = layer.axis if layer.axis >= 0 else rank + layer.axis
        a = g.const_i32(f"{sc}/concat/axis", [ax], [])
        return g.add(f"{sc}/concat", "ConcatV2", xs + [a], N=Attr.i(len(xs)), T=T, Tidx=Attr.type(_I32))
    raise UnsupportedLayer(f"{type(layer).__name__} ({layer.name}) has no TF op mapping here")


# ------------------------------------------------------------------------------------ interpreter
def _decode_attr(buf: bytes):
    f = _parse(buf)
    if 2 in f:
        return f[2][0].decode()
    if 3 in f:
        v = f[3][0]
        return v - (1 << 64) if v >= (1 << 63) else v
    if 4 in f:
        return struct.unpack("<f", struct.pack("<I", f[4][0]))[0]
    if 5 in f:
        return bool(f[5][0])
    if 6 in f:
        return ("type", f[6][0])
    if 7 in f:
        return ("shape", _decode_shape(f[7][0]))
    if 8 in f:
        return _decode_tensor(f[8][0])
    if 1 in f:
        lf = _parse(f[1][0])
        if 2 in lf:
            return [x.decode() for x in lf[2]]
        for num in (3, 6):
            if num in lf:
                return [_signed(v) for v in _unpack_varints(lf[num])]
        return []
    return None


def _signed(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def _unpack_varints(chunks) -> List[int]:
    from .tensor_bundle import _read_varint

    out = []
    for c in chunks:
        if isinstance(c, int):
            out.append(c)
            continue
        pos = 0
        while pos < len(c):
            v, pos = _read_varint(c, pos)
            out.append(v)
    return out


def _decode_shape(buf: bytes):
    f = _parse(buf)
    if f.get(3, [0])[0]:
        return None
    return [_signed(_parse(d).get(1, [0])[0]) for d in f.get(2, [])]


def _decode_tensor(buf: bytes):
    f = _parse(buf)
    dt = f.get(1, [0])[0]
    shape = _decode_shape(f[2][0]) if 2 in f else []
    if dt == DT_STRING:
        vals = [x.decode() for x in f.get(8, [])]
        return np.array(vals if shape else (vals[0] if vals else ""), dtype=object).reshape(shape)
    np_dt = {_F32: np.float32, _I32: np.int32}[dt]
    if 4 in f:
        return np.frombuffer(f[4][0], dtype=np_dt).reshape(shape).copy()
    if dt == _F32:
        vals = [v for c in f.get(5, []) for v in (struct.unpack(f"<{len(c) // 4}f", c) if isinstance(c, bytes)
                                                   else struct.unpack("<f", struct.pack("<I", c)))]
    else:
        vals = [_signed(v) for v in _unpack_varints(f.get(7, []))]
    arr = np.array(vals, dtype=np_dt)
    n = int(np.prod(shape)) if shape else 1
    return (np.full(n, arr[0] if arr.size else 0, dtype=np_dt) if arr.size in (0, 1) else arr).reshape(shape)


def parse_graph_def(buf: bytes) -> Dict[str, dict]:
    """GraphDef bytes -> {node name: {op, inputs, attrs}} (attrs decoded)."""
    nodes = {}
    for nb in _parse(buf).get(1, []):
        f = _parse(nb)
        attrs = {}
        for e in f.get(5, []):
            ef = _parse(e)
            attrs[ef[1][0].decode()] = _decode_attr(ef.get(2, [b""])[0])
        name = f[1][0].decode()
        nodes[name] = {"op": f[2][0].decode(), "inputs": [x.decode() for x in f.get(3, [])], "attrs": attrs}
    return nodes


def run_graph(nodes: Dict[str, dict], fetches: Sequence[str], feeds: Optional[Dict[str, np.ndarray]] = None,
              variables: Optional[Dict[str, np.ndarray]] = None, bundle: Optional[Dict[str, np.ndarray]] = None):
    """Evaluate ``fetches`` ("node" or "node:k") of a parsed graph on the CPU.

    ``variables`` is the resource store (shared name -> array), updated in place by
    AssignVariableOp; ``bundle`` is what RestoreV2 reads (key -> array).  Supports the ops
    ``build_graph`` emits."""
    import torch
    import torch.nn.functional as F

    feeds = dict(feeds or {})
    store = variables if variables is not None else {}
    cache: Dict[str, list] = {}

    def tensor(ref: str):
        name, _, k = ref.partition(":")
        return run(name)[int(k) if k else 0]

    def run(name: str) -> list:
        if name in cache:
            return cache[name]
        if f"{name}:0" in feeds or name in feeds:
            cache[name] = [np.asarray(feeds.get(f"{name}:0", feeds.get(name)))]
            return cache[name]
        nd = nodes[name]
        op, a = nd["op"], nd["attrs"]
        for ctl in (i for i in nd["inputs"] if i.startswith("^")):
            run(ctl[1:])
        ins = [tensor(i) for i in nd["inputs"] if not i.startswith("^")]
        t = lambda v: torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))  # noqa: E731
        nchw = lambda v: t(v).permute(0, 3, 1, 2)  # noqa: E731
        nhwc = lambda v: v.permute(0, 2, 3, 1).contiguous().numpy()  # noqa: E731

        def same_pad(h, k, s, d=1):
            out = -(-h // s)
            tot = max((out - 1) * s + (k - 1) * d + 1 - h, 0)
            return tot // 2, tot - tot // 2

        if op == "Placeholder":
            raise KeyError(f"placeholder {name} not fed")
        elif op in ("Const",):
            out = [a["value"]]
        elif op == "PlaceholderWithDefault":
            out = [ins[0]]
        elif op == "VarHandleOp":
            out = [a["shared_name"]]
        elif op == "ReadVariableOp":
            out = [np.asarray(store[ins[0]], np.float32)]
        elif op == "AssignVariableOp":
            store[ins[0]] = np.array(ins[1], np.float32)
            out = [None]
        elif op == "RestoreV2":
            out = [np.asarray(bundle[k], np.float32) for k in ins[1].reshape(-1)]
        elif op in ("SaveV2", "NoOp"):
            out = [None]
        elif op == "Identity":
            out = [ins[0]]
        elif op == "IdentityN":
            out = list(ins)
        elif op == "Conv2D":
            x, w = nchw(ins[0]), t(ins[1]).permute(3, 2, 0, 1)
            s, d = a["strides"][1:3], a["dilations"][1:3]
            if a["padding"] == "SAME":
                ph = same_pad(x.shape[2], w.shape[2], s[0], d[0])
                pw = same_pad(x.shape[3], w.shape[3], s[1], d[1])
                x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]))
            grp = x.shape[1] // w.shape[1]
            out = [nhwc(F.conv2d(x, w, stride=s, dilation=d, groups=grp))]
        elif op == "BiasAdd":
            out = [ins[0] + ins[1]]
        elif op in ("MaxPool", "AvgPool"):
            x, k, s = nchw(ins[0]), a["ksize"][1:3], a["strides"][1:3]
            if a["padding"] == "SAME":
                ph, pw = same_pad(x.shape[2], k[0], s[0]), same_pad(x.shape[3], k[1], s[1])
                if op == "MaxPool":
                    x = F.pad(x, (pw[0], pw[1], ph[0], ph[1]), value=float("-inf"))
                    y = F.max_pool2d(x, k, s)
                else:
                    ones = F.pad(torch.ones_like(x[:, :1]), (pw[0], pw[1], ph[0], ph[1]))
                    y = F.avg_pool2d(F.pad(x, (pw[0], pw[1], ph[0], ph[1])), k, s) / F.avg_pool2d(ones, k, s)
            else:
                y = F.max_pool2d(x, k, s) if op == "MaxPool" else F.avg_pool2d(x, k, s)
            out = [nhwc(y)]
        elif op in ("Mean", "Max"):
            ax = tuple(int(v) for v in np.asarray(ins[1]).reshape(-1))
            fn = np.mean if op == "Mean" else np.max
            out = [fn(ins[0], axis=ax, keepdims=a.get("keep_dims", False)).astype(np.float32)]
        elif op == "Reshape":
            out = [ins[0].reshape([int(v) for v in np.asarray(ins[1]).reshape(-1)])]
        elif op == "MatMul":
            out = [ins[0] @ ins[1]]
        elif op == "Pad":
            out = [np.pad(ins[0], np.asarray(ins[1]).reshape(-1, 2))]
        elif op == "FusedBatchNormV3":
            x, gm, bt, mu, var = ins
            y = (x - mu) / np.sqrt(var + np.float32(a["epsilon"])) * gm + bt
            out = [y.astype(np.float32), mu, var, mu, var, mu]
        elif op in ("AddV2", "Sub", "Mul", "Maximum", "Minimum"):
            fn = {"AddV2": np.add, "Sub": np.subtract, "Mul": np.multiply, "Maximum": np.maximum,
                  "Minimum": np.minimum}[op]
            out = [fn(ins[0], ins[1]).astype(np.float32)]
        elif op == "AddN":
            out = [np.sum(np.stack(ins), 0).astype(np.float32)]
        elif op == "ConcatV2":
            out = [np.concatenate(ins[:-1], axis=int(np.asarray(ins[-1])))]
        else:
            x = t(ins[0])
            fn = {"Relu": F.relu, "Relu6": F.relu6, "Sigmoid": torch.sigmoid, "Tanh": torch.tanh,
                  "Softmax": lambda v: F.softmax(v, -1), "LogSoftmax": lambda v: F.log_softmax(v, -1),
                  "Elu": F.elu, "Selu": F.selu, "Softplus": F.softplus, "Softsign": F.softsign,
                  "Exp": torch.exp}.get(op)
            if fn is None:
                raise NotImplementedError(f"run_graph: op {op}")
            out = [fn(x).numpy()]
        cache[name] = out
        return out

    return [tensor(f) if not f.startswith("^") else run(f[1:])[0] for f in fetches]
