"""The TensorFlow GraphDef inside ``saved_model.pb`` (ckpt/graph_def.py; README.md:51: the chief saves
the model).  TensorFlow is not installed here, so loading the directory with TF is parity unpinned;
these tests pin what can be pinned without it:

* the bytes parse with the ``protobuf`` runtime against descriptors of TF's GraphDef / NodeDef /
  AttrValue / TensorProto / CollectionDef / VariableDef / MetaGraphDef messages (field numbers of
  tensorflow/core/framework/*.proto), with no unknown fields and nothing lost on re-encoding;
* executing the graph's own bytes (``graph_def.run_graph``: restore op fed with the variables
  bundle, then the serving signature's tensors) reproduces ``model.predict`` -- for the reference
  CNN (tf_dist_example.py:40-48) and for a functional model with BN / residual Add / Concatenate /
  padding / global pooling (the ResNet-50 layer set);
* the variable initializers, the VariableDef collections and the saver names agree with the graph.
"""
import os

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.ckpt import checkpoint as C
from tensorflow_distributed_learning_amd.ckpt import graph_def as GD
from tensorflow_distributed_learning_amd.ckpt import saved_model_pb as SMP
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

keras = tdl.keras
L = keras.layers


def _load(path):
    buf = open(os.path.join(path, "saved_model.pb"), "rb").read()
    mg = SMP.parse_saved_model(buf)["meta_graphs"][0]
    return buf, mg, GD.parse_graph_def(mg["graph_def"])


def _serve(path, x):
    """Restore from variables/ through the graph's own saver, then run serving_default on x."""
    _, mg, nodes = _load(path)
    bundle = {k: v.numpy() for k, v in C.read_bundle(os.path.join(path, "variables", "variables")).items()}
    store = {}
    sv = mg["saver"]
    GD.run_graph(nodes, ["^" + sv["restore_op_name"]], feeds={sv["filename_tensor_name"]: "variables/variables"},
                 variables=store, bundle=bundle)
    sig = mg["signature_def"]["serving_default"]
    (ik, iv), = sig["inputs"].items()
    outs = GD.run_graph(nodes, [o["name"] for o in sig["outputs"].values()], feeds={iv["name"]: x}, variables=store)
    return outs, nodes, mg, store


def test_mnist_cnn_graph_reproduces_predict(tmp_path):
    keras.backend.clear_session()
    keras.utils.set_random_seed(3)
    m = build_mnist_cnn()
    m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=keras.optimizers.SGD(0.01))
    x = torch.rand(5, 28, 28, 1)
    ref = m.predict(x, verbose=0)
    ref = ref.numpy() if hasattr(ref, "numpy") else np.asarray(ref)
    p = str(tmp_path / "sm")
    m.save(p)
    (y,), nodes, mg, store = _serve(p, x.numpy())
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-5)
    ops = {n["op"] for n in nodes.values()}
    assert {"Conv2D", "BiasAdd", "Relu", "MaxPool", "Reshape", "MatMul", "VarHandleOp", "ReadVariableOp",
            "RestoreV2", "SaveV2", "AssignVariableOp"} <= ops
    # every model variable was restored under its Keras name (the bundle key)
    assert sorted(store) == sorted(v.name[:-2] for v in m.weights)
    for v in m.weights:
        np.testing.assert_array_equal(store[v.name[:-2]], v.read_value().numpy())
    # the initializers assign zeros of the variable's shape
    fresh = {}
    GD.run_graph(nodes, ["^conv2d/kernel/Assign"], variables=fresh)
    assert fresh["conv2d/kernel"].shape == (3, 3, 1, 32) and not fresh["conv2d/kernel"].any()
    # VariableDef collections name nodes of the graph
    vdefs = [GD._parse(b) for b in GD._parse(GD._parse(mg["collection_def"]["variables"])[2][0])[1]]
    assert len(vdefs) == 8
    for vd in vdefs:
        for fld in (1, 2, 3, 6):
            assert vd[fld][0].decode().split(":")[0] in nodes
        assert vd[5] == [1]
    assert mg["saver"] == {"filename_tensor_name": "save/Const:0", "save_tensor_name": "save/control_dependency:0",
                           "restore_op_name": "save/restore_all"}


def _resnet_like():
    inp = L.Input(shape=(12, 12, 3), name="image")
    x = L.ZeroPadding2D(((1, 1), (1, 1)))(inp)
    x = L.Conv2D(8, 3, strides=2, use_bias=False)(x)
    x = L.BatchNormalization(epsilon=1.001e-5)(x)
    x = L.Activation("relu")(x)
    s = L.Conv2D(8, 1, use_bias=False)(x)
    y = L.Conv2D(8, 3, padding="same")(x)
    y = L.BatchNormalization()(y)
    y = L.ReLU()(y)
    x = L.Add()([s, y])
    c = L.Concatenate()([x, L.MaxPooling2D(3, strides=1, padding="same")(x)])
    c = L.AveragePooling2D(2)(c)
    g = L.GlobalAveragePooling2D()(c)
    g = L.Dropout(0.5)(g)
    out = L.Dense(4, activation="softmax", name="probs")(g)
    return keras.Model(inp, out)


def test_functional_resnet_like_graph_reproduces_predict(tmp_path):
    keras.backend.clear_session()
    keras.utils.set_random_seed(5)
    m = _resnet_like()
    gen = torch.Generator().manual_seed(0)
    for l in m.layers:  # non-trivial BN statistics / affine
        if isinstance(l, L.BatchNormalization):
            c = l.moving_mean.shape[0]
            l.moving_mean.assign(torch.randn(c, generator=gen) * 0.1)
            l.moving_variance.assign(torch.rand(c, generator=gen) + 0.5)
            l.gamma.assign(torch.rand(c, generator=gen) + 0.5)
            l.beta.assign(torch.randn(c, generator=gen) * 0.1)
    x = torch.randn(3, 12, 12, 3, generator=gen)
    ref = m.predict(x, verbose=0)
    ref = ref.numpy() if hasattr(ref, "numpy") else np.asarray(ref)
    p = str(tmp_path / "fm")
    m.save(p)
    (y,), nodes, mg, _ = _serve(p, x.numpy())
    np.testing.assert_allclose(y, ref, rtol=1e-5, atol=1e-6)
    ops = {n["op"] for n in nodes.values()}
    assert {"Pad", "FusedBatchNormV3", "AddV2", "ConcatV2", "AvgPool", "Mean", "Softmax", "Identity"} <= ops
    sig = mg["signature_def"]["serving_default"]
    assert list(sig["inputs"]) == ["image"] and sig["inputs"]["image"]["name"] == "serving_default_image:0"
    assert list(sig["outputs"]) == ["probs"] and sig["outputs"]["probs"]["name"] == "StatefulPartitionedCall:0"
    # non-trainable BN statistics are variables but not trainable_variables
    n_train = len(GD._parse(GD._parse(mg["collection_def"]["trainable_variables"])[2][0])[1])
    n_all = len(GD._parse(GD._parse(mg["collection_def"]["variables"])[2][0])[1])
    assert n_all - n_train == 4


def test_unsupported_layer_keeps_header_only(tmp_path):
    keras.backend.clear_session()
    inp = L.Input(shape=(4,))
    out = L.Dense(2)(L.Lambda(lambda t: t * 2)(inp))
    m = keras.Model(inp, out)
    p = str(tmp_path / "lm")
    with pytest.warns(UserWarning, match="without a TF graph"):
        m.save(p)
    _, mg, nodes = _load(p)
    assert nodes == {} and mg["signature_def"]["serving_default"]["outputs"]


# ---------------------------------------------------------------- protobuf-runtime conformance
def _messages():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="tdl_graph_def_test.proto", package="tdlg", syntax="proto3")
    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED

    def msg(name, fields, nested=(), oneof=None):
        m = fd.message_type.add(name=name)
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        if oneof:
            m.oneof_decl.add(name=oneof)
        for fname, num, ftype, label, tname, *rest in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
            if rest and rest[0] == "oneof":
                f.oneof_index = 0
        return m

    def entry(name, vname):
        e = descriptor_pb2.DescriptorProto(name=name)
        e.field.add(name="key", number=1, type=F.TYPE_STRING, label=O)
        e.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=O, type_name=vname)
        e.options.map_entry = True
        return e

    dim = descriptor_pb2.DescriptorProto(name="Dim")
    dim.field.add(name="size", number=1, type=F.TYPE_INT64, label=O)
    dim.field.add(name="name", number=2, type=F.TYPE_STRING, label=O)
    msg("TensorShapeProto", [("dim", 2, F.TYPE_MESSAGE, R, ".tdlg.TensorShapeProto.Dim"),
                             ("unknown_rank", 3, F.TYPE_BOOL, O, None)], [dim])
    msg("TensorProto", [("dtype", 1, F.TYPE_ENUM if False else F.TYPE_INT32, O, None),
                        ("tensor_shape", 2, F.TYPE_MESSAGE, O, ".tdlg.TensorShapeProto"),
                        ("version_number", 3, F.TYPE_INT32, O, None), ("tensor_content", 4, F.TYPE_BYTES, O, None),
                        ("float_val", 5, F.TYPE_FLOAT, R, None), ("int_val", 7, F.TYPE_INT32, R, None),
                        ("string_val", 8, F.TYPE_BYTES, R, None)])
    lv = descriptor_pb2.DescriptorProto(name="ListValue")
    for fname, num, ftype, tname in (("s", 2, F.TYPE_BYTES, None), ("i", 3, F.TYPE_INT64, None),
                                     ("f", 4, F.TYPE_FLOAT, None), ("b", 5, F.TYPE_BOOL, None),
                                     ("type", 6, F.TYPE_INT32, None),
                                     ("shape", 7, F.TYPE_MESSAGE, ".tdlg.TensorShapeProto"),
                                     ("tensor", 8, F.TYPE_MESSAGE, ".tdlg.TensorProto")):
        f = lv.field.add(name=fname, number=num, type=ftype, label=R)
        if tname:
            f.type_name = tname
    msg("AttrValue", [("list", 1, F.TYPE_MESSAGE, O, ".tdlg.AttrValue.ListValue", "oneof"),
                      ("s", 2, F.TYPE_BYTES, O, None, "oneof"), ("i", 3, F.TYPE_INT64, O, None, "oneof"),
                      ("f", 4, F.TYPE_FLOAT, O, None, "oneof"), ("b", 5, F.TYPE_BOOL, O, None, "oneof"),
                      ("type", 6, F.TYPE_INT32, O, None, "oneof"),
                      ("shape", 7, F.TYPE_MESSAGE, O, ".tdlg.TensorShapeProto", "oneof"),
                      ("tensor", 8, F.TYPE_MESSAGE, O, ".tdlg.TensorProto", "oneof")], [lv], oneof="value")
    msg("NodeDef", [("name", 1, F.TYPE_STRING, O, None), ("op", 2, F.TYPE_STRING, O, None),
                    ("input", 3, F.TYPE_STRING, R, None), ("device", 4, F.TYPE_STRING, O, None),
                    ("attr", 5, F.TYPE_MESSAGE, R, ".tdlg.NodeDef.AttrEntry")],
        [entry("AttrEntry", ".tdlg.AttrValue")])
    msg("VersionDef", [("producer", 1, F.TYPE_INT32, O, None), ("min_consumer", 2, F.TYPE_INT32, O, None)])
    msg("GraphDef", [("node", 1, F.TYPE_MESSAGE, R, ".tdlg.NodeDef"),
                     ("versions", 4, F.TYPE_MESSAGE, O, ".tdlg.VersionDef")])
    msg("VariableDef", [("variable_name", 1, F.TYPE_STRING, O, None), ("initializer_name", 2, F.TYPE_STRING, O, None),
                        ("snapshot_name", 3, F.TYPE_STRING, O, None), ("is_resource", 5, F.TYPE_BOOL, O, None),
                        ("initial_value_name", 6, F.TYPE_STRING, O, None), ("trainable", 7, F.TYPE_BOOL, O, None)])
    bl = descriptor_pb2.DescriptorProto(name="BytesList")
    bl.field.add(name="value", number=1, type=F.TYPE_BYTES, label=R)
    msg("CollectionDef", [("bytes_list", 2, F.TYPE_MESSAGE, O, ".tdlg.CollectionDef.BytesList")], [bl])
    msg("SaverDef", [("filename_tensor_name", 1, F.TYPE_STRING, O, None),
                     ("save_tensor_name", 2, F.TYPE_STRING, O, None),
                     ("restore_op_name", 3, F.TYPE_STRING, O, None), ("max_to_keep", 4, F.TYPE_INT32, O, None),
                     ("sharded", 5, F.TYPE_BOOL, O, None),
                     ("keep_checkpoint_every_n_hours", 6, F.TYPE_FLOAT, O, None), ("version", 7, F.TYPE_INT32, O, None)])
    ti = descriptor_pb2.DescriptorProto(name="TensorInfo")
    ti.field.add(name="name", number=1, type=F.TYPE_STRING, label=O)
    ti.field.add(name="dtype", number=2, type=F.TYPE_INT32, label=O)
    ti.field.add(name="tensor_shape", number=3, type=F.TYPE_MESSAGE, label=O, type_name=".tdlg.TensorShapeProto")
    fd.message_type.add().CopyFrom(ti)
    msg("SignatureDef", [("inputs", 1, F.TYPE_MESSAGE, R, ".tdlg.SignatureDef.InputsEntry"),
                         ("outputs", 2, F.TYPE_MESSAGE, R, ".tdlg.SignatureDef.OutputsEntry"),
                         ("method_name", 3, F.TYPE_STRING, O, None)],
        [entry("InputsEntry", ".tdlg.TensorInfo"), entry("OutputsEntry", ".tdlg.TensorInfo")])
    msg("MetaInfoDef", [("meta_graph_version", 1, F.TYPE_STRING, O, None), ("tags", 4, F.TYPE_STRING, R, None),
                        ("tensorflow_version", 5, F.TYPE_STRING, O, None),
                        ("tensorflow_git_version", 6, F.TYPE_STRING, O, None),
                        ("stripped_default_attrs", 7, F.TYPE_BOOL, O, None)])
    msg("MetaGraphDef", [("meta_info_def", 1, F.TYPE_MESSAGE, O, ".tdlg.MetaInfoDef"),
                         ("graph_def", 2, F.TYPE_MESSAGE, O, ".tdlg.GraphDef"),
                         ("saver_def", 3, F.TYPE_MESSAGE, O, ".tdlg.SaverDef"),
                         ("collection_def", 4, F.TYPE_MESSAGE, R, ".tdlg.MetaGraphDef.CollectionDefEntry"),
                         ("signature_def", 5, F.TYPE_MESSAGE, R, ".tdlg.MetaGraphDef.SignatureDefEntry")],
        [entry("CollectionDefEntry", ".tdlg.CollectionDef"), entry("SignatureDefEntry", ".tdlg.SignatureDef")])
    msg("SavedModel", [("saved_model_schema_version", 1, F.TYPE_INT64, O, None),
                       ("meta_graphs", 2, F.TYPE_MESSAGE, R, ".tdlg.MetaGraphDef")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(f"tdlg.{n}"))  # noqa: E731
    return get("SavedModel"), get("VariableDef")


def _no_unknown_fields(m):
    from google.protobuf import unknown_fields

    assert len(unknown_fields.UnknownFieldSet(m)) == 0, type(m).__name__
    for fd, v in m.ListFields():
        if fd.message_type is None:
            continue
        items = (v.values() if fd.message_type.GetOptions().map_entry else v) if fd.is_repeated else [v]
        for x in items:
            if hasattr(x, "ListFields"):
                _no_unknown_fields(x)


@pytest.mark.parametrize("which", ["mnist", "functional"])
def test_graph_bytes_conform_to_tf_messages(tmp_path, which):
    keras.backend.clear_session()
    keras.utils.set_random_seed(1)
    m = build_mnist_cnn() if which == "mnist" else _resnet_like()
    m(torch.zeros(2, 28, 28, 1) if which == "mnist" else torch.zeros(2, 12, 12, 3))
    p = str(tmp_path / "sm")
    m.save(p)
    buf = open(os.path.join(p, "saved_model.pb"), "rb").read()
    SavedModel, VariableDef = _messages()
    sm = SavedModel.FromString(buf)
    _no_unknown_fields(sm)
    # every byte is a known field: re-encoding loses nothing (the runtime's map-entry order may
    # differ from the key-sorted order written here, so compare messages and sizes, not bytes)
    again = sm.SerializeToString()
    assert len(again) == len(buf) and SavedModel.FromString(again) == sm
    g = sm.meta_graphs[0]
    names = {n.name for n in g.graph_def.node}
    assert len(names) == len(g.graph_def.node)  # unique node names
    for n in g.graph_def.node:  # every input names an existing node
        for i in n.input:
            assert i.lstrip("^").split(":")[0] in names, (n.name, i)
    conv = next(n for n in g.graph_def.node if n.op == "Conv2D")
    assert conv.attr["padding"].s == b"VALID" and list(conv.attr["strides"].list.i)[0] == 1
    assert conv.attr["T"].type == 1 and conv.attr["data_format"].s == b"NHWC"
    zeros = g.graph_def.node[[n.name for n in g.graph_def.node].index("conv2d/kernel/Initializer/zeros")] \
        if which == "mnist" else None
    if zeros is not None:
        assert [d.size for d in zeros.attr["value"].tensor.tensor_shape.dim] == [3, 3, 1, 32]
    vd = VariableDef.FromString(g.collection_def["variables"].bytes_list.value[0])
    assert vd.is_resource and vd.variable_name.split(":")[0] in names and vd.initializer_name in names
    assert g.saver_def.restore_op_name in names and g.saver_def.version == 2
    assert abs(g.saver_def.keep_checkpoint_every_n_hours - 10000.0) < 1e-3
    out = g.signature_def["serving_default"].outputs
    assert all(t.name.split(":")[0] in names for t in out.values())


def test_resnet50_maps_to_a_graph():
    """BASELINE config 4's model: every layer has a TF op mapping (53 Conv2D / FusedBatchNormV3)."""
    keras.backend.clear_session()
    m = keras.applications.ResNet50(weights=None)
    spec = GD.build_graph(m, SMP.GRAPH_PRODUCER)
    nodes = GD.parse_graph_def(spec.graph_def)
    ops = [n["op"] for n in nodes.values()]
    assert ops.count("Conv2D") == 53 and ops.count("FusedBatchNormV3") == 53 and ops.count("AddV2") == 16
    assert ops.count("VarHandleOp") == len(m.weights) and spec.outputs == ["StatefulPartitionedCall:0"]


def test_two_output_model_uses_identity_n(tmp_path):
    keras.backend.clear_session()
    keras.utils.set_random_seed(2)
    inp = L.Input(shape=(6,), name="x")
    h = L.Dense(5, activation="tanh")(inp)
    a = L.Dense(3, name="head_a")(h)
    b = L.Dense(2, activation="sigmoid", name="head_b")(h)
    m = keras.Model(inp, [a, b])
    x = torch.randn(4, 6)
    ra, rb = [r.numpy() if hasattr(r, "numpy") else np.asarray(r) for r in m.predict(x, verbose=0)]
    p = str(tmp_path / "two")
    m.save(p)
    outs, nodes, mg, _ = _serve(p, x.numpy())
    sig = mg["signature_def"]["serving_default"]["outputs"]
    assert sig["head_a"]["name"] == "StatefulPartitionedCall:0" and sig["head_b"]["name"] == "StatefulPartitionedCall:1"
    assert nodes["StatefulPartitionedCall"]["op"] == "IdentityN"
    got = dict(zip(sig, outs))
    np.testing.assert_allclose(got["head_a"], ra, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(got["head_b"], rb, rtol=1e-5, atol=1e-6)
