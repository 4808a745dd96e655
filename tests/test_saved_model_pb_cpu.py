"""``saved_model.pb`` (ckpt/saved_model_pb.py): written by model.save next to the variables bundle,
round-tripped by the module's own reader, and parsed by the ``protobuf`` runtime against descriptors
of TF's SavedModel / MetaGraphDef / SignatureDef / TensorInfo / SaverDef messages (field numbers of
tensorflow/core/protobuf/*.proto).  TensorFlow itself is not installed: loading the file with
``tf.saved_model.load`` is parity unpinned."""
import os

import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.ckpt import saved_model_pb as SMP
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

keras = tdl.keras


def _messages():
    """Message classes for the SavedModel header, built from a FileDescriptorProto (no .proto files)."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="tdl_saved_model_test.proto", package="tdltest", syntax="proto3")

    def msg(name, fields, nested=()):
        m = fd.message_type.add(name=name)
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        for fname, num, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED

    def entry(name, vtype, vname=None):
        e = descriptor_pb2.DescriptorProto(name=name)
        e.field.add(name="key", number=1, type=F.TYPE_STRING, label=O)
        v = e.field.add(name="value", number=2, type=vtype, label=O)
        if vname:
            v.type_name = vname
        e.options.map_entry = True
        return e

    dim = descriptor_pb2.DescriptorProto(name="Dim")
    dim.field.add(name="size", number=1, type=F.TYPE_INT64, label=O)
    dim.field.add(name="name", number=2, type=F.TYPE_STRING, label=O)
    msg("TensorShapeProto", [("dim", 2, F.TYPE_MESSAGE, R, ".tdltest.TensorShapeProto.Dim"),
                             ("unknown_rank", 3, F.TYPE_BOOL, O, None)], [dim])
    msg("TensorInfo", [("name", 1, F.TYPE_STRING, O, None), ("dtype", 2, F.TYPE_INT32, O, None),
                       ("tensor_shape", 3, F.TYPE_MESSAGE, O, ".tdltest.TensorShapeProto")])
    msg("SignatureDef", [("inputs", 1, F.TYPE_MESSAGE, R, ".tdltest.SignatureDef.InputsEntry"),
                         ("outputs", 2, F.TYPE_MESSAGE, R, ".tdltest.SignatureDef.OutputsEntry"),
                         ("method_name", 3, F.TYPE_STRING, O, None)],
        [entry("InputsEntry", F.TYPE_MESSAGE, ".tdltest.TensorInfo"),
         entry("OutputsEntry", F.TYPE_MESSAGE, ".tdltest.TensorInfo")])
    msg("VersionDef", [("producer", 1, F.TYPE_INT32, O, None), ("min_consumer", 2, F.TYPE_INT32, O, None)])
    # (the graph's nodes and the collections as opaque bytes here: tests/test_graph_def_cpu.py
    # checks them against NodeDef / CollectionDef descriptors)
    msg("GraphDef", [("node", 1, F.TYPE_BYTES, R, None), ("versions", 4, F.TYPE_MESSAGE, O, ".tdltest.VersionDef")])
    msg("SaverDef", [("filename_tensor_name", 1, F.TYPE_STRING, O, None),
                     ("save_tensor_name", 2, F.TYPE_STRING, O, None),
                     ("restore_op_name", 3, F.TYPE_STRING, O, None), ("max_to_keep", 4, F.TYPE_INT32, O, None),
                     ("sharded", 5, F.TYPE_BOOL, O, None),
                     ("keep_checkpoint_every_n_hours", 6, F.TYPE_FLOAT, O, None),
                     ("version", 7, F.TYPE_INT32, O, None)])
    msg("MetaInfoDef", [("meta_graph_version", 1, F.TYPE_STRING, O, None), ("tags", 4, F.TYPE_STRING, R, None),
                        ("tensorflow_version", 5, F.TYPE_STRING, O, None),
                        ("tensorflow_git_version", 6, F.TYPE_STRING, O, None),
                        ("stripped_default_attrs", 7, F.TYPE_BOOL, O, None)])
    msg("MetaGraphDef", [("meta_info_def", 1, F.TYPE_MESSAGE, O, ".tdltest.MetaInfoDef"),
                         ("graph_def", 2, F.TYPE_MESSAGE, O, ".tdltest.GraphDef"),
                         ("saver_def", 3, F.TYPE_MESSAGE, O, ".tdltest.SaverDef"),
                         ("collection_def", 4, F.TYPE_BYTES, R, None),
                         ("signature_def", 5, F.TYPE_MESSAGE, R, ".tdltest.MetaGraphDef.SignatureDefEntry")],
        [entry("SignatureDefEntry", F.TYPE_MESSAGE, ".tdltest.SignatureDef")])
    msg("SavedModel", [("saved_model_schema_version", 1, F.TYPE_INT64, O, None),
                       ("meta_graphs", 2, F.TYPE_MESSAGE, R, ".tdltest.MetaGraphDef")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tdltest.SavedModel"))


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


def test_model_save_writes_saved_model_pb(tmp_path):
    keras.backend.clear_session()
    keras.utils.set_random_seed(1)
    m = build_mnist_cnn()
    m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True), optimizer=keras.optimizers.SGD(0.01))
    m(torch.zeros(2, 28, 28, 1))
    p = str(tmp_path / "sm")
    m.save(p)
    assert set(os.listdir(p)) >= {"saved_model.pb", "saved_model.json", "variables", "assets"}
    buf = open(os.path.join(p, "saved_model.pb"), "rb").read()

    got = SMP.parse_saved_model(buf)
    assert got["saved_model_schema_version"] == 1 and len(got["meta_graphs"]) == 1
    mg = got["meta_graphs"][0]
    assert mg["tags"] == ["serve"] and mg["saver_version"] == 2
    sig = mg["signature_def"]["serving_default"]
    assert sig["method_name"] == "tensorflow/serving/predict"
    (ik, iv), = sig["inputs"].items()
    (ok, ov), = sig["outputs"].items()
    assert iv == {"name": f"serving_default_{ik}:0", "dtype": "float32", "shape": [None, 28, 28, 1]}
    assert ov == {"name": "StatefulPartitionedCall:0", "dtype": "float32", "shape": [None, 10]}

    SavedModel = _messages()
    sm = SavedModel.FromString(buf)
    _no_unknown_fields(sm)
    g = sm.meta_graphs[0]
    assert sm.saved_model_schema_version == 1 and list(g.meta_info_def.tags) == ["serve"]
    assert g.saver_def.version == 2 and g.graph_def.versions.producer == SMP.GRAPH_PRODUCER
    ti = g.signature_def["serving_default"].inputs[ik]
    assert ti.dtype == 1 and [d.size for d in ti.tensor_shape.dim] == [-1, 28, 28, 1]
    assert [d.size for d in g.signature_def["serving_default"].outputs[ok].tensor_shape.dim] == [-1, 10]
    # the protobuf runtime re-serialises it to the same bytes (canonical field order, no unknowns)
    assert sm.SerializeToString() == buf


def test_functional_model_signature_names_inputs_and_outputs():
    keras.backend.clear_session()
    L = keras.layers
    inp = L.Input(shape=(8,), name="features")
    out = L.Dense(3, name="logits")(L.Dense(4)(inp))
    m = keras.Model(inp, out)
    ins, outs = SMP.model_signature(m)
    assert ins == [("features", (None, 8), "float32")] and outs == [("logits", (None, 3), "float32")]
    got = SMP.parse_saved_model(SMP.encode_saved_model(ins, outs))
    assert got["meta_graphs"][0]["signature_def"]["serving_default"]["inputs"]["features"]["shape"] == [None, 8]


def test_unbuilt_model_raises():
    keras.backend.clear_session()
    m = keras.Sequential([keras.layers.Dense(3)])
    with pytest.raises(ValueError):
        SMP.model_signature(m)
