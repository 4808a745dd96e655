"""TDL_DEBUG_CHECKSUMS recorder (utils/checksums.py): per-op forward/backward checksums of the
generic engine's step, identical for identical runs, and the first-difference bisection."""
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.utils import checksums as ck

keras = tdl.keras
L = keras.layers


def _run(lr):
    keras.backend.clear_session()
    keras.utils.set_random_seed(3)
    inp = L.Input(shape=(6, 6, 4))
    x = L.Conv2D(8, 3, padding="same")(inp)
    x = L.Activation("relu")(L.BatchNormalization()(x))
    x = L.GlobalAveragePooling2D()(x)
    m = keras.Model(inp, L.Dense(5)(x))
    m.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=keras.optimizers.SGD(learning_rate=lr, momentum=0.9))
    g = torch.Generator().manual_seed(0)
    ds = tdl.data.Dataset.from_tensor_slices((torch.rand(32, 6, 6, 4, generator=g),
                                              torch.randint(0, 5, (32,), generator=g))).batch(16)
    ck.enable(True)
    ck.reset()
    try:
        m.fit(ds, epochs=1, verbose=0)
    finally:
        ck.enable(False)
    return [{"tag": t, "sum": d[0].item(), "abs": d[1].item(), "hash": d[2].item()} for t, d in ck._REC]


def test_checksums_record_forward_backward_and_slabs():
    a = _run(0.1)
    tags = [e["tag"] for e in a]
    assert any(t.startswith("node:conv2d") for t in tags)
    assert any(t.startswith("grad:node:") for t in tags)
    assert any(t.startswith("slab_grad:") for t in tags)
    assert tags.count("slab_W") == 2  # two steps
    assert ck.first_difference(a, _run(0.1)) is None
    d = ck.first_difference(a, _run(0.2))
    assert d is not None and d[1] == "slab_W"  # same forward/backward, different update
