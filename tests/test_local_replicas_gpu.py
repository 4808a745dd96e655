"""Single-process multi-device MirroredStrategy on the GPU: ONE process drives two
"devices" mapped onto the box's GPU (TDL_SHARE_GPU=1), the reference CNN trains on the fused MI355X
kernels in both replica threads, the replicas stay bit-identical and match one replica on the same
global batches."""
import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn

pytestmark = pytest.mark.gpu


def _fit(strategy, steps=8):
    tdl.keras.utils.set_random_seed(11)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(1024, 28, 28, 1, generator=g)
    y = torch.randint(0, 10, (1024,), generator=g, dtype=torch.int64)
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(128).repeat()
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05),
                  metrics=[tdl.keras.metrics.SparseCategoricalAccuracy()], steps_per_execution=4)
    h = m.fit(ds, epochs=2, steps_per_epoch=steps // 2, verbose=0)
    return m, h


def test_two_devices_one_process_fused_engine(monkeypatch):
    monkeypatch.setenv("TDL_SHARE_GPU", "1")
    s = tdl.distribute.MirroredStrategy(devices=["/gpu:0", "/gpu:1"])
    assert s.num_replicas_in_sync == 2 and s._local_group is not None
    m, h = _fit(s)
    assert m._trainer.kind == "fused", getattr(m, "_fused_reason", None)
    (c,) = m._local_clones
    assert c._trainer.kind == "fused" and c._trainer.rank == 1 and c._trainer.R == 2
    for a, b in zip(m.get_weights(), c.get_weights()):
        assert np.array_equal(a, b), "replicas differ"
    m1, h1 = _fit(tdl.distribute.MirroredStrategy(devices=["/gpu:0"]))
    for a, b in zip(m.get_weights(), m1.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-3, atol=1e-5)
    np.testing.assert_allclose(h.history["loss"], h1.history["loss"], rtol=1e-4)
    assert s.experimental_local_results(1.0) == (1.0,)
    s.shutdown()
