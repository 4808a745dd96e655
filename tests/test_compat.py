"""The reference's API surface through the `tf` compat namespace."""
import os
import subprocess
import sys

import numpy as np
import torch

from tensorflow_distributed_learning_amd.compat import tf, tfds

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_api_names_exist():
    assert tf.distribute.experimental.MultiWorkerMirroredStrategy
    assert tf.distribute.MirroredStrategy
    ids = tf.distribute.experimental.CollectiveCommunication
    assert {ids.AUTO, ids.RING, ids.NCCL}
    assert tf.data.experimental.AutoShardPolicy.OFF.value == -1
    assert tf.keras.layers.Conv2D and tf.keras.layers.MaxPooling2D and tf.keras.layers.Flatten
    assert tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True).from_logits
    assert tf.keras.optimizers.SGD(learning_rate=0.001).current_lr() == 0.001
    assert tf.keras.metrics.SparseCategoricalAccuracy().name == "sparse_categorical_accuracy"
    o = tf.data.Options()
    o.experimental_distribute.auto_shard_policy = tf.data.experimental.AutoShardPolicy.OFF
    opts = tf.distribute.experimental.CommunicationOptions(implementation=tf.distribute.experimental.CommunicationImplementation.RING)
    assert opts.implementation.value == "RING"


def test_cast_does_not_alias():
    x = torch.ones(3)
    y = tf.cast(x, tf.float32)
    y /= 255
    assert torch.equal(x, torch.ones(3))


def test_numpy_to_dataset_readme_snippet():
    train_x, train_y = np.random.rand(10, 4), np.arange(10)
    ds = tf.data.Dataset.from_tensor_slices((train_x, train_y))
    assert ds.cardinality() == 10


def test_gradient_tape_custom_loop():
    strategy = tf.distribute.MirroredStrategy(devices=["/cpu:0"])
    with strategy.scope():
        dense = tf.keras.layers.Dense(1)
        dense.build((None, 3))
    opt = tf.keras.optimizers.SGD(0.1)
    x = torch.randn(32, 3)
    y = x @ torch.tensor([[1.0], [-2.0], [0.5]]) + 0.3
    first = None
    for _ in range(50):
        with tf.GradientTape() as tape:
            loss = ((dense(x) - y) ** 2).mean()
        grads = tape.gradient(loss, dense.trainable_variables)
        opt.apply_gradients(zip(grads, dense.trainable_variables))
        first = first if first is not None else float(loss)
    assert float(loss) < 0.1 * first


def test_strategy_reduce_run_scope():
    s = tf.distribute.MirroredStrategy(devices=["/cpu:0"])
    assert s.num_replicas_in_sync == 1
    out = s.run(lambda a: a * 2, args=(torch.tensor([1.0, 2.0]),))
    assert s.reduce(tf.distribute.ReduceOp.SUM, out, axis=None).tolist() == [2.0, 4.0]
    assert float(s.reduce("MEAN", torch.tensor([1.0, 3.0]), axis=0)) == 2.0
    with s.scope():
        assert tf.distribute.get_strategy() is s and tf.distribute.has_strategy()
        v = tf.Variable(torch.zeros(2))
        assert type(v).__name__ == "MirroredVariable"
    assert not tf.distribute.has_strategy()


def test_example_script_runs_single_worker():
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_EXAMPLE_EPOCHS="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("TF_CONFIG", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "tf_dist_example.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "20/20 [" in r.stdout and "sparse_categorical_accuracy" in r.stdout
