"""The reference walkthrough (tf_dist_example.py / README.md:74-155) on this framework.

Only the two imports differ from the reference.  TF_CONFIG is taken from the environment when
present (the reference overwrites it unconditionally with worker index 1 on every host – quirk
Q1); without it the script trains as a single worker (README.md:34).

    # 2 workers on one machine (README.md:61), CPU or one GPU each:
    python -m tensorflow_distributed_learning_amd.launch --local-workers 2 examples/tf_dist_example.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tensorflow_distributed_learning_amd.compat import tf, tfds  # noqa: E402

if "TF_CONFIG" not in os.environ and os.environ.get("TDL_EXAMPLE_HARDCODED_CLUSTER"):
    os.environ["TF_CONFIG"] = json.dumps({"cluster": {"worker": ["172.16.16.5:12345", "172.16.16.6:12345"]},
                                          "task": {"type": "worker", "index": 1}})

strategy = tf.distribute.experimental.MultiWorkerMirroredStrategy(tf.distribute.experimental.CollectiveCommunication.AUTO)
# strategy = tf.distribute.MirroredStrategy()

tfds.disable_progress_bar()
BUFFER_SIZE = 10000
NUM_WORKERS = strategy.num_replicas_in_sync
GLOBAL_BATCH_SIZE = 64 * NUM_WORKERS
EPOCHS = int(os.environ.get("TDL_EXAMPLE_EPOCHS", "10"))


def make_datasets_unbatched():
    # scale MNIST from [0, 255] to [0., 1.]
    def scale(image, label):
        image = tf.cast(image, tf.float32)
        image /= 255
        return image, label

    datasets, info = tfds.load(with_info=True, name='mnist', as_supervised=True)
    return datasets['train'].map(scale).cache().shuffle(BUFFER_SIZE)


train_datasets = make_datasets_unbatched().batch(GLOBAL_BATCH_SIZE)
options = tf.data.Options()
options.experimental_distribute.auto_shard_policy = tf.data.experimental.AutoShardPolicy.OFF
# dist_dataset = strategy.experimental_distribute_dataset(train_datasets)
dist_dataset = train_datasets.with_options(options)


def build_and_compile_cnn_model():
    model = tf.keras.Sequential([
        tf.keras.layers.Conv2D(32, 3, activation='relu', input_shape=(28, 28, 1)),
        tf.keras.layers.MaxPooling2D(),
        tf.keras.layers.Conv2D(64, 3, activation='relu'),
        tf.keras.layers.MaxPooling2D(),
        tf.keras.layers.Flatten(),
        tf.keras.layers.Dense(128, activation='relu'),
        tf.keras.layers.Dense(10)
    ])
    model.compile(
        loss=tf.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
        optimizer=tf.keras.optimizers.SGD(learning_rate=0.001),
        metrics=[tf.keras.metrics.SparseCategoricalAccuracy()])
    return model


with strategy.scope():
    multi_worker_model = build_and_compile_cnn_model()

history = multi_worker_model.fit(x=dist_dataset, epochs=EPOCHS, steps_per_epoch=20)
if strategy.extended.is_chief:
    print("engine:", multi_worker_model._trainer.kind, "|", strategy)
    print(json.dumps({k: [round(v, 4) for v in vals] for k, vals in history.history.items()}))
