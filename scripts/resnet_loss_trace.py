"""Per-step loss trajectory of keras ResNet-50 on a fixed synthetic set (4 batches, random labels),
SGD(0.01, momentum 0.9) as in scripts/bench_resnet50.py: a healthy run memorises the 4 batches, a
diverging one shows which precision/kernel path blows up.  Usage: resnet_loss_trace.py DTYPE [IMG] [B] [STEPS]"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorflow_distributed_learning_amd as tdl  # noqa: E402


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "mixed_bfloat16"
    img = int(sys.argv[2]) if len(sys.argv) > 2 else 224
    b = int(sys.argv[3]) if len(sys.argv) > 3 else 64
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 24
    lr = float(os.environ.get("LR", "0.01"))
    tdl.keras.mixed_precision.set_global_policy(dtype)
    strategy = tdl.distribute.MirroredStrategy()
    dev = strategy.extended.device
    g = torch.Generator().manual_seed(0)
    x = torch.rand(4 * b, img, img, 3, generator=g).to(dev)
    y = torch.randint(0, 1000, (4 * b,), generator=g).to(dev)
    ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(b, drop_remainder=True).repeat()
    with strategy.scope():
        torch.manual_seed(0)
        model = tdl.keras.applications.ResNet50(weights=None, classes=1000, classifier_activation=None,
                                                input_shape=(img, img, 3))
        model.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=lr, momentum=0.9))
    h = model.fit(ds, epochs=steps, steps_per_epoch=1, verbose=0)
    print(json.dumps({"dtype": dtype, "img": img, "b": b, "lr": lr, "conv": os.environ.get("TDL_CONV", "auto"),
                      "loss": [round(v, 4) for v in h.history["loss"]]}), flush=True)


if __name__ == "__main__":
    main()
