"""Gradient A/B of a whole keras ResNet-50 (mixed_bfloat16) with the hand-written conv kernels
(TDL_CONV=hip) against MIOpen (TDL_CONV=miopen) on the same weights and batch: prints the loss of both
and the variables whose gradients disagree most (relative max error)."""
import os
import sys

import torch

sys.path.insert(0, ".")
import tensorflow_distributed_learning_amd as tdl  # noqa: E402


def run(model, x, y, mode):
    os.environ["TDL_CONV"] = mode
    loss_fn = tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True)
    out = model(x, training=True)
    loss = loss_fn(y, out.float())
    vs = [v.value for v in model.trainable_variables]
    gs = torch.autograd.grad(loss, vs)
    return float(loss), [g.float() for g in gs]


def main():
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    img = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
    with tdl.distribute.MirroredStrategy().scope():
        model = tdl.keras.applications.ResNet50(weights=None, classes=10, classifier_activation=None,
                                                input_shape=(img, img, 3))
    for v in model.variables:
        v._bind(torch.empty(v.shape, dtype=v.dtype, device=dev))
    for v in model.trainable_variables:
        v.value.requires_grad_(True)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.rand(b, img, img, 3, generator=g).to(dev)
    y = torch.randint(0, 10, (b,), generator=g).to(dev)
    l_m, g_m = run(model, x, y, "miopen")
    l_h, g_h = run(model, x, y, "hip")
    print(f"loss miopen {l_m:.6f} hip {l_h:.6f}")
    errs = []
    for v, a, c in zip(model.trainable_variables, g_m, g_h):
        errs.append((float((a - c).abs().max() / a.abs().max().clamp_min(1e-30)), v.name, tuple(a.shape)))
    errs.sort(reverse=True)
    for e in errs[:12]:
        print(f"  rel err {e[0]:.4f}  {e[1]} {e[2]}")
    print(f"median rel err {sorted(e[0] for e in errs)[len(errs) // 2]:.4f}")


if __name__ == "__main__":
    main()
