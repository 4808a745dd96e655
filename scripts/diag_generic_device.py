"""Diagnostic: a generic-engine device execution graph replayed after an epoch boundary vs the same
three steps run eagerly / through a fresh capture, from the same weights and indices, per variable.

Round 6 finding (kept as the regression check): with the conv bias gradient taken by PyTorch's
``dy.sum((0, 1, 2))`` -- a multi-block reduction with a global-memory semaphore buffer zeroed by a
captured memset node -- a captured multi-step graph replayed after eager work on the device (the
epoch-end metric read / reset) produced garbage for that one reduction (9 of 16 channels 0) while a
fresh capture of the same steps was exact.  The bias gradients now come from the weight-gradient
kernel itself (gemm_f32.hip, a column / row of ones), so no such reduction remains in the step.
TDL_GENERIC_DEVICE_EAGER=1 runs the device path without capture for comparison."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tensorflow_distributed_learning_amd as tdl  # noqa: E402

os.environ["TDL_DISABLE_FUSED"] = "1"
os.environ["TDL_GENERIC_DEVICE_DATA"] = "1"
L = tdl.keras.layers
tdl.keras.backend.clear_session()
tdl.keras.utils.set_random_seed(3)
with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
    m = tdl.keras.Sequential([L.Conv2D(16, 3, activation="relu", padding="same", input_shape=(28, 28, 1)),
                              L.MaxPooling2D(), L.Flatten(), L.Dense(64, activation="relu"), L.Dense(10)])
    m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
              optimizer=tdl.keras.optimizers.SGD(0.05), steps_per_execution=3)
g = torch.Generator().manual_seed(0)
x, y = torch.rand(256, 28, 28, 1, generator=g), torch.randint(0, 10, (256,), generator=g)
ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(32).repeat()
m.fit(ds, epochs=1, verbose=0, steps_per_epoch=12)
tr = m._trainer
names = [v.name for v in m._trainable_vars]
views = lambda t: m._layout.views(t)


def diff(a, b):
    return " ".join(f"{n.split('/')[-1][:12]}={float((va - vb).abs().max()):.2g}" for n, va, vb in zip(names, views(a), views(b)))


torch.cuda.synchronize()
W0 = tr.W.clone()
idx = tr._dev_idx[:96].clone()
A = tr._graphs[("dev", 3, 32)]
print("graphs", list(tr._graphs))


def from_w0():
    tr.W.copy_(W0)
    tr._dev_idx[:96].copy_(idx)
    torch.cuda.synchronize()


def eager():
    from_w0()
    for k in range(3):
        tr._dev_step(k, 32, 32, sync_lr=False)
    torch.cuda.synchronize()
    return tr.W.clone(), tr.G.clone()


def replay(gr):
    from_w0()
    gr.replay()
    torch.cuda.synchronize()
    return tr.W.clone(), tr.G.clone()


We, Ge = eager()
Wa, Ga = replay(A)
print("A right after fit   vs eager: W", diff(Wa, We), "| G", diff(Ga, Ge), flush=True)
gb_a, gb_e = views(Ga)[1], views(Ge)[1]
print("conv1 bias grad A    ", [round(float(v), 5) for v in gb_a])
print("conv1 bias grad eager", [round(float(v), 5) for v in gb_e])
Wa1, Ga1 = replay(A)
print("A replayed again     vs A: G", diff(Ga1, Ga), flush=True)
tr.logs()
tr.reset_metrics()
Wa2, Ga2 = replay(A)
print("A after logs/reset  vs eager: W", diff(Wa2, We), "| G", diff(Ga2, Ge), flush=True)
We2, Ge2 = eager()
print("eager after          vs eager: W", diff(We2, We), flush=True)
B = tr._dev_capture(3, 32)
Wb, Gb = replay(B)
print("fresh capture B      vs eager: W", diff(Wb, We), "| G", diff(Gb, Ge), flush=True)
Wa3, Ga3 = replay(A)
print("A after B capture    vs eager: W", diff(Wa3, We), flush=True)
