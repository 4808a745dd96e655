"""The reference's MNIST CNN (tf_dist_example.py:39-53) as a model family of this framework.

* :func:`build_mnist_cnn`   – the Keras-style ``Sequential`` exactly as the reference builds it.
* :data:`MNIST_CNN_VARIABLES` – TF variable names / layouts (HWIO conv kernels, [in,out] dense).
* :func:`reference_logits`  – plain-PyTorch functional forward (NHWC semantics); the fp32/fp64
  oracle for the fused HIP kernels.
* :class:`FusedMnistTrainStep` – one replica's fused train step on the gfx950 kernels of
  ``csrc/kernels/mnist_cnn.hip`` (2 launches for one replica alone on its GPU: fwd + loss head +
  dP2 + conv bwd, then finalize = partial reductions + dense weight gradients [+ SGD]; on a shared
  GPU a separate conv-bwd launch and a K5 launch for dP2 / the dense weight gradients).
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.nn.functional as F

from ..engine.slab import SlabLayout

MNIST_CNN_VARIABLES = [
    ("conv2d/kernel:0", (3, 3, 1, 32)),
    ("conv2d/bias:0", (32,)),
    ("conv2d_1/kernel:0", (3, 3, 32, 64)),
    ("conv2d_1/bias:0", (64,)),
    ("dense/kernel:0", (1600, 128)),
    ("dense/bias:0", (128,)),
    ("dense_1/kernel:0", (128, 10)),
    ("dense_1/bias:0", (10,)),
]
MNIST_NUM_PARAMS = 225_034
FINALIZE_BLOCKS = 375  # workgroups of the fused finalize (kFxBlocks): one exchange slot each


def mnist_layout() -> SlabLayout:
    return SlabLayout.from_shapes(MNIST_CNN_VARIABLES)


def glorot_uniform(shape: Sequence[int], gen: torch.Generator) -> torch.Tensor:
    """Keras glorot_uniform: limit = sqrt(6 / (fan_in + fan_out)); conv fans include the
    receptive field (kh*kw*cin, kh*kw*cout)."""
    if len(shape) == 2:
        fan_in, fan_out = shape
    else:
        rf = int(math.prod(shape[:-2]))
        fan_in, fan_out = shape[-2] * rf, shape[-1] * rf
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return (torch.rand(tuple(shape), generator=gen, dtype=torch.float32) * 2 - 1) * lim


def init_mnist_params(seed: int = 0) -> List[torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    out = []
    for name, shape in MNIST_CNN_VARIABLES:
        out.append(glorot_uniform(shape, g) if name.endswith("kernel:0") else torch.zeros(shape))
    return out


def reference_logits(params: Sequence[torch.Tensor], x: torch.Tensor) -> torch.Tensor:
    """Forward of the reference model in plain PyTorch.  x: [b,28,28,1] NHWC."""
    w1, b1, w2, b2, w3, b3, w4, b4 = params
    h = x.permute(0, 3, 1, 2)
    h = F.relu(F.conv2d(h, w1.permute(3, 2, 0, 1), b1))
    h = F.max_pool2d(h, 2)
    h = F.relu(F.conv2d(h, w2.permute(3, 2, 0, 1), b2))
    h = F.max_pool2d(h, 2)
    h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # Flatten in HWC order (Keras NHWC)
    h = F.relu(h @ w3 + b3)
    return h @ w4 + b4


def reference_loss(params, x, y, num_replicas: int = 1):
    """SparseCategoricalCrossentropy(from_logits=True) averaged over the GLOBAL batch
    (per-replica sum / (b * R)), as tf.distribute + Keras compute it."""
    logits = reference_logits(params, x)
    ce = F.cross_entropy(logits, y.long(), reduction="none")
    return ce.sum() / (x.shape[0] * num_replicas), logits, ce


def build_mnist_cnn(keras_module=None):
    """Build (not compile) the reference's Sequential model with this framework's Keras API."""
    if keras_module is None:
        from .. import keras as keras_module
    L = keras_module.layers
    return keras_module.Sequential(
        [
            L.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
            L.MaxPooling2D(),
            L.Conv2D(64, 3, activation="relu"),
            L.MaxPooling2D(),
            L.Flatten(),
            L.Dense(128, activation="relu"),
            L.Dense(10),
        ]
    )


def dp2_in_forward_ok(b: int, R: int, device: torch.device) -> bool:
    """Whether k_fwd_conv may compute dP2 itself (one launch fewer per step).  Its quarter
    workgroups then wait for their image's loss head, which runs in the image's last-arriving
    workgroup; that is only safe when all 4b workgroups are resident together: 4b <= compute units
    and no other process's kernels on the GPU (not TDL_SHARE_GPU).  Within a replica nothing runs
    alongside k_fwd_conv: every all-reduce of step k (also the side-stream one of the overlap
    option) completes before step k+1's forward.  ``TDL_MNIST_DP2_FWD=0/1`` overrides (1 still
    requires 4b <= CUs)."""
    mode = os.environ.get("TDL_MNIST_DP2_FWD", "auto")
    if mode == "0" or device.type != "cuda":
        return False
    fits = 4 * b <= torch.cuda.get_device_properties(device).multi_processor_count
    if mode == "1":
        return fits
    return fits and os.environ.get("TDL_SHARE_GPU") != "1"


class FusedMnistTrainStep:
    """One replica's MNIST train step on the hand-written gfx950 kernels.

    The dataset lives on the device (``X`` [N,28,28,1] f32, ``Y`` [N] int32); each step reads its
    ``b`` sample ids from ``idx_buf`` at an offset, so a captured hipGraph replays over new data by
    refreshing ``idx_buf`` only.  ``W``/``G`` are the flat parameter / gradient slabs in
    :func:`mnist_layout` order.
    """

    def __init__(self, X: torch.Tensor, Y: torch.Tensor, idx_buf: torch.Tensor, W: torch.Tensor,
                 G: torch.Tensor, layout: SlabLayout, per_replica_batch: int, num_replicas: int,
                 lr: torch.Tensor, metrics: Optional[torch.Tensor] = None, global_batch: Optional[int] = None):
        from .. import ops

        C = ops.hip()
        if [tuple(s.shape) for s in layout.specs] != [s for _, s in MNIST_CNN_VARIABLES]:
            raise ValueError("layout does not match the MNIST CNN variables")
        self.b = int(per_replica_batch)
        self.R = int(num_replicas)
        self.metrics = metrics if metrics is not None else torch.zeros(4, device=W.device)
        self.lr = lr
        self.X, self.Y, self.idx_buf, self.W, self.G = X, Y, idx_buf, W, G
        gb = int(global_batch) if global_batch is not None else self.b * self.R
        self._impl = C.MnistStep(X, Y, idx_buf, W, G, [int(o) for o in layout.offsets], self.b,
                                 1.0 / gb, lr, self.metrics)
        # G[dense_offset:] (dense kernels/biases) is final after forward_dense(); G[:dense_offset]
        # (conv kernels/biases) after backward_conv() + finalize()
        self.dense_offset = int(layout.offsets[4])
        self.dp2_in_forward = dp2_in_forward_ok(self.b, self.R, W.device)
        self._impl.set_dp2_in_forward(self.dp2_in_forward)
        # with dP2 in the forward kernel the conv backward runs there too (one launch for forward
        # + loss + backward; TDL_MNIST_FUSED_BWD=0 keeps the separate k_conv_bwd launch)
        self._impl.set_fused_bwd(os.environ.get("TDL_MNIST_FUSED_BWD", "1") == "1")
        self.fused_bwd = bool(self._impl.fused_bwd())
        self._impl.set_keep_grad(True)
        if (self.fused_bwd and self.R > 1 and os.environ.get("TDL_SHARE_GPU") == "1"
                and "TDL_FX_GRID" not in os.environ):
            # replicas sharing ONE GPU: a replica's exchanging finalize workgroups spin until its
            # peers' arrive, and a peer still in its fused kernel needs whole free CUs for its 4b
            # workgroups (208 VGPRs x 2 waves per SIMD, ~110 KB LDS): spread over every CU, the
            # spinning grid would lock that kernel out until the exchange timed out.  Cap the grid
            # (ranges loop over it) so the others' fused workgroups always find free CUs.
            cus = torch.cuda.get_device_properties(W.device).multi_processor_count
            self._impl.set_fx_grid(max(16, (cus - (self.R - 1) * 4 * self.b) // 2))

    def forward_backward(self, idx_offset: int) -> None:
        self._impl.forward_backward(int(idx_offset))

    def check(self) -> None:
        """Raise if an in-kernel hand-off of this step timed out (host sync).  Such a step gave
        the affected images no gradient and poisoned the loss metric; it indicates that the
        launch did not have the GPU to itself (see :func:`dp2_in_forward_ok`)."""
        if self._impl.error(False):
            raise RuntimeError("fused MNIST step: an in-kernel hand-off timed out (the GPU is shared or not every "
                               "workgroup was resident); set TDL_MNIST_DP2_FWD=0 or TDL_SHARE_GPU=1")

    def forward_eval(self, idx_offset: int, logits: Optional[torch.Tensor] = None) -> None:
        """Forward only (evaluate / predict): loss, correct and sample counts of the b rows at
        ``idx_offset`` accumulate into ``metrics``; ``logits`` [>= b*10] receives their logits."""
        self._impl.forward_eval(int(idx_offset), logits)

    def forward_dense(self, idx_offset: int) -> None:
        """Forward, loss and the dense-layer backward (their gradients land in G)."""
        self._impl.forward_dense(int(idx_offset))

    def backward_conv(self) -> None:
        """Conv backward into per-image partial slabs (reduced into G by finalize)."""
        self._impl.backward_conv()

    def finalize(self, apply_sgd: bool, exchange: bool = False, keep_grad: bool = True) -> None:
        """Partial-slab reductions + dense weight gradients into G (+ SGD).  ``exchange`` (fused
        backward + :meth:`set_exchange`): the same launch all-reduces the gradient across the
        replicas over xGMI before the SGD update (each finalize workgroup exchanges its own range).
        ``keep_grad=False`` (``apply_sgd`` with one replica, or with the exchange): the SGD update is
        applied but G is not written -- nothing reads it then, and its 900 KB of stores cost the
        finalize's kernel-end write-back (K=20 bench +1.2 %, profiles/mnist_fx_no_grad_store_r5.txt)."""
        self._impl.set_keep_grad(bool(keep_grad) or not apply_sgd or (self.R > 1 and not exchange))
        self._impl.finalize(bool(apply_sgd), bool(exchange))

    def set_exchange(self, channel, twoshot: bool = False) -> None:
        """Use this xGMI channel (``_C.XgmiChannel`` with capacity >= the slab and
        >= ``FINALIZE_BLOCKS`` signal slots, connected to every replica) for ``finalize(exchange=True)``;
        ``twoshot``: reduce-scatter + all-gather of the updated weights instead of every rank
        summing every range (2 (R-1)/R instead of (R-1) slabs over the fabric per rank)."""
        self._impl.set_exchange(channel)
        self._impl.set_exchange_algo(1 if twoshot else 0)

    @property
    def exchange_twoshot(self) -> bool:
        return bool(self._impl.exchange_algo())

    @property
    def has_exchange(self) -> bool:
        return bool(self._impl.has_exchange())

    def stage(self, k: int, apply_sgd: bool = False) -> None:
        self._impl.stage(int(k), bool(apply_sgd))

    def set_idx_offset(self, off: int) -> None:
        self._impl.set_idx_offset(int(off))

    def buffers(self) -> Dict[str, torch.Tensor]:
        names = ["P1", "A1", "P2", "A2", "H", "dH", "dP2", "part2", "part1", "part3", "dL"]
        return dict(zip(names, self._impl.buffers()))
