"""Generic f32 convolution / Dense kernels (csrc/kernels/gemm_f32.hip, ops/conv_f32.py) against float64
PyTorch references on the CPU: forward, input gradient and weight gradient over kernel sizes, strides,
asymmetric padding, dilation, channel counts that are not multiples of 4, and reductions long enough
to take the split-K path; Dense forward / dx / dW; and the generic engine's f32 layers (the
reference CNN with 'same' padding, Adam) training with zero library convolutions."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

import tensorflow_distributed_learning_amd as tdl  # noqa: E402
from tensorflow_distributed_learning_amd.ops import conv as _conv  # noqa: E402
from tensorflow_distributed_learning_amd.ops import conv_f32 as CF  # noqa: E402

CASES = [
    # N, H, W, C, K, R, S, stride, pads (t, b, l, r), dilation
    (8, 28, 28, 1, 32, 3, 3, (1, 1), (0, 0, 0, 0), (1, 1)),   # reference CNN conv1
    (8, 13, 13, 32, 64, 3, 3, (1, 1), (0, 0, 0, 0), (1, 1)),  # reference CNN conv2
    (4, 28, 28, 1, 32, 3, 3, (1, 1), (1, 1, 1, 1), (1, 1)),   # 'same'
    (2, 14, 14, 64, 64, 3, 3, (2, 2), (0, 1, 0, 1), (1, 1)),  # 3x3 stride-2 'same' (asymmetric)
    (3, 15, 11, 3, 16, 5, 5, (1, 2), (2, 2, 1, 2), (1, 1)),   # 5x5, mixed strides
    (2, 12, 12, 8, 8, 3, 3, (1, 1), (2, 2, 2, 2), (2, 2)),    # dilation 2
    (4, 7, 7, 130, 70, 1, 1, (1, 1), (0, 0, 0, 0), (1, 1)),   # 1x1, C and K not multiples of 4
    (2, 9, 9, 6, 10, 3, 3, (3, 3), (1, 0, 1, 0), (1, 1)),     # stride 3, odd channels
]


def _ref(x, w, b, stride, pads, dil):
    """float64 CPU autograd reference: NHWC / HWIO through F.conv2d on explicitly padded input."""
    xd = x.detach().double().cpu().requires_grad_(True)
    wd = w.detach().double().cpu().requires_grad_(True)
    bd = b.detach().double().cpu().requires_grad_(True) if b is not None else None
    h = F.pad(xd.permute(0, 3, 1, 2), (pads[2], pads[3], pads[0], pads[1]))
    y = F.conv2d(h, wd.permute(3, 2, 0, 1), bd, stride=stride, dilation=dil).permute(0, 2, 3, 1)
    return y, xd, wd, bd


def _close(got, ref, tol=2e-5):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = ref.abs().max().clamp_min(1e-30)
    err = ((got - ref).abs().max() / scale).item()
    assert err < tol, err


@pytest.mark.parametrize("case", CASES, ids=[f"c{i}" for i in range(len(CASES))])
def test_conv_f32_fwd_dgrad_wgrad(case):
    N, H, W, C, K, R, S, stride, pads, dil = case
    g = torch.Generator().manual_seed(1)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(R, S, C, K, generator=g) / (R * S * C) ** 0.5
    b = torch.randn(K, generator=g)
    yr, xd, wd, bd = _ref(x, w, b, stride, pads, dil)
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())

    xc, wc, bc = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
    _conv.reset_library_calls()
    y = CF.conv2d(xc, wc, bc, stride, pads, dil)
    assert y.shape == yr.shape
    _close(y, yr)
    y.backward(dy.cuda())
    _close(xc.grad, xd.grad)
    _close(wc.grad, wd.grad)
    _close(bc.grad, bd.grad)
    # accumulate into a slab view
    acc = torch.ones_like(wc.grad)
    CF.wgrad(xc.detach(), dy.cuda(), (R, S), stride, pads, dil, out=acc, accumulate=True)
    _close(acc - 1, wd.grad)
    assert _conv.library_calls() == {}


def test_conv_f32_split_k_weight_gradient_is_deterministic():
    """A 36,864-row reduction (64 x 24 x 24 output pixels) on 5 output tiles: split over ~200 slices,
    reduced in slice order -- bit-identical across calls, f64-close."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(64, 26, 26, 32, generator=g)
    dy = torch.randn(64, 24, 24, 64, generator=g)
    a = CF.wgrad(x.cuda(), dy.cuda(), (3, 3), (1, 1), (0, 0, 0, 0))
    b = CF.wgrad(x.cuda(), dy.cuda(), (3, 3), (1, 1), (0, 0, 0, 0))
    assert torch.equal(a, b)
    xd = x.double().permute(0, 3, 1, 2)
    dyd = dy.double().permute(0, 3, 1, 2)
    ref = torch.nn.grad.conv2d_weight(xd, (64, 32, 3, 3), dyd).permute(2, 3, 1, 0)
    _close(a, ref)


@pytest.mark.parametrize("shape", [(64, 9216, 128), (64, 128, 10), (7, 13, 5), (300, 64, 65)])
def test_dense_f32_matches_float64(shape):
    M, D, U = shape
    g = torch.Generator().manual_seed(3)
    x = torch.randn(M, D, generator=g)
    w = torch.randn(D, U, generator=g) / D ** 0.5
    b = torch.randn(U, generator=g)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = xd @ wd + bd
    dy = torch.randn(M, U, generator=g)
    yr.backward(dy.double())
    xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
    y = CF.dense(xc, wc, bc)
    _close(y, yr)
    y.backward(dy.cuda())
    _close(xc.grad, xd.grad)
    _close(wc.grad, wd.grad)
    _close(bc.grad, bd.grad)


def _same_cnn():
    k = tdl.keras
    return k.Sequential([
        k.layers.Input(shape=(28, 28, 1)),
        k.layers.Conv2D(32, 3, padding="same", activation="relu"),
        k.layers.MaxPooling2D(),
        k.layers.Conv2D(64, 3, strides=2, padding="same", activation="relu"),
        k.layers.Flatten(),
        k.layers.Dense(64, activation="relu"),
        k.layers.Dense(10),
    ])


def _fit_same_cnn(device):
    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(5)
    g = np.random.default_rng(0)
    x = g.random((256, 28, 28, 1), dtype=np.float32)
    y = g.integers(0, 10, 256).astype(np.int64)
    os.environ["TDL_DISABLE_FUSED"] = "1"
    try:
        with tdl.distribute.MirroredStrategy(devices=[device]).scope():
            m = _same_cnn()
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.Adam(1e-3))
        h = m.fit(x, y, batch_size=64, epochs=1, verbose=0, shuffle=False)
    finally:
        os.environ.pop("TDL_DISABLE_FUSED", None)
    return m, h


def test_generic_f32_cnn_same_padding_trains_without_library_calls():
    """A 'same'-padded (stride-1 and stride-2) f32 CNN with Adam on the generic engine: every Conv2D
    and Dense runs on gemm_f32.hip (no MIOpen / hipBLASLt conv or GEMM), and it follows the CPU run."""
    _conv.reset_library_calls()
    mg, hg = _fit_same_cnn("/gpu:0")
    assert mg._trainer.kind == "generic"
    assert _conv.library_calls() == {}, _conv.library_calls()
    mc, hc = _fit_same_cnn("/cpu:0")
    np.testing.assert_allclose(hg.history["loss"], hc.history["loss"], rtol=1e-3)
    for a, b in zip(mg.get_weights(), mc.get_weights()):
        np.testing.assert_allclose(a, b, rtol=1e-2, atol=2e-3)


def test_conv_f32_large_problem_matches_float64():
    """Large forward / input-gradient problems (65,536 pixels x 128 channels, 1,024 output tiles);
    float64 reference through im2col on the GPU."""
    N, H, W, C, K = 16, 64, 64, 128, 128
    g = torch.Generator().manual_seed(4)
    x = torch.randn(N, H, W, C, generator=g).cuda()
    w = (torch.randn(3, 3, C, K, generator=g) / (9 * C) ** 0.5).cuda()
    dy = torch.randn(N, H, W, K, generator=g).cuda()
    xd = x.double().permute(0, 3, 1, 2).requires_grad_(True)
    cols = F.unfold(xd, 3, padding=1)
    yr = (w.double().permute(3, 2, 0, 1).reshape(K, C * 9) @ cols).reshape(N, K, H, W).permute(0, 2, 3, 1)
    yr.backward(dy.double())
    xc = x.clone().requires_grad_(True)
    y = CF.conv2d(xc, w, None, (1, 1), (1, 1, 1, 1), (1, 1))
    _close(y, yr)
    y.backward(dy)
    _close(xc.grad, xd.grad.permute(0, 2, 3, 1))


def test_dense_f32_large_gemm_with_ragged_edges():
    """A 2000 x 96 x 4100 GEMM (both tile edges partial) against float64."""
    g = torch.Generator().manual_seed(5)
    a = torch.randn(2000, 96, generator=g).cuda()
    b = torch.randn(96, 4100, generator=g).cuda()
    bias = torch.randn(4100, generator=g).cuda()
    y = CF.dense(a, b, bias)
    _close(y, a.double() @ b.double() + bias.double())


# ---------------------------------------------------------------------------------------------
# Fusions used by the generic engine: ReLU in the forward epilogue, the ReLU mask in the backward
# kernels' operand loads, and the bias gradient from the weight-gradient kernel (a column / row of
# ones), against float64 autograd of relu(conv + b) / relu(x @ w + b).

@pytest.mark.parametrize("case", CASES[:6], ids=[f"c{i}" for i in range(6)])
@pytest.mark.parametrize("targets", [False, True], ids=["autograd", "slab"])
def test_conv_f32_fused_relu_and_bias_grad(case, targets):
    N, H, W, C, K, R, S, stride, pads, dil = case
    g = torch.Generator().manual_seed(2)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(R, S, C, K, generator=g) / (R * S * C) ** 0.5
    b = torch.randn(K, generator=g) * 0.3
    yr, xd, wd, bd = _ref(x, w, b, stride, pads, dil)
    yr = torch.relu(yr)
    dy = torch.randn(yr.shape, generator=g)
    (yr * dy.double()).sum().backward()
    xc = x.cuda().requires_grad_(True)
    if targets:
        gw = torch.full(w.shape, 0.5, device="cuda")  # the kernels ADD into slab views
        gb = torch.full((K,), 0.25, device="cuda")
        wl = w.cuda().requires_grad_(True)
        y = CF.conv2d(xc, w.cuda(), b.cuda(), stride, pads, dil, grad_out=gw, anchor=wl, act=1, gb_out=gb)
        y.backward(dy.cuda())
        _close(gw - 0.5, wd.grad)
        _close(gb - 0.25, bd.grad)
    else:
        wc, bc = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
        y = CF.conv2d(xc, wc, bc, stride, pads, dil, act=1)
        y.backward(dy.cuda())
        _close(wc.grad, wd.grad)
        _close(bc.grad, bd.grad)
    _close(y, yr)
    _close(xc.grad, xd.grad)


@pytest.mark.parametrize("shape", [(64, 1600, 128), (37, 70, 33), (8, 5, 3)])
@pytest.mark.parametrize("targets", [False, True], ids=["autograd", "slab"])
def test_dense_f32_fused_relu_and_bias_grad(shape, targets):
    M, I, O = shape
    g = torch.Generator().manual_seed(3)
    x, w, b = torch.randn(M, I, generator=g), torch.randn(I, O, generator=g) / I ** 0.5, torch.randn(O, generator=g)
    xd, wd, bd = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = torch.relu(xd @ wd + bd)
    dy = torch.randn(M, O, generator=g)
    (yr * dy.double()).sum().backward()
    xc = x.cuda().requires_grad_(True)
    if targets:
        gw, gb = torch.zeros(I, O, device="cuda"), torch.zeros(O, device="cuda")
        y = CF.dense(xc, w.cuda(), b.cuda(), (gw, gb), anchor=w.cuda().requires_grad_(True), act=1)
        y.backward(dy.cuda())
        _close(gw, wd.grad)
        _close(gb, bd.grad)
    else:
        wc, bc = w.cuda().requires_grad_(True), b.cuda().requires_grad_(True)
        y = CF.dense(xc, wc, bc, act=1)
        y.backward(dy.cuda())
        _close(wc.grad, wd.grad)
        _close(bc.grad, bd.grad)
    _close(y, yr)
    _close(xc.grad, xd.grad)


@pytest.mark.parametrize("NK", [(64, 10), (300, 1000), (7, 3), (130, 64), (65, 10), (33, 65)])
def test_xent_head_loss_grad_and_metrics(NK):
    from tensorflow_distributed_learning_amd.ops import dense as D

    N, K = NK
    g = torch.Generator().manual_seed(4)
    z = torch.randn(N, K, generator=g) * 3
    y = torch.randint(0, K, (N,), generator=g)
    gn = 2 * N  # e.g. two replicas
    zd = z.double().requires_grad_(True)
    ref = F.cross_entropy(zd, y, reduction="sum") / gn
    ref.backward()
    accs = [torch.full((), v, dtype=torch.float64, device="cuda") for v in (1.5, 3.0, 2.0, 3.0)]
    zc = z.cuda().requires_grad_(True)
    loss = D.xent_head(zc, y.cuda(), gn, accs[:2], accs[2:])
    (loss * 0.5).backward()
    _close(loss, ref, 1e-6)
    _close(zc.grad, zd.grad * 0.5, 1e-6)
    per = F.cross_entropy(zd.detach(), y, reduction="none")
    np.testing.assert_allclose(float(accs[0]), 1.5 + float(per.sum()), rtol=1e-6)
    assert float(accs[1]) == 3.0 + N and float(accs[3]) == 3.0 + N
    assert float(accs[2]) == 2.0 + float((z.argmax(1) == y).sum())


@pytest.mark.parametrize("shape", [(64, 13, 13, 32, 64), (64, 26, 26, 33, 35), (64, 28, 28, 1, 32), (64, 20, 20, 2, 15)],
                         ids=["cnn_conv2", "ragged", "cnn_conv1_4_per_wave", "ragged_4_per_wave"])
def test_split_k_reduce_16_outputs_per_wave_is_bit_identical(shape):
    """Many-slice split-K reductions sum 16 (>= 8192 outputs) or 4 (>= 256) consecutive partial-slab entries
    per wave (k_gemm_f32_reduce_wave16, 16-B loads; scalar loads when M * N is not a multiple of 4): the weight and
    bias gradients equal the one-output-per-wave reduce bit for bit, and float64."""
    from tensorflow_distributed_learning_amd.ops import hip

    N, H, W, C, K = shape
    g = torch.Generator().manual_seed(4)
    x = torch.randn(N, H, W, C, generator=g)
    w = torch.randn(3, 3, C, K, generator=g) / (9 * C) ** 0.5
    b = torch.randn(K, generator=g)
    yr, xd, wd, bd = _ref(x, w, b, (1, 1), (0, 0, 0, 0), (1, 1))
    dy = torch.randn(yr.shape, generator=g)
    yr.backward(dy.double())
    grads = []
    try:
        for on in (True, False):
            hip().f32_reduce16(on)
            xc, wc, bc = (t.cuda().requires_grad_(True) for t in (x, w, b))
            CF.conv2d(xc, wc, bc, (1, 1), (0, 0, 0, 0)).backward(dy.cuda())
            grads.append((wc.grad, bc.grad))
    finally:
        hip().f32_reduce16(True)
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])
    _close(grads[0][0], wd.grad)
    _close(grads[0][1], bd.grad)
