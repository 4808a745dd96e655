"""Conv2D(relu) -> MaxPooling2D(2) as ONE forward launch on the generic f32 path (csrc/kernels/gemm_f32.hip
pooled epilogue: rows ordered by pool window, conv_f32_fwd_pool) against the unfused pair (conv_f32_fwd +
maxpool_fwd) and float64 PyTorch: conv output on every window pixel, pooled output, argmax, and the
gradients through the fused op's backward (maxpool_bwd + the conv backward) -- including an odd output
size whose last row / column belongs to no window, and 'same' padding."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, H, W, C, K, kernel, pad): the reference CNN's two convs (26x26 and 11x11 outputs), a 'same' conv,
# a ragged one
SHAPES = [(8, 28, 28, 1, 32, 3, 0), (8, 13, 13, 32, 64, 3, 0), (4, 28, 28, 1, 32, 3, 1), (3, 9, 12, 8, 24, 3, 1)]


def _data(shape):
    N, H, W, C, K, k, p = shape
    g = torch.Generator(device="cpu").manual_seed(H * 100 + C)
    x = torch.randn(N, H, W, C, generator=g).cuda()
    w = (torch.randn(k, k, C, K, generator=g) / (k * k * C) ** 0.5).cuda()
    b = (torch.randn(K, generator=g) * 0.1).cuda()
    return x, w, b


@pytest.mark.parametrize("shape", SHAPES)
def test_pooled_epilogue_matches_unfused(shape):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, k, p = shape
    x, w, b = _data(shape)
    OH, OW = H + 2 * p - k + 1, W + 2 * p - k + 1
    y, pooled, arg = C.conv_f32_fwd_pool(x, w, b, OH, OW, 1, 1, p, p, act=1)
    y0 = C.conv_f32_fwd(x, w, b, OH, OW, 1, 1, p, p, act=1)
    PH, PW = OH // 2, OW // 2
    # every pixel inside a window: the unfused conv's value, bit for bit (the pooled conv takes the
    # unfused conv's split-K plan, and its pooled reduce sums the slices in the same order)
    assert torch.equal(y[:, :2 * PH, :2 * PW], y0[:, :2 * PH, :2 * PW])
    p0, a0 = C.maxpool_fwd(y0, 2, 2, 2, 2, 0, 0, PH, PW, False)
    assert torch.equal(pooled, p0) and torch.equal(arg, a0)
    ref = F.max_pool2d(torch.relu(F.conv2d(x.double().permute(0, 3, 1, 2), w.double().permute(3, 2, 0, 1),
                                           b.double(), 1, p)), 2).permute(0, 2, 3, 1)
    torch.testing.assert_close(pooled.double(), ref, rtol=1e-5, atol=1e-5)
    # argmax: the first maximum of the window in (dy, dx) order, as maxpool_fwd
    win = y[:, :2 * PH, :2 * PW].reshape(N, PH, 2, PW, 2, K).permute(0, 1, 3, 2, 4, 5).reshape(N, PH, PW, 4, K)
    assert torch.equal(arg.long(), win.argmax(3)) or torch.equal(torch.gather(win, 3, arg.long().unsqueeze(3))
                                                                  .squeeze(3), pooled)


@pytest.mark.parametrize("shape", SHAPES)
def test_fused_conv_pool_gradients(shape):
    from tensorflow_distributed_learning_amd.ops import conv_f32 as cf
    from tensorflow_distributed_learning_amd.ops import pooling

    N, H, W, Ci, K, k, p = shape
    x, w, b = _data(shape)
    pads = (p, p, p, p)
    outs = []
    for fused in (True, False):
        xv, wv, bv = (t.clone().requires_grad_(True) for t in (x, w, b))
        if fused:
            out = cf.conv2d_pool(xv, wv, bv, (1, 1), pads, act=1)
        else:
            out = pooling.max_pool_nhwc(cf.conv2d(xv, wv, bv, (1, 1), pads, act=1), (2, 2), (2, 2))
        g = torch.Generator(device="cpu").manual_seed(3)
        dout = torch.randn(out.shape, generator=g).cuda()
        out.backward(dout)
        outs.append((out.detach(), xv.grad, wv.grad, bv.grad))
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)


def _fit_reference_cnn(fuse: str, functional: bool = False):
    import os

    import numpy as np

    import tensorflow_distributed_learning_amd as tdl

    tdl.keras.backend.clear_session()
    tdl.keras.utils.set_random_seed(5)
    g = np.random.default_rng(0)
    x = g.random((256, 28, 28, 1), dtype=np.float32)
    y = g.integers(0, 10, 256).astype(np.int64)
    old = {k: os.environ.get(k) for k in ("TDL_DISABLE_FUSED", "TDL_FUSE_CONV_POOL")}
    os.environ["TDL_DISABLE_FUSED"] = "1"
    os.environ["TDL_FUSE_CONV_POOL"] = fuse
    try:
        L = tdl.keras.layers
        with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
            if functional:  # the functional executor's fusion plan (keras/fusion.py conv_pool)
                inp = L.Input(shape=(28, 28, 1))
                h = L.MaxPooling2D()(L.Conv2D(32, 3, activation="relu")(inp))
                h = L.MaxPooling2D()(L.Conv2D(64, 3, activation="relu")(h))
                m = tdl.keras.Model(inp, L.Dense(10)(L.Dense(128, activation="relu")(L.Flatten()(h))))
            else:
                m = tdl.keras.Sequential([L.Conv2D(32, 3, activation="relu", input_shape=(28, 28, 1)),
                                          L.MaxPooling2D(), L.Conv2D(64, 3, activation="relu"), L.MaxPooling2D(),
                                          L.Flatten(), L.Dense(128, activation="relu"), L.Dense(10)])
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(0.05))
        h = m.fit(x, y, batch_size=64, epochs=2, verbose=0, shuffle=False)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return m, h


@pytest.mark.parametrize("functional", [False, True], ids=["sequential", "functional"])
def test_generic_engine_reference_cnn_fused_pool_trains_like_unfused(functional):
    """The generic engine's Sequential forward (and the functional executor's fusion plan) takes the fused
    Conv2D -> MaxPooling2D pairs in training (two launches fewer per step); two epochs match the unfused
    model bit for bit."""
    import numpy as np

    mf, hf = _fit_reference_cnn("1", functional)
    assert mf._trainer.kind == "generic"
    mu, hu = _fit_reference_cnn("0", functional)
    assert hf.history["loss"] == hu.history["loss"]
    for a, b in zip(mf.get_weights(), mu.get_weights()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("shape", SHAPES)
def test_pooled_gradient_loaders_match_maxpool_backward_bitwise(shape, monkeypatch):
    """The fused op's backward reads the POOLED gradient in the input / weight gradient kernels' operand
    loaders (argmax routing + ReLU mask); it matches the max-pool backward pass followed by the plain
    kernels (TDL_FUSE_CONV_POOL_BWD=0) bit for bit, bias gradient included."""
    from tensorflow_distributed_learning_amd.ops import conv_f32 as cf

    x, w, b = _data(shape)
    p = shape[6]
    res = []
    for env in ("1", "0"):
        monkeypatch.setenv("TDL_FUSE_CONV_POOL_BWD", env)
        xv, wv, bv = (t.clone().requires_grad_(True) for t in (x, w, b))
        out = cf.conv2d_pool(xv, wv, bv, (1, 1), (p, p, p, p), act=1)
        g = torch.Generator(device="cpu").manual_seed(11)
        out.backward(torch.randn(out.shape, generator=g).cuda())
        res.append((xv.grad, wv.grad, bv.grad))
    for a, c in zip(res[0], res[1]):
        assert torch.equal(a, c)


@pytest.mark.parametrize("shape", [(8, 26, 26, 32), (8, 11, 11, 64), (3, 9, 12, 24), (2, 7, 7, 16)])
@pytest.mark.parametrize("bf16", [False, True], ids=["f32", "bf16"])
def test_maxpool_2x2_backward_scatter_form(shape, bf16):
    """The 2x2 stride-2 max-pool backward in scatter form (csrc/kernels/pool.hip k_maxpool_bwd_w2: one thread
    per window writes its four pixels, the last window of an odd row / column also the edge zeros) equals the
    gather form bit for bit -- every pixel written, odd sizes included -- and PyTorch's max-pool gradient."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, K = shape
    g = torch.Generator(device="cpu").manual_seed(H * 7 + K)
    x = torch.randn(N, H, W, K, generator=g).cuda()
    if bf16:
        x = x.bfloat16()
    PH, PW = H // 2, W // 2
    y, arg = C.maxpool_fwd(x, 2, 2, 2, 2, 0, 0, PH, PW, False)
    dy = torch.randn(y.shape, generator=g).cuda().to(x.dtype)
    res = []
    try:
        for on in (True, False):
            C.maxpool_w2(on)
            res.append(C.maxpool_bwd(dy, arg, list(x.shape), 2, 2, 2, 2, 0, 0))
    finally:
        C.maxpool_w2(True)
    assert torch.equal(res[0], res[1])
    xr = x.float().permute(0, 3, 1, 2).clone().requires_grad_(True)
    F.max_pool2d(xr, 2).backward(dy.float().permute(0, 3, 1, 2))
    assert torch.equal(res[0].float(), xr.grad.permute(0, 2, 3, 1))
