"""NHWC batch-norm HIP kernels (csrc/kernels/bn.hip) vs a float64 PyTorch reference of the same op:
outputs, moving statistics, and input/gamma/beta gradients."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SHAPES = [((4, 7, 7, 64), torch.float32), ((3, 5, 5, 96), torch.float32), ((2, 5, 5, 2048), torch.bfloat16),
          ((16, 56, 56, 64), torch.bfloat16), ((6, 9, 9, 256), torch.float32), ((1, 1, 3, 8), torch.float32)]


def _ref(x, g, b, mm, mv, mom, eps, relu):
    x64 = x.double().detach().requires_grad_(True)
    g64 = g.double().detach().requires_grad_(True)
    b64 = b.double().detach().requires_grad_(True)
    mm64, mv64 = mm.double().clone(), mv.double().clone()
    h = x64.movedim(-1, 1)
    y = F.batch_norm(h, mm64, mv64, g64, b64, training=True, momentum=1 - mom, eps=eps).movedim(1, -1)
    if relu:
        y = F.relu(y)
    return x64, g64, b64, y, mm64, mv64


@pytest.mark.parametrize("shape,dtype", SHAPES)
@pytest.mark.parametrize("relu", [False, True])
def test_bn_train_matches_fp64(shape, dtype, relu):
    from tensorflow_distributed_learning_amd.ops.batchnorm import batch_norm_train

    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    C = shape[-1]
    x = (torch.randn(shape, device=dev) * 2 + 0.5).to(dtype)
    g = (torch.rand(C, device=dev) + 0.5).requires_grad_(True)
    b = torch.randn(C, device=dev).requires_grad_(True)
    mm, mv = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
    x64, g64, b64, y64, mm64, mv64 = _ref(x, g, b, mm, mv, 0.9, 1e-3, relu)
    xin = x.clone().requires_grad_(True)
    y = batch_norm_train(xin, g, b, mm, mv, 0.9, 1e-3, relu=relu)
    assert y.dtype == dtype and y.shape == x.shape
    tol = dict(atol=2e-4, rtol=2e-4) if dtype == torch.float32 else dict(atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(y.double(), y64, **tol)
    torch.testing.assert_close(mm.double(), mm64, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(mv.double(), mv64, atol=1e-4, rtol=1e-4)
    dy = torch.randn(shape, device=dev).to(dtype)
    y.backward(dy)
    y64.backward(dy.double())
    n = x.numel() // C
    gtol = dict(atol=5e-4, rtol=1e-3) if dtype == torch.float32 else dict(atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(xin.grad.double(), x64.grad, **gtol)
    scale = max(1.0, n ** 0.5 / 8)
    torch.testing.assert_close(g.grad.double(), g64.grad, atol=gtol["atol"] * scale * 4, rtol=gtol["rtol"])
    torch.testing.assert_close(b.grad.double(), b64.grad, atol=gtol["atol"] * scale * 4, rtol=gtol["rtol"])


def test_bn_layer_uses_hip_kernels():
    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.ops import loaded_paths

    x = torch.randn(4, 6, 6, 32, device="cuda:0")
    with tdl.distribute.OneDeviceStrategy("/gpu:0").scope():
        layer = tdl.keras.layers.BatchNormalization()
        layer.build(x.shape)
    for v in (layer.gamma, layer.beta, layer.moving_mean, layer.moving_variance):
        v._value = v._value.to("cuda:0")
    y = layer(x, training=True)
    assert "_C" in loaded_paths()
    ref = F.batch_norm(x.movedim(-1, 1), None, None, training=True, eps=1e-3).movedim(1, -1)
    torch.testing.assert_close(y, ref, atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_bn_add_relu_with_folded_conv_bias(dtype):
    from tensorflow_distributed_learning_amd.ops.batchnorm import batch_norm_train

    torch.manual_seed(1)
    dev = torch.device("cuda:0")
    shape, C = (4, 9, 9, 128), 128
    x = torch.randn(shape, device=dev).to(dtype)
    r = torch.randn(shape, device=dev).to(dtype)
    g = (torch.rand(C, device=dev) + 0.5).requires_grad_(True)
    b = torch.randn(C, device=dev).requires_grad_(True)
    cb = torch.randn(C, device=dev).requires_grad_(True)
    mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    # reference: relu(BN(x + cb) + r) in float64
    x64 = x.double().requires_grad_(True)
    r64 = r.double().requires_grad_(True)
    g64, b64, cb64 = (t.detach().double().requires_grad_(True) for t in (g, b, cb))
    mm64, mv64 = mm.double().clone(), mv.double().clone()
    h = (x64 + cb64).movedim(-1, 1)
    y64 = F.relu(F.batch_norm(h, mm64, mv64, g64, b64, training=True, momentum=0.01, eps=1e-3).movedim(1, -1) + r64)
    xin, rin = x.clone().requires_grad_(True), r.clone().requires_grad_(True)
    y = batch_norm_train(xin, g, b, mm, mv, 0.99, 1e-3, relu=True, residual=rin, conv_bias=cb)
    tol = dict(atol=2e-4, rtol=2e-4) if dtype == torch.float32 else dict(atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(y.double(), y64, **tol)
    torch.testing.assert_close(mm.double(), mm64, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(mv.double(), mv64, atol=1e-4, rtol=1e-4)
    dy = torch.randn(shape, device=dev).to(dtype)
    y.backward(dy)
    y64.backward(dy.double())
    gtol = dict(atol=5e-4, rtol=1e-3) if dtype == torch.float32 else dict(atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(xin.grad.double(), x64.grad, **gtol)
    torch.testing.assert_close(rin.grad.double(), r64.grad, **gtol)
    torch.testing.assert_close(g.grad.double(), g64.grad, atol=gtol["atol"] * 20, rtol=gtol["rtol"])
    torch.testing.assert_close(b.grad.double(), b64.grad, atol=gtol["atol"] * 20, rtol=gtol["rtol"])
    assert float(cb.grad.abs().max()) == 0.0 and float(cb64.grad.abs().max()) < 1e-6


def test_fused_training_graph_matches_unfused_gpu():
    """Same check as tests/test_fusion_cpu.py, with the fused groups on the HIP kernels."""
    import os
    import sys

    sys.path.insert(0, os.path.dirname(__file__))
    from test_fusion_cpu import _tiny_resnet

    import numpy as np
    import tensorflow_distributed_learning_amd as tdl

    tdl.keras.utils.set_random_seed(0)
    m = _tiny_resnet()
    for v in m.weights:
        if v.name.endswith("bias:0"):
            v.assign(np.random.RandomState(1).randn(*v.shape).astype(np.float32))
        v._value = v._value.to("cuda:0")
    x = torch.randn(6, 8, 8, 3, device="cuda:0")
    init = [v._value.clone() for v in m.non_trainable_weights]

    def run(fuse):
        os.environ["TDL_FUSE"] = "1" if fuse else "0"
        m.__dict__.pop("_fusion_plan", None)
        for v, t in zip(m.non_trainable_weights, init):
            v._value.copy_(t)
        leaves = []
        for v in m.trainable_weights:
            v._leaf = v._value.detach().clone().requires_grad_(True)
            leaves.append(v._leaf)
        y = m(x, training=True)
        (y ** 2).sum().backward()
        out = y.detach().clone(), [l.grad.clone() for l in leaves], [v._value.clone() for v in m.non_trainable_weights]
        for v in m.trainable_weights:
            v._leaf = None
        os.environ["TDL_FUSE"] = "1"
        m.__dict__.pop("_fusion_plan", None)
        return out

    y0, g0, s0 = run(False)
    y1, g1, s1 = run(True)
    torch.testing.assert_close(y1, y0, atol=1e-4, rtol=1e-4)
    for a, b, v in zip(g1, g0, m.trainable_weights):
        if "conv" in v.name and v.name.endswith("bias:0"):
            assert float(a.abs().max()) == 0.0 and float(b.abs().max()) < 1e-3
        else:
            torch.testing.assert_close(a, b, atol=1e-3, rtol=1e-3)
    for a, b in zip(s1, s0):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [((3, 3), (2, 2), ((1, 1), (1, 1)), True), ((2, 2), (2, 2), ((0, 0), (0, 0)), False),
                                 ((3, 3), (2, 2), ((0, 1), (0, 1)), False)])
def test_maxpool_nhwc_matches_torch(dtype, geo):
    from tensorflow_distributed_learning_amd.ops.pooling import max_pool_nhwc

    pool, strides, pads, pad_zero = geo
    torch.manual_seed(2)
    x = torch.randn(3, 17, 15, 64, device="cuda:0").to(dtype)
    xa = x.clone().requires_grad_(True)
    xb = x.float().clone().requires_grad_(True)
    y = max_pool_nhwc(xa, pool, strides, pads, pad_zero)
    (pt, pb), (pl, pr) = pads
    h = F.pad(xb.permute(0, 3, 1, 2), (pl, pr, pt, pb), value=0.0 if pad_zero else float("-inf"))
    yr = F.max_pool2d(h, pool, strides).permute(0, 2, 3, 1)
    torch.testing.assert_close(y.float(), yr)
    dy = torch.randn(yr.shape, device="cuda:0").to(dtype)
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(xa.grad.float(), xb.grad, atol=1e-2 if dtype == torch.bfloat16 else 1e-6, rtol=1e-2)


@pytest.mark.parametrize("shape", [(16, 56, 56, 64), (3, 7, 7, 2048), (5, 9, 9, 256), (1, 3, 5, 8)])
def test_bn_elementwise_blocked_matches_grid_stride_bitwise(shape):
    """The blocked elementwise kernels (channels in registers, several vectors per thread in flight,
    ragged last chunk) compute bit-identical apply / dx to the grid-stride ones, for every backward
    mode and with a residual."""
    from tensorflow_distributed_learning_amd.ops import hip

    Ck = hip()
    torch.manual_seed(2)
    dev = torch.device("cuda:0")
    C = shape[-1]
    x = (torch.randn(shape, device=dev) * 2 + 0.5).bfloat16()
    r = torch.randn(shape, device=dev).bfloat16()
    dy = torch.randn(shape, device=dev).bfloat16()
    g, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)

    def run():
        mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        y0, st = Ck.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, True, None, None)
        y1, _ = Ck.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, False, r, None)
        outs = [y0, y1]
        for mode in (0, 1, 2):
            outs += [t for t in Ck.bn_backward(dy, x, y0 if mode == 2 else None, g, st, mode) if t is not None]
        return outs

    try:
        Ck.bn_set_elementwise(0, 4)
        ref = run()
        for vpt in (2, 4, 8):
            Ck.bn_set_elementwise(1, vpt)
            got = run()
            assert len(got) == len(ref)
            for a, e in zip(got, ref):
                assert torch.equal(a, e)
    finally:
        Ck.bn_set_elementwise(1, 4)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("geo", [(1, 1, True), (0, 0, False), (1, 1, False)])
@pytest.mark.parametrize("hw", [(17, 15), (112, 112)])
def test_maxpool_3x3s2_unrolled_matches_generic_bitwise(dtype, geo, hw):
    """The unrolled 3x3 stride-2 max-pool kernels give the generic loops' outputs, argmax and input
    gradient bit for bit (same compare and sum order), with zero and -inf padding."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    pt, pl, pad_zero = geo
    H, W = hw
    torch.manual_seed(3)
    x = torch.randn(2, H, W, 64, device="cuda:0").to(dtype)
    OH, OW = (H + 2 * pt - 3) // 2 + 1, (W + 2 * pl - 3) // 2 + 1
    dy = torch.randn(2, OH, OW, 64, device="cuda:0").to(dtype)
    outs = []
    try:
        for generic in (True, False):
            C.maxpool_force_generic(generic)
            y, arg = C.maxpool_fwd(x, 3, 3, 2, 2, pt, pl, OH, OW, pad_zero)
            dx = C.maxpool_bwd(dy, arg, list(x.shape), 3, 3, 2, 2, pt, pl)
            outs.append((y, arg, dx))
    finally:
        C.maxpool_force_generic(True)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_bn_relu_maxpool_fused_kernels_match_unfused(dtype):
    """maxpool_fwd(bn_stats=st) over the BN input == maxpool over the BN -> ReLU pass's output (values
    and argmax, bitwise); maxpool_bwd_bn's dz == the plain pool backward masked by the recomputed ReLU
    condition (bitwise), and its partial sums add up to sum(dz), sum(dz * x)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    torch.manual_seed(5)
    N, H, Ch = 3, 22, 64
    x = (torch.randn(N, H, H, Ch, device="cuda:0") * 2 + 0.2).to(dtype)
    g, b = torch.rand(Ch, device="cuda:0") + 0.5, torch.randn(Ch, device="cuda:0")
    mm, mv = torch.zeros(Ch, device="cuda:0"), torch.ones(Ch, device="cuda:0")
    y, st = C.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, True, None, None)
    st2 = C.bn_stats_train(x, g, b, mm.clone(), mv.clone(), 0.9, 1e-3)
    assert torch.equal(st, st2)
    OH = (H + 2 - 3) // 2 + 1
    p0, a0 = C.maxpool_fwd(y, 3, 3, 2, 2, 1, 1, OH, OH, True)
    p1, a1 = C.maxpool_fwd(x, 3, 3, 2, 2, 1, 1, OH, OH, True, st)
    assert torch.equal(p0, p1) and torch.equal(a0, a1)
    dy = torch.randn(N, OH, OH, Ch, device="cuda:0").to(dtype)
    d0 = C.maxpool_bwd(dy, a0, list(x.shape), 3, 3, 2, 2, 1, 1)
    dz, part = C.maxpool_bwd_bn(dy, a1, list(x.shape), 3, 3, 2, 2, 1, 1, x, st)
    mask = (x.double() * st[2].double() + st[3].double()) > 0  # the sign of the kernel's f32 fma
    assert torch.equal(dz, torch.where(mask, d0, torch.zeros_like(d0)))
    R = part.shape[0]
    P = next(q for q in range(R + 1) if q + (q + 63) // 64 == R)
    got = part[:P].double().sum(0)
    ref = torch.stack([dz.double().reshape(-1, Ch).sum(0), (dz.double() * x.double()).reshape(-1, Ch).sum(0)])
    torch.testing.assert_close(got, ref, atol=1e-3, rtol=1e-4)


def test_stem_bn_relu_pool_fusion_trains_like_unfused():
    """The stem's BN -> ReLU -> ZeroPadding2D -> MaxPooling2D joined into one group (keras/fusion.py)
    trains like the unfused graph (TDL_FUSE_BN_POOL=0): losses and weights after two SGD steps."""
    import os

    import numpy as np
    import tensorflow_distributed_learning_amd as tdl

    L = tdl.keras.layers

    def run(fuse):
        os.environ["TDL_FUSE_BN_POOL"] = "1" if fuse else "0"
        try:
            tdl.keras.backend.clear_session()
            tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
            tdl.keras.utils.set_random_seed(3)
            inp = L.Input(shape=(32, 32, 3))
            x = L.ZeroPadding2D(3)(inp)
            x = L.Conv2D(64, 7, strides=2)(x)
            x = L.BatchNormalization()(x)
            x = L.Activation("relu")(x)
            x = L.ZeroPadding2D(1)(x)
            x = L.MaxPooling2D(3, strides=2)(x)
            x = L.Conv2D(64, 1)(x)
            x = L.GlobalAveragePooling2D()(x)
            with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
                m = tdl.keras.Model(inp, L.Dense(10)(x))
                m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05))
            gen = torch.Generator().manual_seed(0)
            ds = tdl.data.Dataset.from_tensor_slices((torch.rand(64, 32, 32, 3, generator=gen),
                                                      torch.randint(0, 10, (64,), generator=gen))).batch(32).repeat()
            h = m.fit(ds, epochs=1, steps_per_epoch=2, verbose=0)
            fused = any(gr.pool is not None for gr in m._fusion().groups.values())
            return m.get_weights(), h.history["loss"], fused
        finally:
            os.environ.pop("TDL_FUSE_BN_POOL", None)
            tdl.keras.mixed_precision.set_global_policy("float32")

    wf, lf, ff = run(True)
    wu, lu, fu = run(False)
    assert ff and not fu
    np.testing.assert_allclose(lf, lu, rtol=1e-2)
    for a, b in zip(wf, wu):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=2e-2 * scale, rtol=2e-2)


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 256), (2, 9, 11, 128, 192), (8, 7, 7, 512, 128)])
def test_conv_input_side_bn_relu_matches_materialised_bitwise(shape):
    """conv_fwd / conv_fwd_stats / conv_wgrad with in_bn=st over the BN input == the same kernels over
    the BN -> ReLU pass's output (bitwise: the operand loaders use the apply pass's f32 fma and
    rounding), for every weight-gradient plan the input-side BN takes (ragged pixel and tc tails)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    torch.manual_seed(7)
    N, H, W, Ci, K = shape
    x = (torch.randn(N, H, W, Ci, device="cuda:0") * 2 + 0.3).bfloat16()
    g, b = torch.rand(Ci, device="cuda:0") + 0.5, torch.randn(Ci, device="cuda:0")
    mm, mv = torch.zeros(Ci, device="cuda:0"), torch.ones(Ci, device="cuda:0")
    y, st = C.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, True, None, None)
    w = (torch.randn(K, 1, 1, Ci, device="cuda:0") / Ci ** 0.5).bfloat16()
    assert torch.equal(C.conv_fwd(y, w, H, W, 1, 1, 0, 0), C.conv_fwd(x, w, H, W, 1, 1, 0, 0, in_bn=st))
    y0, p0 = C.conv_fwd_stats(y, w, H, W, 1, 1, 0, 0)
    y1, p1 = C.conv_fwd_stats(x, w, H, W, 1, 1, 0, 0, in_bn=st)
    P = (N * H * W + 127) // 128  # row-tile partial sums (the rows past them are the reduce's scratch)
    assert torch.equal(y0, y1) and torch.equal(p0[:P], p1[:P])
    dy = torch.randn(N, H, W, K, device="cuda:0").bfloat16()
    plans = C.conv_wgrad_plans(list(x.shape), list(dy.shape), 1, 1, 1, 1, 0, 0, 8, in_bn=True)
    assert plans and all(p[0] * p[1] <= 4 and p[4] == 0 for p in plans)
    for p in plans:
        plan = [p[0], p[1], p[3], p[4]]
        a = C.conv_wgrad(y, dy, 1, 1, 1, 1, 0, 0, plan=plan)
        c = C.conv_wgrad(x, dy, 1, 1, 1, 1, 0, 0, plan=plan, in_bn=st)
        assert torch.equal(a, c), plan
    with pytest.raises(RuntimeError):
        C.conv_fwd(x, w, H, W, 1, 1, 0, 0, in_bn=st[:, :8].contiguous())


@pytest.mark.parametrize("mask_stats", [True, False])
def test_bn_apply_deferred_into_1x1_conv_trains_like_unfused(mask_stats):
    """BN -> ReLU -> 1x1 Conv2D with the BN apply taken over by the conv's operand loaders
    (keras/fusion.py ``defer``) trains like the materialised graph (TDL_FUSE_BN_INPUT=0): losses and
    weights after three SGD steps, and the BN backward took its reduction from the conv epilogue.
    With the mask-statistics A/B switch off (TDL_FUSE_BN_MASK_STATS=0) the deferred group must still
    build its ReLU mask from [x*scale + shift > 0], never from the raw BN input x."""
    import os

    from tensorflow_distributed_learning_amd.ops import conv as CV

    import numpy as np
    import tensorflow_distributed_learning_amd as tdl
    from tensorflow_distributed_learning_amd.ops import batchnorm as BN

    L = tdl.keras.layers

    from tensorflow_distributed_learning_amd.keras import fusion

    def run(fuse):
        os.environ["TDL_FUSE_BN_INPUT"] = "1" if fuse else "0"
        os.environ["TDL_CONV"] = "hip"  # the hand-written kernels everywhere (no timing-dependent choices)
        min_px, fusion._DEFER_MIN_PIXELS = fusion._DEFER_MIN_PIXELS, 0  # (a small test image)
        ms, CV._FUSE_BN_MASK_STATS[0] = CV._FUSE_BN_MASK_STATS[0], mask_stats
        try:
            tdl.keras.backend.clear_session()
            tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
            tdl.keras.utils.set_random_seed(3)
            inp = L.Input(shape=(12, 12, 64))
            x = L.Conv2D(64, 3, padding="same")(inp)
            x = L.BatchNormalization()(x)
            x = L.Activation("relu")(x)
            x = L.Conv2D(128, 1)(x)
            x = L.BatchNormalization()(x)
            x = L.Activation("relu")(x)
            x = L.GlobalAveragePooling2D()(x)
            with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
                m = tdl.keras.Model(inp, L.Dense(10)(x))
                m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05))
            gen = torch.Generator().manual_seed(0)
            ds = tdl.data.Dataset.from_tensor_slices((torch.randn(96, 12, 12, 64, generator=gen),
                                                      torch.randint(0, 10, (96,), generator=gen))).batch(32).repeat()
            before = BN.FUSED_BWD_MODES[1]
            h = m.fit(ds, epochs=1, steps_per_epoch=3, verbose=0)
            deferred = any(gr.defer is not None for gr in m._fusion().groups.values())
            return m.get_weights(), h.history["loss"], deferred, BN.FUSED_BWD_MODES[1] - before
        finally:
            os.environ.pop("TDL_FUSE_BN_INPUT", None)
            os.environ.pop("TDL_CONV", None)
            fusion._DEFER_MIN_PIXELS = min_px
            CV._FUSE_BN_MASK_STATS[0] = ms
            tdl.keras.mixed_precision.set_global_policy("float32")

    wf, lf, df, nf = run(True)
    wu, lu, du, nu = run(False)
    assert df and not du
    if mask_stats:
        # both fuse the BN backward reduction into the 1x1 conv's dgrad (counted per host-side call: with
        # the generic engine's device executions the first step runs eagerly, the second is captured,
        # the third replays the graph without Python)
        assert nf >= 2 and nu >= 2
    np.testing.assert_allclose(lf, lu, rtol=1e-2)
    for a, b in zip(wf, wu):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=2e-2 * scale, rtol=2e-2)
