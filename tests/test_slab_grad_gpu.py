"""Direct gradient-slab writes of the generic engine under mixed_bfloat16 (engine/trainer.py):
one bf16 cast of the whole weight slab per step, the conv weight-gradient kernel adding dW straight
into the f32 slab view, the BN backward adding dgamma/dbeta into it, folded conv biases left at zero.
Training must match the plain autograd accumulation path (TDL_CAST_ACCUMULATE=0)."""
import os
import sys

import numpy as np
import pytest
import torch

import tensorflow_distributed_learning_amd as tdl

pytestmark = pytest.mark.gpu


def _model():
    tdl.keras.utils.set_random_seed(5)
    L = tdl.keras.layers
    inp = L.Input(shape=(16, 16, 64))
    x = L.Conv2D(64, 3, padding="same")(inp)
    x = L.BatchNormalization()(x)
    x = L.Activation("relu")(x)
    y = L.Conv2D(64, 1)(x)  # identity block: x feeds this conv and the residual Add (grad tap)
    y = L.BatchNormalization()(y)
    x = L.Activation("relu")(L.Add()([x, y]))
    s = L.Conv2D(128, 1, strides=2)(x)  # projection block: x feeds two strided 1x1 convs (grad box)
    s = L.BatchNormalization()(s)
    m = L.Conv2D(128, 1, strides=2)(x)
    m = L.BatchNormalization()(m)
    m = L.Activation("relu")(m)
    m = L.Conv2D(128, 3, padding="same")(m)
    m = L.BatchNormalization()(m)
    x = L.Activation("relu")(L.Add()([m, s]))
    x = L.GlobalAveragePooling2D()(x)
    out = L.Dense(10)(x)
    return tdl.keras.Model(inp, out)


def _train(direct: bool, steps=2, grad_sum=True, bn_stats=True):
    env = {"TDL_CAST_ACCUMULATE": "1" if direct else "0", "TDL_GRAPH_STEP": "0", "TDL_CONV": "hip",
           "TDL_FUSE_GRAD_SUM": "1" if grad_sum else "0"}
    from tensorflow_distributed_learning_amd.keras import models as _models

    _models._CONV_BN_STATS = bn_stats
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        tdl.keras.backend.clear_session()
        tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
        g = torch.Generator().manual_seed(0)
        x = torch.rand(256, 16, 16, 64, generator=g)
        y = torch.randint(0, 10, (256,), generator=g)
        ds = tdl.data.Dataset.from_tensor_slices((x, y)).batch(64).repeat()
        strategy = tdl.distribute.MirroredStrategy(devices=["/gpu:0"])
        with strategy.scope():
            m = _model()
            m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                      optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
        h = m.fit(ds, epochs=1, steps_per_epoch=steps, verbose=0)
        return m, h
    finally:
        _models._CONV_BN_STATS = True
        tdl.keras.mixed_precision.set_global_policy("float32")
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_direct_slab_gradients_match_autograd_accumulation():
    md, hd = _train(True)
    assert md._trainer.kind == "generic" and md._trainer._Wc is not None
    ma, ha = _train(False)
    assert ma._trainer._Wc is None
    for v, a, b in zip(md.weights, md.get_weights(), ma.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=5e-2 * scale, rtol=2e-2, err_msg=v.name)  # (the direct path keeps dW in f32, autograd rounds it to bf16)
    np.testing.assert_allclose(hd.history["loss"], ha.history["loss"], rtol=2e-2)
    # folded conv biases before a BN keep exactly their initial value (zero gradient)
    for v in md.weights:
        if "conv" in v.name and v.name.endswith("bias:0"):
            assert float(np.abs(v.numpy()).max()) == 0.0, v.name


def test_fused_gradient_sums_match_autograd_adds():
    """Tensors read by a conv and one other node: the conv's input-gradient epilogue adds the other
    contribution (keras/fusion.py grad boxes) instead of autograd's separate add.  (The BN-group
    reductions stay in the BN's own pass in both runs: reduced in the epilogue, their f32 summation
    order differs, and bf16 activations turn that into visible weight differences after two steps.)"""
    from tensorflow_distributed_learning_amd.ops import conv as CV

    CV._FUSE_BN_BWD[0] = False
    try:
        mf, hf = _train(True, grad_sum=True)
        boxes = mf.__dict__["_grad_boxes"]
        assert len(boxes) == 2 and all(b.n == 2 and b.g is None for b in boxes.values())
        mu, hu = _train(True, grad_sum=False)
    finally:
        CV._FUSE_BN_BWD[0] = True
    assert not mu.__dict__["_grad_boxes"]
    for v, a, b in zip(mf.weights, mf.get_weights(), mu.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=2e-2 * scale, rtol=2e-2, err_msg=v.name)
    np.testing.assert_allclose(hf.history["loss"], hu.history["loss"], rtol=1e-2)


@pytest.mark.parametrize("s2", [False, True])
def test_conv_dgrad_residual_epilogue(s2):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    g = torch.Generator(device="cpu").manual_seed(1)
    N, H, W, Ci, K = 4, 14, 14, 128, 256
    k = (torch.randn(1 if s2 else 3, 1 if s2 else 3, Ci, K, generator=g) * 0.05).cuda().bfloat16()
    OH = 7 if s2 else H
    dy = torch.randn(N, OH, OH, K, generator=g).cuda().bfloat16()
    r = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
    if s2:
        a, b = C.conv_dgrad_s2(dy, k, H, W), C.conv_dgrad_s2(dy, k, H, W, r)
    else:
        a, b = C.conv_dgrad(dy, k, H, W, 1, 1), C.conv_dgrad(dy, k, H, W, 1, 1, r)
    assert torch.equal(b, (a.float() + r.float()).bfloat16())


def test_conv_epilogue_bn_statistics_match_bn_pass():
    """BN statistics from the conv forward epilogue vs the BN's own statistics pass."""
    ma, ha = _train(True, bn_stats=True)
    mb, hb = _train(True, bn_stats=False)
    for v, a, b in zip(ma.weights, ma.get_weights(), mb.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=2e-2 * scale, rtol=2e-2, err_msg=v.name)
    np.testing.assert_allclose(ha.history["loss"], hb.history["loss"], rtol=1e-2)


def test_fused_bn_group_backward_in_conv_epilogue():
    """The identity block's first conv computes the previous BN -> Add -> ReLU group's masked
    gradient and BN reductions in its input-gradient epilogue, and each block's 3x3 conv those of
    the BN -> ReLU group it reads; training matches the unfused path."""
    from tensorflow_distributed_learning_amd.ops import batchnorm as B
    from tensorflow_distributed_learning_amd.ops import conv as CV

    L = tdl.keras.layers

    def model():
        tdl.keras.utils.set_random_seed(7)
        inp = L.Input(shape=(8, 8, 64))
        x = L.Conv2D(64, 3, padding="same")(inp)
        x = L.BatchNormalization()(x)
        x = L.Activation("relu")(x)
        for _ in range(2):  # two identity blocks: the first's output feeds the second's conv + Add
            y = L.Conv2D(64, 1)(x)
            y = L.BatchNormalization()(y)
            y = L.Activation("relu")(y)
            y = L.Conv2D(64, 3, padding="same")(y)
            y = L.BatchNormalization()(y)
            x = L.Activation("relu")(L.Add()([x, y]))
        x = L.GlobalAveragePooling2D()(x)
        return tdl.keras.Model(inp, L.Dense(16)(x))

    def run(fuse):
        CV._FUSE_BN_BWD[0] = fuse
        old = {k: os.environ.get(k) for k in ("TDL_GRAPH_STEP", "TDL_CONV")}
        os.environ.update({"TDL_GRAPH_STEP": "0", "TDL_CONV": "hip"})
        try:
            tdl.keras.backend.clear_session()
            tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
            g = torch.Generator().manual_seed(0)
            ds = tdl.data.Dataset.from_tensor_slices((torch.rand(128, 8, 8, 64, generator=g),
                                                      torch.randint(0, 16, (128,), generator=g))).batch(32).repeat()
            with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
                m = model()
                m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tdl.keras.optimizers.SGD(learning_rate=0.05, momentum=0.9))
            n0 = B.FUSED_BWD[0]
            h = m.fit(ds, epochs=1, steps_per_epoch=2, verbose=0)
            return m, h, B.FUSED_BWD[0] - n0
        finally:
            CV._FUSE_BN_BWD[0] = True
            tdl.keras.mixed_precision.set_global_policy("float32")
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    mf, hf, nf = run(True)
    mu, hu, nu = run(False)
    # per step: the first block's output group + the two blocks' inner BN -> ReLU groups; two steps
    assert nf == 6 and nu == 0
    for v, a, b in zip(mf.weights, mf.get_weights(), mu.get_weights()):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=2e-2 * scale, rtol=2e-2, err_msg=v.name)
    np.testing.assert_allclose(hf.history["loss"], hu.history["loss"], rtol=1e-2)


def _diag_run(cfg, steps):
    """scripts/diag_bnfuse.py's ResNet-style model (projection shortcuts, stride-2 blocks, bf16,
    SGD momentum), ``steps`` eager steps in this process: (weights, BN fused-backward modes used)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scripts"))
    from diag_bnfuse import run

    from tensorflow_distributed_learning_amd.ops import batchnorm as B
    from tensorflow_distributed_learning_amd.ops import conv as CV

    old = {k: os.environ.get(k) for k in ("TDL_GRAPH_STEP", "TDL_CONV")}
    m0 = dict(B.FUSED_BWD_MODES)
    try:
        m = run(*{"F": (False, False, False), "T": (True, True, True)}[cfg], steps)
        modes = {k: B.FUSED_BWD_MODES[k] - m0[k] for k in m0}
        return [np.array(w) for w in m.get_weights()], modes
    finally:
        CV._FUSE_BN_BWD[0] = CV._FUSE_BN_BWD_S2[0] = CV._FUSE_BN_BWD_SHORTCUT[0] = True
        tdl.keras.mixed_precision.set_global_policy("float32")
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_fused_bn_backward_projection_shortcut_and_stride2():
    """ResNet conv blocks: the projection-shortcut BN's backward sums come from the same conv
    epilogue as the block output group's (part2), and a group read by two 1x1 stride-2 convs (the
    next stage's conv block) is reduced in the stride-2 input-gradient epilogue; training matches
    the unfused path.  Both configurations run in this process, asynchronously (the round-3
    async-vs-launch-blocking difference was the first conv on MIOpen, keras/layers.py
    _autocast_input)."""
    wf, mf = _diag_run("F", 1)
    wt, mt = _diag_run("T", 1)
    # one step: both shortcut BNs (mode 0); the outputs of blocks 1-3 (block 2's is read by the two
    # stride-2 convs of block 3); the 8 inner BN -> ReLU groups
    assert mt == {0: 2, 1: 8, 2: 3}, mt
    assert mf == {0: 0, 1: 0, 2: 0}, mf
    # (one SGD step: the epilogue sums run in another f32 order, and over more steps bf16
    # activations amplify that into tens of percent on the tiny BN betas of this model; one step
    # bounds the gradients themselves, at the direct-slab test's 5e-2)
    for a, b in zip(wt, wf):
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=5e-2 * scale, rtol=2e-2)


def test_generic_engine_async_matches_launch_blocking_bitwise(tmp_path):
    """Regression pin for the round-3 'async vs HIP_LAUNCH_BLOCKING=1' divergence: two momentum
    steps of the BN-heavy model, fused BN backward on, asynchronous in this process (twice) and
    launch-blocking in a subprocess, give bit-identical weights."""
    import subprocess

    a1, _ = _diag_run("T", 2)
    a2, _ = _diag_run("T", 2)
    out = str(tmp_path / "w_blocking.npz")
    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scripts", "diag_bnfuse2.py")
    r = subprocess.run([sys.executable, script, "T", out, "2"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, HIP_LAUNCH_BLOCKING="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    z = np.load(out)
    b = [z[f"arr_{i}"] for i in range(len(z.files))]
    assert len(a1) == len(a2) == len(b)
    for i, (x, y, w) in enumerate(zip(a1, a2, b)):
        assert np.array_equal(x, y), f"weight {i}: two asynchronous runs differ"
        assert np.array_equal(x, w), f"weight {i}: asynchronous vs launch-blocking differ, max {np.abs(x - w).max()}"


def test_conv_dgrad_s2_bn_epilogue_matches_reference():
    """conv_dgrad_s2_bn / conv_dgrad_bn with bn_x2: dz and every partial-sum row vs fp32 PyTorch."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    g = torch.Generator(device="cpu").manual_seed(3)
    N, H, W, Ci, K = 4, 14, 14, 128, 256
    for s2 in (True, False):
        k = (torch.randn(1 if s2 else 3, 1 if s2 else 3, Ci, K, generator=g) * 0.05).cuda().bfloat16()
        OH = 7 if s2 else H
        dy = torch.randn(N, OH, OH, K, generator=g).cuda().bfloat16()
        r = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
        by = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
        bx = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
        bx2 = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
        if s2:
            base = C.conv_dgrad_s2(dy, k, H, W, r)
            dz, part, part2 = C.conv_dgrad_s2_bn(dy, k, H, W, r, by, bx, bx2)
        else:
            base = C.conv_dgrad(dy, k, H, W, 1, 1, r)
            dz, part, part2 = C.conv_dgrad_bn(dy, k, H, W, 1, 1, r, by, bx, bx2)
        ref = base.float() * (by.float() > 0)
        assert torch.equal(dz.float(), ref.bfloat16().float())
        rows = (N * OH * OH + 127) // 128
        S = part[:rows, 0].sum(0)
        np.testing.assert_allclose(S.cpu().numpy(), ref.bfloat16().float().sum((0, 1, 2)).cpu().numpy(),
                                   rtol=1e-3, atol=1e-2)
        Q = part[:rows, 1].sum(0)
        np.testing.assert_allclose(Q.cpu().numpy(), (dz.float() * bx.float()).sum((0, 1, 2)).cpu().numpy(),
                                   rtol=1e-3, atol=1e-2)
        assert torch.equal(part2[:rows, 0], part[:rows, 0])
        Q2 = part2[:rows, 1].sum(0)
        np.testing.assert_allclose(Q2.cpu().numpy(), (dz.float() * bx2.float()).sum((0, 1, 2)).cpu().numpy(),
                                   rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("kind", ["3x3", "1x1", "s2"])
def test_dgrad_bn_mask_from_stats_matches_mask_from_y_bitwise(kind):
    """A plain BN -> ReLU group's ReLU mask recomputed in the dgrad epilogue from its BN input and the
    forward's scale / shift (bn_stats, no read of the group output) gives the dz and partial sums of
    the mask read from the group output, bit for bit."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    g = torch.Generator(device="cpu").manual_seed(11)
    N, H, Ci, K = 4, 14, 128, 128
    s2 = kind == "s2"
    OH = H // 2 if s2 else H
    bx = (torch.randn(N, H, H, Ci, generator=g) * 2 + 0.3).cuda().bfloat16()
    gam, bet = (torch.rand(Ci, generator=g) + 0.5).cuda(), torch.randn(Ci, generator=g).cuda()
    mm, mv = torch.zeros(Ci, device="cuda"), torch.ones(Ci, device="cuda")
    by, st = C.bn_forward_train(bx, gam, bet, mm, mv, 0.9, 1e-3, True, None, None)
    dy = torch.randn(N, OH, OH, K, generator=g).cuda().bfloat16()
    if s2:
        w = (torch.randn(1, 1, Ci, K, generator=g) * 0.1).cuda().bfloat16()
        a = C.conv_dgrad_s2_bn(dy, w, H, H, None, by, bx)
        b = C.conv_dgrad_s2_bn(dy, w, H, H, None, None, bx, None, st)
    else:
        k = 3 if kind == "3x3" else 1
        w = (torch.randn(k, k, Ci, K, generator=g) * 0.05).cuda().bfloat16()
        a = C.conv_dgrad_bn(dy, w, H, H, k // 2, k // 2, None, by, bx)
        b = C.conv_dgrad_bn(dy, w, H, H, k // 2, k // 2, None, None, bx, None, st)
    assert torch.equal(a[0], b[0])
    R = a[1].shape[0]
    P = next(q for q in range(R + 1) if q + (q + 63) // 64 == R)
    assert torch.equal(a[1][:P], b[1][:P])
    assert int((a[0] == 0).sum()) > 0  # the mask did something


def test_wgrad_side_stream_matches_main_stream_bitwise():
    """Slab weight gradients on the side stream (TDL_WGRAD_STREAM=1: they overlap the input-gradient /
    BN chain) give bit-identical weights to running them on the main stream: same kernels, each slab
    region written by one reduction, joined before the optimizer reads the slab."""
    from tensorflow_distributed_learning_amd.ops import conv as CV

    a, _ = _diag_run("T", 2)
    old = CV._WGRAD_SIDE[0]
    try:
        CV._WGRAD_SIDE[0] = True
        b, _ = _diag_run("T", 2)
    finally:
        CV._WGRAD_SIDE[0] = old
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert np.array_equal(x, y), f"weight {i}: side-stream vs main-stream weight gradients differ"
