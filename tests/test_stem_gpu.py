"""The small-channel stride-2 conv kernels (csrc/kernels/stem.hip, the ResNet-50 stem) vs a plain
PyTorch fp32 reference of the same op: forward, the fused BN statistics, the weight gradient (bf16
out and added into an f32 slab), and the ZeroPadding2D -> Conv2D fusion in a functional model."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

import tensorflow_distributed_learning_amd as tdl

pytestmark = pytest.mark.gpu


def _ref(x, k_hwio, pads, stride):
    xp = F.pad(x.float(), (0, 0, pads[2], pads[3], pads[0], pads[1])).permute(0, 3, 1, 2)
    return F.conv2d(xp, k_hwio.float().permute(3, 2, 0, 1), stride=stride).permute(0, 2, 3, 1)


@pytest.mark.parametrize("geo", [((3, 3, 3, 3), (2, 2), 7, 3, 64, 38), ((1, 2, 0, 1), (1, 2), 5, 4, 128, 21),
                                 ((0, 0, 0, 0), (2, 2), 3, 1, 64, 16)])
@pytest.mark.parametrize("xdtype", [torch.bfloat16, torch.float32])
def test_stem_forward_and_stats(geo, xdtype):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    pads, stride, kk, cin, cout, hw = geo
    g = torch.Generator(device="cpu").manual_seed(0)
    x = torch.randn(3, hw, hw + 3, cin, generator=g).cuda().to(xdtype)
    k = (torch.randn(kk, kk, cin, cout, generator=g) * 0.1).cuda().bfloat16()
    y, xp, part = C.stem_fwd(x, k, *pads, *stride, True)
    ref = _ref(x.bfloat16(), k, pads, stride)
    assert y.shape == ref.shape
    err = (y.float() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 1e-2, err
    M = y.shape[0] * y.shape[1] * y.shape[2]
    P = (M + 255) // 256
    yf = y.float().reshape(-1, cout)
    np.testing.assert_allclose(part[:P, 0].sum(0).cpu().numpy(), yf.sum(0).cpu().numpy(), rtol=1e-4, atol=1e-2)
    np.testing.assert_allclose(part[:P, 1].sum(0).cpu().numpy(), (yf * yf).sum(0).cpu().numpy(), rtol=1e-4,
                               atol=1e-2)


@pytest.mark.parametrize("geo", [((3, 3, 3, 3), (2, 2), 7, 3, 64, 38), ((1, 2, 0, 1), (1, 2), 5, 4, 128, 21)])
def test_stem_weight_gradient(geo):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    pads, stride, kk, cin, cout, hw = geo
    g = torch.Generator(device="cpu").manual_seed(1)
    x = torch.randn(5, hw, hw, cin, generator=g).cuda().bfloat16()
    k = (torch.randn(kk, kk, cin, cout, generator=g) * 0.1).cuda().bfloat16()
    y, xp = C.stem_fwd(x, k, *pads, *stride)
    dy = torch.randn(y.shape, generator=g).cuda().bfloat16()
    kr = k.float().requires_grad_(True)
    _ref(x, kr, pads, stride).backward(dy.float())
    ref = kr.grad
    dw = C.stem_wgrad(xp, dy, kk, kk, cin, stride[0])
    scale = ref.abs().max().item()
    assert (dw.float() - ref).abs().max().item() / scale < 1e-2
    slab = torch.full(ref.shape, 0.5, device="cuda")
    C.stem_wgrad(xp, dy, kk, kk, cin, stride[0], out=slab, accumulate=True)
    assert (slab - 0.5 - ref).abs().max().item() / scale < 1e-4
    # deterministic: the same bits on a second call
    assert torch.equal(dw, C.stem_wgrad(xp, dy, kk, kk, cin, stride[0]))


def test_stem_autograd_and_model_fusion():
    """conv_stem through autograd (image gradient on the library path), and a ZeroPadding2D -> Conv2D
    -> BN -> ReLU stem trained through the fused plan vs the unfused layers."""
    from tensorflow_distributed_learning_amd.ops import conv as CV

    g = torch.Generator(device="cpu").manual_seed(2)
    x = torch.randn(2, 20, 20, 3, generator=g).cuda().bfloat16().requires_grad_(True)
    k = (torch.randn(7, 7, 3, 64, generator=g) * 0.1).cuda().bfloat16().requires_grad_(True)
    y = CV.stem_conv2d_nhwc(x, k, (3, 3, 3, 3), (2, 2))
    dy = torch.randn(y.shape, generator=g).cuda().bfloat16()
    y.backward(dy)
    xr, kr = x.detach().float().requires_grad_(True), k.detach().float().requires_grad_(True)
    _ref(xr, kr, (3, 3, 3, 3), (2, 2)).backward(dy.float())
    assert (x.grad.float() - xr.grad).abs().max().item() / xr.grad.abs().max().item() < 2e-2
    assert (k.grad.float() - kr.grad).abs().max().item() / kr.grad.abs().max().item() < 2e-2

    L = tdl.keras.layers

    def run(fuse):
        old = {kk: os.environ.get(kk) for kk in ("TDL_FUSE", "TDL_GRAPH_STEP")}
        os.environ.update({"TDL_FUSE": "1" if fuse else "0", "TDL_GRAPH_STEP": "0"})
        try:
            tdl.keras.backend.clear_session()
            tdl.keras.mixed_precision.set_global_policy("mixed_bfloat16")
            tdl.keras.utils.set_random_seed(3)
            gg = torch.Generator().manual_seed(0)
            ds = tdl.data.Dataset.from_tensor_slices((torch.rand(64, 32, 32, 3, generator=gg),
                                                      torch.randint(0, 8, (64,), generator=gg))).batch(16).repeat()
            with tdl.distribute.MirroredStrategy(devices=["/gpu:0"]).scope():
                inp = L.Input(shape=(32, 32, 3))
                h = L.ZeroPadding2D(padding=((3, 3), (3, 3)))(inp)
                h = L.Conv2D(64, 7, strides=2)(h)
                h = L.Activation("relu")(L.BatchNormalization()(h))
                h = L.GlobalAveragePooling2D()(h)
                m = tdl.keras.Model(inp, L.Dense(8)(h))
                m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                          optimizer=tdl.keras.optimizers.SGD(learning_rate=0.1))
            hist = m.fit(ds, epochs=1, steps_per_epoch=3, verbose=0)
            return m, hist
        finally:
            tdl.keras.mixed_precision.set_global_policy("float32")
            for kk, v in old.items():
                if v is None:
                    os.environ.pop(kk, None)
                else:
                    os.environ[kk] = v

    mf, hf = run(True)
    plan = mf._fusion()
    assert any(isinstance(n.layer, L.Conv2D) and id(n) in plan.pool_pad for n in mf._nodes)
    mu, hu = run(False)
    for v, a, b in zip(mf.weights, mf.get_weights(), mu.get_weights()):
        if v.name.startswith("conv2d") and v.name.endswith("bias:0"):
            # folded into the BN in the fused plan: exactly zero gradient there, rounding noise (1e-5)
            # through the unfused layers
            assert float(np.abs(a).max()) == 0.0 and float(np.abs(b).max()) < 1e-3
            continue
        scale = max(float(np.abs(b).max()), 1e-3)
        np.testing.assert_allclose(a, b, atol=3e-2 * scale, rtol=3e-2, err_msg=v.name)
    np.testing.assert_allclose(hf.history["loss"], hu.history["loss"], rtol=2e-2)
