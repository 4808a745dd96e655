"""Implicit-GEMM bf16 MFMA convolution kernels (csrc/kernels/conv.hip) vs a float32 PyTorch reference
of the same op (F.conv2d / its input gradient on the bf16-rounded operands)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, H, W, C, K, KH, KW, stride, pad): ResNet-50 tap shapes, shrunk in batch, plus ragged edges
SHAPES = [
    (2, 14, 14, 64, 64, 3, 3, 1, 1),
    (3, 7, 7, 128, 256, 1, 1, 1, 0),
    (2, 9, 11, 64, 128, 3, 3, 2, 1),
    (1, 5, 6, 192, 64, 3, 3, 1, 0),
    (4, 8, 8, 256, 512, 1, 1, 2, 0),
    (2, 13, 13, 64, 64, 5, 3, 1, 2),
    (8, 16, 16, 128, 128, 3, 3, 1, 1),
]


def _mk(shape, dev):
    N, H, W, C, K, KH, KW, s, p = shape
    g = torch.Generator(device="cpu").manual_seed(hash(shape) & 0xFFFF)
    x = torch.randn(N, H, W, C, generator=g).to(dev).bfloat16()
    k = (torch.randn(KH, KW, C, K, generator=g) / (KH * KW * C) ** 0.5).to(dev).bfloat16()
    return x, k


def _ref_fwd(x, k, s, p):
    return F.conv2d(x.float().permute(0, 3, 1, 2), k.float().permute(3, 2, 0, 1), None, s, p).permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fwd_matches_fp32(shape):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    ref = _ref_fwd(x, k, s, p)
    y = C.conv_fwd(x, k.permute(3, 0, 1, 2).contiguous(), ref.shape[1], ref.shape[2], s, s, p, p)
    assert y.dtype == torch.bfloat16 and y.shape == ref.shape
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[7] == 1])
def test_conv_dgrad_matches_fp32(shape):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    xr = x.float().requires_grad_(True)
    y = _ref_fwd(xr, k, s, p)
    dy = torch.randn(y.shape, device="cuda:0").bfloat16()
    y.backward(dy.float())
    dx = C.conv_dgrad(dy, k.contiguous(), H, W, p, p)
    assert dx.dtype == torch.bfloat16 and dx.shape == x.shape
    torch.testing.assert_close(dx.float(), xr.grad, atol=4e-2, rtol=2e-2)


def test_conv2d_layer_on_hip_kernels(monkeypatch):
    """keras Conv2D (bf16, TDL_CONV=hip) forward + backward through the hand-written kernels."""
    monkeypatch.setenv("TDL_CONV", "hip")
    from tensorflow_distributed_learning_amd.ops.conv import conv2d_nhwc

    x, k = _mk((4, 12, 12, 64, 128, 3, 3, 1, 1), "cuda:0")
    x.requires_grad_(True)
    kk = k.float().requires_grad_(True)
    y = conv2d_nhwc(x, kk.bfloat16(), (1, 1), (1, 1))
    dy = torch.randn(y.shape, device="cuda:0").bfloat16()
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    kr = k.float().requires_grad_(True)
    yr = _ref_fwd(xr, kr, 1, 1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(kk.grad, kr.grad, atol=2e-2 * float(kr.grad.abs().max()), rtol=3e-2)


@pytest.mark.parametrize("shape", [(64, 16, 16, 64, 512, 1, 1, 1, 0), (64, 16, 16, 128, 512, 3, 3, 1, 1),
                                   (32, 56, 56, 64, 64, 3, 3, 1, 1), (32, 56, 56, 128, 512, 1, 1, 1, 0),
                                   (64, 32, 32, 64, 512, 3, 3, 1, 1)])
def test_conv_fwd_dgrad_wide_tiles(shape):
    """Large grids take the 128 x 128 and 256 x 128 tile variants."""
    test_conv_fwd_matches_fp32(shape)
    test_conv_dgrad_matches_fp32(shape)


def _ref_grads(x, k, s, p, dy):
    xr = x.float().requires_grad_(True)
    kr = k.float().requires_grad_(True)
    y = _ref_fwd(xr, kr, s, p)
    y.backward(dy.float())
    return xr.grad, kr.grad


WGRAD_SHAPES = SHAPES + [
    (32, 28, 28, 128, 128, 3, 3, 1, 1),  # 3 x 3, 128 x 128 tiles, many slices
    (16, 56, 56, 64, 256, 1, 1, 1, 0),   # direct 1 x 1 path
    (8, 28, 28, 256, 512, 1, 1, 2, 0),   # strided shortcut
    (4, 7, 7, 512, 512, 3, 3, 1, 1),
]


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
def test_conv_wgrad_matches_fp32(shape):
    """Hand-written split-K weight gradient (transposed LDS reads) vs the fp32 autograd gradient;
    also checks the f32 accumulate form and that the result is bitwise deterministic."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    dy = torch.randn(N, OH, OW, K, device="cuda:0").bfloat16()
    _, gw = _ref_grads(x, k, s, p, dy)
    dw = C.conv_wgrad(x, dy, KH, KW, s, s, p, p)
    assert dw.dtype == torch.bfloat16 and dw.shape == k.shape
    scale = gw.abs().max().item()
    torch.testing.assert_close(dw.float(), gw, atol=2e-2 * scale + 1e-3, rtol=2e-2)
    base = torch.full(gw.shape, 0.5, device="cuda:0")
    acc = base.clone()
    C.conv_wgrad(x, dy, KH, KW, s, s, p, p, out=acc, accumulate=True)
    torch.testing.assert_close(acc, base + gw, atol=1e-3 * scale + 1e-4, rtol=1e-3)
    again = base.clone()
    C.conv_wgrad(x, dy, KH, KW, s, s, p, p, out=again, accumulate=True)
    assert torch.equal(acc, again), "weight gradient is not deterministic"
    # a single slice (no split-K) agrees with the split result to f32 rounding
    plan = C.conv_wgrad_plans(list(x.shape), list(dy.shape), KH, KW, s, s, p, p, 1)[0]
    one = C.conv_wgrad(x, dy, KH, KW, s, s, p, p, out=torch.zeros_like(gw), plan=[plan[0], plan[1], 1])
    torch.testing.assert_close(one, acc - base, atol=1e-3 * scale + 1e-4, rtol=1e-3)


@pytest.mark.parametrize("tile", [(1, 1), (1, 2), (2, 1), (2, 2), (1, 4), (4, 1)])
@pytest.mark.parametrize("shape", [(4, 14, 14, 256, 256, 3, 3, 1, 1), (8, 9, 9, 192, 256, 1, 1, 2, 0)])
def test_conv_wgrad_every_tile_shape(shape, tile):
    """Every workgroup tile shape (incl. partial last tc tiles: 192 columns) and a few slice counts."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    dy = torch.randn(N, OH, OW, K, device="cuda:0").bfloat16()
    _, gw = _ref_grads(x, k, s, p, dy)
    scale = gw.abs().max().item()
    for S in (1, 3, 40):
        dw = C.conv_wgrad(x, dy, KH, KW, s, s, p, p, out=torch.empty_like(gw), plan=[tile[0], tile[1], S])
        torch.testing.assert_close(dw, gw, atol=2e-3 * scale + 1e-4, rtol=2e-3)


@pytest.mark.parametrize("shape", [(2, 14, 14, 64, 128, 1, 1, 2, 0), (4, 56, 56, 256, 512, 1, 1, 2, 0),
                                   (3, 7, 9, 128, 64, 1, 1, 2, 0), (2, 28, 28, 512, 1024, 1, 1, 2, 0)])
def test_conv_dgrad_stride2_1x1_matches_fp32(shape):
    """1x1 stride-2 input gradient (scatter epilogue writes the zero pixels too, odd sizes included)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    OH, OW = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    dy = torch.randn(N, OH, OW, K, device="cuda:0").bfloat16()
    gx, _ = _ref_grads(x, k, s, p, dy)
    dx = C.conv_dgrad_s2(dy, k.contiguous(), H, W)
    assert dx.shape == x.shape
    torch.testing.assert_close(dx.float(), gx, atol=4e-2, rtol=2e-2)


def test_conv2d_layer_wgrad_and_strided_on_hip_kernels(monkeypatch):
    """keras Conv2D backward with TDL_CONV=hip runs the weight gradient and the strided 1x1 input
    gradient on the hand-written kernels (no MIOpen call)."""
    monkeypatch.setenv("TDL_CONV", "hip")
    from tensorflow_distributed_learning_amd.ops import conv as conv_ops

    x, k = _mk((4, 16, 16, 128, 256, 1, 1, 2, 0), "cuda:0")
    x.requires_grad_(True)
    kk = k.float().requires_grad_(True)
    calls = []
    orig = torch.ops.aten.convolution_backward
    monkeypatch.setattr(conv_ops, "_miopen_bwd", lambda *a: calls.append(1) or orig(*a))
    y = conv_ops.conv2d_nhwc(x, kk.bfloat16(), (2, 2), (0, 0))
    dy = torch.randn(y.shape, device="cuda:0").bfloat16()
    y.backward(dy)
    gx, gw = _ref_grads(x.detach(), k, 2, 0, dy)
    assert not calls, "backward fell back to MIOpen"
    torch.testing.assert_close(x.grad.float(), gx, atol=4e-2, rtol=2e-2)
    torch.testing.assert_close(kk.grad, gw, atol=2e-2 * gw.abs().max().item(), rtol=3e-2)


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 3, 1, 1), (2, 9, 11, 128, 64, 1, 1, 2, 0),
                                   (8, 28, 28, 256, 256, 1, 1, 1, 0)])
def test_conv_fwd_bn_stats_epilogue(shape):
    """conv_fwd_stats: same y as conv_fwd, and a batch norm fed its partial sums matches one that
    computes its own statistics (moving stats, outputs)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    w = k.permute(3, 0, 1, 2).contiguous()
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    y0 = C.conv_fwd(x, w, OH, OW, s, s, p, p)
    y1, part = C.conv_fwd_stats(x, w, OH, OW, s, s, p, p)
    assert torch.equal(y0, y1)
    g, b = torch.rand(K, device="cuda:0") + 0.5, torch.randn(K, device="cuda:0")
    mm0, mv0 = torch.zeros(K, device="cuda:0"), torch.ones(K, device="cuda:0")
    mm1, mv1 = mm0.clone(), mv0.clone()
    ya, sa = C.bn_forward_train(y0, g, b, mm0, mv0, 0.9, 1e-3, True, None, None)
    yb, sb = C.bn_forward_train(y1, g, b, mm1, mv1, 0.9, 1e-3, True, None, None, part)
    torch.testing.assert_close(sb, sa, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(mm1, mm0, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(mv1, mv0, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(yb.float(), ya.float(), atol=2e-2, rtol=1e-2)


@pytest.mark.parametrize("with_box", [False, True])
def test_conv2d_library_wgrad_reaches_slab(monkeypatch, with_box):
    """When the autotuner picks MIOpen for a weight gradient (forced here through its decision
    cache) the gradient still lands in the slab view ``grad_out``, with and without a GradBox
    shared by two consumers of x (advisor finding, round 2)."""
    monkeypatch.setenv("TDL_CONV", "auto")
    from tensorflow_distributed_learning_amd.ops import conv as CV

    shape = (4, 12, 12, 64, 64, 3, 3, 1, 1)
    x, k = _mk(shape, "cuda:0")
    k2 = (k.float() * 0.5).bfloat16()
    key = (tuple(x.shape), tuple(k.shape), (1, 1), (1, 1))
    saved = dict(CV._choice)
    try:
        CV._choice[("wgrad",) + key] = None  # MIOpen
        gout = torch.zeros(k.shape, device="cuda:0")
        gout2 = torch.zeros(k.shape, device="cuda:0")
        xg = x.clone().requires_grad_(True)
        box = CV.GradBox() if with_box else None
        y = CV.conv2d_nhwc(xg, k, (1, 1), (1, 1), grad_out=gout, grad_box=box)
        dy = torch.randn(y.shape, device="cuda:0").bfloat16()
        if with_box:
            y2 = CV.conv2d_nhwc(xg, k2, (1, 1), (1, 1), grad_out=gout2, grad_box=box)
            dy2 = torch.randn(y2.shape, device="cuda:0").bfloat16()
            torch.autograd.backward([y, y2], [dy, dy2])
        else:
            y.backward(dy)
        dx_ref, dw_ref = _ref_grads(x, k, 1, 1, dy)
        torch.testing.assert_close(gout, dw_ref, atol=2e-2 * float(dw_ref.abs().max()), rtol=3e-2)
        if with_box:
            dx2_ref, dw2_ref = _ref_grads(x, k2, 1, 1, dy2)
            torch.testing.assert_close(gout2, dw2_ref, atol=2e-2 * float(dw2_ref.abs().max()), rtol=3e-2)
            dx_ref = dx_ref + dx2_ref
        torch.testing.assert_close(xg.grad.float(), dx_ref, atol=8e-2, rtol=3e-2)
    finally:
        CV._choice.clear()
        CV._choice.update(saved)


@pytest.mark.parametrize("shape", [(4, 14, 14, 64), (2, 56, 56, 128), (3, 9, 61, 64)])
def test_wgrad3x3_row_kernel_matches_fp32(shape):
    """The 3x3 / C = 64 row kernel (csrc/kernels/wgrad3x3.hip, plan [0, 0, 0]) vs fp32 PyTorch, bf16
    out and added into an f32 slab, deterministic."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, K = shape
    g = torch.Generator(device="cpu").manual_seed(4)
    x = torch.randn(N, H, W, 64, generator=g).cuda().bfloat16()
    dy = torch.randn(N, H, W, K, generator=g).cuda().bfloat16()
    plans = C.conv_wgrad_plans(list(x.shape), list(dy.shape), 3, 3, 1, 1, 1, 1, 2)
    assert plans[0] == [0, 0, 0, 0, 0]
    w = torch.zeros(3, 3, 64, K, device="cuda", requires_grad=True)
    y = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), padding=1)
    y.backward(dy.float().permute(0, 3, 1, 2))
    ref = w.grad
    dw = C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, 1, plan=[0, 0, 0])
    scale = ref.abs().max().item()
    assert (dw.float() - ref).abs().max().item() / scale < 1e-2
    slab = torch.full(ref.shape, 0.25, device="cuda")
    C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, 1, out=slab, accumulate=True, plan=[0, 0, 0])
    assert (slab - 0.25 - ref).abs().max().item() / scale < 1e-4
    assert torch.equal(dw, C.conv_wgrad(x, dy, 3, 3, 1, 1, 1, 1, plan=[0, 0, 0]))


@pytest.mark.parametrize("shape", [(3, 7, 7, 128, 256, 1, 1, 1, 0), (8, 28, 28, 64, 256, 1, 1, 1, 0),
                                   (2, 14, 14, 64, 64, 3, 3, 1, 1)])
def test_conv_main_loop_variants_bitwise(shape):
    """Every main-loop variant of the v1 kernel (single LDS stage at 4 waves per SIMD, single stage with
    register prefetch at 3, register
    prefetch depth 1 and 2, and the default selection that takes the single stage for 1-2 k-tile
    reductions) issues the same MFMAs in the same order: outputs and BN partial sums agree bitwise,
    and match the fp32 reference."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    w = k.permute(3, 0, 1, 2).contiguous()
    ref = _ref_fwd(x, k, s, p)
    OH, OW = ref.shape[1], ref.shape[2]
    outs = []
    try:
        C.conv_force_impl(1)
        for depth in (0, 1, 3, 4, 2):
            C.conv_force_depth(depth)
            outs.append((C.conv_fwd(x, w, OH, OW, s, s, p, p),) + tuple(C.conv_fwd_stats(x, w, OH, OW, s, s, p, p)))
    finally:
        C.conv_force_depth(2)
        C.conv_force_impl(2)
    torch.testing.assert_close(outs[0][0].float(), ref, atol=3e-2, rtol=2e-2)
    for o in outs[1:]:
        assert torch.equal(o[0], outs[0][0]) and torch.equal(o[1], outs[0][1])
        R = o[2].shape[0]  # partial rows [P + ceil(P / 64)]: the trailing scratch rows are not outputs
        P = next(q for q in range(R + 1) if q + (q + 63) // 64 == R)
        assert torch.equal(o[2][:P], outs[0][2][:P])


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 3, 1, 1), (8, 28, 28, 128, 64, 1, 1, 1, 0),
                                   (4, 9, 11, 128, 256, 1, 1, 2, 0)])
def test_conv_wgrad_single_stage_matches_double_buffered_bitwise(shape):
    """The register-staged weight-gradient kernel with one LDS stage and the double-buffered one
    accumulate the same MFMAs in the same order: bit-identical for every v1 tile shape."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    dy = torch.randn(N, OH, OW, K, device="cuda:0").bfloat16()
    for wmw, wnw in ((1, 1), (2, 2), (1, 2), (2, 1)):
        if K % (64 * wmw):
            continue
        outs = []
        try:
            for single in (True, False):
                C.conv_wgrad_force_single(single)
                outs.append(C.conv_wgrad(x, dy, KH, KW, s, s, p, p, plan=[wmw, wnw, 3]))
        finally:
            C.conv_wgrad_force_single(False)
        assert torch.equal(outs[0], outs[1]), (wmw, wnw)


@pytest.mark.parametrize("shape", [(4, 14, 14, 64, 128, 3, 3, 1, 1), (8, 28, 28, 128, 256, 1, 1, 1, 0),
                                   (4, 9, 11, 256, 256, 1, 1, 2, 0), (3, 7, 7, 64, 256, 1, 1, 1, 0)])
def test_conv_wgrad_dma1_matches_register_staged_bitwise(shape):
    """The 2x2-wave weight-gradient tile on the single-stage LDS-DMA kernel and on the register-staged
    one accumulate the same MFMAs in the same order: bit-identical (ragged pixel tails included)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KW) // s + 1
    dy = torch.randn(N, OH, OW, K, device="cuda:0").bfloat16()
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (K, Ci, KH, KW), dy.permute(0, 3, 1, 2).float(),
                                      stride=s, padding=p).permute(2, 3, 1, 0)
    for wmw, wnw in ((2, 2),):
        outs = [C.conv_wgrad(x, dy, KH, KW, s, s, p, p, plan=[wmw, wnw, 2, kind]) for kind in (1, 0)]
        assert torch.equal(outs[0], outs[1]), (wmw, wnw)
        err = (outs[0].float() - ref).abs().max() / ref.abs().max()
        assert err < 2e-2, (wmw, wnw, float(err))


@pytest.mark.parametrize("shape", [s for s in SHAPES if s[7] == 1])
def test_conv_dma1_on_mfma_32x32x16_matches_fp32(shape):
    """The dma1 main loop on v_mfma_f32_32x32x16_bf16 (conv_force_impl(6): 2 x 2 blocks of 32 x 32 per
    wave, its own epilogue accumulator layout) against the fp32 reference, forward and input gradient
    (the A/B of the MFMA form: scripts/bench_conv_mfma32.py)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    N, H, W, Ci, K, KH, KW, s, p = shape
    x, k = _mk(shape, "cuda:0")
    xr = x.float().requires_grad_(True)
    ref = _ref_fwd(xr, k, s, p)
    dy = torch.randn(ref.shape, device="cuda:0").bfloat16()
    ref.backward(dy.float())
    try:
        C.conv_force_impl(6)
        y = C.conv_fwd(x, k.permute(3, 0, 1, 2).contiguous(), ref.shape[1], ref.shape[2], s, s, p, p)
        dx = C.conv_dgrad(dy, k.contiguous(), H, W, p, p)
        torch.cuda.synchronize()
    finally:
        C.conv_force_impl(2)
    torch.testing.assert_close(y.float(), ref.detach(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(dx.float(), xr.grad, atol=4e-2, rtol=2e-2)
