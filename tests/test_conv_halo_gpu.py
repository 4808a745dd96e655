"""The halo (input-reuse) conv main loop (csrc/kernels/conv.hip k_conv_halo: one input window per 256-row
tile and 64-channel chunk, every filter tap reading shifted rows of it) against the default kernels and
a float32 PyTorch reference: forward (+ BN statistics epilogue) and stride-1 input gradient (+ residual,
+ fused BN-group backward).  With one 64-channel chunk the reduction runs in the default kernels' order
(tap-major), so outputs are bit-identical; with more chunks it runs chunk-major (the window is loaded once
per chunk) and agrees to f32 rounding."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from tensorflow_distributed_learning_amd.ops import hip

    c = hip()
    yield c
    c.conv_force_halo(2)
    c.conv_force_impl(2)


def _both(C, fn):
    C.conv_force_halo(0)
    a = fn()
    C.conv_force_halo(1)
    b = fn()
    C.conv_force_halo(2)
    return a, b


def _rows_total(part):
    """Sum of the data rows of a BN partial buffer [P + ceil(P/64)][2][C] (the rest is scratch)."""
    P = part.shape[0]
    while P > 1 and (P - 1) + (P - 1 + 63) // 64 >= part.shape[0]:
        P -= 1
    return part[:P].double().sum(0)


def _close(a, b, exact):
    if exact:
        assert torch.equal(a, b)
    else:
        err = ((a.float() - b.float()).abs().max() / b.float().abs().max()).item()
        assert err < 1e-2, err


# (N, H, W, C, K, KH, KW, pad): every ResNet-50 3x3 stage shape (shrunk batch; BN = 64 and 128 column
# tiles), a ragged last row tile, an asymmetric 5x3 filter, an unpadded conv
SHAPES = [
    (8, 56, 56, 64, 64, 3, 3, 1), (16, 28, 28, 128, 128, 3, 3, 1), (32, 14, 14, 256, 256, 3, 3, 1),
    (64, 7, 7, 512, 512, 3, 3, 1), (3, 13, 13, 64, 128, 5, 3, 2), (1, 5, 6, 192, 64, 3, 3, 0),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_halo_forward_and_stats(C, shape):
    N, H, W, Ci, K, KH, KW, p = shape
    g = torch.Generator(device="cpu").manual_seed(hash(shape) % 1000)
    OH, OW = H + 2 * p - KH + 1, W + 2 * p - KW + 1
    x = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
    w = (torch.randn(KH, KW, Ci, K, generator=g) / (KH * KW * Ci) ** 0.5).cuda().bfloat16()
    wo = w.permute(3, 0, 1, 2).contiguous()
    y0, y1 = _both(C, lambda: C.conv_fwd(x, wo, OH, OW, 1, 1, p, p))
    _close(y1, y0, Ci == 64)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(3, 2, 0, 1), None, 1, p).permute(0, 2, 3, 1)
    assert ((y1.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2
    (z0, s0), (z1, s1) = _both(C, lambda: C.conv_fwd_stats(x, wo, OH, OW, 1, 1, p, p))
    assert torch.equal(z1, y1) and torch.equal(z0, y0)
    want = torch.stack([z1.double().reshape(-1, K).sum(0), (z1.double() ** 2).reshape(-1, K).sum(0)])
    torch.testing.assert_close(_rows_total(s1), want, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("shape", SHAPES)
def test_halo_dgrad_and_bn_epilogues(C, shape):
    N, H, W, Ci, K, KH, KW, p = shape
    g = torch.Generator(device="cpu").manual_seed(7)
    OH, OW = H + 2 * p - KH + 1, W + 2 * p - KW + 1
    dy = torch.randn(N, OH, OW, K, generator=g).cuda().bfloat16()
    w = (torch.randn(KH, KW, Ci, K, generator=g) / (KH * KW * K) ** 0.5).cuda().bfloat16()
    x = torch.randn(N, H, W, Ci, generator=g).cuda().requires_grad_(True)
    y = F.conv2d(x.permute(0, 3, 1, 2), w.float().permute(3, 2, 0, 1), None, 1, p).permute(0, 2, 3, 1)
    y.backward(dy.float())
    d0, d1 = _both(C, lambda: C.conv_dgrad(dy, w, H, W, p, p))
    _close(d1, d0, K == 64)
    assert ((d1.float() - x.grad).abs().max() / x.grad.abs().max()).item() < 1e-2
    r = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
    e0, e1 = _both(C, lambda: C.conv_dgrad(dy, w, H, W, p, p, r))
    _close(e1, e0, K == 64)
    by = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
    bx = torch.randn(N, H, W, Ci, generator=g).cuda().bfloat16()
    (z0, q0, q20), (z1, q1, q21) = _both(C, lambda: C.conv_dgrad_bn(dy, w, H, W, p, p, r, by, bx, bx))
    assert torch.equal(z1, (e1.float() * (by.float() > 0)).bfloat16())
    _close(z1, z0, K == 64)
    want = torch.stack([z1.double().reshape(-1, Ci).sum(0), (z1.double() * bx.double()).reshape(-1, Ci).sum(0)])
    for q in (q1, q21):
        torch.testing.assert_close(_rows_total(q), want, rtol=1e-4, atol=1e-2)
    # plain BN -> ReLU group: the mask recomputed from the BN input and its scale / shift
    st = torch.stack([torch.zeros(Ci), torch.ones(Ci), torch.rand(Ci, generator=g) + 0.5,
                      torch.randn(Ci, generator=g)]).cuda()
    (u0, v0), (u1, v1) = _both(C, lambda: C.conv_dgrad_bn(dy, w, H, W, p, p, None, None, bx, None, st)[:2])
    _close(u1, u0, K == 64)
    torch.testing.assert_close(_rows_total(v1), _rows_total(v0), rtol=1e-3, atol=5e-2)


def test_halo_selection_reports_256_row_tiles(C):
    """The BN partial buffers of a halo launch have one row per 256 output rows."""
    x = torch.randn(4, 28, 28, 128, device="cuda").bfloat16()
    w = (torch.randn(128, 3, 3, 128, device="cuda") * 0.03).bfloat16()
    _, s0 = C.conv_fwd_stats(x, w, 28, 28, 1, 1, 1, 1)  # (not a default halo shape)
    C.conv_force_halo(1)
    try:
        _, s1 = C.conv_fwd_stats(x, w, 28, 28, 1, 1, 1, 1)
    finally:
        C.conv_force_halo(2)
    M = 4 * 28 * 28
    assert s1.shape[0] < s0.shape[0]
    assert s1.shape[0] >= (M + 255) // 256


def test_halo_default_takes_only_the_14x14_class(C):
    """Default selection (TDL_CONV_HALO unset): the halo kernel for 3x3 convs on 14x14-class maps with
    >= 256 channels (256-row partial-sum tiles), the other kernels elsewhere (128-row tiles)."""
    M = 2 * 14 * 14
    x = torch.randn(2, 14, 14, 256, device="cuda").bfloat16()
    w = (torch.randn(256, 3, 3, 256, device="cuda") * 0.02).bfloat16()
    _, s = C.conv_fwd_stats(x, w, 14, 14, 1, 1, 1, 1)
    assert s.shape[0] <= (M + 255) // 256 + 1  # 256-row tiles (+ scratch rows)
    x2 = torch.randn(2, 28, 28, 128, device="cuda").bfloat16()
    w2 = (torch.randn(128, 3, 3, 128, device="cuda") * 0.03).bfloat16()
    _, s2 = C.conv_fwd_stats(x2, w2, 28, 28, 1, 1, 1, 1)
    assert s2.shape[0] >= (2 * 28 * 28 + 127) // 128
