"""The LDS-DMA conv kernels (csrc/kernels/conv.hip k_conv_glds: the 3-stage ring with 256-row tiles,
and the single-stage dma1 variant with 128-row tiles at 4 and 3 waves per SIMD) against the v1
register-staged kernel and fp32 PyTorch, on shapes large enough for the launcher to pick it: the
same per-output MFMA chain over the same k-tile order, so outputs are bit-identical to v1; the BN
partial sums (per 256-row tile instead of 128) agree in total."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C():
    from tensorflow_distributed_learning_amd.ops import hip

    c = hip()
    yield c
    c.conv_force_impl(2)


ALT = [3]


@pytest.fixture(autouse=True, params=[3, 4, 5], ids=["ring", "dma1_w4", "dma1_w3"])
def _alt_impl(request):
    ALT[0] = request.param
    yield


def _both(C, fn):
    C.conv_force_impl(1)
    a = fn()
    # 3: the ring kernel wherever it fits (the default picks it only for long 1x1 reductions);
    # 4 / 5: the single-stage LDS-DMA kernel
    C.conv_force_impl(ALT[0])
    b = fn()
    C.conv_force_impl(2)
    return a, b


def _rows_total(part, _unused=None):
    """Sum of the data rows of a BN partial buffer [P + ceil(P/64)][2][C] (the rest is scratch)."""
    P = part.shape[0]
    while P > 1 and (P - 1) + (P - 1 + 63) // 64 >= part.shape[0]:
        P -= 1
    return part[:P].double().sum(0)


SHAPES = [  # N, H, C, K, kh, stride (M / 256 x column tiles >= 256 workgroups: v2 applies)
    (32, 56, 64, 64, 3, 1), (128, 28, 128, 128, 3, 1), (256, 14, 256, 256, 3, 1), (64, 28, 512, 128, 1, 1),
    (64, 56, 256, 512, 1, 2), (256, 7, 512, 2048, 1, 1),
]


@pytest.mark.parametrize("shape", SHAPES)
def test_v2_forward_bitwise_v1_and_matches_fp32(C, shape):
    N, H, Ci, K, kh, s = shape
    g = torch.Generator(device="cpu").manual_seed(hash(shape) % 1000)
    p = kh // 2
    OH = (H + 2 * p - kh) // s + 1
    x = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    w = (torch.randn(kh, kh, Ci, K, generator=g) * (1.0 / (kh * kh * Ci) ** 0.5)).cuda().bfloat16()
    wo = w.permute(3, 0, 1, 2).contiguous()
    y1, y2 = _both(C, lambda: C.conv_fwd(x, wo, OH, OH, s, s, p, p))
    assert torch.equal(y1, y2)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(3, 2, 0, 1), None, s, p).permute(0, 2, 3, 1)
    err = (y2.float() - ref).abs().max() / ref.abs().max()
    assert err < 1e-2, err
    (z1, s1), (z2, s2) = _both(C, lambda: C.conv_fwd_stats(x, wo, OH, OH, s, s, p, p))
    assert torch.equal(z1, y1) and torch.equal(z2, y1)
    M = N * OH * OH
    t1, t2 = _rows_total(s1, (M + 127) // 128), _rows_total(s2, (M + 255) // 256)
    want = torch.stack([y1.double().reshape(-1, K).sum(0), (y1.double() ** 2).reshape(-1, K).sum(0)])
    torch.testing.assert_close(t2, want, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(t1, t2, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("shape", [sh for sh in SHAPES if sh[5] == 1])
def test_v2_dgrad_and_bn_epilogue(C, shape):
    N, H, Ci, K, kh, s = shape
    g = torch.Generator(device="cpu").manual_seed(7)
    p = kh // 2
    dy = torch.randn(N, H, H, K, generator=g).cuda().bfloat16()
    w = (torch.randn(kh, kh, Ci, K, generator=g) * (1.0 / (kh * kh * K) ** 0.5)).cuda().bfloat16()
    r = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    d1, d2 = _both(C, lambda: C.conv_dgrad(dy, w, H, H, p, p, r))
    assert torch.equal(d1, d2)
    by = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    bx = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    (z1, q1, q21), (z2, q2, q22) = _both(C, lambda: C.conv_dgrad_bn(dy, w, H, H, p, p, r, by, bx, bx))
    assert torch.equal(z1, z2)
    assert torch.equal(z2, (d2.float() * (by.float() > 0)).bfloat16())
    M = N * H * H
    for a, b in ((q1, q2), (q21, q22)):
        torch.testing.assert_close(_rows_total(a, (M + 127) // 128), _rows_total(b, (M + 255) // 256), rtol=1e-4,
                                   atol=1e-2)


def test_v2_dgrad_stride2_scatter(C):
    N, OH, Ci, K = 64, 28, 256, 512
    H = 2 * OH
    g = torch.Generator(device="cpu").manual_seed(11)
    dy = torch.randn(N, OH, OH, K, generator=g).cuda().bfloat16()
    w = (torch.randn(1, 1, Ci, K, generator=g) * 0.05).cuda().bfloat16()
    r = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    a, b = _both(C, lambda: C.conv_dgrad_s2(dy, w, H, H, r))
    assert torch.equal(a, b)
    by = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    bx = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    (z1, q1), (z2, q2) = _both(C, lambda: C.conv_dgrad_s2_bn(dy, w, H, H, r, by, bx))
    assert torch.equal(z1, z2)
    M = N * OH * OH
    torch.testing.assert_close(_rows_total(q1, (M + 127) // 128), _rows_total(q2, (M + 255) // 256), rtol=1e-4,
                               atol=1e-2)


@pytest.mark.parametrize("shape", [(64, 14, 256, 256, 3, 1, 1), (32, 28, 512, 256, 1, 2, 0), (64, 7, 512, 512, 3, 1, 1),
                                   (32, 56, 256, 128, 1, 1, 0)])
def test_v2_wgrad_ring_plans_match_v1_and_fp32(C, shape):
    """The 8-wave LDS-DMA weight-gradient kernel (plans [2, 4, S] / [4, 2, S]) against a v1 plan and
    fp32 PyTorch, including padded taps and a strided conv."""
    N, H, Ci, K, kh, s, p = shape
    g = torch.Generator(device="cpu").manual_seed(5)
    OH = (H + 2 * p - kh) // s + 1
    x = torch.randn(N, H, H, Ci, generator=g).cuda().bfloat16()
    dy = torch.randn(N, OH, OH, K, generator=g).cuda().bfloat16()
    ref = torch.ops.aten.convolution_backward(dy.float().permute(0, 3, 1, 2), x.float().permute(0, 3, 1, 2),
                                              torch.zeros(K, Ci, kh, kh, device="cuda"), None, [s, s], [p, p], [1, 1],
                                              False, [0, 0], 1, [False, True, False])[1].permute(2, 3, 1, 0)
    outs = {}
    for plan in ([2, 2, 3], [2, 4, 3], [4, 2, 5], [2, 4, 1]):
        if K % (64 * plan[0]):
            continue
        o = torch.zeros(kh * kh * Ci * K, device="cuda")
        C.conv_wgrad(x, dy, kh, kh, s, s, p, p, out=o, accumulate=True, plan=plan)
        outs[tuple(plan)] = o.view(kh, kh, Ci, K)
        err = (outs[tuple(plan)] - ref).abs().max() / ref.abs().max()
        assert err < 2e-5 * max(1, N * OH * OH / 1000) ** 0.5 + 1e-4, (plan, float(err))
    # same split count: same per-slice f32 sums in the same order -> bit-identical to the v1 kernel
    if (2, 2, 3) in outs and (2, 4, 3) in outs:
        assert torch.equal(outs[(2, 2, 3)], outs[(2, 4, 3)])
