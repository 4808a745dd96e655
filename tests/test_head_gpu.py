"""Classifier-head kernels (csrc/kernels/gemm.hip, ops/dense.py) vs float32 PyTorch references:
bf16 MFMA GEMM in all four operand storages, NHWC global average pooling, sparse softmax
cross-entropy, and the Dense layer's forward/backward incl. direct gradient-slab accumulation."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _r(*shape, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(*shape, generator=g).cuda()


@pytest.mark.parametrize("ta", [0, 1])
@pytest.mark.parametrize("tb", [0, 1])
@pytest.mark.parametrize("mnk", [(256, 1000, 2048), (136, 200, 40), (8, 8, 8), (264, 1032, 1000)])
def test_gemm_bf16_all_storages(ta, tb, mnk):
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    M, N, K = mnk
    A = _r(M, K, seed=1).bfloat16()
    B = _r(K, N, seed=2).bfloat16()
    a = A.t().contiguous() if ta else A  # stored [K][M] when ta = 1
    b = B.contiguous() if tb else B.t().contiguous()  # stored [K][N] when tb = 1, [N][K] when 0
    ref = A.float() @ B.float()
    bias = _r(N, seed=3)
    y = C.gemm_bf16(a, ta, b, tb, bias=bias)
    assert y.dtype == torch.bfloat16 and y.shape == (M, N)
    scale = ref.abs().max().item()
    torch.testing.assert_close(y.float(), ref + bias, atol=1e-2 * scale, rtol=1e-2)
    out = torch.full((M, N), 0.5, device="cuda")
    C.gemm_bf16(a, ta, b, tb, out=out, accumulate=True, alpha=2.0)
    torch.testing.assert_close(out, 0.5 + 2 * ref, atol=1e-3 * scale, rtol=1e-3)


def test_gap_fwd_bwd():
    from tensorflow_distributed_learning_amd.ops.dense import gap_nhwc

    x = _r(16, 7, 7, 2048).bfloat16().requires_grad_(True)
    y = gap_nhwc(x)
    xr = x.detach().float().requires_grad_(True)
    yr = xr.mean(dim=(1, 2))
    torch.testing.assert_close(y.float(), yr, atol=1e-2, rtol=1e-2)
    dy = _r(16, 2048, seed=4).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=1e-3, rtol=1e-2)


def test_softmax_xent_matches_cross_entropy():
    from tensorflow_distributed_learning_amd.ops.dense import softmax_xent

    z = (_r(256, 1000) * 3).requires_grad_(True)
    y = torch.randint(0, 1000, (256,), device="cuda")
    l = softmax_xent(z, y)
    zr = z.detach().clone().requires_grad_(True)
    lr = F.cross_entropy(zr, y, reduction="none")
    torch.testing.assert_close(l, lr, atol=1e-5, rtol=1e-5)
    w = _r(256, seed=5)
    (l * w).sum().backward()
    (lr * w).sum().backward()
    torch.testing.assert_close(z.grad, zr.grad, atol=1e-6, rtol=1e-4)


def test_dense_layer_bf16_and_slab_targets():
    from tensorflow_distributed_learning_amd.ops.dense import dense_bf16

    x = _r(64, 512).bfloat16().requires_grad_(True)
    w = (_r(512, 1000, seed=6) * 0.05).bfloat16().requires_grad_(True)
    b = _r(1000, seed=7).requires_grad_(True)
    y = dense_bf16(x, w, b)
    xr, wr, br = (t.detach().float().requires_grad_(True) for t in (x, w, b))
    yr = xr @ wr + br
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = _r(64, 1000, seed=8).bfloat16()
    y.backward(dy)
    yr.backward(dy.float())
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(b.grad, br.grad, atol=1e-3, rtol=1e-3)
    # slab targets: gradients ADDED into f32 views, none returned
    gw, gb = torch.ones(512, 1000, device="cuda"), torch.ones(1000, device="cuda")
    x2 = x.detach().requires_grad_(True)
    y2 = dense_bf16(x2, w.detach(), b.detach(), (gw, gb))
    y2.backward(dy)
    torch.testing.assert_close(gw, 1 + wr.grad, atol=2e-2, rtol=1e-2)
    torch.testing.assert_close(gb, 1 + br.grad, atol=1e-3, rtol=1e-3)
    torch.testing.assert_close(x2.grad, x.grad)
