"""Numerics of the fused gfx950 MNIST-CNN train step vs a plain-PyTorch fp64 reference."""
import pytest
import torch

from tensorflow_distributed_learning_amd.models import mnist_cnn as M

pytestmark = pytest.mark.gpu


def _setup(cuda, b, R=1, N=512, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(N, 28, 28, 1, generator=g)
    Y = torch.randint(0, 10, (N,), generator=g, dtype=torch.int32)
    params = M.init_mnist_params(seed)
    # non-zero biases so bias paths are exercised
    for i in (1, 3, 5, 7):
        params[i] = (torch.rand(params[i].shape, generator=g) - 0.5) * 0.1
    layout = M.mnist_layout()
    W = layout.pack(params, device=cuda)
    G = torch.zeros_like(W)
    idx = torch.randperm(N, generator=g)[: 3 * b].to(torch.int32)
    lr = torch.tensor([0.01], device=cuda)
    step = M.FusedMnistTrainStep(X.to(cuda), Y.to(cuda), idx.to(cuda), W, G, layout, b, R, lr)
    return X, Y, params, layout, W, G, idx, lr, step


def _ref_grads(params, x, y, R):
    p = [t.double().clone().requires_grad_(True) for t in params]
    loss, logits, ce = M.reference_loss(p, x.double(), y, R)
    loss.backward()
    return [t.grad for t in p], logits.detach(), ce.detach()


@pytest.mark.parametrize("b,R", [(64, 1), (64, 8), (17, 2), (1, 1), (128, 1)])
def test_fused_grads_match_reference(cuda, b, R):
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, R)
    off = b  # second chunk of idx
    step.forward_backward(off)
    step.finalize(False)
    torch.cuda.synchronize()
    _check_step(step, X, Y, params, layout, G, idx, off, b, R)


@pytest.mark.parametrize("mode,fused", [("0", "1"), ("1", "0"), ("1", "1")])
@pytest.mark.parametrize("split", [False, True])
def test_fused_dp2_modes(cuda, monkeypatch, mode, fused, split):
    """dP2 in the forward kernel (workgroups wait for their image's head) or in the K5 launch, with
    the conv backward in the forward kernel too (fused_bwd) or in its own launch, on the
    single-launch-sequence path and on the R > 1 split (forward_dense / backward_conv)."""
    monkeypatch.setenv("TDL_MNIST_DP2_FWD", mode)
    monkeypatch.setenv("TDL_MNIST_FUSED_BWD", fused)
    b, R = 64, 2
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, R)
    assert step.dp2_in_forward == (mode == "1")
    assert step.fused_bwd == (mode == "1" and fused == "1")
    off = 2 * b
    if split:
        step.forward_dense(off)
        step.backward_conv()
    else:
        step.forward_backward(off)
    step.finalize(False)
    torch.cuda.synchronize()
    _check_step(step, X, Y, params, layout, G, idx, off, b, R)
    step.check()  # no in-kernel hand-off timed out


def test_fused_bwd_steps_match_unfused(cuda, monkeypatch):
    """Several consecutive fused steps (hand-off tags advanced by finalize, not by k_conv_bwd)
    track the unfused launch sequence to f32 rounding."""
    b = 64
    outs = []
    for fused in ("0", "1"):
        monkeypatch.setenv("TDL_MNIST_FUSED_BWD", fused)
        X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, 1)
        assert step.fused_bwd == (fused == "1")
        for k in range(3):
            step.forward_backward(k * b)
            step.finalize(True)
        torch.cuda.synchronize()
        step.check()
        outs.append((W.clone(), step.metrics.clone()))
    torch.testing.assert_close(outs[1][0], outs[0][0], atol=1e-6, rtol=1e-5)
    torch.testing.assert_close(outs[1][1][:3], outs[0][1][:3], atol=1e-3, rtol=1e-5)


def test_dp2_mode_selection(cuda, monkeypatch):
    monkeypatch.delenv("TDL_MNIST_DP2_FWD", raising=False)
    monkeypatch.delenv("TDL_SHARE_GPU", raising=False)
    cus = torch.cuda.get_device_properties(cuda).multi_processor_count
    assert M.dp2_in_forward_ok(cus // 4, 1, cuda)
    assert not M.dp2_in_forward_ok(cus // 4 + 1, 1, cuda)  # not every workgroup resident at once
    assert M.dp2_in_forward_ok(16, 8, cuda)  # replicas: each step's all-reduce ends before the next forward
    monkeypatch.setenv("TDL_SHARE_GPU", "1")
    assert not M.dp2_in_forward_ok(16, 1, cuda)


def _check_step(step, X, Y, params, layout, G, idx, off, b, R):
    ids = idx[off:off + b].long()
    x, y = X[ids], Y[ids]
    grads, logits, ce = _ref_grads(params, x, y, R)
    got = layout.views(G.cpu())
    names = [n for n, _ in M.MNIST_CNN_VARIABLES]
    for name, gr, gg in zip(names, grads, got):
        err = (gg.double() - gr).abs().max().item()
        scale = gr.abs().max().item() + 1e-12
        assert err <= 2e-5 * scale + 1e-9, f"{name}: max err {err} vs scale {scale}"
    m = step.metrics.cpu()
    assert abs(m[0].item() - ce.sum().item()) < 1e-3 * max(1.0, ce.sum().item())
    correct = (logits.argmax(1) == y.long()).sum().item()
    assert m[1].item() == correct
    assert m[2].item() == b


def test_fused_sgd_update(cuda):
    b = 64
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, 1)
    W0 = W.clone()
    step.forward_backward(0)
    step.finalize(True)
    torch.cuda.synchronize()
    assert torch.allclose(W, W0 - 0.01 * G, atol=1e-7, rtol=0)


def test_fused_sgd_without_grad_store(cuda):
    """keep_grad=False (the single-replica fit path): the same SGD update, bit for bit, and the
    gradient slab G is left untouched."""
    b = 64
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, 1)
    W0 = W.clone()
    step.forward_backward(0)
    step.finalize(True)
    W_keep, G_keep = W.clone(), G.clone()
    W.copy_(W0)
    G.fill_(123.0)
    step.forward_backward(0)
    step.finalize(True, keep_grad=False)
    torch.cuda.synchronize()
    assert torch.equal(W, W_keep)
    assert bool((G == 123.0).all()), "keep_grad=False must not write G"
    # the flag is per call: the next default finalize writes G again (slab padding stays as set)
    W.copy_(W0)
    G.zero_()
    step.forward_backward(0)
    step.finalize(True)
    torch.cuda.synchronize()
    assert torch.equal(G, G_keep)


def test_fused_step_graph_capture(cuda):
    b = 64
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, 1)
    W_eager = W.clone()
    # eager reference: 3 steps
    Wsave = W.clone()
    for k in range(3):
        step.forward_backward(k * b)
        step.finalize(True)
    torch.cuda.synchronize()
    W_eager = W.clone()
    W.copy_(Wsave)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        step.forward_backward(0)  # warm-up (not captured)
        step.finalize(False)
    torch.cuda.synchronize()
    with torch.cuda.graph(graph, stream=s):
        for k in range(3):
            step.forward_backward(k * b)
            step.finalize(True)
    W.copy_(Wsave)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(W, W_eager), "graph replay must be bit-identical to eager execution"


def test_fused_deterministic(cuda):
    b = 64
    X, Y, params, layout, W, G, idx, lr, step = _setup(cuda, b, 1)
    step.forward_backward(0)
    step.finalize(False)
    g1 = G.clone()
    step.forward_backward(0)
    step.finalize(False)
    torch.cuda.synchronize()
    assert torch.equal(g1, G)
