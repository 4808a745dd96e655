"""NHWC bf16 convolution on the hand-written implicit-GEMM MFMA kernels (csrc/kernels/conv.hip).

The reference's ``tf.keras.layers.Conv2D`` (tf_dist_example.py:41,43; ResNet-50 of BASELINE configs
4/5) runs on cuDNN inside TensorFlow.  Here a Conv2D with bf16 NHWC activations, C and K multiples
of 64 and symmetric padding has two implementations per direction: the hand-written kernels
(forward; stride-1 input gradient) and MIOpen (through ``torch.nn.functional``).  The weight
gradient, and the input gradient of strided convolutions, stay on MIOpen.

``TDL_CONV`` picks: ``auto`` (default) times both implementations on the first eager call of every
(shape, direction) and keeps the faster one (decisions are cached per process and never measured
while a HIP graph is being captured; an unmeasured shape inside a capture uses MIOpen), ``hip``
forces the hand-written kernels wherever they apply, ``miopen`` disables them.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from . import hip

_choice: dict = {}  # (direction, shape key) -> True (hand-written kernel) / False (MIOpen)
_times: dict = {}  # (direction, shape key) -> (hand-written ms, MIOpen ms) as measured by the autotuner


def mode() -> str:
    return os.environ.get("TDL_CONV", "auto").lower()


def supported(x: torch.Tensor, kernel_hwio: torch.Tensor, groups=1, dilation=(1, 1)) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and groups == 1 and tuple(dilation) == (1, 1)
            and x.shape[-1] % 64 == 0 and kernel_hwio.shape[-1] % 64 == 0 and mode() != "miopen")


def _time(fn, reps=5) -> float:
    """Median of ``reps`` individually timed calls after two untimed ones (the first MIOpen call of a
    shape runs its find-mode solver search)."""
    fn()
    fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e))
    return sorted(ts)[reps // 2]


def _pick(key, hip_fn, ref_fn) -> bool:
    m = mode()
    if m == "hip":
        return True
    got = _choice.get(key)
    if got is not None:
        return got
    if torch.cuda.is_current_stream_capturing():
        return False
    t_ref = _time(ref_fn)
    t_hip = _time(hip_fn)
    got = t_hip < t_ref
    _choice[key] = got
    _times[key] = (t_hip, t_ref)
    return got


def choices() -> dict:
    """The autotuner's decisions so far: {(direction, shape key): 'hip' | 'miopen'}."""
    return {k: ("hip" if v else "miopen") for k, v in _choice.items()}


def _ref_fwd(x, w_oihw, stride, pad):
    return F.conv2d(x.permute(0, 3, 1, 2), w_oihw, None, stride, pad).permute(0, 2, 3, 1)


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, stride, pad):
        C = hip()
        x = x.contiguous()
        if x.data_ptr() % 16:
            x = x.clone()
        kh, kw, cin, cout = kernel.shape
        sh, sw = stride
        ph, pw = pad
        oh, ow = (x.shape[1] + 2 * ph - kh) // sh + 1, (x.shape[2] + 2 * pw - kw) // sw + 1
        w_oihw = kernel.permute(3, 2, 0, 1)
        key = ("fwd", tuple(x.shape), tuple(kernel.shape), stride, pad)
        w_ohwi = kernel.permute(3, 0, 1, 2).contiguous()
        hip_fn = lambda: C.conv_fwd(x, w_ohwi, oh, ow, sh, sw, ph, pw)  # noqa: E731
        if _pick(key, hip_fn, lambda: _ref_fwd(x, w_oihw, stride, pad)):
            y = hip_fn()
        else:
            y = _ref_fwd(x, w_oihw, stride, pad).contiguous()
        ctx.save_for_backward(x, kernel)
        ctx.geo = (stride, pad)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        x, kernel = ctx.saved_tensors
        stride, pad = ctx.geo
        dy = dy.contiguous()
        if dy.data_ptr() % 16:
            dy = dy.clone()
        w_oihw = kernel.permute(3, 2, 0, 1)
        x_nchw, dy_nchw = x.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2)
        dx = None
        want_dx = ctx.needs_input_grad[0]
        if want_dx and stride == (1, 1):
            kc = kernel.contiguous()
            key = ("dgrad", tuple(x.shape), tuple(kernel.shape), stride, pad)
            hip_fn = lambda: C.conv_dgrad(dy, kc, x.shape[1], x.shape[2], pad[0], pad[1])  # noqa: E731
            ref_fn = lambda: torch.ops.aten.convolution_backward(  # noqa: E731
                dy_nchw, x_nchw, w_oihw, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
                [True, False, False])[0]
            if _pick(key, hip_fn, ref_fn):
                dx = hip_fn()
        gx, gw, _ = torch.ops.aten.convolution_backward(
            dy_nchw, x_nchw, w_oihw, None, list(stride), list(pad), [1, 1], False, [0, 0], 1,
            [want_dx and dx is None, ctx.needs_input_grad[1], False])
        if dx is None and gx is not None:
            dx = gx.permute(0, 2, 3, 1)
        dk = gw.permute(2, 3, 1, 0) if gw is not None else None
        return dx, dk, None, None


def conv2d_nhwc(x, kernel_hwio, stride=(1, 1), pad=(0, 0)):
    """y[N,OH,OW,K] = conv(x[N,H,W,C], kernel[KH,KW,C,K]) with symmetric zero padding ``pad = (ph, pw)``,
    bf16; the caller checked :func:`supported`."""
    return _Conv.apply(x, kernel_hwio, tuple(stride), tuple(pad))
