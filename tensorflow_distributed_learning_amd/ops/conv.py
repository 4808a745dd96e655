"""NHWC bf16 convolution on the hand-written implicit-GEMM MFMA kernels (csrc/kernels/conv.hip).

The reference's ``tf.keras.layers.Conv2D`` (tf_dist_example.py:41,43; ResNet-50 of BASELINE configs
4/5) runs on cuDNN inside TensorFlow.  Here a Conv2D with bf16 NHWC activations, C and K multiples
of 64 and symmetric padding has two implementations per direction: the hand-written kernels
(forward; stride-1 and 1x1 stride-2 input gradient, csrc/kernels/conv.hip; weight gradient,
csrc/kernels/conv_wgrad.hip) and MIOpen (through ``torch.nn.functional``, a test oracle).  The
directions and shapes those bf16 kernels do not tile (other strided input gradients, >= 2^24-row
weight gradients) and every f32 / odd-channel / asymmetric-padding / dilated conv run on the
generic f32-MFMA kernels of ops/conv_f32.py (csrc/kernels/gemm_f32.hip).

``TDL_CONV`` picks: ``hip`` (default) runs the hand-written kernels for every shape they cover;
``auto`` times both implementations on the first eager call of every (shape, direction) and keeps
the faster one (decisions are cached per process and never measured while a HIP graph is being
captured: an unmeasured shape inside a capture takes the hand-written kernel); ``miopen`` disables
them (a test oracle).  Every convolution that still runs on the library -- a shape or dtype no
hand-written kernel covers, ``miopen`` / ``auto`` choices, the very large weight gradients -- is
counted in :data:`LIB_CALLS` (``library_calls()``; bench JSON ``fallbacks``).
"""
from __future__ import annotations

import collections
import os
import threading

import torch
import torch.nn.functional as F

from . import hip

_FUSE_BN_BWD = [os.environ.get("TDL_FUSE_BN_BWD", "1") == "1"]
# the two extensions of that fusion, separately switchable: the 1x1 stride-2 input gradient's epilogue,
# and the projection-shortcut BN's sums (part2) beside the block-output group's
_FUSE_BN_BWD_S2 = [os.environ.get("TDL_FUSE_BN_BWD_S2", "1") == "1"]
_FUSE_BN_BWD_SHORTCUT = [os.environ.get("TDL_FUSE_BN_BWD_SHORTCUT", "1") == "1"]
# a plain BN -> ReLU group's mask recomputed from its BN input and statistics (one read less)
_FUSE_BN_MASK_STATS = [os.environ.get("TDL_FUSE_BN_MASK_STATS", "1") == "1"]

# Weight gradients into a trainer's slab on a side stream, overlapping the input-gradient / BN chain
# of the main stream (the trainer opens the window around loss.backward() and joins it before the
# slab is read: side_stream_window / join_side).  The side stream forks from the main stream at each
# wgrad (so it sees dy and x), the tensors it reads stay referenced until the join (no allocator
# reuse while it may still read them).  Off by default (TDL_WGRAD_STREAM=1 enables it): measured on
# ResNet-50 b=256 the kernels do run concurrently (summed kernel time 26.4 ms in a 21.2 ms step) but
# the step does not get shorter -- the main chain's grids already fill the GPU, and the latency-bound
# BN finalize / split-K reduce kernels only slow down beside the wgrads
# (profiles/resnet50_steady_state_breakdown_r4_wgrad_side_stream.txt).
_WGRAD_SIDE = [os.environ.get("TDL_WGRAD_STREAM", "0") == "1"]
_SIDE: dict = {}  # device index -> torch.cuda.Stream
_SIDE_HELD: list = []  # tensors queued side-stream work reads
_SIDE_STATE = {"open": False, "used": False}


def _side_stream(dev):
    s = _SIDE.get(dev.index)
    if s is None:
        s = _SIDE[dev.index] = torch.cuda.Stream(dev)
    return s


def side_stream_window(open_: bool) -> None:
    """The trainer's backward window: while open, slab weight gradients go to the side stream."""
    _SIDE_STATE["open"] = bool(open_) and _WGRAD_SIDE[0]


def join_side() -> None:
    """Order each device's current stream after every weight gradient queued on its side stream (before
    the slab is read: bucket all-reduce, optimizer) and release the tensors that work reads."""
    if not _SIDE_STATE["used"]:
        return
    for idx, s in _SIDE.items():
        torch.cuda.current_stream(torch.device("cuda", idx)).wait_stream(s)
    _SIDE_HELD.clear()
    _SIDE_STATE["used"] = False
_choice: dict = {}  # (direction, shape key) -> True (hand-written kernel) / False (MIOpen)
_times: dict = {}  # (direction, shape key) -> (hand-written ms, MIOpen ms) as measured by the autotuner


def mode() -> str:
    return os.environ.get("TDL_CONV", "hip").lower()


# convolution work that ran on the library (MIOpen through torch) instead of a hand-written kernel:
# (direction, reason) -> calls.  Empty on the hot path of every model whose convs the kernels cover.
LIB_CALLS: "collections.Counter" = collections.Counter()


def _lib(direction: str, reason: str) -> None:
    LIB_CALLS[(direction, reason)] += 1


def library_calls() -> dict:
    """{(direction, reason): calls} of convolutions that ran on MIOpen since the last reset."""
    return dict(LIB_CALLS)


def reset_library_calls() -> None:
    LIB_CALLS.clear()


def supported(x: torch.Tensor, kernel_hwio: torch.Tensor, groups=1, dilation=(1, 1)) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and groups == 1 and tuple(dilation) == (1, 1)
            and x.shape[-1] % 64 == 0 and kernel_hwio.shape[-1] % 64 == 0 and mode() != "miopen")


class GradBox:
    """Rendezvous of the two backward contributions to a tensor with two consumers, at least one of
    them a hand-written conv (keras/fusion.py plans them).  Participants register in the forward
    (``n``); in the backward the first participant parks its contribution in ``g`` and returns
    nothing for the tensor, the second adds it in: a conv input gradient inside its epilogue (no
    separate add pass), a :class:`_GradTap` with one add.  With fewer than two registered
    participants (a conv that fell back to a library path) everybody returns gradients normally."""

    __slots__ = ("n", "g")

    def __init__(self):
        self.n = 0
        self.g = None

    @property
    def active(self) -> bool:
        return self.n == 2


class _GradTap(torch.autograd.Function):
    """Identity in the forward; in the backward a :class:`GradBox` participant."""

    @staticmethod
    def forward(ctx, t, box):
        box.n += 1
        ctx.box = box
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        box = ctx.box
        if not box.active:
            return g, None
        if box.g is None:
            box.g = g
            return None, None
        s = g + box.g
        box.g = None
        return s, None


def grad_tap(t: torch.Tensor, box: GradBox) -> torch.Tensor:
    return _GradTap.apply(t, box)


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


# the hand-written kernel is kept unless the library is more than this much faster: single timings of
# near-equal candidates flip from run to run (profiles/resnet50_steady_state_breakdown_r3b.txt had a
# 3x3 wgrad on MIOpen that the bench run before had on the hand-written kernel), and a stable choice
# keeps the step's kernel set -- and its numerics -- the same across runs
_PREFER_HIP = float(os.environ.get("TDL_CONV_PREFER_HIP", "1.05"))
_HBM_BYTES_PER_MS = 4.5e9  # streaming rate the BN/add kernels reach on MI355X (profiles/bn_tuning_sweep_r2.jsonl)


# the job's communicator while a multi-replica trainer runs (engine/trainer.py binds it): rank 0
# makes every autotuning decision and broadcasts it, so that all replicas run the same kernel set
# (the same numerics, the same step time) instead of timing candidates each on its own
_COMM = [None]
# the binding of the calling thread: replicas of a single-process MirroredStrategy are threads of one
# process (parallel/local_replicas.py), each with its own rank in its own communicator
_COMM_TLS = threading.local()
_FALLBACK_LOGGED: set = set()


def bind_communicator(comm) -> None:
    c = comm if comm is not None and getattr(comm, "world_size", 1) > 1 else None
    _COMM[0] = c
    _COMM_TLS.comm = c


def _bound_comm():
    return getattr(_COMM_TLS, "comm", _COMM[0])


def _capture_fallback(key) -> None:
    """``auto`` mode: a shape first met inside a graph capture cannot be timed (nor agreed on
    collectively): it takes the hand-written kernel untimed.  Said once per shape."""
    if key not in _FALLBACK_LOGGED:
        _FALLBACK_LOGGED.add(key)
        import warnings

        warnings.warn(f"conv autotuner: {key[0]} shape {key[1:]} first seen inside a hipGraph capture; "
                      "using the hand-written kernel untimed (run one eager step of every shape before capturing)")


_AGREE_WIDTH = 5  # [chosen, wmw, wnw, nsplit, kind]


def _agree(local_decide, encode, decode):
    """Rank 0 decides (``local_decide``), every rank gets rank 0's decision.  Collective: every
    replica reaches the same key at the same point of the same model's first eager step."""
    comm = _bound_comm()
    if comm is None:
        return local_decide()
    v = local_decide() if comm.rank == 0 else None
    on = comm.device if getattr(comm, "name", "") == "rccl" else torch.device("cpu")
    e = encode(v) if v is not None else []
    assert len(e) <= _AGREE_WIDTH, e
    t = torch.tensor(e + [0] * (_AGREE_WIDTH - len(e)), dtype=torch.int64, device=on)  # same size on every rank
    comm.broadcast(t, 0)
    return decode(t.tolist())


def _pick(key, hip_fn, ref_fn, saved_bytes: int = 0) -> bool:
    """``saved_bytes``: HBM traffic of the passes the hand-written kernel's fused epilogue removes
    (BN statistics, gradient sums) that the library path would still run; credited to it."""
    m = mode()
    if m == "hip":
        return True
    got = _choice.get(key)
    if got is not None:
        return got
    if torch.cuda.is_current_stream_capturing():
        _capture_fallback(key)
        return True

    def decide():
        t_ref = _time(ref_fn) + saved_bytes / _HBM_BYTES_PER_MS
        t_hip = _time(hip_fn)
        _times[key] = (t_hip, t_ref)
        return t_hip < t_ref * _PREFER_HIP

    got = _agree(decide, lambda v: [int(v)], lambda a: bool(a[0]))
    _choice[key] = got
    return got


def _pick_wgrad(key, C, x, dy, kh, kw, stride, pad, ref_fn):
    """Weight gradient: time the cost model's first ``TDL_WGRAD_CANDIDATES`` (default 6) tile/slice
    plans and MIOpen on the first eager call of a shape; returns the winning plan
    ``[wmw, wnw, nsplit, kind]`` or None (MIOpen).  TDL_CONV=hip: the cost model's first plan, cached under
    its own key -- a plan an earlier auto-mode call timed for the same shape (another split-K order)
    must not leak into a forced-hip run, nor the reverse."""
    m = mode()
    if m == "hip":
        key = ("hip",) + tuple(key)
    if key in _choice:
        return _choice[key]
    n = 1 if m == "hip" or torch.cuda.is_current_stream_capturing() else int(os.environ.get("TDL_WGRAD_CANDIDATES", 6))
    plans = [[p[0], p[1], p[3], p[4]] for p in C.conv_wgrad_plans(list(x.shape), list(dy.shape), kh, kw, stride[0],
                                                            stride[1], pad[0], pad[1], n)]
    if m == "hip":
        _choice[key] = plans[0]
        return plans[0]
    if torch.cuda.is_current_stream_capturing():
        _capture_fallback(key)
        return plans[0]

    def decide():
        t_ref = _time(ref_fn)
        best, t_best = None, float("inf")
        for p in plans:
            t = _time(lambda: C.conv_wgrad(x, dy, kh, kw, stride[0], stride[1], pad[0], pad[1], plan=p))
            if t < t_best:
                best, t_best = p, t
        _times[key] = (t_best, t_ref)
        return best if t_best < t_ref * _PREFER_HIP else None

    best = _agree(decide, lambda v: [1] + [int(u) for u in v] if v is not None else [0],
                  lambda a: [int(u) for u in a[1:]] if a[0] else None)
    _choice[key] = best
    return best


def choices() -> dict:
    """The autotuner's decisions so far: {(direction, shape key): 'hip' | 'miopen'} (forced-hip
    weight-gradient plans, cached under ("hip", ...) keys, are not decisions)."""
    return {k: ("hip" if (v is True or isinstance(v, list)) else "miopen") for k, v in _choice.items()
            if k[0] != "hip"}


def _ref_fwd(x, w_oihw, stride, pad):
    return F.conv2d(x.permute(0, 3, 1, 2), w_oihw, None, stride, pad).permute(0, 2, 3, 1)


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, kernel, stride, pad, grad_out, w_ohwi=None, box=None, stats_out=None, bn_src=None,
                bn_src2=None, anchor=None, bn_stats_src=None, bn_in=None):
        C = hip()
        x = x.contiguous()
        if x.data_ptr() % 16:
            x = x.clone()
        ctx.bn_in = bn_in
        kh, kw, cin, cout = kernel.shape
        sh, sw = stride
        ph, pw = pad
        oh, ow = (x.shape[1] + 2 * ph - kh) // sh + 1, (x.shape[2] + 2 * pw - kw) // sw + 1
        w_oihw = kernel.permute(3, 2, 0, 1)
        # with BN statistics in the epilogue the library path would also pay a read of y
        key = ("fwd", tuple(x.shape), tuple(kernel.shape), stride, pad, stats_out is not None)
        y_bytes = x.shape[0] * oh * ow * cout * x.element_size()
        if w_ohwi is None:
            w_ohwi = kernel.permute(3, 0, 1, 2).contiguous()
        hip_fn = lambda: C.conv_fwd(x, w_ohwi, oh, ow, sh, sw, ph, pw)  # noqa: E731
        if bn_in is not None:
            # x is a BN -> ReLU's input: the operand loader applies it (no library equivalent, no timing)
            if stats_out is not None:
                y, stats_out[0] = C.conv_fwd_stats(x, w_ohwi, oh, ow, sh, sw, ph, pw, in_bn=bn_in)
            else:
                y = C.conv_fwd(x, w_ohwi, oh, ow, sh, sw, ph, pw, in_bn=bn_in)
        elif _pick(key, hip_fn, lambda: _ref_fwd(x, w_oihw, stride, pad), y_bytes if stats_out is not None else 0):
            if stats_out is not None:  # + the following batch norm's partial channel sums
                y, stats_out[0] = C.conv_fwd_stats(x, w_ohwi, oh, ow, sh, sw, ph, pw)
            else:
                y = hip_fn()
        else:
            _lib("fwd", f"{mode()} mode chose MIOpen")
            y = _ref_fwd(x, w_oihw, stride, pad).contiguous()
        ctx.save_for_backward(x, kernel)
        ctx.geo = (stride, pad)
        ctx.grad_out = grad_out
        ctx.box = box
        ctx.bn_src = bn_src if (bn_src is not None and tuple(bn_src.shape) == tuple(x.shape)
                                and bn_src.dtype == x.dtype) else None
        ctx.bn_src2 = bn_src2 if (ctx.bn_src is not None and bn_src2 is not None
                                  and tuple(bn_src2.shape) == tuple(x.shape) and bn_src2.dtype == x.dtype) else None
        # a plain BN -> ReLU group's [4][C] statistics: the dgrad epilogue recomputes the mask from bn_src.
        # With bn_in (deferred BN -> ReLU) x IS the raw BN input, so a mask taken from x itself would be
        # [x > 0] instead of [x*scale + shift > 0]: the statistics are then mandatory, whatever the A/B switch.
        ctx.bn_stats_src = bn_stats_src if (ctx.bn_src is not None and ctx.bn_src2 is None
                                            and (_FUSE_BN_MASK_STATS[0] or bn_in is not None)
                                            and bn_stats_src is not None
                                            and bn_stats_src.numel() == 4 * x.shape[-1]) else None
        if bn_in is not None and ctx.bn_src is not None and ctx.bn_stats_src is None:
            # no statistics to rebuild the mask from: skip the fused BN epilogue (plain dgrad + BN backward)
            ctx.bn_src = None
        if box is not None:
            box.n += 1
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
        kh, kw = kernel.shape[0], kernel.shape[1]
        bn_in = ctx.bn_in
        gout = ctx.grad_out  # f32 HWIO slab view: dW is ADDED into it and not returned
        want_dx, want_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1] or gout is not None
        shape_key = (tuple(x.shape), tuple(kernel.shape), stride, pad)
        dx = dw = None

        def ref(mask):
            if bn_in is not None:  # the library reads the materialised relu(bn(x)) (weight gradient only)
                return lambda: _miopen_bwd(dy_nchw, _bn_relu_ref(x, bn_in).permute(0, 3, 1, 2) if mask[1] else x_nchw,
                                           w_oihw, list(stride), list(pad), mask)
            return lambda: _miopen_bwd(dy_nchw, x_nchw, w_oihw, list(stride), list(pad), mask)

        box = ctx.box if (ctx.box is not None and ctx.box.active and want_dx) else None
        other = None  # the other consumer's gradient contribution, added into dx
        first = False
        if box is not None:
            other, box.g = box.g, None
            first = other is None
            if other is not None:
                other = other.contiguous()
                if other.data_ptr() % 16:
                    other = other.clone()
        if want_dx:
            kc = kernel.contiguous()
            hip_fn = key = None
            if stride == (1, 1):
                hip_fn = lambda r=None: C.conv_dgrad(dy, kc, x.shape[1], x.shape[2], pad[0], pad[1], r)  # noqa: E731
                key = ("dgrad",) + shape_key
            elif stride == (2, 2) and (kh, kw) == (1, 1) and pad == (0, 0):
                hip_fn = lambda r=None: C.conv_dgrad_s2(dy, kc, x.shape[1], x.shape[2], r)  # noqa: E731
                key = ("dgrad_s2",) + shape_key
            # fused epilogues: a gradient sum saves an add pass (2 reads + 1 write of dx, one read back),
            # the BN group reduction a read of dz, x, y and a write of dz
            # the BN-group fusion needs the complete gradient of x: the second GradBox participant,
            # or the only reader of x (no box)
            fuse_bn = (ctx.bn_src is not None and (other is not None or ctx.box is None) and hip_fn is not None
                       and _FUSE_BN_BWD[0] and (stride == (1, 1) or _FUSE_BN_BWD_S2[0]))
            dx_bytes = x.numel() * x.element_size()
            saved = (2 * dx_bytes if other is not None else 0) + (2 * dx_bytes if fuse_bn else 0)
            key = (key + (other is not None, fuse_bn)) if hip_fn is not None else None
            if hip_fn is not None and _pick(key, hip_fn, lambda: ref([True, False, False])()[0], saved):
                src = ctx.bn_src
                if fuse_bn:
                    # full gradient of the BN (-> Add) -> ReLU group output x: mask it and reduce it for
                    # the group's BN backward in the same epilogue (ops/batchnorm.py uses the part);
                    # with bn_src2 also the reduction of the projection-shortcut BN feeding its Add
                    src, src2 = _aligned(src), ctx.bn_src2 if _FUSE_BN_BWD_SHORTCUT[0] else None
                    src2 = _aligned(src2) if src2 is not None else None
                    # plain BN -> ReLU group: no read of x for the mask (recomputed from src and the stats)
                    st = ctx.bn_stats_src
                    xm = x if st is None else None
                    if stride == (1, 1):
                        out = C.conv_dgrad_bn(dy, kc, x.shape[1], x.shape[2], pad[0], pad[1], other, xm, src, src2, st)
                    else:
                        out = C.conv_dgrad_s2_bn(dy, kc, x.shape[1], x.shape[2], other, xm, src, src2, st)
                    dx = out[0]
                    dx._tdl_bn_bwd_part = out[1]
                    if src2 is not None:
                        dx._tdl_bn_bwd_part2 = out[2]
                    if _DEBUG_PARTS:
                        _check_parts(dx, src, out[1], "part")
                        if src2 is not None:
                            _check_parts(dx, src2, out[2], "part2")
                else:
                    dx = hip_fn(other)
                other = None
        if want_dw and x.shape[0] * dy.shape[1] * dy.shape[2] < (1 << 24):
            if bn_in is not None:
                plan = _pick_wgrad_bn_in(("wgrad_bn_in",) + shape_key, C, x, dy, bn_in)
            else:
                plan = _pick_wgrad(("wgrad",) + shape_key, C, x, dy, kh, kw, stride, pad,
                                   lambda: ref([False, True, False])()[1])
            if plan is not None and bn_in is not None:
                if gout is not None:
                    C.conv_wgrad(x, dy, 1, 1, 1, 1, 0, 0, out=gout, accumulate=True, plan=plan, in_bn=bn_in)
                    want_dw = False
                else:
                    dw = C.conv_wgrad(x, dy, 1, 1, 1, 1, 0, 0, plan=plan, in_bn=bn_in)
            elif plan is not None:
                if gout is not None and _SIDE_STATE["open"] and x.is_cuda:
                    side = _side_stream(x.device)
                    side.wait_stream(torch.cuda.current_stream(x.device))
                    with torch.cuda.stream(side):
                        C.conv_wgrad(x, dy, kh, kw, stride[0], stride[1], pad[0], pad[1], out=gout, accumulate=True,
                                     plan=plan)
                    _SIDE_HELD.append((x, dy))
                    _SIDE_STATE["used"] = True
                    want_dw = False
                elif gout is not None:
                    C.conv_wgrad(x, dy, kh, kw, stride[0], stride[1], pad[0], pad[1], out=gout, accumulate=True,
                                 plan=plan)
                    want_dw = False
                else:
                    dw = C.conv_wgrad(x, dy, kh, kw, stride[0], stride[1], pad[0], pad[1], plan=plan)
        need_dx, need_dw = want_dx and dx is None, want_dw and dw is None
        if (need_dx or need_dw) and mode() == "hip":
            # no bf16 kernel for this direction / size (strided 3x3 input gradients, >= 2^24-row weight
            # gradients): the generic f32-MFMA kernels of ops/conv_f32.py, not the library
            from . import conv_f32 as _cf

            pads4 = (pad[0], pad[0], pad[1], pad[1])
            if need_dx:
                dx = _cf.dgrad(dy, kernel, (x.shape[1], x.shape[2]), stride, pads4).to(x.dtype)
            if need_dw:
                xs = _bn_relu_ref(x, bn_in) if bn_in is not None else x
                if gout is not None:
                    _cf.wgrad(xs, dy, (kh, kw), stride, pads4, out=gout, accumulate=True)
                else:
                    dw = _cf.wgrad(xs, dy, (kh, kw), stride, pads4).to(kernel.dtype)
            need_dx = need_dw = False
        if need_dx or need_dw:
            if need_dx:
                _lib("dgrad", f"stride {tuple(stride)} {kh}x{kw}" if hip_fn is None else f"{mode()} mode chose MIOpen")
            if need_dw:
                _lib("wgrad", f"{mode()} mode chose MIOpen" if x.shape[0] * dy.shape[1] * dy.shape[2] < (1 << 24)
                     else "reduction >= 2^24 rows")
            gx, gw, _ = ref([need_dx, need_dw, False])()
            if need_dx:
                dx = gx.permute(0, 2, 3, 1)
            if need_dw:  # library weight gradient: into the slab view, or returned
                dw = gw.permute(2, 3, 1, 0)
                if gout is not None:
                    gout.add_(dw)
                    dw = None
        if other is not None:  # library input gradient: one add
            dx = dx + other.view_as(dx)
        if first:  # park this contribution for the other consumer's backward
            box.g, dx = dx, None
        return dx, dw, None, None, None, None, None, None, None, None, None, None, None


def _bn_relu_ref(x, st):
    """relu(x * scale + shift) with the BN apply pass's f32 arithmetic (st: [4][C] statistics)."""
    return torch.relu(torch.addcmul(st[3], x.float(), st[2])).to(x.dtype)


def _pick_wgrad_bn_in(key, C, x, dy, st):
    """Weight gradient of a 1x1 conv over relu(bn(x)) (the input-side BN): the register-staged plans
    only, timed among themselves on the first eager call (MIOpen would need the applied tensor)."""
    if key in _choice:
        return _choice[key]
    n = 1 if mode() == "hip" or torch.cuda.is_current_stream_capturing() else int(os.environ.get("TDL_WGRAD_CANDIDATES", 6))
    plans = [[p[0], p[1], p[3], p[4]] for p in C.conv_wgrad_plans(list(x.shape), list(dy.shape), 1, 1, 1, 1, 0, 0, n,
                                                                    in_bn=True)]
    if len(plans) == 1:
        _choice[key] = plans[0]
        return plans[0]

    def decide():
        ts = [_time(lambda: C.conv_wgrad(x, dy, 1, 1, 1, 1, 0, 0, plan=p, in_bn=st)) for p in plans]
        i = min(range(len(plans)), key=ts.__getitem__)
        _times[key] = (ts[i], float("nan"))
        return plans[i]

    best = _agree(decide, lambda v: [1] + [int(u) for u in v], lambda a: [int(u) for u in a[1:]])
    _choice[key] = best
    return best


_DEBUG_PARTS = os.environ.get("TDL_DEBUG_BN_PARTS") == "1"


def _check_parts(dz, xb, part, what):
    """TDL_DEBUG_BN_PARTS=1: an epilogue's BN sums vs PyTorch over the tensors (stderr)."""
    import sys

    C = dz.shape[-1]
    P = part.shape[0]
    while P > 1 and (P - 1) + (P - 1 + 63) // 64 >= part.shape[0]:
        P -= 1
    got = part[:P].double().sum(0)
    d, x = dz.double().reshape(-1, C), xb.double().reshape(-1, C)
    ref = torch.stack([d.sum(0), (d * x).sum(0)])
    err = ((got - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
    print(f"[tdl parts] {what} {tuple(dz.shape)} rows {P}/{part.shape[0]} rel err {err:.3g}", file=sys.stderr, flush=True)


def _aligned(t):
    t = t.contiguous()
    return t.clone() if t.data_ptr() % 16 else t


def _miopen_bwd(dy_nchw, x_nchw, w_oihw, stride, pad, mask):
    """MIOpen convolution backward (input / weight gradients as selected by ``mask``)."""
    return torch.ops.aten.convolution_backward(dy_nchw, x_nchw, w_oihw, None, stride, pad, [1, 1], False, [0, 0], 1,
                                               mask)


def conv2d_nhwc(x, kernel_hwio, stride=(1, 1), pad=(0, 0), grad_out=None, w_ohwi=None, grad_box=None,
                bn_stats=False, bn_src=None, bn_src2=None, anchor=None, bn_stats_src=None, bn_in=None):
    """y[N,OH,OW,K] = conv(x[N,H,W,C], kernel[KH,KW,C,K]) with symmetric zero padding ``pad = (ph, pw)``,
    bf16; the caller checked :func:`supported`.  ``grad_out``: f32 [KH,KW,C,K] tensor the weight
    gradient is added into (a trainer's gradient slab view; ``kernel_hwio`` then needs no autograd);
    ``w_ohwi``: the same kernel already in OHWI [K,KH,KW,C] layout (skips the per-call transpose);
    ``grad_box``: a :class:`GradBox` shared with the other consumer of ``x``; ``bn_stats``: the
    hand-written forward also writes the batch-norm partial channel sums of y, attached as
    ``y._tdl_bn_part`` for the BN that consumes it (ops/batchnorm.py skips its statistics pass);
    ``bn_src``: x is the output relu(bn(bn_src) + r) of a fused BN group; when this conv's input
    gradient is the complete gradient of x (second GradBox participant), its epilogue also applies
    the group's ReLU mask and reduces the group's BN backward sums; ``bn_src2``: the input of the
    plain (projection-shortcut) BN whose output is that group's residual: the same epilogue reduces
    its backward sums too.  ``anchor``: with ``grad_out``, the variable's leaf tensor, so that the
    backward runs although neither the input (the first layer's batch) nor the detached compute-dtype
    kernel needs a gradient (the kernel's gradient goes into ``grad_out``; the anchor gets none).
    ``bn_stats_src``: with ``bn_src`` of a plain BN -> ReLU group, that BN's [4][C] batch statistics: the
    epilogue recomputes the ReLU mask from ``bn_src`` instead of reading x.
    ``bn_in``: x is the INPUT of a plain BN -> ReLU group and ``bn_in`` its [4][C] statistics (1x1 stride-1
    unpadded convs): the forward and weight-gradient operand loaders apply relu(x * scale + shift), so
    the group output is never written (keras/fusion.py ``defer``); pass ``bn_src=x, bn_stats_src=bn_in``
    for the fused input-gradient epilogue."""
    if bn_in is not None and not (tuple(kernel_hwio.shape[:2]) == (1, 1) and tuple(stride) == (1, 1)
                                  and tuple(pad) == (0, 0) and bn_in.numel() == 4 * x.shape[-1] and x.shape[-1] <= 512):
        raise ValueError("conv2d_nhwc: bn_in takes 1x1 stride-1 unpadded convolutions of <= 512 input channels "
                         "and [4][C] statistics")
    holder = [None] if bn_stats else None
    y = _Conv.apply(x, kernel_hwio, tuple(stride), tuple(pad), grad_out, w_ohwi, grad_box, holder, bn_src, bn_src2,
                    anchor, bn_stats_src, bn_in)
    if holder is not None and holder[0] is not None:
        y._tdl_bn_part = holder[0]
    return y


def stem_supported(x: torch.Tensor, kernel_hwio: torch.Tensor, strides, groups=1, dilation=(1, 1)) -> bool:
    """The small-channel stride-2 kernel (csrc/kernels/stem.hip): the ResNet stem, 3 -> 64 channels."""
    kh, kw, cin, cout = kernel_hwio.shape
    return (x.is_cuda and x.dtype in (torch.bfloat16, torch.float32) and x.dim() == 4 and groups == 1
            and tuple(dilation) == (1, 1) and x.shape[-1] == cin and 1 <= cin <= 4 and 1 <= kh <= 8 and 1 <= kw <= 8
            and int(strides[1]) == 2 and cout % 64 == 0 and mode() != "miopen")


class _Stem(torch.autograd.Function):
    """Small-channel stride-2 conv with its zero padding folded in (stem.hip): forward on the packed
    NHWC4 image (kept for the weight gradient), weight gradient on MFMA with transposed LDS reads."""

    @staticmethod
    def forward(ctx, x, kernel, pads, stride, grad_out, holder, anchor=None):
        C = hip()
        x = _aligned(x)
        kc = _aligned(kernel.to(torch.bfloat16))
        out = C.stem_fwd(x, kc, pads[0], pads[1], pads[2], pads[3], stride[0], stride[1], holder is not None)
        if holder is not None:
            holder[0] = out[2]
        ctx.save_for_backward(out[1], kernel, x if ctx.needs_input_grad[0] else None)
        ctx.geo = (pads, stride)
        ctx.grad_out = grad_out
        return out[0]

    @staticmethod
    def backward(ctx, dy):
        C = hip()
        xp, kernel, x = ctx.saved_tensors
        pads, stride = ctx.geo
        dy = _aligned(dy.to(torch.bfloat16))
        kh, kw, cin, _ = kernel.shape
        dw = dx = None
        if ctx.grad_out is not None:  # f32 slab view: dW added straight into it
            C.stem_wgrad(xp, dy, kh, kw, cin, stride[0], out=ctx.grad_out, accumulate=True)
        elif ctx.needs_input_grad[1]:
            dw = C.stem_wgrad(xp, dy, kh, kw, cin, stride[0]).to(kernel.dtype)
        if ctx.needs_input_grad[0]:  # image gradient (not needed for training): the generic f32 kernel
            from . import conv_f32 as _cf

            dx = _cf.dgrad(dy, kernel, (x.shape[1], x.shape[2]), stride, pads).to(x.dtype)
        return dx, dw, None, None, None, None, None


def stem_conv2d_nhwc(x, kernel_hwio, pads, stride, grad_out=None, bn_stats=False, anchor=None):
    """y = conv(zero_pad(x, pads = (top, bottom, left, right)), kernel_hwio) for a <= 4-channel image,
    column stride 2 (:func:`stem_supported`); ``grad_out`` / ``bn_stats`` as for :func:`conv2d_nhwc`.
    ``anchor``: with ``grad_out``, the variable's leaf tensor, so that the backward runs although
    neither the image nor the detached compute-dtype kernel needs a gradient (its gradient goes
    into ``grad_out``; the anchor itself gets none)."""
    holder = [None] if bn_stats else None
    y = _Stem.apply(x, kernel_hwio, tuple(int(p) for p in pads), tuple(int(s) for s in stride), grad_out, holder,
                    anchor)
    if holder is not None and holder[0] is not None:
        y._tdl_bn_part = holder[0]
    return y
