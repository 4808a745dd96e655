"""Graph-level fusion for training-mode functional models on the GPU.

The functional executor (models.Model._run_graph) asks :func:`plan` for a fusion plan of its node
list; the plan rewrites, at execution time only (the layer graph, variables, checkpoints and
``model.summary()`` are untouched):

* ``Conv2D(use_bias, linear) -> BatchNormalization``: the conv runs without its bias; the bias is
  folded into the BN (only the moving mean sees it; its gradient is exactly zero in training mode),
  and the hand-written conv forward's epilogue computes the BN's batch statistics (per-tile
  channel sums of its bf16 output), so the BN skips its statistics pass over the tensor.
* ``BatchNormalization -> ReLU``: one fused kernel pass (ops/batchnorm.py); when a Conv2D is the
  only reader of the output, that conv's input-gradient epilogue applies the ReLU mask and reduces
  the BN backward sums (the BN backward then skips its reduction pass over the tensor).
* ``BatchNormalization -> Add(other) -> ReLU``: the ResNet block tail, one fused pass that also
  produces the residual's gradient.
* ``ZeroPadding2D -> MaxPooling2D('valid')``: one pooling pass with implicit zero padding.
* ``BatchNormalization -> ReLU -> Conv2D(1x1, stride 1)`` where the conv is the only reader (the ResNet
  bottleneck's last conv): the BN computes its statistics only and the conv's forward and weight-gradient
  operand loaders apply relu(x * scale + shift) to the BN input; the normalised tensor is never written.
* ``BatchNormalization -> ReLU -> [ZeroPadding2D ->] MaxPooling2D('valid')`` (the ResNet stem): the pool
  runs on the BN input with the normalisation in its kernel and reduces the BN backward sums in its
  backward pass; the normalised tensor is never written.
* ``ZeroPadding2D -> Conv2D`` with <= 4 input channels, 'valid', column stride 2 (the ResNet stem):
  the padding goes into the stem kernel's packed image (ops/conv.py ``stem_conv2d_nhwc``).
* a tensor read by a Conv2D and by one other node (the ResNet block input: the shortcut / the
  residual of the block tail, and the first 1x1 conv): the two backward contributions meet in a
  ``GradBox`` (ops/conv.py) and the conv's input-gradient kernel adds the other one in its
  epilogue, instead of autograd's separate add pass over the tensor.

Every intermediate tensor of a fused group must have exactly one consumer.  A group executes at
the position of its last node, when all its external inputs exist.  Eval / CPU calls run the
original node by node.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

from . import activations as A
from . import layers as L


class Group:
    __slots__ = ("bn_node", "relu", "residual", "conv_layer", "out", "last", "conv_reader", "add_node", "res_bn",
                 "pool", "defer")

    def __init__(self, bn_node, relu, residual, conv_layer, out, last, conv_reader=False, add_node=None):
        self.bn_node, self.relu, self.residual, self.conv_layer, self.out, self.last = (
            bn_node, relu, residual, conv_layer, out, last)
        # BN -> ReLU whose output is read by exactly one Conv2D: that conv's input gradient is the
        # group's whole output gradient, so its epilogue can run the group's backward reduction
        self.conv_reader = conv_reader
        self.add_node = add_node  # the absorbed Add of a BN -> Add -> ReLU group
        # the plain BN group (a projection shortcut's BN) whose output is this group's residual and
        # is read by nothing else: its output gradient is this group's dz, so the conv epilogue that
        # reduces this group's backward sums can reduce that BN's as well
        self.res_bn = None
        # (MaxPooling2D layer, pads, pad_zero): a BN -> ReLU -> [ZeroPadding2D ->] MaxPooling2D chain whose
        # pool is the group output's only reader -- the pool runs on the BN input with the normalisation
        # in its kernel (ops/pooling.py bn_relu_max_pool) and the normalised tensor is never written
        self.pool = None
        # the reading 1x1 stride-1 Conv2D layer of a BN -> ReLU group whose apply it takes over (the
        # group output is never materialised; decided again at run time: GPU, bf16, kernel shapes)
        self.defer = None


class Plan:
    def __init__(self):
        self.skip = set()        # node ids absorbed into a group that runs elsewhere
        self.conv_nobias = set()  # conv node ids whose bias is folded into their BN
        self.groups: Dict[int, Group] = {}  # id(last node) -> group
        self.pool_pad: Dict[int, tuple] = {}  # id(max-pool / stem conv node) -> (padding input, padding)
        self.conv_box: Dict[int, int] = {}   # id(conv node) -> id(input tensor) of its GradBox
        self.taps: Dict[int, set] = {}       # id(node or group last node) -> ids of inputs read through a tap
        self.conv_pool: Dict[int, object] = {}  # id(conv node) -> the 2x2 MaxPooling2D node it runs (Conv2D._pool)

    def __len__(self):
        return len(self.groups)


def _is_plain_relu(layer) -> bool:
    if isinstance(layer, L.Activation):
        return layer.activation is A.relu
    if isinstance(layer, L.ReLU):
        return layer.max_value is None and layer.negative_slope == 0 and layer.threshold == 0
    return False


def _single_tensor(x):
    return x if isinstance(x, L.KerasTensor) else None


def plan(nodes: List[L.Node], outputs) -> Plan:
    p = Plan()
    if os.environ.get("TDL_FUSE", "1") != "1":
        return p
    consumers: Dict[int, List[L.Node]] = {}
    for n in nodes:
        for t in L._flat(n.inputs):
            consumers.setdefault(id(t), []).append(n)
    outs = {id(t) for t in L._flat(outputs)}

    def only_consumer(t) -> Optional[L.Node]:
        if t is None or id(t) in outs:
            return None
        c = consumers.get(id(t), [])
        return c[0] if len(c) == 1 else None

    producer = {id(t): n for n in nodes for t in L._flat(n.outputs)}
    for n in nodes:  # ZeroPadding2D -> MaxPooling2D('valid'): one pooling pass with zero padding
        if isinstance(n.layer, L.MaxPooling2D) and n.layer.padding == "valid":
            x_t = _single_tensor(n.inputs)
            prod = producer.get(id(x_t)) if x_t is not None else None
            if prod is not None and isinstance(prod.layer, L.ZeroPadding2D) and only_consumer(x_t) is n:
                p.pool_pad[id(n)] = (prod.inputs, prod.layer.padding)
                p.skip.add(id(prod))
    for n in nodes:  # ZeroPadding2D -> small-channel stride-2 'valid' Conv2D (the stem): padding folded in
        if isinstance(n.layer, L.Conv2D) and n.layer.padding == "valid" and n.layer.strides[1] == 2 and \
                n.layer.groups == 1 and tuple(n.layer.dilation_rate) == (1, 1) and max(n.layer.kernel_size) <= 8:
            x_t = _single_tensor(n.inputs)
            prod = producer.get(id(x_t)) if x_t is not None else None
            if prod is not None and isinstance(prod.layer, L.ZeroPadding2D) and only_consumer(x_t) is n and \
                    x_t.shape[-1] is not None and int(x_t.shape[-1]) <= 4:
                p.pool_pad[id(n)] = (prod.inputs, prod.layer.padding)
                p.skip.add(id(prod))
    for n in nodes:
        bn = n.layer
        if not (isinstance(bn, L.BatchNormalization) and bn.trainable and bn.axis in (-1, 3)):
            continue
        x_t = _single_tensor(n.inputs)
        out_t = _single_tensor(n.outputs)
        if x_t is None or out_t is None or len(x_t.shape) != 4:
            continue
        conv_layer = None
        prod = producer.get(id(x_t))
        if prod is not None and isinstance(prod.layer, L.Conv2D) and prod.layer.use_bias and \
                prod.layer.activation is A.linear and prod.layer.trainable and only_consumer(x_t) is n:
            conv_layer = prod.layer
            p.conv_nobias.add(id(prod))
        relu, residual, last, out, add_node = False, None, n, out_t, None
        c1 = only_consumer(out_t)
        if c1 is not None and _is_plain_relu(c1.layer):
            relu, last, out = True, c1, _single_tensor(c1.outputs)
        elif c1 is not None and isinstance(c1.layer, L.Add) and isinstance(c1.inputs, (list, tuple)) and \
                len(c1.inputs) == 2 and id(c1) not in p.skip:  # (a projection shortcut's BN may own it)
            add_out = _single_tensor(c1.outputs)
            c2 = only_consumer(add_out)
            other = c1.inputs[1] if c1.inputs[0] is out_t else c1.inputs[0]
            if c2 is not None and _is_plain_relu(c2.layer) and other is not out_t and \
                    tuple(other.shape) == tuple(out_t.shape):
                relu, residual, last, out, add_node = True, other, c2, _single_tensor(c2.outputs), c1
                p.skip.add(id(c1))
        if last is not n:
            p.skip.add(id(n))
        reader = only_consumer(out) if relu and residual is None else None
        conv_reader = reader is not None and isinstance(reader.layer, L.Conv2D) and reader.inputs is out
        p.groups[id(last)] = Group(n, relu, residual, conv_layer, out, last, conv_reader, add_node)
    by_out = {id(g.out): g for g in p.groups.values()}
    for g in p.groups.values():
        pg = by_out.get(id(g.residual)) if g.residual is not None else None
        if pg is not None and not pg.relu and pg.residual is None and pg.last is pg.bn_node and \
                only_consumer(g.residual) is g.add_node:
            g.res_bn = pg
    if os.environ.get("TDL_FUSE_BN_POOL", "1") == "1":
        _plan_bn_pool(p, only_consumer)
    if os.environ.get("TDL_FUSE_BN_INPUT", "1") == "1":
        for g in p.groups.values():
            if g.relu and g.residual is None and g.conv_reader and g.pool is None:
                c = only_consumer(g.out).layer
                if tuple(c.kernel_size) == (1, 1) and tuple(c.strides) == (1, 1) and \
                        tuple(c.dilation_rate) == (1, 1) and c.groups == 1 and c.filters % 64 == 0:
                    g.defer = c
    if os.environ.get("TDL_FUSE_GRAD_SUM", "1") == "1":
        _plan_grad_sums(p, nodes, consumers, outs)
    # Conv2D -> MaxPooling2D(2, 2, 'valid') whose conv output has no other reader and which no other plan
    # touches: the pool runs inside the conv's call (one launch on the generic f32 path, Conv2D._pool)
    in_groups = {id(g.bn_node) for g in p.groups.values()} | {id(g.last) for g in p.groups.values()}
    for n in nodes:
        if id(n) in p.skip or id(n) in p.conv_nobias or id(n) in p.conv_box or id(n) in p.pool_pad or \
                id(n) in p.taps or id(n) in in_groups:
            continue
        out_t = _single_tensor(n.outputs)
        c = only_consumer(out_t) if out_t is not None and isinstance(n.layer, L.Conv2D) else None
        if c is None or not L.conv_pool_pair(n.layer, c.layer) or c.inputs is not out_t or id(c) in p.skip or \
                id(c) in p.pool_pad or id(c) in p.taps or id(c) in in_groups:
            continue
        p.conv_pool[id(n)] = c
        p.skip.add(id(c))
    return p


def _plan_bn_pool(p: Plan, only_consumer):
    """BN -> ReLU groups whose output's only reader is a 'valid' MaxPooling2D, directly or through a
    ZeroPadding2D already folded into it (the ResNet stem): the pool joins the group."""
    for key, g in list(p.groups.items()):
        if not g.relu or g.residual is not None or g.conv_reader:
            continue
        c = only_consumer(g.out)
        pool_n, pads, pad_zero = None, ((0, 0), (0, 0)), False
        if c is not None and isinstance(c.layer, L.ZeroPadding2D):
            c2 = only_consumer(_single_tensor(c.outputs))
            pp = p.pool_pad.get(id(c2)) if c2 is not None else None
            if pp is not None and isinstance(c2.layer, L.MaxPooling2D) and pp[0] is g.out:
                pool_n, pads, pad_zero = c2, pp[1], True
        elif c is not None and isinstance(c.layer, L.MaxPooling2D) and c.layer.padding == "valid" and c.inputs is g.out:
            pool_n = c
        if pool_n is None or _single_tensor(pool_n.outputs) is None:
            continue
        p.pool_pad.pop(id(pool_n), None)
        if g.last is not g.bn_node:
            p.skip.add(id(g.last))
        del p.groups[key]
        g.pool = (pool_n.layer, pads, pad_zero)
        g.last, g.out = pool_n, _single_tensor(pool_n.outputs)
        p.groups[id(pool_n)] = g


def _plan_grad_sums(p: Plan, nodes, consumers, outs):
    """Tensors with exactly two consumers, at least one a Conv2D reading it as its only input."""
    owner = {}  # id(node absorbed in a group) -> id(group's last node)
    for last_id, g in p.groups.items():
        if g.residual is not None:
            for c in consumers.get(id(g.residual), []):
                if isinstance(c.layer, L.Add) and id(c) in p.skip:
                    owner[id(c)] = last_id

    def is_conv_reader(c, t):
        return isinstance(c.layer, L.Conv2D) and c.inputs is t and id(c) not in p.skip

    seen = set()
    for n in nodes:
        for t in L._flat(n.inputs):
            tid = id(t)
            if tid in seen or tid in outs:
                continue
            seen.add(tid)
            cs = consumers.get(tid, [])
            if len(cs) != 2 or cs[0] is cs[1] or not any(is_conv_reader(c, t) for c in cs):
                continue
            for c in cs:
                if is_conv_reader(c, t):
                    p.conv_box[id(c)] = tid
                elif id(c) in owner:  # the residual of a fused BN -> Add -> ReLU group
                    p.taps.setdefault(owner[id(c)], set()).add(tid)
                elif id(c) not in p.skip:
                    p.taps.setdefault(id(c), set()).add(tid)
                else:  # absorbed elsewhere: leave this tensor to autograd
                    p.conv_box = {k: v for k, v in p.conv_box.items() if v != tid}
                    for v in p.taps.values():
                        v.discard(tid)
                    break


_DEFER_MIN_PIXELS = int(os.environ.get("TDL_FUSE_BN_INPUT_MIN_PIXELS", 131072))


def _defer_ok(x) -> bool:
    """The hand-written 1x1 kernels take this BN input (what Conv2D.call's kernel path requires), and
    the tensor is large enough for the saved apply pass to outweigh the loaders' extra work: per
    ResNet-50 bottleneck shape (scripts/bench_bn_in.py, profiles/bn_input_side_r4.txt) the fused
    forward + weight gradient beat apply + plain kernels at 56x56 and 28x28 (b=256) and lost at
    14x14 and 7x7, where the weight gradient also gives up the single-stage LDS-DMA plans."""
    import torch

    from ..ops import conv as _conv

    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[-1] % 64 == 0
            and x.shape[-1] <= 512 and x.numel() < (1 << 30) and _conv.mode() != "miopen"
            and x.shape[0] * x.shape[1] * x.shape[2] >= _DEFER_MIN_PIXELS)


def run_group(g: Group, vals, training, taps=None, boxes=None):
    from ..ops.batchnorm import batch_norm_train

    bn = g.bn_node.layer
    x = vals[id(g.bn_node.inputs)]
    r = vals[id(g.residual)] if g.residual is not None else None
    if r is not None and taps and id(g.residual) in taps:
        from ..ops.conv import GradBox, grad_tap

        r = grad_tap(r, boxes.setdefault(id(g.residual), GradBox()))
    cb = None
    if g.conv_layer is not None:
        cbv = g.conv_layer.bias
        # the folded bias's gradient is exactly zero: with a gradient slab bound, leave its (zeroed)
        # slab entries alone instead of accumulating zeros
        cb = cbv.value.detach() if cbv.grad_target() is not None else cbv.value
    if g.pool is not None:
        from ..ops import pooling as _pool

        pool_layer, pads, pad_zero = g.pool
        if training and _pool.bn_pool_supported(x):
            y = _pool.bn_relu_max_pool(x, bn.gamma.value if bn.gamma is not None else None,
                                       bn.beta.value if bn.beta is not None else None, bn.moving_mean.value,
                                       bn.moving_variance.value, bn.momentum, bn.epsilon, pool_layer.pool_size,
                                       pool_layer.strides, pads, pad_zero, conv_bias=cb,
                                       grad_out=bn._grad_targets(), part=getattr(x, "_tdl_bn_part", None))
        else:
            y = batch_norm_train(x, bn.gamma.value if bn.gamma is not None else None,
                                 bn.beta.value if bn.beta is not None else None, bn.moving_mean.value,
                                 bn.moving_variance.value, bn.momentum, bn.epsilon, relu=True, conv_bias=cb,
                                 grad_out=bn._grad_targets(), part=getattr(x, "_tdl_bn_part", None))
            y = pool_layer(y, training=training, **({"_zero_pad": pads} if pad_zero else {}))
        vals[id(g.out)] = y
        return
    st = [] if (g.relu and r is None) else None
    defer = g.defer is not None and training and _defer_ok(x)
    y = batch_norm_train(x, bn.gamma.value if bn.gamma is not None else None,
                         bn.beta.value if bn.beta is not None else None, bn.moving_mean.value,
                         bn.moving_variance.value, bn.momentum, bn.epsilon, relu=g.relu, residual=r, conv_bias=cb,
                         grad_out=bn._grad_targets(), part=getattr(x, "_tdl_bn_part", None), stats_out=st,
                         defer_apply=defer)
    if defer:  # y is a stand-in: the reading 1x1 conv applies relu(bn(x)) in its operand loaders
        y._tdl_bn_in = st[0]
    if g.relu and (r is not None or g.conv_reader) and y.is_cuda:
        # a conv reading this group's output can fuse the group's backward reduction into its
        # input-gradient epilogue (ops/conv.py): it needs the BN input, and for a plain BN -> ReLU
        # group the batch statistics, from which the epilogue recomputes the ReLU mask (no read of y)
        y._tdl_bn_src = x
        if st:
            y._tdl_bn_stats = st[0]
        if g.res_bn is not None:
            y._tdl_bn_src2 = vals[id(g.res_bn.bn_node.inputs)]
    vals[id(g.out)] = y
