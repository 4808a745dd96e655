"""The MI355X fast path of ``fit`` for the reference model (tf_dist_example.py:39-59).

``compile()`` + ``fit()`` on the reference's Sequential (Conv2D(32,3,relu) MaxPool Conv2D(64,3,relu)
MaxPool Flatten Dense(128,relu) Dense(10); SparseCategoricalCrossentropy(from_logits) ; SGD ;
SparseCategoricalAccuracy) on a GPU replica is compiled into:

* the model's flat parameter/gradient slabs (the same storage its MirroredVariables view);
* a device-resident dataset (data/device.py) with per-step index vectors;
* :class:`~..models.mnist_cnn.FusedMnistTrainStep` (hand-written gfx950 kernels);
* the cross-replica gradient all-reduce (``world > 1``): on one node the xGMI all-reduce kernel
  with the SGD update fused into it, one 900 KB message per step; RCCL otherwise, followed by the
  SGD kernel;
* ONE hipGraph per execution of ``steps_per_execution`` steps, replayed with a new index vector,
  the all-reduce captured inside it on the step's stream (serial; the side-stream overlap of a
  dense bucket with the conv backward is opt-in, TDL_OVERLAP_ALLREDUCE=1, and measured slower:
  profiles/mnist_side_stream_ab_r2.txt).

Host work per execution: one H2D copy of K*B int32 indices and one graph launch.  Metrics (loss
sum, correct count, sample count) are accumulated by the loss kernel on the device and reduced
across replicas only when logs are read.
"""
from __future__ import annotations

import gc
import os
import queue
import threading
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..data import device as DD
from ..models import mnist_cnn as M
from ..parallel import input_lib


def _is_reference_cnn(model) -> bool:
    from ..keras import activations as A
    from ..keras import layers as L
    from ..keras.models import Sequential

    if not isinstance(model, Sequential):
        return False
    ls = [l for l in model.layers if not isinstance(l, L.InputLayer)]
    pat = [L.Conv2D, L.MaxPooling2D, L.Conv2D, L.MaxPooling2D, L.Flatten, L.Dense, L.Dense]
    if len(ls) != len(pat) or any(type(l) is not p for l, p in zip(ls, pat)):
        return False
    c1, p1, c2, p2, _, d1, d2 = ls
    for c, f in ((c1, 32), (c2, 64)):
        if not (c.filters == f and c.kernel_size == (3, 3) and c.strides == (1, 1) and c.padding == "valid" and
                c.dilation_rate == (1, 1) and c.groups == 1 and c.use_bias and c.activation is A.relu):
            return False
    for p in (p1, p2):
        if not (p.pool_size == (2, 2) and p.strides == (2, 2) and p.padding == "valid"):
            return False
    if not (d1.units == 128 and d1.use_bias and d1.activation is A.relu):
        return False
    if not (d2.units == 10 and d2.use_bias and d2.activation is A.linear):
        return False
    if tuple(model._built_input_shape[1:]) != (28, 28, 1):
        return False
    if any(getattr(l, "kernel_regularizer", None) or getattr(l, "bias_regularizer", None) for l in ls):
        return False
    return all(l.trainable for l in ls)


def eligible(model, dataset=None) -> Optional[str]:
    """None if the fused path applies, else the reason it does not."""
    from .. import ops
    from ..keras import losses, metrics, optimizers

    if os.environ.get("TDL_DISABLE_FUSED") == "1":
        return "disabled by TDL_DISABLE_FUSED"
    s = model._get_strategy()
    if s.extended.device.type != "cuda":
        return "replica is not on a GPU"
    if not ops.hip_available():
        ops.hip()  # GPU replica without the HIP kernels: fail loudly
    if not _is_reference_cnn(model):
        return "model is not the reference CNN"
    if model._dtype_policy() != "float32":
        return "non-f32 dtype policy"
    lo = model.loss
    if not (isinstance(lo, losses.SparseCategoricalCrossentropy) and lo.from_logits and lo.ignore_class is None and
            lo.reduction in (losses.Reduction.AUTO, losses.Reduction.SUM_OVER_BATCH_SIZE)):
        return "loss is not SparseCategoricalCrossentropy(from_logits=True)"
    opt = model.optimizer
    if type(opt) not in (optimizers.SGD, optimizers.Adam, optimizers.AdamW, optimizers.RMSprop, optimizers.Adagrad):
        return f"optimizer {type(opt).__name__} has no fused update"
    if opt.clipnorm or opt.clipvalue or opt.global_clipnorm:
        return "gradient clipping (a global norm) is not fused"
    if opt.weight_decay and not isinstance(opt, optimizers.Adam):
        return "decoupled weight decay is fused for Adam/AdamW only"
    kern = {"Adam": "adam", "AdamW": "adam", "RMSprop": "rmsprop", "Adagrad": "adagrad"}.get(type(opt).__name__)
    if kern is not None and not hasattr(ops.hip(), kern):
        return f"the extension has no {kern} kernel (rebuild: python build_native.py)"
    for m in model.compiled_metrics:
        if not isinstance(m, metrics.SparseCategoricalAccuracy):
            return f"metric {m.name} not supported by the fused step"
    return None


def overlap_enabled() -> bool:
    """TDL_OVERLAP_ALLREDUCE=1: R > 1 steps all-reduce the dense bucket on a side stream while the
    conv backward runs (a forked execution graph); default serial."""
    return os.environ.get("TDL_OVERLAP_ALLREDUCE", "0") == "1"



def _source_key(x, y):
    """Identity of a host data source: the tensors themselves (strong references, so a freed
    tensor's id can never be reused for a different dataset) plus their in-place version counters."""
    return (x, y, x._version, None if y is None else y._version)


def _same_source(a, b) -> bool:
    return a is not None and b is not None and a[0] is b[0] and a[1] is b[1] and a[2:] == b[2:]


class FusedMnistTrainer:
    kind = "fused"

    def __init__(self, model):
        self.model = model
        self.strategy = model._get_strategy()
        self.device = self.strategy.extended.device
        self.comm = self.strategy.extended.communicator
        self.R = self.strategy.num_replicas_in_sync
        self.rank = self.strategy.extended.rank
        model._ensure_slabs()
        self.layout = model._layout
        self.W, self.G = model._W, model._G
        for v in model._trainable_vars:
            v._leaf = None
        self.optimizer = model.optimizer
        self.optimizer.build(self.W.numel(), self.device)
        self.K = max(1, int(model._steps_per_execution))
        self.metrics_dev = torch.zeros(4, dtype=torch.float32, device=self.device)
        self._steps = {}
        self._graphs = {}
        self._data_key = None
        # (no capture for the replica threads of a single-process MirroredStrategy: their
        # collectives are host rendezvous, and concurrent captures in threads of one process are not
        # safe with torch's process-global capture mode)
        self.capture = os.environ.get("TDL_GRAPH", "1") == "1" and not getattr(self.comm, "threaded", False)
        # With R > 1 the cross-replica all-reduce is recorded inside the execution graph (RCCL
        # supports hipGraph capture) unless TDL_CAPTURE_ALLREDUCE=0 or the collective capture probe
        # fails on some rank; then each step's graph is followed by an eager all-reduce + update.
        self._capture_comm = None
        self._comm_stream = None
        self.allreduce_mode = "local" if self.R == 1 else None
        self.fallbacks = []  # why a faster path was not taken (bench.py reports them)
        # R > 1: the dense bucket's all-reduce on a side stream overlapping the conv backward is
        # opt-in; serial is the default: on one MI355X (2 replica processes sharing it) the forked
        # execution graph ran 350 us/step against 68.6 serial (profiles/mnist_side_stream_ab_r2.txt)
        self.overlap = overlap_enabled()
        # index-upload slots (one captured graph each): the host may run this many executions ahead
        # of the GPU, which absorbs host hiccups such as an epoch's shuffle (~ms) without starving it
        self._nslots = max(2, int(os.environ.get("TDL_INDEX_SLOTS", "4")))
        self._ragged_bufs, self._ragged_stage, self._ragged_ev = {}, None, None
        # diagnostics: host seconds per execution (index take, upload, graph launch)
        self._host_times = [] if os.environ.get("TDL_HOST_TIMING") == "1" else None
        # one execution's indices taken and uploaded ahead of its launch (prefetch())
        self._ready = None

    @property
    def capture_comm(self) -> bool:
        if self._capture_comm is None:
            if self.R == 1:
                self._capture_comm = True
            elif os.environ.get("TDL_CAPTURE_ALLREDUCE", "1") != "1" or not self.capture:
                self._capture_comm = False
            else:
                self._capture_comm = bool(self.comm.capture_probe())
                if not self._capture_comm:
                    self.fallbacks.append("all-reduce not capturable into the execution graph (probe failed)")
        return self._capture_comm

    # ------------------------------------------------------------------ data
    def prepare(self, dataset):
        lp = DD.lower(dataset)
        if lp is None:
            return None
        x, y = (lp.columns if isinstance(lp.columns, (tuple, list)) else (None, None))[:2]
        if x is None or y is None or tuple(x.shape[1:]) not in ((28, 28, 1), (28, 28)) or \
                x.dtype != torch.float32 or y.dim() != 1:
            return None
        if lp.batch_size % self.R:
            raise ValueError(f"global batch {lp.batch_size} is not divisible by {self.R} replicas")
        key = _source_key(x, y)
        if not _same_source(self._data_key, key):
            self.X = x.reshape(len(x), 28, 28, 1).to(self.device, torch.float32).contiguous()
            self.Y = y.to(self.device, torch.int32).contiguous()
            self._data_key = key
            self._steps, self._graphs = {}, {}
        policy = input_lib.effective_policy(dataset) if self.R > 1 else None
        seed = input_lib.shared_seed(self.strategy) if policy is not None and policy.name in ("DATA", "FILE") else None
        h = DeviceHandler(lp, seed, self.rank, self.R)
        self._handlers_b = [h.b]
        return h

    # ------------------------------------------------------------------ steps
    def _step(self, b: int, idx_buf: torch.Tensor, global_b: Optional[int] = None):
        key = (b, idx_buf.data_ptr(), global_b)
        st = self._steps.get(key)
        if st is None:
            st = M.FusedMnistTrainStep(self.X, self.Y, idx_buf, self.W, self.G, self.layout, b, self.R,
                                       self.optimizer.lr_dev, self.metrics_dev, global_batch=global_b)
            self._steps[key] = st
        return st

    def _apply(self, st, global_b: int, k: int = 0):
        """finalize + (all-reduce) + optimizer for one step (step ``k`` of its execution).  R > 1
        with plain SGD: one all-reduce of the whole 900 KB slab with the SGD update fused into it
        (xGMI kernel), when the communicator has one.  Other optimizers: finalize leaves the
        gradient in G, their flat-slab kernel (csrc/kernels/optim.hip) applies it."""
        opt = self.optimizer
        self._step_k = k
        plain = getattr(opt, "momentum", None) == 0 and type(opt).__name__ == "SGD"
        if self.R == 1 and plain:
            st.finalize(True, keep_grad=False)  # (nothing reads G on this path)
            return
        if self.R > 1 and plain and st.has_exchange:
            # fused backward: the finalize launch itself all-reduces over xGMI and applies SGD
            st.finalize(True, exchange=True, keep_grad=False)  # (G is not read on this path)
            return
        st.finalize(False)
        if self.R > 1 and plain and self.comm.all_reduce_sgd(self.G, self.W, opt.lr_dev):
            return
        self._reduce_and_update()

    def _train_step(self, st, off: int, global_b: int):
        """One whole step on the current stream.  R > 1 default (serial): forward + backward,
        finalize, then ONE all-reduce of the 900 KB gradient slab with the SGD update fused into it
        (_apply).  With TDL_OVERLAP_ALLREDUCE=1 the gradient all-reduce instead runs as two
        buckets: the dense-layer bucket (G[dense_offset:], 91% of the bytes) is final after
        forward_dense() and reduces on a side stream while the conv backward runs; the conv bucket
        follows finalize().  With the xGMI one-shot communicator each bucket's all-reduce also
        applies plain SGD to its own parameter range (W[dense_offset:] is not read again in the
        step), so no separate optimizer kernel runs; otherwise the optimizer waits for both."""
        if self.R == 1 or not self.overlap or not self._plain_sgd:
            st.forward_backward(off)
            self._apply(st, global_b, off // max(1, st.b))
            return
        main = torch.cuda.current_stream(self.device)
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(self.device)
        cs = self._comm_stream
        d0 = st.dense_offset
        G, W = self.G, self.W
        fuse = self.optimizer.momentum == 0
        lr = self.optimizer.lr_dev
        st.forward_dense(off)
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            dense_fused = fuse and self.comm.all_reduce_sgd(G[d0:], W[d0:], lr)
            if not dense_fused:
                self.comm.all_reduce(G[d0:], "sum")
        st.backward_conv()
        st.finalize(False)
        if dense_fused and self.comm.all_reduce_sgd(G[:d0], W[:d0], lr):
            main.wait_stream(cs)
            return
        cs.wait_stream(main)
        with torch.cuda.stream(cs):
            self.comm.all_reduce(G[:d0], "sum")
        main.wait_stream(cs)
        if dense_fused:
            self._update(0, d0)
        else:
            self._update()

    def _prepare_comm(self, st):
        """Collective set-up of the communicator's all-reduce channels for this step's buckets
        (must precede any graph capture; every rank reaches it at the same point).  With the fused
        backward and plain SGD the finalize kernel all-reduces through a dedicated xGMI channel
        (one exchange slot per finalize workgroup)."""
        if self.R == 1:
            return
        if not getattr(self, "_comm_prepared", False):
            n, d0 = self.W.numel(), st.dense_offset
            self.comm.prepare_all_reduce(n - d0, d0, n)
            self._xchg = None
            # one-shot moves (R-1) slabs per rank over the fabric, two-shot 2 (R-1)/R in two rounds
            self._xchg_twoshot = self.R >= int(os.environ.get("TDL_FX_TWOSHOT_MIN_R", "3"))
            if st.fused_bwd and self._plain_sgd and os.environ.get("TDL_MNIST_FINALIZE_XCHG", "1") == "1":
                self._xchg = self.comm.exchange_channel(n, M.FINALIZE_BLOCKS)
                if self._xchg is not None and not self._selftest_exchange(st.b):
                    self._xchg = None
            self.allreduce_mode = (("xgmi-in-finalize-twoshot" if self._xchg_twoshot else "xgmi-in-finalize")
                                   if self._xchg is not None else getattr(self.comm, "algorithm", self.comm.name))
            self._comm_prepared = True
        if self._xchg is not None and st.fused_bwd and not st.has_exchange:
            st.set_exchange(self._xchg, twoshot=self._xchg_twoshot)

    def _selftest_exchange(self, b: int) -> bool:
        """Collective start-up check of the exchange-in-finalize path on this job's devices: one
        real step (replica-specific samples) through a scratch step object with the exchange, whose
        updated weights must equal W0 - lr * (sum of the replicas' local gradients) taken through
        the communicator's own (self-tested) all-reduce, and be bit-identical on every replica.
        Parameters, gradients and metrics are restored afterwards.  Any failure on any rank: every
        rank keeps the serial all-reduce (TDL_XCHG_SELFTEST=0 skips the check)."""
        if os.environ.get("TDL_XCHG_SELFTEST", "1") != "1":
            return True
        import warnings

        from ..parallel import consistency

        dev = self.device
        n = len(self.X)
        idx = ((torch.arange(b, dtype=torch.int64) * 7919 + self.rank * 104729) % n).to(torch.int32).to(dev)
        saved = (self.W.clone(), self.G.clone())
        # phase 1, local work only: one step through the exchange.  Whatever happens here, every
        # rank then reaches the same agreement collective (a rank that raised must not wander into
        # a different collective than its peers)
        ok, why, timed_out, w_x, g_local = True, "", False, None, None
        try:
            tst = M.FusedMnistTrainStep(self.X, self.Y, idx, self.W, self.G, self.layout, b, self.R,
                                        self.optimizer.lr_dev, torch.zeros(4, dtype=torch.float32, device=dev),
                                        global_batch=b * self.R)
            if not tst.fused_bwd:
                raise RuntimeError("fused backward unavailable")
            tst.set_exchange(self._xchg, twoshot=self._xchg_twoshot)
            torch.cuda.synchronize(dev)
            if os.environ.get("TDL_FAULT_XCHG_SELFTEST_RAISE") == str(self.rank):  # fault injection (tests)
                raise RuntimeError("injected self-test failure before the exchange")
            tst.forward_backward(0)
            tst.finalize(True, exchange=True)
            torch.cuda.synchronize(dev)
            timed_out = bool(self._xchg.error())
            if timed_out:
                raise RuntimeError("exchange timed out")
            tst.check()
            w_x, g_local = self.W.clone(), self.G.clone()
            del tst
        except Exception as e:  # noqa: BLE001 - any failure means the serial path
            ok, why = False, f"{type(e).__name__}: {e}"
            timed_out = timed_out or bool(self._xchg.error())
        # agreement on the control plane (never through the xGMI kernel: its device may now carry a
        # sticky error word): [step ok everywhere, no rank timed out]
        ok_all, no_timeout = self._agree_flags([ok, not timed_out])
        if not no_timeout:
            # a bounded wait expired: the error word disables every xGMI kernel on that device, so
            # the serial all-reduce could not run there either -- fail the job on every rank
            self.W.copy_(saved[0])
            raise RuntimeError("exchange-in-finalize self-test: a peer did not arrive at the xGMI exchange "
                               f"({why or 'on another rank'}); the device fabric or a peer is broken")
        if ok_all:
            # phase 2, every rank: the reference reduction and the cross-replica identity check
            self.comm.all_reduce(g_local, "sum")
            lr = float(self.optimizer.lr_dev.item())
            w_ref = saved[0] - lr * g_local
            if os.environ.get("TDL_FAULT_XCHG_SELFTEST") == str(self.rank):  # fault injection (tests)
                w_ref = w_ref + 1.0
            if not torch.allclose(w_x, w_ref, rtol=1e-5, atol=1e-7):
                ok, why = False, f"max |W - W_ref| = {float((w_x - w_ref).abs().max()):.3g}"
            if not consistency.replicas_identical(self.comm, w_x):
                ok, why = False, "replicas differ"
            ok_all = self._agree_flags([ok])[0]
        self.W.copy_(saved[0])
        self.G.copy_(saved[1])
        if not ok_all:
            self.fallbacks.append(f"exchange-in-finalize self-test failed ({why or 'on another rank'})")
            if self.rank == 0:
                warnings.warn(f"exchange-in-finalize self-test failed ({why or 'on another rank'}); "
                              "using the serial gradient all-reduce")
        return ok_all

    def _agree_flags(self, flags) -> list:
        """MIN over ranks of boolean flags through the process group itself (not the communicator's
        xGMI fast path)."""
        import torch.distributed as dist

        on = self.device if self.comm.name == "rccl" else torch.device("cpu")
        f = torch.tensor([1.0 if x else 0.0 for x in flags], device=on)
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        return [bool(v > 0.5) for v in f.tolist()]

    @property
    def _plain_sgd(self) -> bool:
        opt = self.optimizer
        return type(opt).__name__ == "SGD" and opt.momentum == 0

    def _update(self, lo: int = 0, hi: Optional[int] = None):
        from .. import ops

        opt = self.optimizer
        C = ops.hip()
        W, G = self.W[lo:hi], self.G[lo:hi]
        if type(opt).__name__ != "SGD":
            # whole slab only (lo, hi cover it: the two-bucket split is SGD-only); Adam's step offset
            # inside the execution is baked into the captured graph
            if not opt.device_update(W, G, getattr(self, "_step_k", 0)):
                raise RuntimeError(f"fused trainer: {type(opt).__name__} has no device update on {W.device}")
            return
        if opt.momentum == 0:
            C.sgd(W, G, opt.lr_dev)
        else:
            C.sgd_momentum(W, G, opt._slots["momentum"][lo:hi], opt.lr_dev, opt.momentum, opt.nesterov)

    def _reduce_and_update(self):
        if self.R > 1:
            self.comm.all_reduce(self.G, "sum")
        self._update()

    def _run_eager(self, idx_np: np.ndarray, b: int, global_b: int):
        if b == 0:
            # this replica got no samples of a tiny final batch: contribute zero gradients
            self.G.zero_()
            if self.R > 1:
                self.comm.all_reduce(self.G, "sum")
            self.optimizer.apply_flat(self.W, self.G)
            return
        # one persistent index buffer per ragged size (the step object is cached by its address),
        # filled through a pinned staging buffer without a host sync
        key = ("ragged", b)
        idx_buf = self._ragged_bufs.get(key)
        if idx_buf is None:
            idx_buf = torch.zeros(b, dtype=torch.int32, device=self.device)
            self._ragged_bufs[key] = idx_buf
        if self._ragged_ev is not None:
            self._ragged_ev.synchronize()
        if self._ragged_stage is None or self._ragged_stage.numel() < b:
            self._ragged_stage = torch.empty(max(b, 256), dtype=torch.int32, pin_memory=True)
        self._ragged_stage[:b].numpy()[:] = idx_np
        idx_buf.copy_(self._ragged_stage[:b], non_blocking=True)
        self._ragged_ev = torch.cuda.Event()
        self._ragged_ev.record(torch.cuda.current_stream(self.device))
        st = self._step(b, idx_buf, global_b)
        self._prepare_comm(st)
        self._train_step(st, 0, global_b)
        self.optimizer.iterations += 1

    def _graph_for(self, K: int, b: int, slot: int = 0):
        """Graph of one K-step execution reading its sample ids from its own index buffer; the
        slots rotate so the host uploads execution i+1's indices while execution i runs."""
        g = self._graphs.get((K, b, slot))
        if g is not None:
            return g
        idx_buf = torch.zeros(K * b, dtype=torch.int32, device=self.device)
        st = self._step(b, idx_buf)
        self._prepare_comm(st)
        graph = None
        if self.capture:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            torch.cuda.synchronize(self.device)
            saved = (self.W.clone(), self.metrics_dev.clone(),
                     {k: v.clone() for k, v in self.optimizer.slots().items()})
            if self.capture_comm:
                # whole execution (K steps incl. all-reduce + optimizer) in one graph
                graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(graph, stream=s):
                    for k in range(K):
                        self._train_step(st, k * b, b * self.R)
            else:
                # one graph per step holding the fused fwd/bwd/finalize; the RCCL all-reduce and
                # the SGD kernel are issued eagerly between replays
                graph = []
                for k in range(K):
                    gk = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(gk, stream=s):
                        st.forward_backward(k * b)
                        st.finalize(False)
                    graph.append(gk)
            torch.cuda.synchronize(self.device)
            # capture does not execute, but be safe: restore state
            self.W.copy_(saved[0])
            self.metrics_dev.copy_(saved[1])
            for k, v in saved[2].items():
                self.optimizer.slots()[k].copy_(v)
        g = (graph, idx_buf, st)
        self._graphs[(K, b, slot)] = g
        return g

    def warm_graphs(self, steps: int, b: Optional[int] = None):
        """Capture every graph ``run_train(steps)`` will replay, ahead of a timed region."""
        if b is None and getattr(self, "_handlers_b", None):
            b = self._handlers_b[0]
        if b is None:
            return
        sizes = {self.K} if steps >= self.K else set()
        if steps % self.K:
            sizes.add(steps % self.K)
        for K in sizes:
            for slot in range(self._nslots):
                self._graph_for(K, b, slot)
        # pinned staging buffers of every slot at full size now: a pinned (hipHostMalloc)
        # allocation inside the launch loop waited ~30 ms for the device
        if sizes:
            self._ensure_stage(max(sizes) * b)

    def _ensure_stage(self, n: int):
        if not hasattr(self, "_stage"):
            self._stage, self._stage_ev, self._slot = [None] * self._nslots, [None] * self._nslots, 0
        for slot in range(self._nslots):
            if self._stage[slot] is None or self._stage[slot].numel() < n:
                if self._stage_ev[slot] is not None:
                    self._stage_ev[slot].synchronize()
                self._stage[slot] = torch.empty(max(n, 1024), dtype=torch.int32, pin_memory=True)

    def _upload(self, idx: np.ndarray, idx_buf: torch.Tensor, slot: int):
        """Asynchronous H2D copy of an execution's indices through a pinned staging buffer."""
        n = idx.size
        stage = self._stage[slot]
        if stage is None or stage.numel() < n:
            stage = torch.empty(max(n, 1024), dtype=torch.int32, pin_memory=True)
            self._stage[slot] = stage
        elif self._stage_ev[slot] is not None:
            self._stage_ev[slot].synchronize()  # the previous copy out of this buffer has run
        stage[:n].numpy()[:] = idx
        idx_buf[:n].copy_(stage[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._stage_ev[slot] = ev

    def _take_upload(self, handler: "DeviceHandler", K: int):
        """Take the next K full batches' indices and start their upload into the next index slot
        (None at a ragged tail / the end of finite data)."""
        ta = time.perf_counter()
        idx = handler.take(K)
        tb = time.perf_counter()
        if idx is None:
            return None
        if not hasattr(self, "_stage"):
            self._stage, self._stage_ev, self._slot = [None] * self._nslots, [None] * self._nslots, 0
        slot = self._slot
        self._slot = (slot + 1) % self._nslots
        graph, idx_buf, st = self._graph_for(K, handler.b, slot)
        tc = time.perf_counter()
        self._upload(idx, idx_buf, slot)
        self._last_take = (tb - ta, tc - tb, time.perf_counter() - tc)
        return (handler, K, idx.size // handler.b, graph, st)

    def prefetch(self, handler: "DeviceHandler", K: int) -> bool:
        """Input prefetch of depth one execution (tf.data ``prefetch`` semantics): take and upload
        the indices of the next K-step execution now, so the next ``run_train`` launches its first
        graph without waiting for the host's batch assembly.  Returns False at a ragged tail."""
        K = min(int(K), self.K)
        if self._ready is not None:
            return self._ready[1] == K
        self._ready = self._take_upload(handler, K)
        return self._ready is not None

    def run_train(self, handler: "DeviceHandler", steps: int) -> int:
        # everything allocated so far (modules, model, graphs) is long-lived: move it out of the
        # cyclic GC's generations so a collection in the launch loop scans only per-step garbage
        # (a full collection of the torch-sized heap stalled the host ~30 ms mid-run)
        gc.freeze()
        done = 0
        b = handler.b
        opt = self.optimizer
        if not hasattr(self, "_stage"):
            self._stage, self._stage_ev, self._slot = [None] * self._nslots, [None] * self._nslots, 0
        timing = self._host_times is not None
        while done < steps:
            K = min(self.K, steps - done)
            t0 = time.perf_counter() if timing else 0.0
            r, self._ready = self._ready, None
            if r is not None and (r[0] is not handler or r[1] != K):
                raise RuntimeError("fused trainer: prefetched execution does not match the requested steps")
            if r is None:
                r = self._take_upload(handler, K)
            t1 = t2 = time.perf_counter() if timing else 0.0
            if r is None:
                # ragged tail (end of finite data) -> eager steps of their own sizes
                one = handler.next_ragged()
                if one is None:
                    break
                opt._sync_lr()
                self._run_eager(*one)
                done += 1
                continue
            opt._sync_lr()
            _, _, Kr, graph, st = r
            if Kr < K:
                # the full batches in front of an epoch's partial batch: same slot buffers and
                # step object, launched eagerly (no per-step host sync, no new graph size)
                for k in range(Kr):
                    self._train_step(st, k * b, b * self.R)
                K = Kr
            elif isinstance(graph, list):
                for k, gk in enumerate(graph):
                    gk.replay()
                    self._step_k = k
                    self._reduce_and_update()
            elif graph is not None:
                graph.replay()
            else:
                for k in range(K):
                    self._train_step(st, k * b, b * self.R)
            if timing:
                tk = getattr(self, "_last_take", (0.0, 0.0, 0.0)) if t1 - t0 > 1e-4 else (t1 - t0, 0.0, 0.0)
                self._host_times.append((tk[0], tk[1] + tk[2], time.perf_counter() - t2))
            opt.iterations += K
            done += K
        return done

    # ------------------------------------------------------------------ evaluate / predict
    def _eval_columns(self, lp, labels: bool):
        """Device copies of an evaluation pipeline's columns (the last one is cached), or None
        when they are not the reference model's input."""
        cols = lp.columns if isinstance(lp.columns, (tuple, list)) else (lp.columns,)
        x = cols[0]
        y = cols[1] if len(cols) > 1 else None
        if not isinstance(x, torch.Tensor) or tuple(x.shape[1:]) not in ((28, 28, 1), (28, 28)) or \
                x.dtype != torch.float32:
            return None
        if labels and (not isinstance(y, torch.Tensor) or y.dim() != 1):
            return None
        key = _source_key(x, y if labels else None)
        cached = getattr(self, "_eval_cache", None)
        if cached is None or not _same_source(cached[0], key):
            X = x.reshape(len(x), 28, 28, 1).to(self.device, torch.float32).contiguous()
            Y = (y.to(self.device, torch.int32) if labels else torch.zeros(len(x), dtype=torch.int32, device=self.device)).contiguous()
            self._eval_cache = cached = (key, X, Y, {})
        return cached[1], cached[2], cached[3]

    def _eval_step(self, steps: dict, X, Y, b: int, cap: int, metrics):
        st = steps.get(b)
        if st is None or st.idx_buf.numel() < cap * b:
            idx_buf = torch.zeros(max(cap, 1) * b, dtype=torch.int32, device=self.device)
            st = M.FusedMnistTrainStep(X, Y, idx_buf, self.W, self.G, self.layout, b, self.R, self.optimizer.lr_dev,
                                       metrics)
            steps[b] = st
        st.metrics = metrics
        st._impl.set_metrics(metrics)
        return st

    def _forward_batches(self, handler: "DeviceHandler", X, Y, cache, steps, metrics, logits_out=None):
        """Forward-only passes over the handler's batches on the hand-written kernels."""
        K = 64
        done = 0
        while steps is None or done < steps:
            n = K if steps is None else min(K, steps - done)
            idx = handler.take(n)
            if idx is None:
                one = handler.next_ragged()
                if one is None:
                    break
                ids, nb, _ = one
                if nb > 0:
                    st = self._eval_step(cache, X, Y, nb, 1, metrics)
                    st.idx_buf[:nb].copy_(torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int32)))
                    lg = None if logits_out is None else torch.empty(nb * 10, device=self.device)
                    st.forward_eval(0, lg)
                    if lg is not None:
                        logits_out.append(lg.view(nb, 10))
                done += 1
                continue
            b = handler.b
            kb = idx.size // b
            st = self._eval_step(cache, X, Y, b, K, metrics)
            st.idx_buf[:idx.size].copy_(torch.from_numpy(np.ascontiguousarray(idx, dtype=np.int32)))
            lg = None if logits_out is None else torch.empty(kb * b * 10, device=self.device)
            for k in range(kb):
                st.forward_eval(k * b, None if lg is None else lg[k * b * 10:])
            if lg is not None:
                logits_out.append(lg.view(kb * b, 10))
            done += kb
        return done

    def evaluate(self, dataset, steps: Optional[int] = None) -> Optional[Dict[str, float]]:
        """``Model.evaluate`` on the gfx950 forward kernel (head mode 2): each replica evaluates its
        slice of every global batch of the device-resident pipeline; loss / accuracy sums are
        all-reduced once at the end.  None when the pipeline does not lower to the device."""
        lp = DD.lower(dataset)
        if lp is None:
            return None
        cols = self._eval_columns(lp, labels=True)
        if cols is None:
            return None
        X, Y, cache = cols
        if lp.batch_size % self.R:
            return None
        h = DeviceHandler(lp, None, self.rank, self.R)
        h._async = False
        metrics = torch.zeros(4, dtype=torch.float32, device=self.device)
        try:
            self._forward_batches(h, X, Y, cache, steps, metrics)
        finally:
            h.close()
        if self.R > 1:
            self.comm.check_health()
            self.comm.all_reduce(metrics, "sum")
        loss_sum, correct, count = (float(v) for v in metrics[:3].cpu())
        out = {"loss": loss_sum / max(count, 1.0)}
        for m in self.model.compiled_metrics:
            out[m.name] = correct / max(count, 1.0)
        return out

    def predict(self, dataset, steps: Optional[int] = None) -> Optional[np.ndarray]:
        """``Model.predict`` on the gfx950 forward kernel: logits of every sample in order.  Every
        replica computes all of them (inference is replica-independent; no collective)."""
        lp = DD.lower(dataset)
        if lp is None:
            return None
        cols = self._eval_columns(lp, labels=False)
        if cols is None:
            return None
        X, Y, cache = cols
        h = DeviceHandler(lp, None, 0, 1)
        h._async = False
        metrics = torch.zeros(4, dtype=torch.float32, device=self.device)
        out = []
        try:
            self._forward_batches(h, X, Y, cache, steps, metrics, logits_out=out)
        finally:
            h.close()
        if not out:
            return np.zeros((0, 10), dtype=np.float32)
        return torch.cat(out).cpu().numpy()

    def reset_metrics(self):
        self.metrics_dev.zero_()
        self.model._loss_tracker.reset_state()
        for m in self.model.compiled_metrics:
            m.reset_state()

    def logs(self) -> Dict[str, float]:
        for st in list(self._steps.values()):
            st.check()
        t = self.metrics_dev.clone()
        if self.R > 1:
            self.comm.check_health()
            self.comm.all_reduce(t, "sum")
        loss_sum, correct, count = (float(v) for v in t[:3].cpu())
        out = {"loss": loss_sum / max(count, 1.0)}
        for m in self.model.compiled_metrics:
            out[m.name] = correct / max(count, 1.0)
        # mirror into the Keras metric objects so model.metrics results agree
        lt = self.model._loss_tracker
        lt._to(self.device)
        lt.total._value.fill_(float(self.metrics_dev[0]))
        lt.count._value.fill_(float(self.metrics_dev[2]))
        for m in self.model.compiled_metrics:
            m._to(self.device)
            m.total._value.fill_(float(self.metrics_dev[1]))
            m.count._value.fill_(float(self.metrics_dev[2]))
        return out

    def finish(self):
        torch.cuda.synchronize(self.device)

    def on_replica_divergence(self):
        """The replicas' parameters differed after the custom xGMI all-reduce path (detected by
        keras/models.py _check_replicas and already repaired from rank 0): drop that path and the
        graphs that captured it; later executions all-reduce over RCCL / the ring."""
        if getattr(self.comm, "xgmi", None) is not None:
            self.comm.xgmi = None
            self.comm.algorithm = "rccl" if self.comm.name == "rccl" else self.comm.name
            self.comm._capture_ok = None  # re-probe: without xGMI a gloo group cannot be captured
        self._graphs = {}
        self._steps = {}
        self._capture_comm = None
        self._comm_prepared = False
        self._xchg = None
        self.allreduce_mode = getattr(self.comm, "algorithm", self.comm.name)


class _IndexProducer:
    """Background thread producing the global-batch index arrays of an IndexStream into a bounded
    queue, so an epoch's shuffle (native, GIL released) never stalls the launch loop."""

    def __init__(self, stream: "DD.IndexStream", depth: int = 512):
        self.stream = stream
        self.q: "queue.Queue" = queue.Queue(maxsize=depth)
        self._stop = threading.Event()
        self._ended = False
        self.t = threading.Thread(target=self._run, name="tdl-index-producer", daemon=True)
        self.t.start()

    def _run(self):
        while not self._stop.is_set():
            g = self.stream.next_batch()
            item = (g, self.stream._epoch)  # epochs the stream had to generate to produce g
            while not self._stop.is_set():
                try:
                    self.q.put(item, timeout=0.1)
                    break
                except queue.Full:
                    continue
            if g is None:
                return

    def get(self):
        """(batch or None at the end, epochs generated up to it)."""
        if self._ended:
            return None, None
        g, ep = self.q.get()
        if g is None:
            self._ended = True
        return g, ep

    def close(self):
        self._stop.set()
        while True:
            try:
                self.q.get_nowait()
            except queue.Empty:
                break
        self.t.join(timeout=5)


class DeviceHandler:
    """Index vectors for this replica: its slice of every global batch."""

    def __init__(self, lp: DD.LoweredPipeline, seed: Optional[int], rank: int, R: int):
        self.lp = lp
        self.rank, self.R = rank, R
        self.B = lp.batch_size
        self.b = lp.batch_size // R
        self.stream = DD.IndexStream(lp, seed)
        self._pending = []
        self._async = os.environ.get("TDL_ASYNC_INDICES", "1") == "1"
        self._producer: Optional[_IndexProducer] = None
        self._epochs_used = 0

    def new_iterator(self):
        self.close()
        self.stream = DD.IndexStream(self.lp, self.stream._seed)
        self._pending = []
        self._epochs_used = 0

    def close(self):
        if self._producer is not None:
            self._producer.close()
            self._producer = None
        self.stream.commit(self._epochs_used)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _next_global(self):
        if self._pending:
            return self._pending.pop(0)
        if not self._async:
            g = self.stream.next_batch()
            self._epochs_used = self.stream._epoch
            return g
        if self._producer is None:
            self._producer = _IndexProducer(self.stream)
        g, ep = self._producer.get()
        if ep is not None:
            self._epochs_used = ep
        return g

    def take(self, K: int) -> Optional[np.ndarray]:
        """Up to K full global batches -> this replica's [K'*b] indices.  Stops early in front of
        a partial batch (the epoch's remainder, left pending for ``next_ragged``) or the end of
        finite data; None when the next batch is not a full one."""
        got = []
        for _ in range(K):
            g = self._next_global()
            if g is None or len(g) < self.B:
                if g is not None:
                    self._pending.insert(0, g)
                break
            got.append(g)
        if not got:
            return None
        return np.concatenate([g[self.rank * self.b:(self.rank + 1) * self.b] for g in got])

    def next_ragged(self):
        g = self._next_global()
        if g is None:
            return None
        sizes = input_lib.split_sizes(len(g), self.R)
        lo = sum(sizes[: self.rank])
        n = sizes[self.rank]
        return g[lo:lo + n], n, len(g)
