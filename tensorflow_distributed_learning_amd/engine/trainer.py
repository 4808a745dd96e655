"""Training engines behind ``Model.fit`` / ``evaluate``.

:class:`GenericTrainer` – any model: PyTorch autograd over the layer ``call``s, parameters as
  autograd leaves that SHARE STORAGE with the replica's flat slab and whose ``.grad`` is a view of
  the flat gradient slab; after backward the gradient slab is all-reduced (bucketed, overlapped
  with backward through post-accumulate-grad hooks when the communicator is asynchronous) and the
  optimizer updates the whole slab at once.  Mixed precision (``keras.mixed_precision`` policy
  ``mixed_bfloat16``) runs the forward/backward under bf16 autocast with f32 master weights.

:class:`~.fused.FusedMnistTrainer` – the reference model on MI355X: hand-written HIP kernels,
  device-resident data, hipGraph-captured multi-step executions (engine/fused.py).

Both share the data handling and the cross-replica metric reduction defined here.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..data import dataset as D
from ..parallel import input_lib
from ..utils.tracing import trace_range


class LazyLogs(dict):
    """Logs dict whose values are computed (host sync + cross-replica reduce) on first access."""

    def __init__(self, fn):
        super().__init__()
        self._fn = fn
        self._done = False

    def _force(self):
        if not self._done:
            self._done = True
            super().update(self._fn())

    def __getitem__(self, k):
        self._force()
        return super().__getitem__(k)

    def get(self, k, d=None):
        self._force()
        return super().get(k, d)

    def items(self):
        self._force()
        return super().items()

    def keys(self):
        self._force()
        return super().keys()

    def values(self):
        self._force()
        return super().values()

    def __iter__(self):
        self._force()
        return super().__iter__()

    def __len__(self):
        self._force()
        return super().__len__()

    def __contains__(self, k):
        self._force()
        return super().__contains__(k)

    def __bool__(self):
        return True


def _async_ok(t: torch.Tensor) -> bool:
    """An asynchronous host->device copy is safe only from pinned memory (PyTorch's host allocator
    keeps a pinned block until the copies reading it complete).  A pageable batch may be freed and
    its memory reused by the next batch right after ``.to`` returns, while the copy still reads it."""
    return t.is_cuda or t.is_pinned()


def _to_device(batch, device):
    return D.map_structure(lambda t: t.to(device, non_blocking=_async_ok(t)) if isinstance(t, torch.Tensor) else t,
                           batch)


def _split_xy(batch):
    if isinstance(batch, (tuple, list)):
        if len(batch) == 1:
            return batch[0], None, None
        if len(batch) == 2:
            return batch[0], batch[1], None
        return batch[0], batch[1], batch[2]
    if isinstance(batch, dict) and "x" in batch:
        return batch["x"], batch.get("y"), batch.get("sample_weight")
    return batch, None, None


class HostDataHandler:
    """Per-replica batches from a (distributed) host pipeline."""

    def __init__(self, dataset: D.Dataset, strategy):
        self.dist = input_lib.DistributedDataset(dataset, strategy)
        self.strategy = strategy
        self._it = None

    def new_iterator(self):
        self._it = iter(self.dist)

    def next(self):
        if self._it is None:
            self.new_iterator()
        return next(self._it)

    def global_size(self, local_n: int) -> int:
        """Actual global batch size of the current step (per-replica sizes follow split_sizes)."""
        gb = self.dist.global_batch_size
        R = self.dist.num_replicas
        if R == 1:
            return local_n
        if gb is not None and local_n == gb // R and gb % R == 0:
            return gb
        t = torch.tensor([float(local_n)], dtype=torch.float64)
        comm = self.strategy.extended.communicator
        if comm.name == "rccl":
            t = t.to(self.strategy.extended.device)
        comm.all_reduce(t, "sum")
        return int(t.item())


class GenericTrainer:
    kind = "generic"

    def __init__(self, model):
        self.model = model
        self.strategy = model._get_strategy()
        self.device = self.strategy.extended.device
        self.comm = self.strategy.extended.communicator
        model._ensure_slabs()
        self.W, self.G = model._W, model._G
        self._make_leaves()
        self.optimizer = model.optimizer
        self.optimizer.build(self.W.numel(), self.device)
        self.loss = model.loss
        self.loss_tracker = model._loss_tracker
        self.metrics = model.compiled_metrics
        self._policy = model._dtype_policy()
        self._Wc = None
        self._Wt = None
        if self._policy == "mixed_bfloat16" and self.device.type == "cuda" and \
                os.environ.get("TDL_CAST_ACCUMULATE", "1") == "1":
            # bf16 compute copy of the whole weight slab: one cast kernel per step instead of one
            # per layer; Variable.cast / compute_view hand out views of it inside the step
            self._Wc = torch.empty(self.W.numel(), dtype=torch.bfloat16, device=self.device)
            self._bind_compute_views()
        self._buckets = self._make_buckets()
        self._bind_cast_accumulate()
        # whole-step hipGraphs (forward + backward + all-reduce + optimizer + metrics), keyed by
        # the batch signature; the first two steps of a signature run eagerly (solver search,
        # allocator warm-up), the third is captured and every later one is a single replay
        self._graphs: Dict[tuple, tuple] = {}
        self._seen: Dict[tuple, int] = {}
        self._graph_ok: Optional[bool] = None
        # metric accumulators start from zero for callers that drive run_train() directly
        # (fit() resets them per epoch; scripts/bench_resnet50.py did not, and reported stale state)
        self.reset_metrics()
        if self.device.type == "cuda":
            from ..ops import conv as _conv

            _conv.bind_communicator(self.comm)  # rank 0 makes the autotuning decisions for all replicas
        # TDL_CONV_AUTOTUNE=1, like TF's cuDNN autotuning (TF_CUDNN_USE_AUTOTUNE=1): MIOpen find-mode
        # search of the solvers per shape on first use, for the convs that fall back to MIOpen (scoped
        # to this trainer's steps, not left set process-wide).  Off by default: every ResNet-50 conv
        # runs on the hand-written kernels now, and MIOpen's find-mode GenericSearch worker threads
        # aborted the process on tiny f32 shapes on several boxes (tests/test_fit_gpu.py)
        self._conv_search = self.device.type == "cuda" and os.environ.get("TDL_CONV_AUTOTUNE", "0") == "1"

    # ------------------------------------------------------------------ parameters
    def _make_leaves(self):
        layout = self.model._layout
        for v, view, gview in zip(self.model._trainable_vars, layout.views(self.W), layout.views(self.G)):
            leaf = view.detach().requires_grad_(True)
            leaf.grad = gview
            v._leaf = leaf
        self._leaves = [v._leaf for v in self.model._trainable_vars]
        if getattr(self, "_buckets", None) is not None:
            # new leaves (after evaluate/predict): the bucket all-reduce hooks move with them
            self._register_bucket_hooks()
        if hasattr(self, "_buckets"):
            self._bind_cast_accumulate()
        self._bind_compute_views()

    def _bind_compute_views(self):
        if getattr(self, "_Wc", None) is None:
            return
        layout = self.model._layout
        for leaf, cv in zip(self._leaves, layout.views(self._Wc)):
            leaf._tdl_cview = cv
        # 4-D (conv) kernels also get an OHWI bf16 copy (the implicit-GEMM forward's weight rows),
        # refreshed with the cast by one transpose kernel over the whole slab
        if getattr(self, "_Wt", None) is None:
            entries, tiles = [], []
            for i, (spec, off) in enumerate(zip(layout.specs, layout.offsets)):
                if len(spec.shape) != 4 or i >= len(self._leaves):
                    continue
                R, K = spec.shape[0] * spec.shape[1] * spec.shape[2], spec.shape[3]
                e = len(entries)
                entries.append([off, off, R, K])
                tiles += [[e, a, b, 0] for a in range((R + 63) // 64) for b in range((K + 63) // 64)]
            self._Wt = torch.empty_like(self._Wc) if entries else False
            if entries:
                assert max(o + r * k for o, _, r, k in entries) <= self.W.numel()
                self._wt_tables = (torch.tensor(entries, dtype=torch.int32, device=self.device),
                                   torch.tensor(tiles, dtype=torch.int32, device=self.device))
        if self._Wt is not False:
            for leaf, spec, off in zip(self._leaves, layout.specs, layout.offsets):
                if len(spec.shape) == 4:
                    kh, kw, c, k = spec.shape
                    leaf._tdl_tview = self._Wt[off: off + spec.size].view(k, kh, kw, c)

    def _bind_cast_accumulate(self):
        if self._buckets is None and os.environ.get("TDL_CAST_ACCUMULATE", "1") == "1":
            # no bucket hooks to fire: compute-dtype weight copies accumulate their gradient
            # straight into the slab view (Variable.cast)
            for leaf in self._leaves:
                leaf._tdl_gview = leaf.grad

    def _make_buckets(self):
        """Overlap of the gradient all-reduce with backward: contiguous slab buckets (reverse
        layer order) are launched asynchronously as soon as every gradient inside is final.  The
        bucket size comes from compile(bucket_bytes=...), else CommunicationOptions.bytes_per_pack,
        else the size/topology plan of parallel/bucketing.py; CommunicationOptions.all_reduce_dtype
        sets the dtype on the wire."""
        from ..parallel import bucketing

        opts = getattr(self.strategy.extended, "communication_options", None)
        self._wire = (getattr(opts, "all_reduce_dtype", None) or "float32") if self.device.type == "cuda" else "float32"
        wb = bucketing.DTYPE_BYTES[self._wire]
        explicit = self.model._bucket_bytes
        per_pack = explicit if explicit is not None else int(getattr(opts, "bytes_per_pack", 0) or 0)
        lw = int(os.environ.get("LOCAL_WORLD_SIZE", self.comm.world_size) or self.comm.world_size)
        self.plan = bucketing.plan(self.G.numel(), self.comm.world_size, lw, self._wire, per_pack,
                                   algorithm=getattr(self.comm, "algorithm", self.comm.name))
        self._wire_full = None
        if self.comm.world_size == 1:
            return None
        if explicit == 0:
            self.plan.n_buckets, self.plan.bucket_bytes = 1, self.plan.wire_bytes
            return None
        xg = getattr(self.comm, "xgmi", None)
        if self.comm.name != "rccl":
            # no RCCL (replicas sharing one GPU: gloo control plane): the xGMI kernel is the
            # device data plane, f32 on the wire, buckets within its message limit
            if xg is None:
                return None
            self._wire, wb = "float32", 4
            self.plan.wire_dtype, self.plan.wire_bytes = "float32", self.G.numel() * 4
            self.plan.bucket_bytes = min(self.plan.bucket_bytes, xg.limit * 4)
            self.plan.algorithm = getattr(self.comm, "algorithm", "xgmi")
        layout = self.model._layout
        ranges = layout.buckets(self.plan.bucket_bytes, elem_bytes=wb)
        self.plan.n_buckets = len(ranges)
        if len(ranges) <= 1 and self.comm.name == "rccl":
            return None
        # collective (every rank computes the same ranges): RCCL, or an xGMI channel per size
        capable = getattr(self.comm, "device_bucket_capable", None)
        if capable is not None and not capable([e - s for s, e in ranges]):
            return None
        var_bucket = {}
        for bi, (s, e) in enumerate(ranges):
            for i, off in enumerate(layout.offsets):
                if s <= off < e:
                    var_bucket[i] = bi
        self._pending = [sum(1 for i in var_bucket if var_bucket[i] == b) for b in range(len(ranges))]
        self._bucket_ranges = ranges
        # low-precision wire copies of every bucket, allocated once (graph-capture safe)
        self._wire_bufs = None if self._wire == "float32" else [
            torch.empty(e - s, dtype=getattr(torch, self._wire), device=self.device) for s, e in ranges]
        self._var_bucket = var_bucket
        self._works = []
        self._counts = list(self._pending)
        self._register_bucket_hooks()
        return ranges

    def _register_bucket_hooks(self):
        """Post-accumulate hooks on the CURRENT leaves: the last gradient of a bucket launches that
        bucket's asynchronous all-reduce."""
        var_bucket = self._var_bucket

        def hook_for(i):
            b = var_bucket[i]

            def hook(_p):
                self._counts[b] -= 1
                if self._counts[b] == 0:
                    from ..ops import conv as _conv

                    _conv.join_side()  # this bucket's weight gradients may still be on the side stream
                    s, e = self._bucket_ranges[b]
                    if getattr(self, "_skip_comm", False):  # fault injection: this rank leaves it out
                        from ..parallel.communicator import _Done

                        self._works.append(_Done())
                    elif self._wire_bufs is None:
                        self._works.append(self.comm.all_reduce_async(self.G[s:e], "sum"))
                    else:
                        buf = self._wire_bufs[b]
                        buf.copy_(self.G[s:e])
                        self._works.append((self.comm.all_reduce_async(buf, "sum"), b))
            return hook

        for i, leaf in enumerate(self._leaves):
            leaf.register_post_accumulate_grad_hook(hook_for(i))

    # ------------------------------------------------------------------ steps
    def _forward_loss(self, x, y, sw, global_n):
        model = self.model
        if self._policy == "mixed_bfloat16" and self.device.type == "cuda":
            # no cast cache: a cached bf16 weight copy must not outlive a captured step graph
            ctx = torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False)
        else:
            ctx = torch.autocast(self.device.type, enabled=False)
        with ctx:
            y_pred = model(x, training=True)
        fused = self._fused_head(y, y_pred, sw)
        if fused is not None:
            loss = fused(global_n)
            reg = model._regularization_loss()
            if reg is not None:
                loss = loss + reg / self.strategy.num_replicas_in_sync
            return loss, None, y_pred
        per_ex = self.loss.per_example(y, y_pred.float() if y_pred.dtype != torch.float32 else y_pred)
        if sw is not None:
            per_ex = per_ex * sw.to(per_ex.dtype)
        # tf.nn.compute_average_loss: per-replica sum / GLOBAL batch -> SUM all-reduce = global mean
        loss = per_ex.sum() / float(global_n)
        reg = model._regularization_loss()
        if reg is not None:
            loss = loss + reg / self.strategy.num_replicas_in_sync
        return loss, per_ex, y_pred

    def _seed(self) -> torch.Tensor:
        """The backward seed d(loss)/d(loss) = 1, allocated once (autograd would fill a new one every
        step; the fused loss head recognises this one and skips its scaling kernel)."""
        s = getattr(self, "_seed_t", None)
        if s is None:
            s = self._seed_t = torch.ones((), dtype=torch.float32, device=self.device)
        return s

    def _fused_head(self, y, y_pred, sw):
        """The one-kernel loss head (ops/dense.py xent_head) when the step's loss and metrics are what it
        computes: SparseCategoricalCrossentropy(from_logits=True) on f32 2-D logits, no sample weights,
        metrics none or SparseCategoricalAccuracy.  Returns ``f(global_n) -> loss`` (the metric
        accumulators are advanced by the kernel), or None."""
        from ..keras import losses as _losses
        from ..keras import metrics as _metrics
        from ..ops import dense as _dense

        if (sw is not None or y is None or os.environ.get("TDL_FUSED_HEAD", "1") != "1" or
                not isinstance(self.loss, _losses.SparseCategoricalCrossentropy) or not self.loss.from_logits or
                self.loss.ignore_class is not None or y_pred.dim() != 2 or y.dim() != 1 or
                y_pred.dtype not in (torch.float32, torch.bfloat16, torch.float16)):
            return None
        # (mixed precision: the loss is computed on f32 logits, as the unfused path's y_pred.float())
        y_pred = y_pred.float() if y_pred.dtype != torch.float32 else y_pred
        if not _dense.xent_head_supported(y_pred, y.long()):
            return None
        if len(self.metrics) > 1 or (self.metrics and type(self.metrics[0]) is not _metrics.SparseCategoricalAccuracy):
            return None
        accs = []
        for m in [self.loss_tracker] + list(self.metrics):
            m._to(y_pred.device)
            accs += [m.total._value, m.count._value]
        while len(accs) < 4:
            accs.append(None)
        labels = y.long()
        return lambda gn: _dense.xent_head(y_pred, labels, gn, accs[:2], accs[2:], seed=self._seed())

    def train_step(self, batch, global_n: int, sync_lr: bool = True, t_add: int = 0):
        """One whole step.  ``t_add``: the step's offset inside a multi-step execution graph whose
        first step count is the optimizer's device ``t_dev`` (Adam's bias correction)."""
        x, y, sw = _split_xy(_to_device(batch, self.device))
        from ..utils import fault

        # fault injection (tests): this rank leaves out this step's gradient all-reduce
        self._skip_comm = self.comm.world_size > 1 and fault.maybe_skip_collective(self.comm.rank,
                                                                                   int(self.optimizer.iterations))
        G = self.G
        if getattr(self, "_g_clean", None) == G.data_ptr():  # the previous step's optimizer kernel zeroed G
            self._g_clean = None
        else:
            G.zero_()
        if self._buckets is not None:
            self._counts = list(self._pending)
            self._works = []
        from ..parallel import values as V

        if self._Wc is not None:
            from ..ops import hip

            hip().slab_cast_bf16(self.W, self._Wc)  # the step's bf16 weights, one kernel
            if self._Wt is not False:
                hip().slab_transpose_bf16(self.W, self._Wt, *self._wt_tables)  # OHWI conv rows, one kernel
        V.CAST_ACCUMULATE[0] += 1  # Variable.cast may add straight into the slab only in here
        search_prev = torch.backends.cudnn.benchmark
        torch.backends.cudnn.benchmark = search_prev or self._conv_search
        try:
            with trace_range("tdl.forward"):
                loss, per_ex, y_pred = self._forward_loss(x, y, sw, global_n)
        except BaseException:
            torch.backends.cudnn.benchmark = search_prev
            raise
        finally:
            V.CAST_ACCUMULATE[0] -= 1
        from ..utils import checksums as _ck

        if _ck.enabled():
            _ck.record("input:x", x)
            _ck.record("input:y", y)
            _ck.record("loss", loss)
        from ..ops import conv as _conv

        _conv.side_stream_window(self.device.type == "cuda")
        try:
            with trace_range("tdl.backward"):
                loss.backward(self._seed())
        finally:
            _conv.side_stream_window(False)
            _conv.join_side()  # every slab weight gradient queued on the side stream is in G
            torch.backends.cudnn.benchmark = search_prev
        if _ck.enabled():
            for v, gv in zip(self.model._trainable_vars, self.model._layout.views(G)):
                _ck.record("slab_grad:" + v.name, gv)
        for b in (self.model.__dict__.get("_grad_boxes") or {}).values():
            if b.g is not None:  # a parked gradient contribution nobody collected
                raise RuntimeError("fused gradient sum lost a contribution (keras/fusion.py grad boxes)")
        if self.comm.world_size > 1 and not self._skip_comm:
            with trace_range("tdl.allreduce"):
                if self._buckets is not None:
                    for w in self._works:
                        if isinstance(w, tuple):  # low-precision wire copy: cast back into G
                            w[0].wait()
                            s, e = self._bucket_ranges[w[1]]
                            G[s:e].copy_(self._wire_bufs[w[1]])
                        else:
                            w.wait()
                    if len(self._works) != len(self._bucket_ranges):
                        raise RuntimeError("gradient bucket hooks did not fire for every bucket (unused parameters?)")
                elif self._wire != "float32":
                    if self._wire_full is None:
                        self._wire_full = torch.empty(G.numel(), dtype=getattr(torch, self._wire), device=G.device)
                    self._wire_full.copy_(G)
                    self.comm.all_reduce(self._wire_full, "sum")
                    G.copy_(self._wire_full)
                else:
                    self.comm.all_reduce(G, "sum")
        with torch.no_grad(), trace_range("tdl.optimizer"):
            opt = self.optimizer
            opt._zero_grad_after, opt._zeroed_grad = G.is_cuda, False
            try:
                opt.apply_flat(self.W, G, sync_lr=sync_lr, t_add=t_add)
            finally:
                opt._zero_grad_after = False
            # (only an optimizer kernel that zeroed G after reading it marks this slab clean)
            self._g_clean = G.data_ptr() if opt._zeroed_grad else None
            opt._zeroed_grad = False
            if _ck.enabled():
                _ck.record("slab_W", self.W)
            if per_ex is not None:  # (the fused loss head advanced the metric accumulators itself)
                self.loss_tracker.update_state(per_ex.detach())
                yp = y_pred.detach()
                for m in self.metrics:
                    m.update_state(y, yp, sw)

    def run_train(self, handler, steps: int) -> int:
        from .fused import DeviceHandler

        if isinstance(handler, DeviceHandler):  # (prepare(): device-resident input, execution graphs)
            return self._run_device(handler, steps)
        done = 0
        for _ in range(steps):
            try:
                batch = handler.next()
            except StopIteration:
                break
            n = len(D.flatten(batch)[0])
            gn = handler.global_size(n)
            if not self._graphed_step(batch, gn):
                self.train_step(batch, gn)
            done += 1
        return done

    # ------------------------------------------------------------------ whole-step graphs
    def _graphable(self) -> bool:
        if self._graph_ok is None:
            ok = (self.device.type == "cuda" and os.environ.get("TDL_GRAPH_STEP", "1") == "1" and
                  getattr(self.optimizer, "graph_safe", False) and not self.optimizer.weight_decay)
            if ok and self.comm.world_size > 1:
                ok = self.comm.capture_probe()  # collective: every rank takes the same decision
            self._graph_ok = bool(ok)
        return self._graph_ok

    def _graphed_step(self, batch, global_n: int) -> bool:
        flat = D.flatten(batch)
        if not all(isinstance(t, torch.Tensor) for t in flat):
            return False
        if not self._graphable():
            return False
        key = (global_n,) + tuple((tuple(t.shape), t.dtype) for t in flat)
        ent = self._graphs.get(key)
        if ent is None:
            seen = self._seen.get(key, 0) + 1
            self._seen[key] = seen
            if seen <= 2:
                return False
            try:
                ent = self._capture(batch, global_n)
            except Exception as e:  # noqa: BLE001 - a layer with host-side logic: stay eager
                import warnings

                warnings.warn(f"whole-step graph capture failed, training eagerly: {type(e).__name__}: {e}")
                torch.cuda.synchronize(self.device)
                self._graph_ok = False
                return False
            self._graphs[key] = ent
        static, graph = ent
        for s_, t in zip(static, flat):
            s_.copy_(t, non_blocking=_async_ok(t))
        self.optimizer._sync_lr()
        graph.replay()
        self.optimizer.iterations += 1
        return True

    def _capture(self, batch, global_n: int):
        flat = D.flatten(batch)
        static = [torch.empty_like(t, device=self.device).copy_(t) for t in flat]
        it = iter(static)
        sbatch = D.map_structure(lambda _t: next(it), batch)
        dev = self.device
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        it0 = self.optimizer.iterations
        try:
            with torch.cuda.graph(graph, stream=s):
                self.train_step(sbatch, global_n, sync_lr=False)
        finally:
            self.optimizer.iterations = it0  # capture records, it does not run a step
        torch.cuda.current_stream(dev).wait_stream(s)
        return static, graph

    # ------------------------------------------------------------------ device-resident executions
    def prepare(self, dataset):
        """Device-resident input for ANY model (the fused engine's data path, data/device.py): an
        in-memory ``[map].cache().shuffle().batch().repeat()`` pipeline of (features, labels) is
        uploaded to HBM once, and each execution of ``steps_per_execution`` steps is ONE captured
        hipGraph that gathers its batches from HBM by the execution's index vector (one async H2D
        copy per execution) and runs K whole steps: forward, backward, all-reduce, optimizer and
        metrics (TF's ``steps_per_execution``: K steps per ``tf.function`` call).  None: host pipeline.
        TDL_GENERIC_DEVICE_DATA=0 keeps the host pipeline."""
        if self.device.type != "cuda" or os.environ.get("TDL_GENERIC_DEVICE_DATA", "1") != "1":
            return None
        from ..data import device as DD
        from . import fused as F

        lp = DD.lower(dataset)
        if lp is None or not isinstance(lp.columns, (tuple, list)) or len(lp.columns) != 2:
            return None
        x, y = lp.columns
        if not (isinstance(x, torch.Tensor) and isinstance(y, torch.Tensor)) or not x.is_floating_point():
            return None
        R = self.comm.world_size
        if lp.batch_size % R or not self._graphable():  # (_graphable is collective at R > 1: every rank is here)
            return None
        key = (x.data_ptr(), tuple(x.shape), y.data_ptr(), tuple(y.shape), x._version, y._version)
        if getattr(self, "_dev_key", None) != key:
            self._X = x.to(self.device).contiguous()
            self._Y = y.to(self.device).contiguous()
            self._dev_key = key
        from ..ops import hip

        self._gather_xy = (self._X.dtype == torch.float32 and self._Y.dim() == 1 and
                           self._Y.dtype in (torch.int64, torch.int32) and hasattr(hip(), "gather_xy") and
                           self._X.data_ptr() % 16 == 0)
        policy = input_lib.effective_policy(dataset) if R > 1 else None
        seed = input_lib.shared_seed(self.strategy) if policy is not None and policy.name in ("DATA", "FILE") else None
        return F.DeviceHandler(lp, seed, self.comm.rank, R)

    def _dev_upload(self, idx) -> None:
        """The execution's sample ids into the device index buffer (stream-ordered after the previous
        execution's graph, which reads the same buffer), through a ring of pinned staging buffers."""
        n = int(idx.size)
        if getattr(self, "_dev_idx", None) is None or self._dev_idx.numel() < n:
            self._dev_idx = torch.zeros(max(n, 1024), dtype=torch.int32, device=self.device)
            self._graphs = {k: v for k, v in self._graphs.items() if k[0] != "dev"}  # they read the old buffer
            self._dev_stage = [None] * 4
            self._dev_ev = [None] * 4
            self._dev_slot = 0
        s = self._dev_slot
        self._dev_slot = (s + 1) % len(self._dev_stage)
        if self._dev_stage[s] is None or self._dev_stage[s].numel() < n:
            self._dev_stage[s] = torch.empty(self._dev_idx.numel(), dtype=torch.int32, pin_memory=True)
        elif self._dev_ev[s] is not None:
            self._dev_ev[s].synchronize()  # the copy out of this staging buffer has run
        self._dev_stage[s][:n].numpy()[:] = idx
        self._dev_idx[:n].copy_(self._dev_stage[s][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self._dev_ev[s] = ev

    def _dev_step(self, k: int, b: int, global_n: int, sync_lr: bool):
        ii = self._dev_idx[k * b:(k + 1) * b]
        if self._gather_xy:  # features and labels of the batch in one hand-written kernel
            from ..ops import hip

            x, y = hip().gather_xy(self._X, self._Y, ii)
        else:
            x, y = self._X.index_select(0, ii), self._Y.index_select(0, ii)
        self.train_step((x, y), global_n, sync_lr=sync_lr, t_add=k)

    def warm_graphs(self, steps: int, b: Optional[int] = None):
        """Capture (without running) the execution graphs ``run_train(steps)`` will replay, once a
        step of this batch size has run eagerly (bench.py: ahead of the timed region)."""
        b = b if b is not None else getattr(self, "_dev_b", None)
        if b is None or b not in getattr(self, "_dev_warm", ()) or self._graph_ok is False:
            return
        K = max(1, self.model._steps_per_execution)
        sizes = ({K} if steps >= K else set()) | ({steps % K} if steps % K else set())
        if getattr(self, "_dev_idx", None) is None or self._dev_idx.numel() < max(sizes) * b:
            self._dev_upload(np.zeros(max(sizes) * b, dtype=np.int32))
        for k in sizes:
            if ("dev", k, b) not in self._graphs:
                self._dev_capture(k, b)

    def _run_device(self, handler, steps: int) -> int:
        import gc

        gc.freeze()  # long-lived state out of the cyclic GC's generations (engine/fused.py run_train)
        done, b, opt = 0, handler.b, self.optimizer
        self._dev_b = b
        if not hasattr(self, "_dev_warm"):
            self._dev_warm = set()
        spe = max(1, self.model._steps_per_execution)
        while done < steps:
            idx = handler.take(min(spe, steps - done))
            if idx is None:
                one = handler.next_ragged()  # an epoch's partial batch: one eager step of its size
                if one is None:
                    break
                ids, n, gb = one
                if n == 0:
                    raise RuntimeError("generic device path: a replica got no samples of a partial batch")
                self._dev_upload(ids)
                opt._sync_lr()
                self._dev_step(0, n, gb, sync_lr=False)
                done += 1
                continue
            K = idx.size // b
            self._dev_upload(idx)
            opt._sync_lr()
            graph = self._graphs.get(("dev", K, b))
            if (graph is None and b in self._dev_warm and self._graph_ok is not False and
                    os.environ.get("TDL_GENERIC_DEVICE_EAGER", "0") != "1"):
                graph = self._dev_capture(K, b)
            if graph is None:
                # the first execution at this batch size runs eagerly (allocator warm-up, autotuning
                # decisions), or every one does when a layer cannot be captured
                t0 = opt.iterations
                for k in range(K):
                    self._dev_step(k, b, b * self.comm.world_size, sync_lr=False)
                opt.iterations = t0 + K
                self._dev_warm.add(b)
            else:
                graph.replay()
                opt.iterations += K
            done += K
        return done

    def _dev_capture(self, K: int, b: int):
        dev = self.device
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        it0 = self.optimizer.iterations
        try:
            with torch.cuda.graph(graph, stream=s):
                for k in range(K):
                    self._dev_step(k, b, b * self.comm.world_size, sync_lr=False)
        except Exception as e:  # noqa: BLE001 - a layer with host-side logic: stay eager
            import warnings

            warnings.warn(f"execution graph capture failed, training eagerly: {type(e).__name__}: {e}")
            torch.cuda.synchronize(dev)
            self._graph_ok = False
            return None
        finally:
            self.optimizer.iterations = it0  # capture records, it does not run a step
        torch.cuda.current_stream(dev).wait_stream(s)
        self._graphs[("dev", K, b)] = graph
        return graph

    @torch.no_grad()
    def test_step(self, batch):
        x, y, sw = _split_xy(_to_device(batch, self.device))
        y_pred = self.model(x, training=False)
        per_ex = self.loss.per_example(y, y_pred.float())
        if sw is not None:
            per_ex = per_ex * sw.to(per_ex.dtype)
        self.loss_tracker.update_state(per_ex)
        for m in self.metrics:
            m.update_state(y, y_pred, sw)

    def run_test(self, handler: HostDataHandler, steps: Optional[int]) -> int:
        done = 0
        while steps is None or done < steps:
            try:
                batch = handler.next()
            except StopIteration:
                break
            self.test_step(batch)
            done += 1
        return done

    def reset_metrics(self):
        self.loss_tracker.reset_state()
        for m in self.metrics:
            m.reset_state()

    def logs(self) -> Dict[str, float]:
        from ..parallel.strategy import _cross_replica

        if self.comm.world_size > 1:
            # raises if a custom (xGMI) all-reduce of the executions since the last read timed out
            self.comm.check_health()
        with _cross_replica():
            out = {"loss": float(self.loss_tracker.result())}
            for m in self.metrics:
                out[m.name] = float(m.result())
        return out

    def finish(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
