"""``fit`` of a single-process multi-device MirroredStrategy (tf_dist_example.py:13, README.md:15-19):
ONE training loop (callbacks, progress bar, History, ``stop_training``, learning-rate schedules all
live once, on the user's model) driving G replicas.

* :class:`MirroredFusedTrainer` -- the reference CNN on the device path.  ONE host thread, one
  stream per device, no replica threads: each replica's execution of K steps is captured once into
  a hipGraph on its own device (engine/fused.py's fused MNIST step), and every execution launches
  the G graphs back to back (``hipGraphLaunch`` is asynchronous).  The gradient all-reduce is
  inside those graphs: each finalize workgroup exchanges its gradient range with the same
  workgroup of every other device over xGMI and applies SGD (``allreduce: xgmi-in-finalize``), or,
  where the fused backward does not apply, the standalone xGMI all-reduce kernel with SGD fused.
  The channels are wired in-process (csrc/xgmi_channel.h ``connect_local`` after peer access;
  parallel/device_group.py).  A start-up self-test compares one real step against
  ``W0 - lr * sum(local gradients)`` and otherwise falls back to per-step graphs with the all-reduce
  between them (an RCCL clique of the devices, or event-ordered copies).
* :class:`ThreadedGroupTrainer` -- every other model: the generic engine of each replica runs its
  steps in the group's turn-taking replica threads (parallel/local_replicas.py), one global input
  pipeline split into per-replica slices on the host.

Both keep the replicas' optimizers in lock step with replica 0's (learning rate incl. schedules and
callbacks, iterations) and re-broadcast replica 0's weights and optimizer state whenever the loop
may have changed them (``broadcast_from_primary``: start of fit, after ``on_train_begin``).
"""
from __future__ import annotations

import gc
import os
from typing import Dict, List, Optional

import numpy as np
import torch

from ..data import device as DD
from ..parallel import input_lib
from . import fused as F


def _models_and_group(model):
    g = model._get_strategy()._local_group
    return model._local_replicas(), g


def make_group_trainer(model):
    """The group trainer of replica 0's model (the user's) of a single-process MirroredStrategy."""
    models, group = _models_and_group(model)
    if all(d.type == "cuda" for d in group.devices) and os.environ.get("TDL_MIRRORED_DEVICE_PATH", "1") == "1":
        reason = F.eligible(model)
        if reason is None:
            return MirroredFusedTrainer(model, models, group)
        model._fused_reason = reason
    return ThreadedGroupTrainer(model, models, group)


def _sync_optimizer(dst, src):
    """dst follows src: learning rate (value or schedule) and step count."""
    dst._lr = src._lr
    dst.iterations = src.iterations


def _copy_optimizer_state(dst, src):
    _sync_optimizer(dst, src)
    for k, v in src.slots().items():
        d = dst.slots().get(k)
        if d is not None and d.numel() == v.numel():
            d.copy_(v.to(d.device))


class _ReplicaFused(F.FusedMnistTrainer):
    """Replica r's fused engine inside a :class:`MirroredFusedTrainer`: its execution graph holds
    the cross-device all-reduce of the group (never a host collective)."""

    def __init__(self, model, grp: "MirroredFusedTrainer", r: int):
        super().__init__(model)
        self.grp, self.r = grp, r
        self.capture = os.environ.get("TDL_GRAPH", "1") == "1"
        self.overlap = False
        self.allreduce_mode = None

    @property
    def capture_comm(self) -> bool:
        return self.grp.mode in ("xchg", "xgmi")

    def _prepare_comm(self, st):
        if self.grp.mode == "xchg" and st.fused_bwd and self._plain_sgd and not st.has_exchange:
            st.set_exchange(self.grp.xchg[self.r], twoshot=self.grp.twoshot)

    def _apply(self, st, global_b: int, k: int = 0):
        self._step_k = k
        mode = self.grp.mode
        if mode == "xchg" and st.has_exchange:
            st.finalize(True, exchange=True, keep_grad=False)
            return
        if mode in ("xchg", "xgmi"):
            st.finalize(False)
            ch = self.grp.ar[self.r]
            if self._plain_sgd:
                ch.all_reduce_sgd(self.G, self.W, self.optimizer.lr_dev, 1.0)
            else:
                ch.all_reduce(self.G, self.G, 1.0)
                self._update()
            return
        raise RuntimeError("mirrored fused trainer: no in-graph all-reduce in serial mode")


class _SliceHandler:
    """Replica r's slices of precomputed global batches (evaluation)."""

    def __init__(self, batches: List[np.ndarray], r: int, G: int, B: int):
        self.batches, self.r, self.G = list(batches), r, G
        self.B, self.b = B, B // G

    def take(self, K: int) -> Optional[np.ndarray]:
        got = []
        while self.batches and len(got) < K and len(self.batches[0]) == self.B:
            got.append(self.batches.pop(0))
        if not got:
            return None
        return np.concatenate([g[self.r * self.b:(self.r + 1) * self.b] for g in got])

    def next_ragged(self):
        if not self.batches:
            return None
        g = self.batches.pop(0)
        sizes = input_lib.split_sizes(len(g), self.G)
        lo = sum(sizes[:self.r])
        return g[lo:lo + sizes[self.r]], sizes[self.r], len(g)


class MirroredFusedTrainer:
    """See module docstring."""

    kind = "fused"
    is_group = True

    def __init__(self, model, models, group):
        self.model, self.models, self.group = model, models, group
        self.G = group.G
        self.devices = group.devices
        self.dc = group.device_comm()
        self.subs = []
        for r, m in enumerate(models):
            with torch.cuda.device(self.devices[r]):
                self.subs.append(_ReplicaFused(m, self, r))
        for m, s in zip(models[1:], self.subs[1:]):
            m._trainer = s  # a clone's own engine (evaluate / predict inside replica regions)
        self.optimizer = model.optimizer
        self.W, self.G_ = self.subs[0].W, self.subs[0].G
        self.K = self.subs[0].K
        self.capture = self.subs[0].capture
        self.mode: Optional[str] = None  # "xchg" | "xgmi" | "serial" (decided at the first prepare)
        self.twoshot = False
        self.xchg = self.ar = None
        self.allreduce_mode = None
        self.fallbacks: List[str] = []
        self._nslots = self.subs[0]._nslots
        self._slot = 0
        self._ready = None
        self._data_key = None
        self._b = None
        self.broadcast_from_primary()

    # ------------------------------------------------------------------ replicas
    def replica_trainer(self, model):
        for m, s in zip(self.models, self.subs):
            if m is model:
                return s
        raise KeyError("model is not a replica of this trainer")

    @property
    def metrics_dev(self):
        return self.subs[0].metrics_dev

    @property
    def capture_comm(self) -> bool:
        """The all-reduce is recorded inside every device's execution graph."""
        return self.mode in ("xchg", "xgmi") and self.capture

    def broadcast_from_primary(self):
        """Replica 0's weights and optimizer state onto every replica (mirrored variables)."""
        s0 = self.subs[0]
        self.dc.synchronize()
        for s in self.subs[1:]:
            s.W.copy_(s0.W.to(s.W.device))
            _copy_optimizer_state(s.optimizer, s0.optimizer)
        self.dc.synchronize()

    def _sync_optimizers(self):
        o0 = self.subs[0].optimizer
        for s in self.subs[1:]:
            _sync_optimizer(s.optimizer, o0)

    # ------------------------------------------------------------------ data
    def prepare(self, dataset):
        lp = DD.lower(dataset)
        if lp is None:
            return None
        cols = lp.columns if isinstance(lp.columns, (tuple, list)) else (None, None)
        x, y = cols[:2]
        if x is None or y is None or tuple(x.shape[1:]) not in ((28, 28, 1), (28, 28)) or \
                x.dtype != torch.float32 or y.dim() != 1:
            return None
        if lp.batch_size % self.G:
            raise ValueError(f"global batch {lp.batch_size} is not divisible by {self.G} replicas")
        key = F._source_key(x, y)
        if not F._same_source(self._data_key, key):
            per_dev = {}
            for s in self.subs:
                d = s.device
                if d not in per_dev:
                    per_dev[d] = (x.reshape(len(x), 28, 28, 1).to(d, torch.float32).contiguous(),
                                  y.to(d, torch.int32).contiguous())
                s.X, s.Y = per_dev[d]
                s._data_key = key
                s._steps, s._graphs = {}, {}
            self._data_key = key
        # ONE pipeline for the process (TF: the global batch is split over the local replicas)
        h = F.DeviceHandler(lp, None, 0, 1)
        self._b = lp.batch_size // self.G
        for s in self.subs:
            s._handlers_b = [self._b]
        if self.mode is None:
            self._choose_mode(self._b)
        return h

    def _choose_mode(self, b: int):
        """The in-graph all-reduce path, decided once (every replica the same)."""
        s0 = self.subs[0]
        n = s0.W.numel()
        plain = s0._plain_sgd
        self.twoshot = self.G >= int(os.environ.get("TDL_FX_TWOSHOT_MIN_R", "3"))
        mode = "serial"
        if self.capture and self.dc.xgmi_ok():
            from ..models import mnist_cnn as M

            self.ar = self.dc.channels(n)
            mode = "xgmi"
            probe = self._probe_step(b)
            if probe.fused_bwd and plain and os.environ.get("TDL_MNIST_FINALIZE_XCHG", "1") == "1":
                self.xchg = self.dc.channels(n, M.FINALIZE_BLOCKS, algo=0)
                mode = "xchg"
            self.mode = mode
            ok, why = self._selftest(b)
            if not ok and mode == "xchg":
                self.fallbacks.append(f"exchange-in-finalize self-test failed ({why})")
                self.mode = mode = "xgmi"
                for s in self.subs:
                    s._steps, s._graphs = {}, {}
                ok, why = self._selftest(b)
            if not ok:
                self.fallbacks.append(f"in-graph xGMI all-reduce self-test failed ({why})")
                mode = "serial"
        elif self.capture:
            self.fallbacks.append(f"in-process xGMI unavailable ({self.dc.reason})")
        self.mode = mode
        for s in self.subs:
            s._steps, s._graphs = {}, {}
        if mode == "xchg":
            self.allreduce_mode = "xgmi-in-finalize-twoshot" if self.twoshot else "xgmi-in-finalize"
        elif mode == "xgmi":
            self.allreduce_mode = "xgmi-" + ("twoshot" if self.ar[0].algo == 1 else "oneshot") + "-in-graph"
        else:
            cl = self.dc.clique()
            self.allreduce_mode = "serial-" + ("rccl-clique" if cl is not None else "copies")

    def _probe_step(self, b: int):
        from ..models import mnist_cnn as M

        s0 = self.subs[0]
        idx = torch.zeros(b, dtype=torch.int32, device=s0.device)
        with torch.cuda.device(s0.device):
            return M.FusedMnistTrainStep(s0.X, s0.Y, idx, s0.W, s0.G, s0.layout, b, self.G, s0.optimizer.lr_dev,
                                         torch.zeros(4, device=s0.device))

    def _selftest(self, b: int):
        """One real step of every replica through the chosen path (scratch step objects, replica-
        specific samples) against W0 - lr * (rank-order sum of the local gradients); parameters,
        gradients and metrics restored afterwards.  TDL_XCHG_SELFTEST=0 skips it."""
        if os.environ.get("TDL_XCHG_SELFTEST", "1") != "1":
            return True, ""
        from ..models import mnist_cnn as M

        dc = self.dc
        saved = [(s.W.clone(), s.G.clone()) for s in self.subs]
        n = len(self.subs[0].X)
        try:
            steps = []
            for r, s in enumerate(self.subs):
                idx = ((torch.arange(b, dtype=torch.int64) * 7919 + r * 104729) % n).to(torch.int32).to(s.device)
                with torch.cuda.device(s.device):
                    st = M.FusedMnistTrainStep(s.X, s.Y, idx, s.W, s.G, s.layout, b, self.G, s.optimizer.lr_dev,
                                               torch.zeros(4, device=s.device), global_batch=b * self.G)
                s._prepare_comm(st)
                steps.append(st)
            # local gradients (no exchange)
            for r, (s, st) in enumerate(zip(self.subs, steps)):
                with dc.on(r):
                    st.forward_backward(0)
                    st.finalize(False)
            dc.synchronize()
            g = saved[0][1]  # (shape only)
            total = torch.zeros_like(g, device="cpu")
            for s in self.subs:
                total += s.G.cpu()
            lr = float(self.subs[0].optimizer.lr_dev.item())
            w_ref = saved[0][0].cpu() - lr * total
            # the real path (plain SGD: the fused update; other optimizers: the in-graph gradient
            # all-reduce their kernels then consume)
            plain = self.subs[0]._plain_sgd
            for r, (s, st) in enumerate(zip(self.subs, steps)):
                with dc.on(r):
                    st.forward_backward(0)
                    if plain:
                        s._apply(st, b * self.G)
                    else:
                        st.finalize(False)
                        self.ar[r].all_reduce(s.G, s.G, 1.0)
            dc.synchronize()
            if dc.error():
                raise RuntimeError("an xGMI wait timed out")
            for st in steps:
                st.check()
            got = [(s.W if plain else s.G).cpu() for s in self.subs]
            want = w_ref if plain else total
            if os.environ.get("TDL_FAULT_XCHG_SELFTEST") == "1":
                want = want + 1.0
            if not all(torch.equal(got[0], w) for w in got[1:]):
                return False, "replicas differ"
            if not torch.allclose(got[0], want, rtol=1e-5, atol=1e-7):
                return False, f"max |result - reference| = {float((got[0] - want).abs().max()):.3g}"
            return True, ""
        except Exception as e:  # noqa: BLE001 - any failure means the serial path
            return False, f"{type(e).__name__}: {e}"
        finally:
            for s, (w, gr) in zip(self.subs, saved):
                s.W.copy_(w)
                s.G.copy_(gr)
            dc.synchronize()

    # ------------------------------------------------------------------ executions
    def warm_graphs(self, steps: int, b: Optional[int] = None):
        b = b or self._b
        if b is None:
            return
        for r, s in enumerate(self.subs):
            with torch.cuda.device(s.device):
                s.warm_graphs(steps, b)

    def _slices(self, idx: np.ndarray, K: int) -> List[np.ndarray]:
        B = self._b * self.G
        a = idx.reshape(K, B)
        return [np.ascontiguousarray(a[:, r * self._b:(r + 1) * self._b]).reshape(-1) for r in range(self.G)]

    def _take_upload(self, handler, K: int):
        idx = handler.take(K)
        if idx is None:
            return None
        Kr = idx.size // handler.b
        slot = self._slot
        self._slot = (slot + 1) % self._nslots
        # every replica's graph exists before any of this execution is launched (a capture syncs
        # its device, which must never wait on a launched replica whose peers are not launched yet)
        ents = []
        for s in self.subs:
            with torch.cuda.device(s.device):
                if not hasattr(s, "_stage"):
                    s._stage, s._stage_ev, s._slot = [None] * s._nslots, [None] * s._nslots, 0
                ents.append(s._graph_for(K, self._b, slot))
        for r, (s, sl) in enumerate(zip(self.subs, self._slices(idx, Kr))):
            with self.dc.on(r):
                s._upload(sl, ents[r][1], slot)
        return handler, K, Kr, ents

    def prefetch(self, handler, K: int) -> bool:
        K = min(int(K), self.K)
        if self._ready is not None:
            return self._ready[1] == K
        self._ready = self._take_upload(handler, K)
        return self._ready is not None

    def run_train(self, handler, steps: int) -> int:
        gc.freeze()
        done = 0
        b = self._b
        self._sync_optimizers()
        while done < steps:
            K = min(self.K, steps - done)
            ent, self._ready = self._ready, None
            if ent is not None and (ent[0] is not handler or ent[1] != K):
                raise RuntimeError("mirrored fused trainer: prefetched execution does not match the requested steps")
            if ent is None:
                ent = self._take_upload(handler, K)
            if ent is None:
                one = handler.next_ragged()
                if one is None:
                    break
                self._ragged_step(one[0])
                done += 1
                continue
            _, _, Kr, ents = ent
            for r, s in enumerate(self.subs):
                with self.dc.on(r):
                    s.optimizer._sync_lr()
            if self.mode == "serial":
                self._serial_execution(ents, Kr)
            else:
                for r, (s, (graph, _, st)) in enumerate(zip(self.subs, ents)):
                    with self.dc.on(r):
                        if Kr < K or graph is None:
                            for k in range(Kr):
                                s._train_step(st, k * b, b * self.G)
                        else:
                            graph.replay()
            for s in self.subs:
                s.optimizer.iterations += Kr
            done += Kr
        return done

    def _serial_execution(self, ents, Kr: int):
        """Per step: every replica's forward/backward/finalize (graph replay when captured), then the
        group all-reduce of the G gradient slabs, then every replica's optimizer update."""
        b = self._b
        for k in range(Kr):
            for r, (s, (graph, _, st)) in enumerate(zip(self.subs, ents)):
                with self.dc.on(r):
                    if isinstance(graph, list) and len(graph) > k:
                        graph[k].replay()
                    else:
                        st.forward_backward(k * b)
                        st.finalize(False)
            self._reduce_update(k)

    def _reduce_update(self, k: int = 0):
        self.dc.all_reduce([s.G for s in self.subs], "sum")
        for r, s in enumerate(self.subs):
            with self.dc.on(r):
                s._step_k = k
                s._update()

    def _ragged_step(self, g: np.ndarray):
        """A partial global batch: split over the replicas, local gradients, group all-reduce
        (serial), updates."""
        sizes = input_lib.split_sizes(len(g), self.G)
        lo = 0
        for r, s in enumerate(self.subs):
            n = sizes[r]
            ids = g[lo:lo + n]
            lo += n
            with self.dc.on(r):
                s.optimizer._sync_lr()
                if n == 0:
                    s.G.zero_()
                    continue
                key = ("ragged", n)
                buf = s._ragged_bufs.get(key)
                if buf is None:
                    buf = torch.zeros(n, dtype=torch.int32, device=s.device)
                    s._ragged_bufs[key] = buf
                buf.copy_(torch.from_numpy(np.ascontiguousarray(ids, dtype=np.int32)))
                st = s._step(n, buf, len(g))
                st.forward_backward(0)
                st.finalize(False)
        self._reduce_update(0)
        for s in self.subs:
            s.optimizer.iterations += 1

    # ------------------------------------------------------------------ metrics / checks
    def reset_metrics(self):
        for s in self.subs:
            s.metrics_dev.zero_()
        self.subs[0].reset_metrics()

    def logs(self) -> Dict[str, float]:
        self.dc.synchronize()
        for s in self.subs:
            for st in list(s._steps.values()):
                st.check()
        if self.dc.error():
            raise RuntimeError("in-process xGMI all-reduce: a device's wait for a peer timed out "
                               "(replicas out of step)")
        tot = np.zeros(3, dtype=np.float64)
        for s in self.subs:
            tot += s.metrics_dev[:3].double().cpu().numpy()
        loss_sum, correct, count = (float(v) for v in tot)
        out = {"loss": loss_sum / max(count, 1.0)}
        for m in self.model.compiled_metrics:
            out[m.name] = correct / max(count, 1.0)
        dev0 = self.subs[0].device
        lt = self.model._loss_tracker
        lt._to(dev0)
        lt.total._value.fill_(loss_sum)
        lt.count._value.fill_(count)
        for m in self.model.compiled_metrics:
            m._to(dev0)
            m.total._value.fill_(correct)
            m.count._value.fill_(count)
        return out

    def finish(self):
        self.dc.synchronize()

    def check_replicas(self) -> bool:
        """Collective-free replica check (one process): every replica's parameters must equal
        replica 0's bit for bit; a mismatch is repaired from replica 0 and the in-graph xGMI path
        is dropped (serial all-reduce from then on)."""
        self.dc.synchronize()
        w0 = self.subs[0].W
        same = all(torch.equal(w0, s.W.to(w0.device)) for s in self.subs[1:])
        if not same:
            import warnings

            warnings.warn("mirrored replicas diverged; restored from replica 0, using the serial all-reduce")
            self.broadcast_from_primary()
            self.on_replica_divergence()
        return same

    def replicas_identical(self) -> bool:
        self.dc.synchronize()
        w0 = self.subs[0].W
        return all(torch.equal(w0, s.W.to(w0.device)) for s in self.subs[1:])

    def on_replica_divergence(self):
        self.mode = "serial"
        self.allreduce_mode = "serial-" + ("rccl-clique" if self.dc.clique() is not None else "copies")
        for s in self.subs:
            s._steps, s._graphs = {}, {}

    # ------------------------------------------------------------------ evaluate / predict
    def evaluate(self, dataset, steps: Optional[int] = None):
        lp = DD.lower(dataset)
        if lp is None or lp.batch_size % self.G:
            return None
        cols = [s._eval_columns(lp, labels=True) for s in self.subs]
        if any(c is None for c in cols):
            return None
        h = F.DeviceHandler(lp, None, 0, 1)
        h._async = False
        batches = []
        try:
            while steps is None or len(batches) < steps:
                g = h._next_global()
                if g is None:
                    break
                batches.append(g)
        finally:
            h.close()
        mets = []
        for r, (s, (X, Y, cache)) in enumerate(zip(self.subs, cols)):
            with self.dc.on(r):
                m = torch.zeros(4, dtype=torch.float32, device=s.device)
                s._forward_batches(_SliceHandler(batches, r, self.G, lp.batch_size), X, Y, cache, None, m)
                mets.append(m)
        self.dc.synchronize()
        tot = np.zeros(3, dtype=np.float64)
        for m in mets:
            tot += m[:3].double().cpu().numpy()
        loss_sum, correct, count = (float(v) for v in tot)
        out = {"loss": loss_sum / max(count, 1.0)}
        for m in self.model.compiled_metrics:
            out[m.name] = correct / max(count, 1.0)
        return out

    def predict(self, dataset, steps: Optional[int] = None):
        return self.subs[0].predict(dataset, steps)


class _ListHandler:
    """A replica's pre-split batches of one execution (ThreadedGroupTrainer)."""

    def __init__(self, batches, sizes):
        self.batches, self.sizes = list(batches), list(sizes)

    def next(self):
        if not self.batches:
            raise StopIteration
        self.sizes_cur = self.sizes.pop(0)
        return self.batches.pop(0)

    def global_size(self, local_n: int) -> int:
        return self.sizes_cur


class GroupHostHandler:
    """ONE host input pipeline for the whole process; each global batch is split into per-replica
    slices (split_sizes), as TF's single-worker MirroredStrategy distributes a dataset."""

    def __init__(self, dataset, G: int):
        from ..data import dataset as D

        self.D = D
        self.dataset = dataset
        self.G = G
        self._it = None
        self.dist = self  # (fit reads handler.dist.cardinality())

    def cardinality(self):
        return self.dataset.cardinality()

    def new_iterator(self):
        self._it = iter(self.dataset)

    def take(self, n: int):
        """Up to n global batches -> ([per-replica batch lists], [global sizes])."""
        if self._it is None:
            self.new_iterator()
        per = [[] for _ in range(self.G)]
        sizes = []
        for _ in range(n):
            try:
                batch = next(self._it)
            except StopIteration:
                break
            m = len(self.D.flatten(batch)[0])
            sz = input_lib.split_sizes(m, self.G)
            lo = 0
            for r in range(self.G):
                per[r].append(self.D.map_structure(lambda t, lo=lo, hi=lo + sz[r]: t[lo:hi], batch))
                lo += sz[r]
            sizes.append(m)
        return per, sizes


class ThreadedGroupTrainer:
    """See module docstring: the generic engine of every replica, steps in turn-taking threads."""

    kind = "generic"
    is_group = True

    def __init__(self, model, models, group):
        self.model, self.models, self.group = model, models, group
        self.G = group.G

        def make(r):
            from .trainer import GenericTrainer

            return GenericTrainer(models[r])

        self.trainers = group.run(make)
        for m, t in zip(models[1:], self.trainers[1:]):
            m._trainer = t
        self.optimizer = model.optimizer
        self.broadcast_from_primary()

    def replica_trainer(self, model):
        for m, t in zip(self.models, self.trainers):
            if m is model:
                return t
        raise KeyError("model is not a replica of this trainer")

    def broadcast_from_primary(self):
        t0 = self.trainers[0]
        for t in self.trainers[1:]:
            t.W.copy_(t0.W.to(t.W.device))
            if t.model._NT is not None and t0.model._NT is not None:
                t.model._NT.copy_(t0.model._NT.to(t.model._NT.device))
            _copy_optimizer_state(t.optimizer, t0.optimizer)

    def prepare(self, dataset):
        return None  # no device-resident path: host pipeline (host_handler)

    def host_handler(self, dataset):
        return GroupHostHandler(dataset, self.G)

    def run_train(self, handler: GroupHostHandler, steps: int) -> int:
        per, sizes = handler.take(steps)
        if not sizes:
            return 0
        o0 = self.trainers[0].optimizer
        for t in self.trainers[1:]:
            _sync_optimizer(t.optimizer, o0)
        out = self.group.run(lambda r: self.trainers[r].run_train(_ListHandler(per[r], sizes), len(sizes)))
        return out[0]

    def reset_metrics(self):
        for t in self.trainers:
            t.reset_metrics()

    def logs(self) -> Dict[str, float]:
        return self.group.run(lambda r: self.trainers[r].logs())[0]

    def finish(self):
        for t in self.trainers:
            t.finish()

    def check_replicas(self) -> bool:
        w0 = self.trainers[0].W
        same = all(torch.equal(w0, t.W.to(w0.device)) for t in self.trainers[1:])
        if not same:
            import warnings

            warnings.warn("mirrored replicas diverged; restored from replica 0")
            self.broadcast_from_primary()
        return same
