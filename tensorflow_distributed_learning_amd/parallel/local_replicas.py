"""Single-process multi-device MirroredStrategy: ONE process drives G local devices
(tf_dist_example.py:13 ``tf.distribute.MirroredStrategy()``, README.md:15-19: one replica per GPU,
every variable mirrored onto each device, the script body runs once).

The framework's scaling mode stays one process per GPU (parallel/launch.py, torchrun); this module
is what a plain script gets from ``MirroredStrategy(devices=[...G devices...])``, as in TF:

* :class:`LocalReplicaGroup` -- the G replicas of the process.  ``run(fn)`` executes ``fn(r)`` for
  every replica concurrently, replica 0 on the calling thread and replicas 1..G-1 on worker
  threads, each with its own device and its own HIP stream, so the replicas' kernels are
  independent streams on independent devices (or share one GPU under ``TDL_SHARE_GPU=1``).
* :class:`LocalReplicaCommunicator` -- the cross-replica collectives between those threads.  Every
  all-reduce is a host rendezvous followed by device work only: each replica's stream waits on
  its peers' "ready" events, sums the G tensors IN RANK ORDER on its own device (peer tensors are
  read directly: same device, or a peer-to-peer copy over xGMI), signals "read done", and only
  after every peer has read its tensor writes the sum back.  The f32 adds run in the same order on
  every replica, so replicas stay bit-identical.  Nothing spins on the device, so G replicas can
  share one GPU without any residency assumption.
* :class:`ReplicaView` -- replica r's strategy object (device r, rank r of G, its communicator).
  Replica r's model clone is created in its view's ``scope()``, so the engines (fused MNIST
  kernels, generic autograd trainer) run on it exactly as they run in a replica process.

``keras.Model.fit / evaluate / predict`` on a model of such a strategy run their body once per
replica inside :meth:`LocalReplicaGroup.run` (keras/models.py ``_local_run``): replica 0 is the
user's model, replicas 1..G-1 are clones with replica 0's weights; callbacks, progress bar and
History belong to replica 0 (TF runs them once).
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch

from .communicator import Communicator, _Done


class LocalReplicaGroup:
    """G replicas of ONE process (see module docstring)."""

    def __init__(self, devices: List[torch.device], timeout: float = 600.0):
        self.devices = [torch.device(d) for d in devices]
        self.G = len(self.devices)
        self.timeout = float(timeout)
        self._barrier = threading.Barrier(self.G, timeout=self.timeout)
        self.slots: List[Optional[torch.Tensor]] = [None] * self.G
        self.ready: List[Optional[torch.cuda.Event]] = [None] * self.G
        self.done: List[Optional[torch.cuda.Event]] = [None] * self.G
        self._tls = threading.local()
        self._streams = {}
        self.comms = [LocalReplicaCommunicator(r, self) for r in range(self.G)]
        self.views: List["ReplicaView"] = []

    # ---- regions ---------------------------------------------------------------------------
    def replica(self) -> Optional[int]:
        """The replica the calling thread executes inside :meth:`run`, else None."""
        return getattr(self._tls, "rank", None)

    def in_region(self) -> bool:
        return self.replica() is not None

    def stream(self, r: int):
        d = self.devices[r]
        if d.type != "cuda":
            return None
        s = self._streams.get(r)
        if s is None:
            s = self._streams[r] = torch.cuda.Stream(d)
        return s

    def run(self, fn: Callable[[int], object]) -> list:
        """``fn(r)`` for every replica r concurrently; returns the G results.  The first error of any
        replica is raised (the others are released from their rendezvous instead of waiting)."""
        if self.in_region():
            raise RuntimeError("LocalReplicaGroup.run: already inside a replica region")
        results: list = [None] * self.G
        errors: list = [None] * self.G
        # the caller's current stream of every device: each replica stream starts behind it (e.g.
        # weights the caller just wrote) and it continues behind every replica's work
        base = {}
        for d in self.devices:
            if d.type == "cuda" and d not in base:
                base[d] = torch.cuda.current_stream(d)

        def body(r: int):
            self._tls.rank = r
            dev, s = self.devices[r], self.stream(r)
            try:
                if s is not None:
                    torch.cuda.set_device(dev)
                    s.wait_stream(base[dev])
                    with torch.cuda.stream(s):
                        results[r] = fn(r)
                else:
                    results[r] = fn(r)
            except BaseException as e:  # noqa: BLE001 - re-raised on the calling thread
                errors[r] = e
                self._barrier.abort()
            finally:
                self._tls.rank = None

        threads = [threading.Thread(target=body, args=(r,), name=f"tdl-replica-{r}", daemon=True)
                   for r in range(1, self.G)]
        for t in threads:
            t.start()
        body(0)
        for t in threads:
            t.join()
        if self.devices[0].type == "cuda":
            torch.cuda.set_device(self.devices[0])
        for r in range(self.G):
            s = self._streams.get(r)
            if s is not None:
                base[self.devices[r]].wait_stream(s)
        if self._barrier.broken:
            self._barrier.reset()
        real = [e for e in errors if e is not None and not isinstance(e, threading.BrokenBarrierError)]
        if real or any(e is not None for e in errors):
            raise (real or [e for e in errors if e is not None])[0]
        return results

    def wait(self):
        self._barrier.wait()


class LocalReplicaCommunicator(Communicator):
    """Collectives between the replica threads of one :class:`LocalReplicaGroup` (module docstring).
    Outside a replica region (the user's thread acting as replica 0 alone, e.g. building weights
    before fit) a broadcast from replica 0 is a no-op; the other collectives need every replica."""

    name = "local-threads"
    capturable = False  # host rendezvous: never inside a hipGraph capture
    threaded = True  # engines: no whole-execution graph capture (concurrent captures in threads)

    def __init__(self, rank: int, group: LocalReplicaGroup):
        super().__init__(rank, group.G, group.devices[rank])
        self.group = group
        self.algorithm = "in-process rank-order sum"
        self.xgmi = None

    def _solo(self) -> bool:
        return not self.group.in_region()

    def _publish(self, t: torch.Tensor):
        g = self.group
        g.slots[self.rank] = t
        if t.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(t.device))
            g.ready[self.rank] = ev
        g.wait()
        if t.is_cuda:
            s = torch.cuda.current_stream(t.device)
            for q in range(self.world_size):
                if q != self.rank and g.ready[q] is not None:
                    s.wait_event(g.ready[q])
                    pd = g.slots[q].device
                    if pd != t.device:
                        # a peer-to-peer copy is issued on the SOURCE device's current stream (of this
                        # thread), then joined into ours by torch: order it behind the peer's work too
                        torch.cuda.current_stream(pd).wait_event(g.ready[q])
        return list(g.slots)

    def _finish(self, t: torch.Tensor):
        """Every peer has issued its reads of every published tensor before anyone overwrites its
        own (device order through the 'done' events)."""
        g = self.group
        if t.is_cuda:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(t.device))
            g.done[self.rank] = ev
        g.wait()
        if t.is_cuda:
            s = torch.cuda.current_stream(t.device)
            for q in range(self.world_size):
                if q != self.rank and g.done[q] is not None:
                    s.wait_event(g.done[q])

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self._solo():
            raise RuntimeError("cross-replica all-reduce outside a replica region (MirroredStrategy.run / fit)")
        srcs = self._publish(t)
        acc = srcs[0].to(t.device, copy=True)
        for q in range(1, self.world_size):  # rank order on every replica: bit-identical results
            x = srcs[q].to(t.device)
            if op in ("sum", "mean"):
                acc += x
            elif op == "max":
                acc = torch.maximum(acc, x)
            elif op == "min":
                acc = torch.minimum(acc, x)
            elif op == "prod":
                acc *= x
            else:
                raise ValueError(f"unknown reduce op {op}")
        if op == "mean":
            acc = acc / self.world_size if acc.is_floating_point() else acc // self.world_size
        self._finish(t)
        t.copy_(acc)
        return t

    def all_reduce_async(self, t, op="sum"):
        self.all_reduce(t, op)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self._solo():
            if src != self.rank:
                raise RuntimeError("cross-replica broadcast outside a replica region")
            return t  # only replica 0 exists outside a region: nothing to send
        srcs = self._publish(t)
        val = srcs[src].to(t.device, copy=True) if self.rank != src else None
        self._finish(t)
        if val is not None:
            t.copy_(val)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self._solo():
            raise RuntimeError("cross-replica all-gather outside a replica region")
        srcs = self._publish(t)
        out = torch.stack([s.to(t.device) for s in srcs])
        self._finish(t)
        return out

    def barrier(self) -> None:
        if self._solo():
            return
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self.group.wait()

    def device_bucket_capable(self, numels) -> bool:
        return False  # one all-reduce after backward, on the replica's own thread (no hooks)


def make_views(strategy, group: LocalReplicaGroup) -> list:
    """Replica r's strategy object for r = 1..G-1 (replica 0 is ``strategy`` itself)."""
    views = []
    for r in range(1, group.G):
        views.append(ReplicaView(strategy, r, group))
    return views


class ReplicaView:
    """Replica r of a single-process MirroredStrategy as a strategy object of its own: device r,
    rank r of G, the group's communicator r.  Models built in ``view.scope()`` mirror replica r."""

    def __init__(self, parent, r: int, group: LocalReplicaGroup):
        from .strategy import StrategyExtended

        self._parent = parent
        self._local_group = group
        self.cluster_resolver = None
        self.extended = StrategyExtended(self, group.devices[r], r, group.G, r, group.comms[r],
                                         parent.extended.communication_options)

    @property
    def num_replicas_in_sync(self) -> int:
        return self.extended.world_size

    def scope(self):
        from .strategy import Strategy

        return Strategy.scope(self)

    def __getattr__(self, name):  # everything else behaves like the parent strategy
        return getattr(self._parent, name)

    def __repr__(self):
        return f"ReplicaView(replica={self.extended.rank}/{self.num_replicas_in_sync}, device={self.extended.device})"
