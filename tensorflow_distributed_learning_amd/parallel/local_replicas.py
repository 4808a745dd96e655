"""Single-process multi-device MirroredStrategy: ONE process drives G local devices
(tf_dist_example.py:13 ``tf.distribute.MirroredStrategy()``, README.md:15-19: one replica per GPU,
every variable mirrored onto each device, the script body runs once).

The framework's scaling mode stays one process per GPU (parallel/launch.py, torchrun); this module
is what a plain script gets from ``MirroredStrategy()`` / ``MirroredStrategy(devices=[...])``, as in TF:

* ``fit`` of the reference CNN runs on the device path (engine/mirrored.py): ONE host thread
  launches every device's captured execution graph back to back, and the gradient all-reduce
  happens inside those graphs (the xGMI exchange in the fused finalize kernel) -- no replica
  threads, no host rendezvous per step.
* :class:`LocalReplicaGroup` -- the G replicas of the process, for everything else (``strategy.run``
  of user functions, the generic engine's steps).  ``run(fn)`` executes ``fn(r)`` for every replica
  in a thread of its own, with its own device and HIP stream, but the threads TAKE TURNS, as TF's
  mirrored run does (its replica threads run one at a time and hand control over at merge calls):
  replica r runs until it reaches a collective, then replica r+1 runs, and when the last replica
  has reached it the collective completes and replica 0 continues.  Host work is therefore never
  concurrent (process-global state such as a GradientTape or autocast flags stays consistent),
  while each replica's device work is asynchronous on its own stream.
* :class:`LocalReplicaCommunicator` -- replica r's view of the group's collectives.  The LAST replica
  to arrive issues the collective for all G at once through the group's
  :class:`~.device_group.DeviceGroupComm` (xGMI kernels over locally connected channels, an RCCL
  clique, or event-ordered rank-order copies), like TF's batch all-reduce in a merge call.
* :class:`ReplicaView` -- replica r's strategy object (device r, rank r of G, its communicator).
  Replica r's model clone is created in its view's ``scope()``.
"""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

import torch

from .communicator import Communicator, _Done


class _Broken(Exception):
    pass


# the device of the replica the calling thread executes inside LocalReplicaGroup.run (None outside):
# a variable of replica 0 read there is mirrored onto that device (parallel/values.py Variable.value)
CURRENT = threading.local()


def current_device() -> Optional[torch.device]:
    return getattr(CURRENT, "device", None)


class LocalReplicaGroup:
    """G replicas of ONE process (see module docstring)."""

    def __init__(self, devices: List[torch.device], timeout: float = 600.0):
        self.devices = [torch.device(d) for d in devices]
        self.G = len(self.devices)
        self.timeout = float(timeout)
        self._tls = threading.local()
        self._streams = {}
        self.comms = [LocalReplicaCommunicator(r, self) for r in range(self.G)]
        self.views: List["ReplicaView"] = []
        self._dev_comm = None
        # turn-taking state (guarded by _cv)
        self._cv = threading.Condition()
        self._turn: Optional[int] = None
        self._finished: List[bool] = [True] * self.G
        self._arrived: List[Optional[object]] = [None] * self.G  # per replica: the payload it brought
        self._gen = 0
        self._result = None
        self._broken: Optional[BaseException] = None

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

    def device_comm(self):
        """The group's single-thread cross-device communicator (parallel/device_group.py)."""
        if self._dev_comm is None:
            from .device_group import DeviceGroupComm

            self._dev_comm = DeviceGroupComm(self.devices, [self.stream(r) for r in range(self.G)],
                                             timeout=self.timeout)
        return self._dev_comm

    # ---- turn taking -----------------------------------------------------------------------
    def _pass_turn(self, r: int):
        """Caller holds _cv: give the turn to the next unfinished replica after r (wrapping)."""
        for k in range(1, self.G + 1):
            q = (r + k) % self.G
            if not self._finished[q]:
                if self._arrived[q] is not None and self._broken is None:
                    # the turn came back to a replica already waiting at the open collective: every
                    # live replica is there, yet a finished one never arrived -- it can never complete
                    self._broken = RuntimeError(
                        "replicas reached different collectives (a replica finished without the collective "
                        "its peers wait in)")
                self._turn = q
                self._cv.notify_all()
                return
        self._turn = None
        self._cv.notify_all()

    def _wait_turn(self, r: int, gen: Optional[int] = None):
        """Caller holds _cv: block until it is replica r's turn (and, with ``gen``, the rendezvous
        of generation ``gen`` has completed)."""
        ok = self._cv.wait_for(lambda: self._broken is not None or
                               (self._turn == r and (gen is None or self._gen != gen)), timeout=self.timeout)
        if self._broken is not None:
            raise _Broken() from None
        if not ok:
            self._broken = TimeoutError(f"replica {r}: a peer replica did not reach the collective within "
                                        f"{self.timeout:.0f} s")
            self._cv.notify_all()
            raise self._broken

    def rendezvous(self, payload=None, combine: Optional[Callable[[list], object]] = None):
        """Collective point of the calling replica: its payload is deposited and the turn passes on;
        the LAST replica to arrive runs ``combine(payloads)`` (for all G at once), whose result every
        replica returns.  Replicas then continue one at a time in rank order."""
        r = self.replica()
        if r is None:
            raise RuntimeError("cross-replica collective outside a replica region (MirroredStrategy.run / fit)")
        with self._cv:
            if self._broken is not None:
                raise _Broken()
            self._arrived[r] = (payload,)
            if all(a is not None for a in self._arrived):
                payloads = [a[0] for a in self._arrived]
                self._arrived = [None] * self.G
                try:
                    self._result = combine(payloads) if combine is not None else None
                except BaseException as e:
                    self._broken = e
                    self._cv.notify_all()
                    raise
                self._gen += 1
                res = self._result
                self._turn = 0
                self._cv.notify_all()
                if r != 0:
                    self._wait_turn(r)
                return res
            gen = self._gen
            self._pass_turn(r)
            self._wait_turn(r, gen)
            return self._result

    def wait(self):
        self.rendezvous()

    def run(self, fn: Callable[[int], object]) -> list:
        """``fn(r)`` for every replica r, the replicas taking turns (module docstring); returns the
        G results.  The first error of any replica is raised (the others are released from their
        rendezvous instead of waiting)."""
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
        with self._cv:
            self._finished = [False] * self.G
            self._arrived = [None] * self.G
            self._broken = None
            self._turn = 0

        def body(r: int):
            self._tls.rank = r
            dev, s = self.devices[r], self.stream(r)
            CURRENT.device = dev
            try:
                with self._cv:
                    self._wait_turn(r)
                if s is not None:
                    torch.cuda.set_device(dev)
                    s.wait_stream(base[dev])
                    with torch.cuda.stream(s):
                        results[r] = fn(r)
                else:
                    results[r] = fn(r)
            except BaseException as e:  # noqa: BLE001 - re-raised on the calling thread
                errors[r] = e
                with self._cv:
                    if self._broken is None:
                        self._broken = e
                    self._cv.notify_all()
            finally:
                self._tls.rank = None
                CURRENT.device = None
                with self._cv:
                    self._finished[r] = True
                    if self._turn == r:
                        self._pass_turn(r)

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
        real = [e for e in errors if e is not None and not isinstance(e, _Broken)]
        if real:
            raise real[0]
        if any(e is not None for e in errors):
            if isinstance(self._broken, BaseException) and not isinstance(self._broken, _Broken):
                raise self._broken
            raise RuntimeError("a replica region was aborted")
        return results


class LocalReplicaCommunicator(Communicator):
    """Collectives between the replica threads of one :class:`LocalReplicaGroup` (module docstring).
    Outside a replica region (the user's thread acting as replica 0 alone, e.g. building weights
    before fit) a broadcast from replica 0 is a no-op; the other collectives need every replica."""

    name = "local-threads"
    capturable = False  # host rendezvous: never inside a hipGraph capture
    threaded = True  # engines: no whole-execution graph capture from replica threads

    def __init__(self, rank: int, group: LocalReplicaGroup):
        super().__init__(rank, group.G, group.devices[rank])
        self.group = group
        self.xgmi = None

    @property
    def algorithm(self) -> str:
        dc = self.group._dev_comm
        return "in-process " + (dc.algorithm if dc is not None else "rank-order sum")

    def _solo(self) -> bool:
        return not self.group.in_region()

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if self._solo():
            raise RuntimeError("cross-replica all-reduce outside a replica region (MirroredStrategy.run / fit)")
        g = self.group
        g.rendezvous(t, lambda ts: g.device_comm().all_reduce(ts, op))
        return t

    def all_reduce_async(self, t, op="sum"):
        self.all_reduce(t, op)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self._solo():
            if src != self.rank:
                raise RuntimeError("cross-replica broadcast outside a replica region")
            return t  # only replica 0 exists outside a region: nothing to send
        g = self.group
        g.rendezvous(t, lambda ts: g.device_comm().broadcast(ts, src))
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        if self._solo():
            raise RuntimeError("cross-replica all-gather outside a replica region")
        g = self.group
        outs = g.rendezvous(t, lambda ts: g.device_comm().all_gather(ts))
        return outs[self.rank]

    def barrier(self) -> None:
        if self._solo():
            return
        if self.device.type == "cuda":
            torch.cuda.current_stream(self.device).synchronize()
        self.group.wait()

    def check_health(self) -> None:
        dc = self.group._dev_comm
        if dc is not None and dc.error():
            raise RuntimeError("in-process xGMI all-reduce: a replica's wait timed out")

    def device_bucket_capable(self, numels) -> bool:
        return False  # one all-reduce after backward (no hooks inside autograd)


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
