"""Distribution strategies: synchronous mirrored data parallelism (README.md:11-29).

MI355X-first process model: ONE PROCESS PER REPLICA (per GPU).  ``num_replicas_in_sync`` is the
number of replica processes in the job; cross-replica reductions go through a
:class:`~.communicator.Communicator` (RCCL over xGMI for GPU replicas, the native TCP ring for
CPU replicas / ``CollectiveCommunication.RING``).

* :class:`MirroredStrategy` (README.md:15-19, tf_dist_example.py:13): all GPUs of one node.
  Started by a launcher (``torchrun``/``python -m tensorflow_distributed_learning_amd.launch``)
  each process becomes one replica (the scaling mode).  Started as a plain script with several
  devices selected, ONE process drives them all, as in TF (parallel/local_replicas.py: a replica
  thread per device, in-process rank-order all-reduces, the script body runs once);
  ``spawn=True`` / ``TDL_MIRRORED_MODE=process`` instead spawns one child process per extra device
  (the parent is replica 0) before touching the GPU.
* :class:`MultiWorkerMirroredStrategy` (tf_dist_example.py:12, README.md:21-29): the cluster comes
  from TF_CONFIG; tasks meet at the chief over the native TCP store (cluster/rendezvous.py) and
  every GPU of every worker is one replica.  No TF_CONFIG / a single task degrades to
  MirroredStrategy; no GPU degrades to CPU replicas with ring all-reduce (README.md:34).
"""
from __future__ import annotations

import atexit
import contextlib
import enum
import os
import threading
from typing import Any, Callable, List, Optional, Sequence

import torch

from ..cluster.tf_config import ClusterConfigError, TFConfig, TFConfigClusterResolver, parse_tf_config
from .communication import (
    CollectiveCommunication,
    CommunicationImplementation,
    CommunicationOptions,
    collective_timeout,
    default_timeout,
    normalize_options,
)
from .communicator import Communicator, LocalCommunicator, RingCommunicator, TorchCommunicator


class ReduceOp(enum.Enum):
    SUM = "SUM"
    MEAN = "MEAN"


_state = threading.local()


def _stack() -> List["Strategy"]:
    if not hasattr(_state, "stack"):
        _state.stack = []
    return _state.stack


def get_strategy() -> "Strategy":
    s = _stack()
    if s:
        return s[-1]
    return _default_strategy()


def has_strategy() -> bool:
    return bool(_stack())


def in_cross_replica_context() -> bool:
    return getattr(_state, "replica_ctx", None) is None


def get_replica_context() -> Optional["ReplicaContext"]:
    ctx = getattr(_state, "replica_ctx", None)
    if ctx is not None:
        return ctx
    if not has_strategy():
        return ReplicaContext(_default_strategy())
    return None


_DEFAULT = None


def _default_strategy() -> "Strategy":
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = _DefaultStrategy()
    return _DEFAULT


def parse_device(d) -> torch.device:
    """'/gpu:1', 'GPU:1', '/job:worker/replica:0/task:0/device:GPU:1', 'cuda:1', '/cpu:0' -> torch.device"""
    if isinstance(d, torch.device):
        return d
    s = str(d).strip().lower()
    if "device:" in s:
        s = s.split("device:")[-1]
    s = s.lstrip("/")
    if s.startswith("gpu") or s.startswith("cuda"):
        idx = s.split(":")[-1] if ":" in s else "0"
        return torch.device("cuda", int(idx))
    if s.startswith("cpu"):
        return torch.device("cpu")
    raise ValueError(f"unrecognised device spec {d!r}")


def _launched() -> Optional[dict]:
    """Replica placement provided by a launcher (torchrun-compatible env)."""
    env = os.environ
    if "WORLD_SIZE" in env and "RANK" in env:
        return {
            "rank": int(env["RANK"]),
            "world_size": int(env["WORLD_SIZE"]),
            "local_rank": int(env.get("LOCAL_RANK", env["RANK"])),
            "local_world_size": int(env.get("LOCAL_WORLD_SIZE", env["WORLD_SIZE"])),
        }
    return None


class ReplicaContext:
    """tf.distribute.ReplicaContext: what `strategy.run` functions see."""

    def __init__(self, strategy: "Strategy"):
        self.strategy = strategy

    @property
    def num_replicas_in_sync(self) -> int:
        return self.strategy.num_replicas_in_sync

    @property
    def replica_id_in_sync_group(self) -> int:
        return self.strategy.extended.rank

    def all_reduce(self, reduce_op, value):
        return self.strategy.extended.all_reduce(reduce_op, value)

    def merge_call(self, merge_fn, args=(), kwargs=None):
        with _cross_replica():
            return merge_fn(self.strategy, *args, **(kwargs or {}))


@contextlib.contextmanager
def _replica(ctx):
    prev = getattr(_state, "replica_ctx", None)
    _state.replica_ctx = ctx
    try:
        yield
    finally:
        _state.replica_ctx = prev


@contextlib.contextmanager
def _cross_replica():
    prev = getattr(_state, "replica_ctx", None)
    _state.replica_ctx = None
    try:
        yield
    finally:
        _state.replica_ctx = prev


class StrategyExtended:
    """Per-process replica placement + communicator (tf.distribute.StrategyExtended)."""

    def __init__(self, strategy, device: torch.device, rank: int, world_size: int, local_rank: int,
                 communicator: Communicator, options: CommunicationOptions, tf_config: Optional[TFConfig] = None,
                 rendezvous=None):
        self._strategy = strategy
        if device.type == "cuda" and os.environ.get("TDL_HIP_SCHEDULE"):
            from ..utils import hipsync

            hipsync.configure(devices=[device.index or 0])  # this replica's device only
        self.device = device
        self.rank = rank
        self.world_size = world_size
        self.local_rank = local_rank
        self.communicator = communicator
        self.communication_options = options
        self.tf_config = tf_config
        self.rendezvous = rendezvous

    @property
    def worker_devices(self):
        return (str(self.device),)

    @property
    def parameter_devices(self):
        return (str(self.device),)

    @property
    def task_type(self):
        if self.tf_config and self.tf_config.task:
            return self.tf_config.task.type
        return None

    @property
    def task_id(self):
        if self.tf_config and self.tf_config.task:
            return self.tf_config.task.index
        return None

    @property
    def is_chief(self) -> bool:
        """The chief does checkpoints / event logs (README.md:51).  With several replica
        processes per task, only global rank 0 (the chief task's first replica) acts."""
        return self.rank == 0

    should_checkpoint = property(lambda self: self.is_chief)
    should_save_summary = property(lambda self: self.is_chief)
    experimental_should_init = property(lambda self: True)
    experimental_between_graph = property(lambda self: True)

    def all_reduce(self, reduce_op, value):
        op = reduce_op.value if isinstance(reduce_op, ReduceOp) else str(reduce_op).upper()
        t = torch.as_tensor(value)
        if not t.is_floating_point() and op == "MEAN":
            t = t.double()
        t = t.clone()
        self.communicator.all_reduce(t, "mean" if op == "MEAN" else "sum")
        return t

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        return self.communicator.broadcast(t, src)


class Strategy:
    """Base class (tf.distribute.Strategy)."""

    def __init__(self, extended: StrategyExtended, cluster_resolver=None):
        self.extended = extended
        self.cluster_resolver = cluster_resolver
        self._closed = False
        atexit.register(self.shutdown)

    # --------------------------------------------------------------------------------------
    @property
    def num_replicas_in_sync(self) -> int:
        return self.extended.world_size

    @contextlib.contextmanager
    def scope(self):
        """Variables (models) created in this scope are mirrored onto every replica."""
        _stack().append(self)
        try:
            yield self
        finally:
            _stack().pop()

    _local_group = None  # single-process multi-device MirroredStrategy (parallel/local_replicas.py)

    def _replica_strategy(self, r: int):
        """Replica r's strategy object in single-process multi-device mode (r = 0: self)."""
        return self if r == 0 else self._local_group.views[r - 1]

    def run(self, fn: Callable, args=(), kwargs=None, options=None):
        g = self._local_group
        if g is None or g.in_region():
            with self.scope(), _replica(ReplicaContext(self)):
                return fn(*args, **(kwargs or {}))
        from .values import PerReplica

        def pick(v, r):
            if isinstance(v, PerReplica):
                return v.values[r]
            if isinstance(v, dict):
                return {k: pick(x, r) for k, x in v.items()}
            if isinstance(v, (tuple, list)):
                return type(v)(pick(x, r) for x in v)
            return v

        def one(r):
            st = self._replica_strategy(r)
            a = tuple(pick(v, r) for v in args)
            kw = {k: pick(v, r) for k, v in (kwargs or {}).items()}
            with st.scope(), _replica(ReplicaContext(st)):
                return fn(*a, **kw)

        out = g.run(one)
        if isinstance(out[0], (tuple, list)):  # a structure of per-replica values
            return type(out[0])(PerReplica([o[i] for o in out]) for i in range(len(out[0])))
        if isinstance(out[0], dict):
            return {k: PerReplica([o[k] for o in out]) for k in out[0]}
        return PerReplica(out)

    def reduce(self, reduce_op, value, axis=None):
        """Cross-replica reduction of a per-replica value (optionally along `axis` first)."""
        op = reduce_op.value if isinstance(reduce_op, ReduceOp) else str(reduce_op).upper()
        from .values import PerReplica

        if isinstance(value, PerReplica):  # single-process replicas: reduce the local values here
            dev = self.extended.device
            vals = [torch.as_tensor(v).to(dev) for v in value.values]
            if axis is not None:
                cnt = sum(v.shape[axis] for v in vals)
                vals = [v.sum(dim=axis) for v in vals]
            total = vals[0].clone()
            for v in vals[1:]:  # rank order
                total = total + v
            if op == "SUM":
                return total
            n = cnt if axis is not None else len(vals)
            return total / n if total.is_floating_point() else total.double() / n
        t = torch.as_tensor(value)
        if axis is None:
            return self.extended.all_reduce(op, t)
        dev = t.device
        local_sum = t.sum(dim=axis).to(torch.float64 if not t.is_floating_point() else t.dtype)
        total = self.extended.all_reduce("SUM", local_sum.to(dev))
        if op == "SUM":
            return total
        cnt = torch.tensor(float(t.shape[axis]), device=dev, dtype=torch.float64)
        n = self.extended.all_reduce("SUM", cnt)
        return total / n.to(total.dtype)

    def gather(self, value, axis=0):
        from .values import PerReplica

        if isinstance(value, PerReplica):
            return torch.cat([torch.as_tensor(v).to(self.extended.device) for v in value.values], dim=axis)
        t = torch.as_tensor(value)
        g = self.extended.communicator.all_gather(t.to(self.extended.device))
        return torch.cat(list(g.unbind(0)), dim=axis)

    def experimental_local_results(self, value):
        """The values of this process's replicas: one per local device in single-process
        multi-device mode, else this process's one replica."""
        from .values import PerReplica

        if isinstance(value, PerReplica):
            return value.values
        return (value,)

    def experimental_distribute_dataset(self, dataset, options=None):
        from .input_lib import DistributedDataset, LocalDistributedDataset

        if self._local_group is not None and not self._local_group.in_region():
            return LocalDistributedDataset(dataset, self, options)  # PerReplica slices, one pipeline
        return DistributedDataset(dataset, self, options)

    def distribute_datasets_from_function(self, dataset_fn, options=None):
        from .input_lib import (DistributedDatasetFromFunction, InputContext,
                                LocalDistributedDatasetFromFunction)

        if self._local_group is not None and not self._local_group.in_region():
            ctx = InputContext(num_input_pipelines=1, input_pipeline_id=0,
                               num_replicas_in_sync=self.num_replicas_in_sync)
            return LocalDistributedDatasetFromFunction(dataset_fn(ctx), self, ctx)
        ctx = InputContext(
            num_input_pipelines=self.num_replicas_in_sync,
            input_pipeline_id=self.extended.rank,
            num_replicas_in_sync=self.num_replicas_in_sync,
        )
        return DistributedDatasetFromFunction(dataset_fn(ctx), self, ctx)

    experimental_distribute_datasets_from_function = distribute_datasets_from_function

    def barrier(self):
        self.extended.communicator.barrier()

    def shutdown(self):
        if self._closed:
            return
        self._closed = True
        wd = getattr(self.extended, "watchdog", None)
        if wd is not None:
            wd.stop()
            self.extended.watchdog = None
            lv = getattr(wd, "liveness", None)
            if lv is not None:
                lv.shutdown()
        try:
            self.extended.communicator.shutdown()
        except Exception:
            pass
        rdv = self.extended.rendezvous
        if rdv is not None:
            try:
                rdv.shutdown()
            except Exception:
                pass

    def __repr__(self):
        e = self.extended
        return (f"{type(self).__name__}(num_replicas_in_sync={self.num_replicas_in_sync}, rank={e.rank}, "
                f"device={e.device}, communicator={e.communicator.name})")


class _DefaultStrategy(Strategy):
    """No-op strategy used outside any scope: one replica on the default device."""

    def __init__(self):
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
        ext = StrategyExtended(self, dev, 0, 1, 0, LocalCommunicator(dev), CommunicationOptions())
        super().__init__(ext)


# ------------------------------------------------------------------------------------------------
def _select_communicator(impl: CommunicationImplementation, device: torch.device, rank: int, world: int,
                         store=None, host_hint: str = "127.0.0.1", timeout: Optional[float] = None,
                         prefer_native_ring: bool = True) -> Communicator:
    if world == 1:
        return LocalCommunicator(device)
    timeout = float(timeout or default_timeout())
    gpu = device.type == "cuda"
    if impl == CommunicationImplementation.NCCL and not gpu:
        raise ValueError("CollectiveCommunication.NCCL (RCCL) requires GPU replicas; this replica is on the CPU")
    if impl == CommunicationImplementation.RING or (not gpu and impl == CommunicationImplementation.AUTO):
        from .. import ops

        if store is None:
            import torch.distributed as dist

            if not dist.is_initialized():
                dist.init_process_group("gloo", rank=rank, world_size=world)
            store = _PGStore()
        if prefer_native_ring and ops.native_available():
            return RingCommunicator(rank, world, device, store, host_hint=host_hint, timeout=min(timeout, 600.0))
        import torch.distributed as dist

        return TorchCommunicator("gloo", rank, world, device, store=None if dist.is_initialized() else store,
                                 timeout=timeout)
    if impl == CommunicationImplementation.AUTO and os.environ.get("TDL_SHARE_GPU") == "1":
        # replica processes sharing one GPU: RCCL refuses duplicate devices; gloo control plane +
        # the xGMI kernel over IPC-mapped buffers of the same device
        import torch.distributed as dist

        if store is None and not dist.is_initialized():
            dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = TorchCommunicator("gloo", rank, world, device, store=None if dist.is_initialized() else store,
                                 timeout=timeout)
        comm.enable_xgmi(timeout)
        return comm
    # Default: torch's RCCL process group (ProcessGroupNCCL over the same librccl).  The framework's
    # own communicator stays opt-in because no multi-rank RCCL run is possible on the one-GPU
    # development box (RCCL refuses two ranks on one device), so its world >= 2 path has never
    # executed, while torch's group has; the abort path is wired either way (the job watchdog's
    # on_abort is communicator.abort: ncclCommAbort through torch's group or through ours).
    if os.environ.get("TDL_NATIVE_RCCL") == "1":
        # the framework's own RCCL communicator (csrc/rccl_comm.cpp: async-error query, abort)
        from .communicator import NativeRcclCommunicator

        comm = NativeRcclCommunicator(rank, world, device, store=store, timeout=timeout)
    else:
        comm = TorchCommunicator("nccl", rank, world, device, store=store, timeout=timeout)
    if impl != CommunicationImplementation.NCCL:  # AUTO: topology/size-aware algorithm choice
        comm.enable_xgmi(timeout)
    return comm


def _PGStore():
    """The default process group's own store (ring address exchange when launched by torchrun)."""
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store()


class MirroredStrategy(Strategy):
    """tf.distribute.MirroredStrategy(devices=None, cross_device_ops=None)."""

    def __init__(self, devices: Optional[Sequence] = None, cross_device_ops=None, *, communication=None,
                 communication_options=None, spawn: Optional[bool] = None):
        opts = normalize_options(communication if communication is not None or communication_options is not None
                                 else _cdo_to_impl(cross_device_ops), communication_options)
        launched = _launched()
        if devices is not None:
            devs = [parse_device(d) for d in devices]
            if not devs:
                raise ValueError("MirroredStrategy(devices=[]) needs at least one device")
        else:
            n = torch.cuda.device_count()  # does not initialise the GPU
            devs = [torch.device("cuda", i) for i in range(n)] or [torch.device("cpu")]
        if launched is None and len(devs) > 1:
            mode = "process" if spawn is True else ("threads" if spawn is False else
                                                    os.environ.get("TDL_MIRRORED_MODE", "threads"))
            if mode == "process":
                from .launch import maybe_spawn_local_replicas

                launched = maybe_spawn_local_replicas(len(devs), spawn=True)
                if launched is None:  # (maybe_spawn_local_replicas warned and said why)
                    devs = devs[:1]
            else:
                self._init_local(devs, opts)
                return
        if launched is None:
            dev = _shared_gpu(devs[0])
            comm = LocalCommunicator(dev)
            ext = StrategyExtended(self, dev, 0, 1, 0, comm, opts)
        else:
            lr = launched["local_rank"]
            if devices is not None:
                if lr >= len(devs):
                    raise ValueError(f"local rank {lr} has no device in {devices}")
                dev = _shared_gpu(_task_device(devs[lr], lr))
            else:
                dev = _replica_device(lr)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            comm = _select_communicator(opts.implementation, dev, launched["rank"], launched["world_size"],
                                        timeout=collective_timeout(opts))
            ext = StrategyExtended(self, dev, launched["rank"], launched["world_size"], lr, comm, opts)
        super().__init__(ext)
        if ext.world_size > 1:
            from ..cluster.liveness import start_for_process_group

            ext.watchdog = start_for_process_group(ext.rank, ext.world_size)
            if ext.watchdog is not None:
                ext.watchdog.on_abort = ext.communicator.abort
            ext.communicator.barrier()


    def _init_local(self, devs, opts):
        """ONE process, G local replicas (parallel/local_replicas.py): replica 0 is this strategy
        (device 0, communicator 0 of the group), replicas 1..G-1 are views of it."""
        from .local_replicas import LocalReplicaGroup, make_views

        local = [_shared_gpu(d) if d.type == "cuda" else d for d in devs]
        if any(d.type == "cuda" for d in local) and not torch.cuda.is_available():
            raise RuntimeError(f"MirroredStrategy: devices {devs} include GPUs but none is visible")
        group = LocalReplicaGroup(local, timeout=collective_timeout(opts))
        ext = StrategyExtended(self, local[0], 0, len(local), 0, group.comms[0], opts)
        Strategy.__init__(self, ext)
        self._local_group = group
        group.views = make_views(self, group)
        if local[0].type == "cuda":
            torch.cuda.set_device(local[0])

    @property
    def extended_local_devices(self):
        g = self._local_group
        return tuple(str(d) for d in g.devices) if g is not None else (str(self.extended.device),)


def _cdo_to_impl(cross_device_ops):
    if cross_device_ops is None:
        return None
    name = type(cross_device_ops).__name__.lower() if not isinstance(cross_device_ops, str) else cross_device_ops.lower()
    if "nccl" in name:
        return CommunicationImplementation.NCCL
    if "ring" in name or "reductiontoonedevice" in name or "hierarchical" in name:
        return CommunicationImplementation.RING
    return None


class NcclAllReduce:
    """tf.distribute.NcclAllReduce marker (selects RCCL)."""

    def __init__(self, num_packs=1):
        self.num_packs = num_packs


class HierarchicalCopyAllReduce(NcclAllReduce):
    pass


class ReductionToOneDevice:
    def __init__(self, reduce_to_device=None, accumulation_fn=None):
        self.reduce_to_device = reduce_to_device


class MultiWorkerMirroredStrategy(Strategy):
    """tf.distribute(.experimental).MultiWorkerMirroredStrategy.

    Accepts the TF 2.0-2.3 positional ``communication`` (tf_dist_example.py:12) and the TF >= 2.4
    ``communication_options``.  Reads the cluster from TF_CONFIG at construction (README.md:82:
    TF_CONFIG must be set before the strategy is created)."""

    def __init__(self, communication=None, cluster_resolver=None, communication_options=None, *,
                 gpus_per_worker: Optional[int] = None, timeout: float = 300.0):
        opts = normalize_options(communication, communication_options)
        resolver = cluster_resolver or TFConfigClusterResolver()
        cfg = resolver.config if isinstance(resolver, TFConfigClusterResolver) else parse_tf_config()
        launched = _launched()
        rendezvous = None
        watchdog = None
        if cfg is not None and cfg.task is not None and not cfg.is_training_task:
            raise ClusterConfigError(
                f"this process is the '{cfg.task.type}' task; MultiWorkerMirroredStrategy trains only on "
                "chief/worker tasks (ps/evaluator belong to ParameterServerStrategy, README.md:55-57)")
        if cfg is None or cfg.is_single_worker:
            # README.md:34 — a single worker degrades to MirroredStrategy
            local = _LocalPlacement.resolve(launched, gpus_per_worker)
            rank, world, lr, dev = local
            comm = _select_communicator(opts.implementation, dev, rank, world,
                                        timeout=collective_timeout(opts)) if world > 1 else LocalCommunicator(dev)
            if world > 1:
                from ..cluster.liveness import start_for_process_group

                watchdog = start_for_process_group(rank, world)
        else:
            from ..cluster.rendezvous import Rendezvous

            lr = int(os.environ.get("LOCAL_RANK", "0")) if launched else 0
            nlocal = int(os.environ.get("LOCAL_WORLD_SIZE", "1")) if launched else 1
            if gpus_per_worker is not None and not launched and gpus_per_worker > 1:
                raise ClusterConfigError(
                    "gpus_per_worker > 1 needs one process per GPU: start each task with "
                    "`python -m tensorflow_distributed_learning_amd.launch --nproc-per-node G`")
            dev = _replica_device(lr)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            rendezvous = Rendezvous(cfg, local_rank=lr, num_local=nlocal, timeout=timeout)
            layout = rendezvous.join()
            rank, world = layout.rank, layout.world_size
            host_hint = cfg.task_address[0] if cfg.task_address else "127.0.0.1"
            comm = _select_communicator(opts.implementation, dev, rank, world, store=rendezvous.store,
                                        host_hint=host_hint, timeout=collective_timeout(opts))
        ext = StrategyExtended(self, dev, rank, world, lr, comm, opts, tf_config=cfg, rendezvous=rendezvous)
        ext.watchdog = watchdog
        super().__init__(ext, cluster_resolver=resolver)
        if rendezvous is not None and world > 1 and os.environ.get("TDL_WATCHDOG", "1") == "1":
            from ..utils.fault import PeerWatchdog

            ext.watchdog = PeerWatchdog(rendezvous, stale_after=float(os.environ.get("TDL_HEARTBEAT_TIMEOUT", "60")),
                                        grace=float(os.environ.get("TDL_ABORT_GRACE", "30"))).start()
        if ext.watchdog is not None:
            ext.watchdog.on_abort = comm.abort
        if world > 1:
            comm.barrier()


class _LocalPlacement:
    @staticmethod
    def resolve(launched, gpus_per_worker):
        if launched is not None:
            lr = launched["local_rank"]
            dev = _replica_device(lr)
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            return launched["rank"], launched["world_size"], lr, dev
        dev = torch.device("cuda", 0) if torch.cuda.device_count() > 0 else torch.device("cpu")
        return 0, 1, 0, dev


class OneDeviceStrategy(Strategy):
    """tf.distribute.OneDeviceStrategy(device)."""

    def __init__(self, device):
        dev = parse_device(device)
        super().__init__(StrategyExtended(self, dev, 0, 1, 0, LocalCommunicator(dev), CommunicationOptions()))


class experimental:  # noqa: N801 - tf.distribute.experimental namespace
    MultiWorkerMirroredStrategy = MultiWorkerMirroredStrategy
    CollectiveCommunication = CollectiveCommunication
    CommunicationImplementation = CommunicationImplementation
    CommunicationOptions = CommunicationOptions


def _shared_gpu(dev: torch.device) -> torch.device:
    """TDL_SHARE_GPU=1: an explicit '/gpu:i' maps onto the visible GPUs round-robin (N replicas
    on a one-GPU box for tests); otherwise the device is used as given."""
    if dev.type == "cuda" and os.environ.get("TDL_SHARE_GPU") == "1":
        n = torch.cuda.device_count()
        if n > 0:
            return torch.device("cuda", (dev.index or 0) % n)
    return dev


def _task_device(dev: torch.device, local_rank: int) -> torch.device:
    """An explicit ``devices=`` entry of a task started by ``launch --local-workers``: the task's
    devices are numbered from its first GPU (TDL_DEVICE_INDEX = first GPU + local rank), as if the
    task ran alone on its own host."""
    pinned = os.environ.get("TDL_DEVICE_INDEX")
    if dev.type != "cuda" or not pinned:
        return dev
    first = int(pinned) - local_rank
    return torch.device("cuda", first + (dev.index or 0))


def _replica_device(local_rank: int) -> torch.device:
    """GPU of a replica process: cuda:<local_rank> (one process per GPU).  TDL_SHARE_GPU=1 maps
    several replica processes onto the visible GPUs round-robin (tests with the RING communicator on
    a one-GPU box; RCCL itself refuses two ranks on one device)."""
    n = torch.cuda.device_count()
    if n == 0:
        return torch.device("cpu")
    pinned = os.environ.get("TDL_DEVICE_INDEX")
    if pinned:  # set by launch_local_workers: the node-global device of this replica
        i = int(pinned)
        return torch.device("cuda", i % n if os.environ.get("TDL_SHARE_GPU") == "1" else i)
    if os.environ.get("TDL_SHARE_GPU") == "1":
        return torch.device("cuda", local_rank % n)
    return torch.device("cuda", local_rank) if n > local_rank else torch.device("cpu")
