"""Cross-replica communicators (the DP communication backend).

One process drives one replica (one GPU, or the CPU).  A communicator reduces tensors across all
replicas of the job:

* :class:`LocalCommunicator`  – single replica: every collective is the identity.
* :class:`TorchCommunicator`  – ``torch.distributed`` process group.  Backend ``"nccl"`` is RCCL on
  ROCm: ring/tree collectives over the xGMI links of an MI355X node, capturable into hipGraphs.
  Backend ``"gloo"`` is kept as a CPU oracle for tests.
* :class:`RingCommunicator`   – the native C++ TCP ring (``CollectiveCommunication.RING`` and CPU
  replicas); GPU tensors are staged through pinned host memory.

All communicators reduce in place and produce bit-identical results on every rank.
"""
from __future__ import annotations

import os
import socket
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import ops

_OPS = {"sum", "mean", "max", "min", "prod"}


class Communicator:
    name = "base"
    capturable = False  # can be recorded inside a hipGraph capture

    def __init__(self, rank: int, world_size: int, device: torch.device):
        self.rank = int(rank)
        self.world_size = int(world_size)
        self.device = torch.device(device)

    # -- collectives (in place) --------------------------------------------------------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        raise NotImplementedError

    def all_reduce_async(self, t: torch.Tensor, op: str = "sum"):
        """Start an all-reduce; returns an object with ``wait()``.  Default: synchronous."""
        self.all_reduce(t, op)
        return _Done()

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        raise NotImplementedError

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Returns a new tensor [world_size, *t.shape]."""
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError

    def capture_probe(self) -> bool:
        """True when this communicator's collectives can be recorded into a hipGraph."""
        return self.capturable

    def check_health(self) -> None:
        """Raise if an asynchronous collective failed (host sync; called when logs are read)."""

    def prepare_all_reduce(self, *numels: int) -> None:
        """Collective set-up for all-reduces of these sizes (before any graph capture)."""

    def all_reduce_sgd(self, g: torch.Tensor, w: torch.Tensor, lr: torch.Tensor) -> bool:
        """``w -= lr * all_reduce_sum(g)`` as one fused operation when the communicator has one
        (returns False otherwise; the caller then all-reduces and applies SGD itself)."""
        return False

    def exchange_channel(self, numel: int, min_blocks: int):
        """Collective: a device exchange channel for kernels that all-reduce inside their own
        workgroups (xGMI); None when the communicator has none."""
        return None

    def device_bucket_capable(self, numels) -> bool:
        """Collective: whether bucketed all-reduces of these sizes can run asynchronously on the
        device and inside a captured hipGraph (RCCL, or the xGMI kernel)."""
        return self.name == "rccl"

    def shutdown(self) -> None:
        pass

    def abort(self) -> None:
        """Unblock this rank's collectives after a job fault (called from the watchdog thread, so
        that a rank stuck in a collective raises instead of waiting for its timeout).  Best effort;
        the communicator is unusable afterwards."""

    def __repr__(self):
        return f"{type(self).__name__}(rank={self.rank}, world_size={self.world_size}, device={self.device})"


class _Done:
    def wait(self):
        return None

    def is_completed(self):
        return True


class LocalCommunicator(Communicator):
    name = "local"
    capturable = True

    def __init__(self, device: torch.device):
        super().__init__(0, 1, device)

    def all_reduce(self, t, op="sum"):
        if op not in _OPS:
            raise ValueError(f"unknown reduce op {op}")
        return t

    def broadcast(self, t, src=0):
        return t

    def all_gather(self, t):
        return t.unsqueeze(0).clone()

    def barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)


_TORCH_OPS = {
    "sum": dist.ReduceOp.SUM,
    "max": dist.ReduceOp.MAX,
    "min": dist.ReduceOp.MIN,
    "prod": dist.ReduceOp.PRODUCT,
}


class TorchCommunicator(Communicator):
    """torch.distributed process group (``nccl`` = RCCL over xGMI, or ``gloo``)."""

    def __init__(self, backend: str, rank: int, world_size: int, device: torch.device, store=None,
                 timeout: Optional[float] = None, init: bool = True):
        super().__init__(rank, world_size, device)
        from .communication import default_timeout

        timeout = float(timeout or default_timeout())
        self.timeout = timeout
        self.backend = backend
        self.name = "rccl" if backend == "nccl" else backend
        self.capturable = backend == "nccl"
        self._owns_group = False
        if init and not dist.is_initialized():
            from datetime import timedelta

            kw = {}
            if backend == "nccl" and self.device.type == "cuda":
                kw["device_id"] = self.device
            if store is not None:
                dist.init_process_group(backend, store=store, rank=rank, world_size=world_size,
                                        timeout=timedelta(seconds=timeout), **kw)
            else:
                dist.init_process_group(backend, rank=rank, world_size=world_size,
                                        timeout=timedelta(seconds=timeout), **kw)
            self._owns_group = True
        self._avg_native = backend == "nccl"
        self.xgmi = None  # parallel/xgmi.py one-shot path for small f32 messages (single node)
        self.xgmi_reason = ""  # why the xGMI path was dropped (bench.py reports it)
        self.algorithm = "ring" if backend == "gloo" else "rccl"

    def enable_xgmi(self, timeout: Optional[float] = None) -> bool:
        """Route small f32 sum/mean all-reduces through the xGMI one-shot kernel when every rank
        is on this node (collective; the self-test runs on the first prepared channel).  Over a
        gloo group (replica processes sharing one GPU, where RCCL cannot run) the kernel is the
        only device data plane; gloo carries the control messages."""
        from . import xgmi

        if self.device.type != "cuda" or self.world_size > 8 or not xgmi.enabled_by_env():
            return False
        if not xgmi.single_node():
            return False
        ctrl = self.device if self.backend == "nccl" else torch.device("cpu")
        self.xgmi = xgmi.XgmiAllReduce(self.rank, self.world_size, self.device, ctrl_device=ctrl,
                                       timeout=timeout or self.timeout)
        # over gloo the kernel is the only device data plane: messages above its limit go in chunks
        self.xgmi.chunked = self.backend != "nccl"
        return True

    def prepare_all_reduce(self, *numels):
        if self.xgmi is not None:
            if self.xgmi.prepare(*numels):
                from .xgmi import choose_algo

                two = any(choose_algo(int(n), self.world_size) == 1 for n in numels if 0 < int(n) <= self.xgmi.limit)
                self.algorithm = ("xgmi-twoshot+" if two else "xgmi-oneshot+") + \
                    ("rccl" if self.backend == "nccl" else self.backend)
            else:
                self.xgmi_reason = self.xgmi.reason or "disabled"
                self.xgmi = None

    def all_reduce_sgd(self, g, w, lr):
        return self.xgmi is not None and self.xgmi.all_reduce_sgd(g, w, lr)

    def exchange_channel(self, numel: int, min_blocks: int):
        """Collective: a dedicated xGMI channel for a kernel with a built-in exchange (None when
        this communicator has no xGMI path)."""
        if self.xgmi is None:
            return None
        return self.xgmi.dedicated(numel, min_blocks)

    def check_health(self):
        if self.xgmi is not None:
            self.xgmi.check()

    def _no_host_collective_in_capture(self, t):
        # a gloo collective stages through the host (a device sync), which would invalidate a
        # graph capture for the whole process; fail before issuing anything, so that the capture
        # ends cleanly and the caller can fall back to eager steps
        if self.backend != "nccl" and t.is_cuda and torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"{self.backend} all-reduce of {t.numel()} elements cannot be recorded in a hipGraph")

    def all_reduce(self, t, op="sum"):
        if self.xgmi is not None and self.xgmi.all_reduce(t, op):
            return t
        self._no_host_collective_in_capture(t)
        if op == "mean":
            if self._avg_native:
                dist.all_reduce(t, op=dist.ReduceOp.AVG)
            else:
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
                t.div_(self.world_size)
            return t
        dist.all_reduce(t, op=_TORCH_OPS[op])
        return t

    def all_reduce_async(self, t, op="sum"):
        if self.xgmi is not None and op in ("sum", "mean") and self.xgmi.applicable(t) and \
                self.xgmi.has_channel(t.numel()):
            # xGMI kernel on a side stream (forked from the current one, joined by wait()): the
            # bucket's exchange overlaps the rest of the backward and records into a hipGraph
            return _SideStreamWork(self, t, op)
        self._no_host_collective_in_capture(t)
        if op == "mean" and not self._avg_native:
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, async_op=True)
            return _ScaleOnWait(work, t, 1.0 / self.world_size)
        rop = dist.ReduceOp.AVG if op == "mean" else _TORCH_OPS[op]
        return dist.all_reduce(t, op=rop, async_op=True)

    def device_bucket_capable(self, numels) -> bool:
        """Whether bucketed all-reduces of these sizes can be issued asynchronously from backward
        hooks and recorded into a whole-step hipGraph: RCCL, or the xGMI kernel for every size
        (channels prepared collectively here; the only device data plane of replicas sharing a GPU)."""
        if self.backend == "nccl":
            return True
        if self.xgmi is None:
            return False
        numels = [int(n) for n in numels]
        if any(n > self.xgmi.limit for n in numels) and not self.xgmi.chunked:
            return False
        self.prepare_all_reduce(*numels)
        return self.xgmi is not None and all(self.xgmi.has_channel(n) for n in numels)

    def broadcast(self, t, src=0):
        dist.broadcast(t, src=src)
        return t

    def all_gather(self, t):
        # flat output (gloo's all-gather-into-tensor takes only a [world * numel] buffer), then viewed
        out = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, t.contiguous().view(-1))
        return out.view((self.world_size,) + tuple(t.shape))

    def barrier(self):
        if self.backend == "nccl" and self.device.type == "cuda":
            dist.barrier(device_ids=[self.device.index or 0])
        else:
            dist.barrier()

    def capture_probe(self) -> bool:
        """Collectively decide whether RCCL all-reduces can live inside a hipGraph on this job.

        Every rank captures a graph with one all-reduce; the ranks agree (eager MIN) on whether
        all captures succeeded before any of them replays, replay once, verify the sum, and agree
        again — so all ranks take the same path and issue the same collective sequence.
        """
        if getattr(self, "_capture_ok", None) is not None:
            return self._capture_ok
        if self.backend != "nccl" and self.xgmi is not None:
            # gloo control plane: the device collectives are the (capturable) xGMI kernels
            self._capture_ok = bool(self.xgmi._ensure_tested())
            return self._capture_ok
        if not self.capturable or self.device.type != "cuda":
            self._capture_ok = False
            return False
        dev = self.device
        flag = torch.ones(1, device=dev)
        t = torch.full((64,), float(self.rank + 1), device=dev)
        u = torch.full((4096,), float(self.rank + 1), device=dev)
        dist.all_reduce(t)  # warm the communicator outside capture
        torch.cuda.synchronize(dev)
        # (no eager async warm-up: with torch's cached collective events, an eager async work the
        # PG watchdog still tracks can see its event re-recorded inside the capture below)
        g = None
        try:
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                # the two patterns the engines record: a synchronous all-reduce, and an async one
                # launched mid-computation (as from a backward hook) and waited for later
                dist.all_reduce(t)
                u.mul_(1.0)
                work = self.all_reduce_async(u)
                t.add_(0.0)
                work.wait()
            torch.cuda.synchronize(dev)
        except Exception:  # capture unsupported by this RCCL/torch build
            g = None
            flag.zero_()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        ok = bool(flag.item() > 0.5)
        if ok:
            t.fill_(float(self.rank + 1))
            u.fill_(float(self.rank + 1))
            g.replay()
            torch.cuda.synchronize(dev)
            want = float(self.world_size * (self.world_size + 1) // 2)
            flag.fill_(1.0 if bool(torch.all(t == want)) and bool(torch.all(u == want)) else 0.0)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            ok = bool(flag.item() > 0.5)
        self._capture_ok = ok
        return ok

    def abort(self):
        """RCCL: ncclCommAbort on every communicator of the job (torch's process-group abort), which
        makes a collective blocked in RCCL return an error on this rank.  gloo has no abort (its own
        timeout applies)."""
        if self.backend == "nccl" and dist.is_initialized():
            try:
                from torch.distributed import distributed_c10d as c10d

                c10d._abort_process_group()
            except Exception:  # noqa: BLE001 - best effort from the watchdog thread
                pass

    def shutdown(self):
        if self.xgmi is not None:
            try:
                self.barrier()  # no peer may still be reading our exchange buffers
            except Exception:
                pass
            self.xgmi.close()
            self.xgmi = None
        if self._owns_group and dist.is_initialized():
            try:
                dist.destroy_process_group()
            except Exception:
                pass
            self._owns_group = False


class NativeRcclCommunicator(TorchCommunicator):
    """The framework's OWN RCCL communicator (csrc/rccl_comm.cpp): device
    collectives go straight to ncclAllReduce / ncclBroadcast / ncclAllGather on the caller's HIP
    stream (capturable into hipGraphs), the communicator's asynchronous errors are polled by
    :meth:`check_health`, and :meth:`abort` is ncclCommAbort (from the job watchdog's thread: a rank
    stuck in a collective returns instead of hanging the GPU queue).  A gloo process group carries
    the control plane (unique-id exchange, host tensors, barriers).  The xGMI kernel path for small
    single-node messages works on top of it as on the torch RCCL group (``enable_xgmi``).

    Selected with ``TDL_NATIVE_RCCL=1`` for GPU replicas (``CollectiveCommunication.NCCL`` / ``AUTO``)."""

    # communicators created so far by this process; every rank creates them in the same order
    # (collective construction), so the count is the same everywhere and versions the id key
    _generation = 0

    def __init__(self, rank: int, world_size: int, device: torch.device, store=None,
                 timeout: Optional[float] = None):
        super().__init__("gloo", rank, world_size, device, store=store, timeout=timeout)
        self.name = "rccl"
        self.capturable = True
        self._avg_native = True
        self.algorithm = "rccl-native"
        from torch.distributed import distributed_c10d as c10d

        C = ops.hip()
        kv = c10d._get_default_store()
        # one key per communicator generation: a second communicator of the same job (strategy
        # re-created, tests) must never read the previous generation's id (mismatched comms hang)
        gen = NativeRcclCommunicator._generation
        NativeRcclCommunicator._generation += 1
        key = f"tdl/rccl/unique_id/{gen}"
        if rank == 0:
            kv.set(key, C.RcclComm.unique_id())
        uid = kv.get(key)
        torch.cuda.set_device(self.device)
        self.rccl = C.RcclComm(bytes(uid), rank, world_size, self.device.index or 0)
        self.rccl_version = int(C.RcclComm.version())

    def enable_xgmi(self, timeout: Optional[float] = None) -> bool:
        ok = super().enable_xgmi(timeout)
        if ok and self.xgmi is not None:
            self.xgmi.chunked = False  # large messages belong to RCCL's rings, as on the torch group
        return ok

    def prepare_all_reduce(self, *numels):
        super().prepare_all_reduce(*numels)
        self.algorithm = self.algorithm.replace("+gloo", "+rccl-native")

    # ---- device data plane ------------------------------------------------------------------
    _OPC = {"sum": 0, "prod": 1, "max": 2, "min": 3, "mean": 4}

    def all_reduce(self, t, op="sum"):
        if not t.is_cuda:
            return super().all_reduce(t, op)
        if self.xgmi is not None and self.xgmi.all_reduce(t, op):
            return t
        if op not in self._OPC:
            raise ValueError(f"unknown reduce op {op}")
        if op == "mean" and not t.is_floating_point():
            raise ValueError("mean all-reduce of an integer tensor")
        if t.is_contiguous():
            self.rccl.all_reduce(t, self._OPC[op])
        else:  # reduce a contiguous copy, then write the result back into t
            c = t.contiguous()
            self.rccl.all_reduce(c, self._OPC[op])
            t.copy_(c)
        return t

    def all_reduce_async(self, t, op="sum"):
        if not t.is_cuda:
            return super().all_reduce_async(t, op)
        if self.xgmi is not None and op in ("sum", "mean") and self.xgmi.applicable(t) and \
                self.xgmi.has_channel(t.numel()):
            return _SideStreamWork(self, t, op)
        return _RcclSideWork(self, t, op)

    def broadcast(self, t, src=0):
        if not t.is_cuda:
            return super().broadcast(t, src)
        self.rccl.broadcast(t, int(src))
        return t

    def all_gather(self, t):
        if not t.is_cuda:
            return super().all_gather(t)
        out = torch.empty(self.world_size * t.numel(), dtype=t.dtype, device=t.device)
        self.rccl.all_gather(out, t.contiguous().view(-1))
        return out.view((self.world_size,) + tuple(t.shape))

    def barrier(self):
        torch.cuda.synchronize(self.device)
        dist.barrier()

    def _no_host_collective_in_capture(self, t):
        if not t.is_cuda:
            super()._no_host_collective_in_capture(t)

    def device_bucket_capable(self, numels) -> bool:
        return True

    def capture_probe(self) -> bool:
        """Collectively: an RCCL all-reduce recorded into a hipGraph replays correctly on every
        rank (agreement on the gloo control plane, so every rank takes the same path)."""
        if getattr(self, "_capture_ok", None) is not None:
            return self._capture_ok
        dev = self.device
        t = torch.full((64,), float(self.rank + 1), device=dev)
        ok = True
        try:
            self.rccl.all_reduce(t, 0)
            torch.cuda.synchronize(dev)
            s = torch.cuda.Stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                # (a kernel in front of the collective: at world 1 RCCL's in-place all-reduce records
                # no node, and an empty graph proves nothing about replay)
                t.mul_(1.0)
                self.rccl.all_reduce(t, 0)
            torch.cuda.synchronize(dev)
        except Exception:  # noqa: BLE001 - capture unsupported: eager collectives
            ok = False
        f = torch.tensor([1.0 if ok else 0.0])
        dist.all_reduce(f, op=dist.ReduceOp.MIN)
        ok = bool(f.item() > 0.5)
        if ok:
            t.fill_(float(self.rank + 1))
            g.replay()
            torch.cuda.synchronize(dev)
            want = float(self.world_size * (self.world_size + 1) // 2)
            f.fill_(1.0 if bool(torch.all(t == want)) else 0.0)
            dist.all_reduce(f, op=dist.ReduceOp.MIN)
            ok = bool(f.item() > 0.5)
        self._capture_ok = ok
        return ok

    # ---- failure handling ------------------------------------------------------------------
    def check_health(self):
        super().check_health()
        e = self.rccl.async_error()
        if e != 0:
            raise RuntimeError(f"rccl: asynchronous communicator error: {self.rccl.error_string(e)}")

    def abort(self):
        """ncclCommAbort: every pending collective of this communicator returns (watchdog thread)."""
        try:
            self.rccl.abort()
        except Exception:  # noqa: BLE001 - best effort
            pass

    def shutdown(self):
        if not self.rccl.aborted:
            try:
                torch.cuda.synchronize(self.device)
            except Exception:  # noqa: BLE001
                pass
        super().shutdown()


class _RcclSideWork:
    """An RCCL all-reduce enqueued on the communicator's side stream (forked from the current one):
    it overlaps the rest of the backward on the GPU; ``wait()`` joins it back."""

    def __init__(self, comm, t, op):
        dev = t.device
        if getattr(comm, "_side", None) is None:
            comm._side = torch.cuda.Stream(dev)
        side = comm._side
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            comm.all_reduce(t, op)
        self._side, self._dev = side, dev

    def wait(self):
        torch.cuda.current_stream(self._dev).wait_stream(self._side)

    def is_completed(self):
        return self._side.query()


class _SideStreamWork:
    """An all-reduce issued on the communicator's side stream (forked from the caller's current
    stream); ``wait()`` joins it back into the stream current at wait time."""

    def __init__(self, comm, t, op):
        dev = t.device
        if getattr(comm, "_side", None) is None:
            comm._side = torch.cuda.Stream(dev)
        side = comm._side
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            comm.xgmi.all_reduce(t, op)
        self._side, self._dev = side, dev

    def wait(self):
        torch.cuda.current_stream(self._dev).wait_stream(self._side)

    def is_completed(self):
        return self._side.query()


class _ScaleOnWait:
    def __init__(self, work, t, s):
        self.work, self.t, self.s = work, t, s

    def wait(self):
        self.work.wait()
        self.t.mul_(self.s)

    def is_completed(self):
        return self.work.is_completed()


def _my_ring_host(default: str) -> str:
    h = os.environ.get("TDL_RING_HOST")
    if h:
        return h
    if default in ("127.0.0.1", "localhost", ""):
        return "127.0.0.1"
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return default


class RingCommunicator(Communicator):
    """Native C++ TCP ring collectives (csrc/native/ring.cpp)."""

    name = "ring"

    def __init__(self, rank: int, world_size: int, device: torch.device, store, host_hint: str = "127.0.0.1",
                 timeout: float = 300.0, tag: str = "ring"):
        super().__init__(rank, world_size, device)
        N = ops.native()
        self._ring = N.RingComm(self.rank, self.world_size, "0.0.0.0", int(timeout * 1000))
        if self.world_size > 1:
            me = _my_ring_host(host_hint)
            store.set(f"{tag}/addr/{self.rank}", f"{me}:{self._ring.port}".encode())
            right = (self.rank + 1) % self.world_size
            addr = bytes(store.get(f"{tag}/addr/{right}")).decode()
            h, p = addr.rsplit(":", 1)
            self._ring.connect(h, int(p))
        self._stage: Optional[torch.Tensor] = None

    def _host(self, t: torch.Tensor):
        if t.device.type == "cpu":
            return t.contiguous(), False
        n = t.numel() * t.element_size()
        if self._stage is None or self._stage.numel() < n:
            self._stage = torch.empty(max(n, 1 << 20), dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        h = self._stage[:n].view(t.dtype).view(t.shape)
        h.copy_(t)
        return h, True

    def all_reduce(self, t, op="sum"):
        if self.world_size == 1:
            return t
        rop = "sum" if op == "mean" else op
        work = t
        conv = None
        if t.dtype in (torch.float16, torch.bfloat16):
            conv = t
            work = t.float()
        h, staged = self._host(work)
        self._ring.all_reduce(h, rop)
        if op == "mean":
            h.div_(self.world_size)
        if staged or h.data_ptr() != work.data_ptr():
            work.copy_(h)
        if conv is not None:
            conv.copy_(work)
        return t

    def broadcast(self, t, src=0):
        if self.world_size == 1:
            return t
        h, staged = self._host(t)
        self._ring.broadcast(h, int(src))
        if staged or h.data_ptr() != t.data_ptr():
            t.copy_(h)
        return t

    def all_gather(self, t):
        src = t.detach().contiguous().cpu()
        out = torch.empty((self.world_size,) + tuple(t.shape), dtype=t.dtype)
        self._ring.all_gather(src, out)
        return out.to(t.device)

    def barrier(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self._ring.barrier()

    def abort(self):
        self._ring.abort()

    def shutdown(self):
        self._ring.close()


def all_reduce_coalesced(comm: Communicator, tensors: List[torch.Tensor], op: str = "sum") -> None:
    """All-reduce a list of tensors as one flat buffer (TF's pack-by-size with one pack)."""
    if comm.world_size == 1 or not tensors:
        return
    flat = torch.cat([x.reshape(-1) for x in tensors])
    comm.all_reduce(flat, op)
    off = 0
    for x in tensors:
        n = x.numel()
        x.copy_(flat[off : off + n].view_as(x))
        off += n
