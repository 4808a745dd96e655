"""Cross-device collectives of ONE process driving G devices from ONE host thread.

This is the data plane of the single-process ``MirroredStrategy`` (tf_dist_example.py:13,
README.md:15-19: one process, one replica per GPU, variables mirrored on every GPU, the NCCL
all-reduce between them -- README.md:17).  TF issues that all-reduce once for all local devices
(``NcclAllReduce`` inside a merge call); here the same call takes the G replicas' tensors at once and
enqueues each device's part on that replica's stream, so no host thread ever waits for another:

* ``xgmi``   -- the hand-written xGMI all-reduce kernel (csrc/kernels/xgmi.hip).  The G channels live
  in this process and are wired with plain pointers (``XgmiChannel.connect_local``) after enabling
  peer access between every ordered device pair; each device's kernel reads the other devices'
  exchange buffers directly over the point-to-point links and waits for them on the device (bounded
  waits, rank-order sums: bit-identical on every replica).  One launch per device, capturable into
  each device's hipGraph.  The fused MNIST engine uses the same channels for the exchange inside its
  finalize kernel (engine/mirrored.py).
* ``rccl``   -- an RCCL clique of this process's devices (``ncclCommInitAll``; every collective a
  ``ncclGroupStart/End`` of the G per-device calls, csrc/rccl_comm.cpp ``RcclClique``).
* ``copies`` -- rank-order sums through device-to-device copies ordered by events (CPU replicas,
  replicas sharing one GPU when spinning kernels are unsafe, or a failed self-test).

Spinning kernels of several replicas on ONE GPU (``TDL_SHARE_GPU=1`` tests) need every replica's
stream on its own hardware queue: streams that share a queue are serialised, so a replica's waiting
kernel would block the peer it waits for.  HIP gives a process ``GPU_MAX_HW_QUEUES`` (default 4)
queues per device; with more replicas per device than that leaves free, the group uses ``copies``.
"""
from __future__ import annotations

import contextlib
import os
import warnings
from typing import Dict, List, Optional, Sequence

import torch

BLOCK = 1024  # f32 elements per xGMI workgroup (kXgmiBlockElems)


def hw_queues() -> int:
    return int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)


class DeviceGroupComm:
    """Collectives over the G replicas of one process, issued from one thread (module docstring).

    ``streams[r]`` is replica r's stream; every collective enqueues replica r's part on it and
    returns without a host wait (the ``copies`` path included: events order the reads and writes)."""

    def __init__(self, devices: Sequence[torch.device], streams: Sequence[Optional[torch.cuda.Stream]],
                 timeout: float = 120.0):
        self.devices = [torch.device(d) for d in devices]
        self.G = len(self.devices)
        self.streams = list(streams)
        self.gpu = all(d.type == "cuda" for d in self.devices)
        self.timeout = float(os.environ.get("TDL_XGMI_TIMEOUT", min(float(timeout), 120.0)))
        phys = [d.index or 0 for d in self.devices] if self.gpu else []
        self.per_device = max((phys.count(i) for i in set(phys)), default=1)
        self.distinct = self.gpu and len(set(phys)) == self.G
        self._xgmi: Optional[bool] = None
        self.reason = ""
        self._chans: Dict[tuple, list] = {}
        self._clique = None
        self._clique_tried = False
        self.algorithm = "copies"

    # ------------------------------------------------------------------ placement
    @contextlib.contextmanager
    def on(self, r: int):
        """Replica r's device and stream as the current ones."""
        d = self.devices[r]
        if d.type != "cuda" or self.streams[r] is None:
            yield
            return
        with torch.cuda.device(d), torch.cuda.stream(self.streams[r]):
            yield

    @contextlib.contextmanager
    def all_streams(self):
        """Every replica's stream current on its device at once (a cross-device copy is ordered
        against the CURRENT streams of both devices)."""
        with contextlib.ExitStack() as es:
            for r, d in enumerate(self.devices):
                if d.type == "cuda" and self.streams[r] is not None:
                    es.enter_context(torch.cuda.stream(self.streams[r]))
            yield

    # ------------------------------------------------------------------ xGMI channels
    def spin_safe(self) -> bool:
        """Whether kernels that wait on the device for a peer replica can run: distinct GPUs, or
        replicas sharing a GPU with a hardware queue each (plus one for the default stream)."""
        if not self.gpu:
            return False
        return self.distinct or self.per_device <= hw_queues() - 1

    def xgmi_ok(self) -> bool:
        """Peer access + a start-up self-test of the in-process xGMI channels (once)."""
        if self._xgmi is None:
            self._xgmi = False
            if os.environ.get("TDL_XGMI", "1") != "1":
                self.reason = "disabled by TDL_XGMI=0"
            elif not self.spin_safe():
                self.reason = (f"{self.per_device} replicas share one GPU but only {hw_queues()} hardware queues "
                               "(GPU_MAX_HW_QUEUES)" if self.gpu else "CPU replicas")
            elif torch.cuda.is_current_stream_capturing():
                self._xgmi = None
                return False
            else:
                try:
                    self._enable_peers()
                    self._xgmi = self._selftest()
                    if not self._xgmi:
                        self.reason = "self-test mismatch"
                except Exception as e:  # noqa: BLE001 - any failure means the fallback path
                    self._xgmi, self.reason = False, f"{type(e).__name__}: {e}"
                if not self._xgmi:
                    warnings.warn(f"in-process xGMI all-reduce disabled ({self.reason})")
        if self._xgmi:
            self.algorithm = "xgmi"
        return bool(self._xgmi)

    def _enable_peers(self):
        from .. import ops

        C = ops.hip()
        idx = sorted({d.index or 0 for d in self.devices})
        for a in idx:
            for b in idx:
                if a != b and not C.enable_peer_access(a, b):
                    raise RuntimeError(f"no peer access from GPU {a} to GPU {b}")

    def channels(self, numel: int, min_blocks: int = 0, algo: Optional[int] = None) -> Optional[list]:
        """G locally connected channels (rank r on device r) for messages of ``numel`` f32 (two-shot
        calls must use exactly that size); None without xGMI.  ``min_blocks``: signal slots for a
        kernel that runs the exchange in its own workgroups."""
        if not self.xgmi_ok():
            return None
        from .. import ops
        from .xgmi import choose_algo

        a = choose_algo(numel, self.G) if algo is None else int(algo)
        key = (int(numel), a, int(min_blocks))
        chans = self._chans.get(key)
        if chans is None:
            C = ops.hip()
            chans = [C.XgmiChannel(r, self.G, int(numel), d.index or 0, self.timeout, a, int(min_blocks))
                     for r, d in enumerate(self.devices)]
            for ch in chans:
                ch.connect_local(chans)
            self._chans[key] = chans
        return chans

    def _selftest(self) -> bool:
        """Both algorithms, eager and graph-replayed, plus the fused SGD form, against the rank-order
        sum of the replicas' inputs computed on the host (bit-identical expected)."""
        ok = True
        for n in (3 * BLOCK + 37, 70 * BLOCK + 5):
            for algo in (0, 1) if self.G > 1 else (0,):
                chans = self._raw_channels(n, algo)
                g = torch.Generator().manual_seed(4242 + n + algo)
                xs = [torch.randn(n, generator=g) for _ in range(self.G)]
                want = xs[0].clone()
                for x in xs[1:]:
                    want += x
                dev = [x.to(d) for x, d in zip(xs, self.devices)]
                outs = [torch.empty_like(x) for x in dev]
                for r in range(self.G):
                    with self.on(r):
                        chans[r].all_reduce(dev[r], outs[r], 1.0)
                self.synchronize()
                ok &= all(torch.equal(o.cpu(), want) for o in outs)
                # graph replay on each device (the engines capture these calls)
                graphs = []
                for r in range(self.G):
                    with torch.cuda.device(self.devices[r]):
                        s = torch.cuda.Stream(self.devices[r])
                        s.wait_stream(torch.cuda.current_stream(self.devices[r]))
                        gr = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gr, stream=s):
                            chans[r].all_reduce(dev[r], outs[r], 1.0)
                        graphs.append(gr)
                self.synchronize()
                for _ in range(2):
                    for o in outs:
                        o.zero_()
                    self.synchronize()
                    for r in range(self.G):
                        with self.on(r):
                            graphs[r].replay()
                    self.synchronize()
                    ok &= all(torch.equal(o.cpu(), want) for o in outs)
                w0 = torch.randn(n, generator=g)
                ws = [w0.to(d) for d in self.devices]
                lrs = [torch.tensor([0.5], device=d) for d in self.devices]
                for r in range(self.G):
                    with self.on(r):
                        chans[r].all_reduce_sgd(dev[r], ws[r], lrs[r], 1.0)
                self.synchronize()
                wref = w0 - 0.5 * want
                ok &= all(torch.allclose(w.cpu(), wref, rtol=0, atol=1e-6) for w in ws)
                ok &= all(torch.equal(ws[0].cpu(), w.cpu()) for w in ws[1:])
                ok &= all(ch.error() == 0 for ch in chans)
        return bool(ok)

    def _raw_channels(self, n: int, algo: int) -> list:
        from .. import ops

        C = ops.hip()
        chans = [C.XgmiChannel(r, self.G, n, d.index or 0, 10.0, algo, 0) for r, d in enumerate(self.devices)]
        for ch in chans:
            ch.connect_local(chans)
        self._chans[("selftest", n, algo)] = chans  # kept alive: graphs may reference them
        return chans

    def error(self) -> bool:
        """Whether an xGMI wait timed out on any device (host sync)."""
        for chans in self._chans.values():
            if any(ch.error() for ch in chans):
                return True
        return False

    # ------------------------------------------------------------------ RCCL clique
    def clique(self):
        if not self._clique_tried:
            self._clique_tried = True
            if self.distinct and os.environ.get("TDL_LOCAL_RCCL", "1") == "1":
                try:
                    from .. import ops

                    self._clique = ops.hip().RcclClique([d.index or 0 for d in self.devices])
                except Exception as e:  # noqa: BLE001 - RCCL unavailable: copies
                    self.reason = (self.reason + "; " if self.reason else "") + f"rccl clique: {e}"
        return self._clique

    # ------------------------------------------------------------------ collectives
    def synchronize(self):
        for d in {d for d in self.devices if d.type == "cuda"}:
            torch.cuda.synchronize(d)

    def all_reduce(self, ts: List[torch.Tensor], op: str = "sum") -> str:
        """In-place all-reduce of replica r's ``ts[r]`` (on device r) for every r; returns the path
        taken.  Sum/mean of contiguous f32 -> xGMI; otherwise the RCCL clique; otherwise copies."""
        if len(ts) != self.G:
            raise ValueError(f"all_reduce: {len(ts)} tensors for {self.G} replicas")
        if op in ("sum", "mean") and all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and
                                         t.data_ptr() % 16 == 0 for t in ts) and self.xgmi_ok():
            n = ts[0].numel()
            lim = int(os.environ.get("TDL_XGMI_MAX_BYTES", str(4 << 20))) // 4
            if not self.distinct:
                # replicas sharing a GPU: every replica's launch must be resident beside the others'
                # (each workgroup spins until the same workgroup of every peer arrives)
                lim = min(lim, int(os.environ.get("TDL_XGMI_CHUNK_ELEMS", str(256 * BLOCK))))
            chunk = min(lim, n) if n else 0
            scale = 1.0 / self.G if op == "mean" else 1.0
            for o in range(0, n, max(chunk, 1)):
                c = min(chunk, n - o)
                chans = self.channels(c)
                for r in range(self.G):
                    with self.on(r):
                        x = ts[r].view(-1)[o:o + c]
                        chans[r].all_reduce(x, x, scale)
            return "xgmi"
        cl = self.clique() if op in ("sum", "max", "min", "prod", "mean") else None
        if cl is not None and all(t.is_cuda and t.is_contiguous() for t in ts):
            code = {"sum": 0, "prod": 1, "max": 2, "min": 3, "mean": 4}[op]
            with self.all_streams():
                cl.all_reduce(list(ts), code)
            return "rccl"
        self._copies(ts, op)
        return "copies"

    def all_reduce_sgd(self, gs: List[torch.Tensor], ws: List[torch.Tensor], lrs: List[torch.Tensor]) -> bool:
        """``w_r -= lr_r * sum_q g_q`` on every replica in one xGMI launch per device; False when
        xGMI is unavailable (the caller all-reduces and applies SGD itself)."""
        if not self.xgmi_ok():
            return False
        n = gs[0].numel()
        chans = self.channels(n)
        for r in range(self.G):
            with self.on(r):
                chans[r].all_reduce_sgd(gs[r], ws[r], lrs[r], 1.0)
        return True

    def join_streams(self) -> None:
        """Every replica stream waits for the work already enqueued on every other replica stream
        (orders cross-replica reads/writes also when replicas share one device)."""
        evs = []
        for r in range(self.G):
            s = self.streams[r]
            if s is None:
                continue
            ev = torch.cuda.Event()
            ev.record(s)
            evs.append((r, ev))
        for r in range(self.G):
            s = self.streams[r]
            if s is not None:
                for q, ev in evs:
                    if q != r:
                        s.wait_event(ev)

    def broadcast(self, ts: List[torch.Tensor], src: int = 0) -> None:
        self.join_streams()
        with self.all_streams():
            for r in range(self.G):
                if r != src:
                    with self.on(r):
                        ts[r].copy_(ts[src].to(self.devices[r]))
        self.join_streams()

    def all_gather(self, ts: List[torch.Tensor]) -> List[torch.Tensor]:
        """[G, *shape] on every replica's device (its own stream)."""
        self.join_streams()
        outs = []
        with self.all_streams():
            for r in range(self.G):
                with self.on(r):
                    outs.append(torch.stack([x.to(ts[r].device) for x in ts]))
        self.join_streams()
        return outs

    def _copies(self, ts: List[torch.Tensor], op: str):
        """Rank-order reduction through device-to-device copies: replica r's stream waits for every
        replica's tensor, sums them in rank order on device r, and overwrites its own tensor only
        after every replica has read it."""
        cuda = [t.is_cuda for t in ts]
        ready = []
        for r, t in enumerate(ts):
            if cuda[r] and self.streams[r] is not None:
                ev = torch.cuda.Event()
                ev.record(self.streams[r])
                ready.append(ev)
            else:
                ready.append(None)
        accs = []
        with self.all_streams():
            for r, t in enumerate(ts):
                with self.on(r):
                    if cuda[r]:
                        for q, ev in enumerate(ready):
                            if ev is not None and q != r:
                                torch.cuda.current_stream(t.device).wait_event(ev)
                    acc = ts[0].to(t.device, copy=True)
                    for q in range(1, self.G):
                        x = ts[q].to(t.device)
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
                        acc = acc / self.G if acc.is_floating_point() else acc // self.G
                    accs.append(acc)
            done = []
            for r, t in enumerate(ts):
                if cuda[r] and self.streams[r] is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.streams[r])
                    done.append(ev)
                else:
                    done.append(None)
            for r, t in enumerate(ts):
                with self.on(r):
                    if cuda[r]:
                        for q, ev in enumerate(done):
                            if ev is not None and q != r:
                                torch.cuda.current_stream(t.device).wait_event(ev)
                    t.copy_(accs[r])

    def close(self):
        self._chans.clear()
        self._clique = None
