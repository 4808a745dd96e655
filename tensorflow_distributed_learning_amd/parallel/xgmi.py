"""One-shot xGMI all-reduce for small messages (SURVEY.md §2.8 "algorithm selection", §5 comm row).

RCCL's ring all-reduce of a sub-MiB message pays 2(R-1) dependent hops over one xGMI link per hop.
On one MI355X node every GPU has a direct link to every other GPU, so for messages up to a few MiB
each rank pulls every peer's slice in ONE hop and reduces it locally
(``csrc/kernels/xgmi.hip``); the SGD update can ride in the same kernel.  TF's ``AUTO``
collective selection by "hardware, network topology, tensor size" (README.md:21) is this choice:
xGMI one-shot below ``TDL_XGMI_MAX_BYTES`` (default 4 MiB) on a single node, RCCL otherwise.

Exchange buffers are exported with HIP IPC and opened by every peer (one channel per message size;
channel set-up is collective, so it happens outside graph capture: :meth:`XgmiAllReduce.prepare`).
A self-test against an all-gather reference runs when the first channel is made; if any rank
fails it (or cannot map its peers), every rank falls back to RCCL.  Waits inside the kernel are
bounded (``TDL_XGMI_TIMEOUT`` seconds): a peer that never arrives raises an error on the host at
the next :meth:`check` instead of hanging the GPU.
"""
from __future__ import annotations

import os
import socket
import warnings
from typing import Dict, Optional

import torch
import torch.distributed as dist

BLOCK = 1024  # f32 elements per workgroup (kXgmiBlockElems)


def enabled_by_env() -> bool:
    return os.environ.get("TDL_XGMI", "1") == "1"


def max_bytes() -> int:
    return int(os.environ.get("TDL_XGMI_MAX_BYTES", str(4 << 20)))


def choose_algo(numel: int, world: int) -> int:
    """0 = one-shot, 1 = two-shot.  One-shot moves (R-1) x n bytes over a rank's links, two-shot
    2 (R-1)/R x n in two hops: above ``TDL_XGMI_ONESHOT_MAX_BYTES`` (256 KiB) at R >= 3 the
    bandwidth term wins over the extra hop."""
    lim = int(os.environ.get("TDL_XGMI_ONESHOT_MAX_BYTES", str(256 << 10)))
    return 1 if world >= 3 and 4 * numel > lim else 0


class XgmiAllReduce:
    """Channel manager of one process group (every rank on this node, one GPU each)."""

    def __init__(self, rank: int, world: int, device: torch.device, group=None, ctrl_device=None,
                 timeout: Optional[float] = None):
        from .. import ops

        self.C = ops.hip()
        self.rank, self.world, self.device, self.group = rank, world, torch.device(device), group
        # device of the small control collectives (the process group's own: cpu for gloo)
        self.ctrl = torch.device(ctrl_device) if ctrl_device is not None else self.device
        # bounded in-kernel waits: a peer that does not arrive within this many seconds sets the
        # device's error word; every later exchange then returns at entry and the host raises at the
        # next health check (log read / execution boundary).  Default: the job's collective timeout
        # (the process group's), so a slow but live peer is no more fatal here than under RCCL --
        # capped at 120 s: a GPU spinning in an exchange holds its queue, and the peers of a
        # synchronous step arrive within milliseconds of each other when they are alive
        if timeout is None:
            from .communication import default_timeout

            timeout = min(default_timeout(), 120.0)
        self.timeout = float(os.environ.get("TDL_XGMI_TIMEOUT", timeout))
        self.limit = max_bytes() // 4
        self._chans: Dict[int, object] = {}
        self._selftest_chans = []
        self._dedicated = []
        self.ok: Optional[bool] = None  # None = not yet tested
        self.reason = ""
        # messages above the channel limit in limit-sized chunks (one launch each) -- only where the
        # kernel is the job's sole device data plane (gloo control plane: replicas sharing a GPU);
        # with RCCL beside it, large messages belong to RCCL's bandwidth-optimal rings
        self.chunked = False
        # chunked mode: elements per launch.  Replicas sharing one GPU spin in their exchange
        # workgroups until the peer's workgroup of the same index arrives, so every replica's launch
        # (beside the backward kernels still running) must fit on the GPU at once: 256 workgroups
        # per launch, not the 1024 of a full 4 MiB channel
        self.chunk = min(self.limit, int(os.environ.get("TDL_XGMI_CHUNK_ELEMS", str(256 * BLOCK))))

    # ------------------------------------------------------------------ set-up (collective)
    def _make(self, numel: int, timeout: Optional[float] = None, min_blocks: int = 0):
        ch = self.C.XgmiChannel(self.rank, self.world, numel, self.device.index or 0,
                                self.timeout if timeout is None else timeout, choose_algo(numel, self.world),
                                int(min_blocks))
        mine = (bytes(ch.handle(False)), bytes(ch.handle(True)))
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=self.group)
        err = ""
        try:
            ch.open([h[0] for h in allh], [h[1] for h in allh])
        except Exception as e:  # noqa: BLE001 - reported collectively below
            err = f"{type(e).__name__}: {e}"
        if not self._agree(not err):
            raise RuntimeError(f"xgmi: peer buffers could not be mapped on every rank ({err or 'another rank failed'})")
        return ch

    def _agree(self, ok: bool) -> bool:
        f = torch.tensor([1.0 if ok else 0.0], device=self.ctrl)
        dist.all_reduce(f, op=dist.ReduceOp.MIN, group=self.group)
        return bool(f.item() > 0.5)

    def _chunks(self, n: int):
        """[(offset, size)] of a message of n elements: one piece, or (chunked) ``chunk``-sized
        pieces (offsets multiples of the chunk: 16-B aligned) and the remainder."""
        n = int(n)
        if not self.chunked:
            return [(0, n)]
        return [(o, min(self.chunk, n - o)) for o in range(0, n, self.chunk)]

    def prepare(self, *numels: int) -> bool:
        """Create (collectively) the channels for these message sizes; False if disabled."""
        if not self._ensure_tested():
            return False
        for n in numels:
            for _, c in self._chunks(int(n)):
                if 0 < c <= self.limit and c not in self._chans:
                    self._chans[c] = self._make(c)
        return True

    def _ensure_tested(self) -> bool:
        if self.ok is None and torch.cuda.is_current_stream_capturing():
            return False  # the self-test is collective: never inside a capture (all ranks agree)
        if self.ok is None:
            try:
                self.ok = self._selftest()
                if not self.ok:
                    self.reason = "self-test mismatch"
            except Exception as e:  # noqa: BLE001 - any failure means RCCL
                self.ok, self.reason = False, f"{type(e).__name__}: {e}"
            if not self.ok and self.rank == 0:
                warnings.warn(f"xGMI one-shot all-reduce disabled, using RCCL ({self.reason})")
        return self.ok

    def _selftest(self) -> bool:
        """Both algorithms (a small and a large message): eager, repeated (both buffer halves),
        graph-replayed and fused-SGD calls against an exact all-gather reference summed in rank
        order (bit-identical expected)."""
        ok = True
        for n in (3 * BLOCK + 37, 70 * BLOCK + 5):
            ok &= self._selftest_one(n)
        return self._agree(ok)

    def _selftest_one(self, n: int) -> bool:
        # short bounded waits: a protocol failure on this machine must fall back, not stall
        ch = self._make(n, timeout=10.0)
        dev = self.device
        g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
        ok = True

        def ref(x):
            parts = [torch.empty(x.numel(), dtype=x.dtype, device=self.ctrl) for _ in range(self.world)]
            dist.all_gather(parts, x.to(self.ctrl), group=self.group)
            acc = parts[0].clone()
            for r in range(1, self.world):
                acc += parts[r]
            return acc.to(dev)

        for it in range(3):
            x = torch.randn(n, generator=g).to(dev)
            y = torch.empty_like(x)
            ch.all_reduce(x, y, 1.0)
            ok &= bool(torch.equal(y, ref(x)))
        x = torch.randn(n, generator=g).to(dev)
        want = ref(x)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        y = torch.zeros_like(x)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=s):
            ch.all_reduce(x, y, 1.0)
        torch.cuda.synchronize(dev)
        for _ in range(3):
            y.zero_()
            graph.replay()
            torch.cuda.synchronize(dev)
            ok &= bool(torch.equal(y, want))
        # the same parameters on every rank, as in training: the two-shot SGD epilogue updates each
        # shard on its owner and the other ranks copy the owner's result
        w = torch.randn(n, generator=torch.Generator(device="cpu").manual_seed(4321)).to(dev)
        w_ref = w - 0.5 * want
        lr = torch.tensor([0.5], device=dev)
        ch.all_reduce_sgd(x, w, lr, 1.0)
        torch.cuda.synchronize(dev)
        ok &= bool(torch.allclose(w, w_ref, rtol=0, atol=1e-6))
        ok &= ch.error() == 0
        self._selftest_chans.append(ch)  # kept alive (see close); not reused for traffic
        return bool(ok)

    def dedicated(self, numel: int, min_blocks: int):
        """Collective: a channel of its own (not shared with ``all_reduce``) for a kernel that runs
        the exchange protocol in its own workgroups (``min_blocks`` signal slots); None if xGMI is
        disabled on this job."""
        if not self._ensure_tested():
            return None
        ch = self._make(int(numel), min_blocks=int(min_blocks))
        self._dedicated.append(ch)
        return ch

    # ------------------------------------------------------------------ collectives
    def _channel(self, n: int):
        ch = self._chans.get(n)
        if ch is not None or n > self.limit or not self.ok:
            return ch
        if torch.cuda.is_current_stream_capturing():
            return None  # set-up is collective and cannot run inside a capture: RCCL for this one
        self._chans[n] = self._make(n)
        return self._chans[n]

    def has_channel(self, n: int) -> bool:
        return bool(self.ok) and int(n) > 0 and all(c in self._chans for _, c in self._chunks(int(n)))

    def applicable(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0 and
                0 < t.numel() and (t.numel() <= self.limit or self.chunked))

    def _pieces(self, n: int):
        """[(offset, size, channel)] for a message of n elements, or None (some channel missing)."""
        out = []
        for o, c in self._chunks(n):
            ch = self._channel(c)
            if ch is None:
                return None
            out.append((o, c, ch))
        return out

    def all_reduce(self, t: torch.Tensor, op: str) -> bool:
        """In-place sum/mean of ``t`` on the current stream; False = not handled (use RCCL)."""
        if op not in ("sum", "mean") or not self.applicable(t) or not self._ensure_tested():
            return False
        pieces = self._pieces(t.numel())
        if pieces is None:
            return False
        flat = t.view(-1)
        scale = 1.0 / self.world if op == "mean" else 1.0
        for o, c, ch in pieces:
            x = flat[o:o + c]
            ch.all_reduce(x, x, scale)
        return True

    def all_reduce_sgd(self, g: torch.Tensor, w: torch.Tensor, lr: torch.Tensor) -> bool:
        """``w -= lr * sum_over_ranks(g)`` (one kernel per piece); False = not handled."""
        if not (self.applicable(g) and self.applicable(w)) or g.numel() != w.numel() or not self._ensure_tested():
            return False
        pieces = self._pieces(g.numel())
        if pieces is None:
            return False
        gf, wf = g.view(-1), w.view(-1)
        for o, c, ch in pieces:
            ch.all_reduce_sgd(gf[o:o + c], wf[o:o + c], lr, 1.0)
        return True

    def _any_channel(self):
        for group in (list(self._chans.values()), self._dedicated, self._selftest_chans):
            if group:
                return group[0]
        return None

    def error(self) -> bool:
        """Whether any xGMI kernel on this device timed out waiting for a peer (host sync; one
        error word per device, shared by every channel: any channel reads it)."""
        ch = self._any_channel()
        return bool(ch is not None and ch.error())

    def check(self) -> None:
        """Raise if any kernel of this rank timed out waiting for a peer (host sync)."""
        if self.error():
            raise RuntimeError(f"xgmi all-reduce: a peer did not arrive within {self.timeout:.0f} s; "
                               "the job's ranks are out of step or one died")

    def disable(self, reason: str) -> None:
        """Stop routing collectives through the kernel (every rank must call this at the same point)."""
        self.ok, self.reason = False, reason

    def close(self) -> None:
        self._chans.clear()
        self._selftest_chans.clear()
        self._dedicated.clear()


def single_node(group=None) -> bool:
    """True when every rank of the (initialised) default group runs on this host."""
    me = socket.gethostname()
    names = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, me, group=group)
    return all(n == me for n in names)
