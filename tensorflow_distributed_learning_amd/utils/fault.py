"""Failure detection and fault injection for multi-worker jobs (test tier T-fault).

The reference assumes every gRPC server comes up and stays up (README.md:65-68): a dead worker
stalls the job.  Here a job fails fast and says why:

* **Detection.**  The chief's native KV server (csrc/native/store.cpp) marks a client whose TCP
  connection drops without an orderly BYE as *lost*, and every rank keeps a heartbeat connection
  (cluster/rendezvous.py).  :class:`PeerWatchdog` runs on every rank: on the chief it turns a lost or
  stale heartbeat into the job-wide key ``job/abort``; on every rank it polls that key and notices
  when the chief itself disappears.
* **Reaction.**  ``Model.fit`` calls :func:`check` at every execution boundary, which raises
  :class:`PeerLostError` on a fault.  A rank blocked inside a collective cannot reach that check,
  so after ``grace`` seconds the watchdog ends the process with exit status
  :data:`EXIT_PEER_LOST`, having printed the reason.  (The collective timeouts of the TCP ring and
  of RCCL/gloo stay as the last line of defence.)
* **Injection.**  ``TDL_FAULT_KILL_AT_STEP="rank:step"`` makes that rank die abruptly
  (``os._exit``) once its optimizer has taken ``step`` steps — the fault the tests inject.
  ``TDL_FAULT_CORRUPT_AT_STEP="rank:step"`` silently perturbs that rank's parameters instead
  (caught by the periodic replica-consistency check of ``fit``).

The job is not elastic: recovery is a restart that resumes from the chief's checkpoint
(``keras.callbacks.BackupAndRestore``), as with TF.
"""
from __future__ import annotations

import os
import sys
import threading
import time
from typing import Optional

EXIT_PEER_LOST = 75
EXIT_INJECTED = 43

_ACTIVE: Optional["PeerWatchdog"] = None


class PeerLostError(RuntimeError):
    """A peer of this multi-worker job died, hung, or the job was aborted."""


def _kill_spec():
    spec = os.environ.get("TDL_FAULT_KILL_AT_STEP")
    if not spec:
        return None
    r, s = spec.split(":")
    return int(r), int(s)


def maybe_inject(rank: int, step: int) -> None:
    """Fault injection hook: die abruptly when ``TDL_FAULT_KILL_AT_STEP`` names this rank/step."""
    spec = _kill_spec()
    if spec is not None and spec[0] == rank and step >= spec[1]:
        sys.stderr.write(f"[tdl] fault injection: rank {rank} exits at step {step}\n")
        sys.stderr.flush()
        os._exit(EXIT_INJECTED)


_CORRUPTED = set()


def maybe_corrupt(rank: int, step: int, slab) -> bool:
    """Fault injection hook: ``TDL_FAULT_CORRUPT_AT_STEP="rank:step"`` silently perturbs that
    rank's parameter slab once, at the first execution boundary at or after ``step`` (a broken
    fabric hand-off that no collective reports).  The periodic replica-consistency check of
    ``fit`` must catch it (parallel/consistency.py)."""
    spec = os.environ.get("TDL_FAULT_CORRUPT_AT_STEP")
    if not spec or slab is None:
        return False
    r, s = (int(v) for v in spec.split(":"))
    if r != rank or step < s or (r, s) in _CORRUPTED:
        return False
    _CORRUPTED.add((r, s))
    import torch

    with torch.no_grad():
        slab.view(-1)[: min(64, slab.numel())] += 0.5
    sys.stderr.write(f"[tdl] fault injection: rank {rank} parameters perturbed at step {step}\n")
    sys.stderr.flush()
    return True


def maybe_skip_collective(rank: int, step: int) -> bool:
    """Fault injection hook: ``TDL_FAULT_SKIP_ALLREDUCE_AT_STEP="rank:step"`` makes that rank leave
    out its gradient all-reduce once (a live rank out of step with its peers: the hung-collective
    case the progress watchdog and the collective timeouts must end)."""
    spec = os.environ.get("TDL_FAULT_SKIP_ALLREDUCE_AT_STEP")
    if not spec:
        return False
    r, s = (int(v) for v in spec.split(":"))
    if r != rank or step != s:
        return False
    sys.stderr.write(f"[tdl] fault injection: rank {rank} skips its gradient all-reduce at step {step}\n")
    sys.stderr.flush()
    return True


# this rank's training progress, published by its watchdog thread: [steps done, busy flag, seconds
# the last execution took].  busy = the host is inside a training execution or its log read (waiting
# on the device or on peers); a rank that stays busy without progressing for longer than its stall
# threshold is stuck
_PROGRESS = [0, False, 0.0]
_BUSY_SINCE = [None]


def note_progress(count: Optional[int] = None, busy: Optional[bool] = None) -> None:
    if count is not None:
        _PROGRESS[0] = int(count)
        if _BUSY_SINCE[0] is not None:  # an execution just completed: remember how long it took
            _PROGRESS[2] = time.monotonic() - _BUSY_SINCE[0]
            _BUSY_SINCE[0] = time.monotonic()
    if busy is not None:
        _PROGRESS[1] = bool(busy)
        _BUSY_SINCE[0] = time.monotonic() if busy else None


def stall_threshold(base: float, explicit: bool, count: int, last_exec_s: float) -> float:
    """Seconds a busy rank may go without progress before the job is declared stuck.

    An explicit ``TDL_STALL_TIMEOUT`` is taken as is.  Otherwise the threshold is the collective
    timeout, stretched to 10x the rank's own last execution (a long ``steps_per_execution`` or a
    chief-only checkpoint is not a stall), and the first execution (autotuning, graph capture,
    first-use compilation) gets 3x that and at least 15 minutes."""
    if explicit:
        return base
    t = max(base, 10.0 * last_exec_s)
    return max(3.0 * t, 900.0) if count == 0 else t


def check() -> None:
    """Raise :class:`PeerLostError` if the job has been aborted."""
    w = _ACTIVE
    if w is not None and w.reason is not None:
        w.acknowledged = True
        raise PeerLostError(w.reason)


class PeerWatchdog:
    """Per-rank failure detector over the rendezvous store (see module docstring)."""

    def __init__(self, rendezvous, interval: float = 0.5, stale_after: float = 60.0, grace: float = 30.0,
                 stall_after: Optional[float] = None):
        from .. import ops
        from ..parallel.communication import default_timeout

        self.rdv = rendezvous
        self.interval = float(interval)
        self.stale_after = float(stale_after)
        self.grace = float(grace)
        # a live rank (heartbeat fine) stuck inside an execution: a collective a peer never joins,
        # or a device wait that never ends (an all-reduce inside a replayed hipGraph is invisible
        # to the process group's own timeout)
        self._stall_explicit = "TDL_STALL_TIMEOUT" in os.environ
        self.stall_after = float(os.environ.get("TDL_STALL_TIMEOUT", stall_after or default_timeout()))
        self._published = None
        self._seen = {}  # chief: rank -> (progress record, monotonic time it last changed)
        self.on_abort = None  # e.g. the communicator's abort (strategy.py sets it)
        self.reason: Optional[str] = None
        self.acknowledged = False
        self._stop = threading.Event()
        lay = rendezvous.layout
        self.rank = lay.rank
        self.world = lay.world_size
        self._client = ops.native().KVClient(rendezvous.store_host, rendezvous.store_port, 10000,
                                             f"watchdog/{self.rank}")
        self._thread = threading.Thread(target=self._run, name="tdl-watchdog", daemon=True)

    def start(self) -> "PeerWatchdog":
        global _ACTIVE
        _ACTIVE = self
        self._thread.start()
        return self

    def stop(self):
        global _ACTIVE
        self._stop.set()
        if _ACTIVE is self:
            _ACTIVE = None
        self._thread.join(timeout=5 * self.interval + 1)
        try:
            self._client.close()
        except Exception:
            pass

    # ------------------------------------------------------------------------------------------
    def _chief_scan(self) -> Optional[str]:
        srv = self.rdv.server
        lost = [c for c in srv.lost_clients() if c.startswith("hb/")]
        if lost:
            return f"lost connection to {', '.join(sorted('rank ' + c[3:] for c in lost))} (process died)"
        stale = self.rdv.dead_peers(self.stale_after)
        if stale:
            return f"no heartbeat from {', '.join(sorted('rank ' + c[3:] for c in stale))} for {self.stale_after:.0f}s"
        return self._stall_scan()

    def _publish_progress(self):
        rec = f"{_PROGRESS[0]} {int(_PROGRESS[1])} {_PROGRESS[2]:.3f}"
        if rec != self._published:
            self._client.set(f"progress/{self.rank}", rec.encode())
            self._published = rec

    def _stall_scan(self) -> Optional[str]:
        """Chief: ranks busy in an execution whose progress record has not changed for
        ``stall_after`` seconds."""
        if self.stall_after <= 0:
            return None
        now = time.monotonic()
        stuck, counts = [], {}
        for r in range(self.world):
            key = f"progress/{r}"
            if not self._client.check([key]):
                continue
            rec = bytes(self._client.get(key)).decode()
            prev = self._seen.get(r)
            if prev is None or prev[0] != rec:
                self._seen[r] = (rec, now)
                prev = self._seen[r]
            f = rec.split()
            n, busy, last = f[0], f[1], float(f[2]) if len(f) > 2 else 0.0
            counts[r] = int(n)
            lim = stall_threshold(self.stall_after, self._stall_explicit, int(n), last)
            if busy == "1" and now - prev[1] > lim:
                stuck.append(r)
        if not stuck:
            return None
        where = ", ".join(f"rank {r} at execution {counts[r]}" for r in stuck)
        others = ", ".join(f"rank {r}: {c}" for r, c in sorted(counts.items()) if r not in stuck)
        return (f"no training progress past the stall threshold ({self.stall_after:.0f}s base) on {where} (heartbeats alive: a collective a peer "
                f"never joined, or a hung device wait){'; ' + others if others else ''}")

    def _abort(self, reason: str):
        if self.reason is None:
            self.reason = reason
            sys.stderr.write(f"[tdl] rank {self.rank}: aborting multi-worker job: {reason}\n")
            sys.stderr.flush()
            if self.on_abort is not None:  # unblock a collective this rank may be stuck in
                try:
                    self.on_abort()
                except Exception:  # noqa: BLE001 - best effort; the grace-period exit follows
                    pass

    def _run(self):
        aborted_at = None
        while not self._stop.wait(self.interval):
            if self.reason is None:
                try:
                    self._publish_progress()
                    if self.rdv.server is not None:
                        why = self._chief_scan()
                        if why is not None:
                            self._client.set("job/abort", why.encode())
                    if self._client.check(["job/abort"]):
                        self._abort(bytes(self._client.get("job/abort")).decode())
                except Exception as e:  # the chief's store is gone
                    if self._stop.is_set():
                        return
                    self._abort(f"lost connection to the chief's rendezvous store ({e})")
            if self.reason is not None:
                aborted_at = aborted_at or time.monotonic()
                if not self.acknowledged and time.monotonic() - aborted_at > self.grace:
                    sys.stderr.write(f"[tdl] rank {self.rank}: still blocked {self.grace:.0f}s after the abort; "
                                     f"exiting ({self.reason})\n")
                    sys.stderr.flush()
                    os._exit(EXIT_PEER_LOST)
                if self.acknowledged:
                    return
