"""Job liveness for replica groups started WITHOUT a TF_CONFIG rendezvous (launcher, torchrun,
self-spawned ``MirroredStrategy`` replicas, ``bench.py``).

The reference's cluster flow (README.md:65-68) assumes every task stays up; a dead worker stalls
the job.  Multi-worker jobs here get failure detection from the rendezvous store
(cluster/rendezvous.py + utils/fault.py).  A job that bootstrapped through ``torch.distributed``
(``MASTER_ADDR``/``MASTER_PORT``) has no such store, so this module gives it the same detector:

* rank 0 starts a native :class:`KVServer` (csrc/native/store.cpp) on an ephemeral port and
  publishes ``host:port`` through the process group's own store;
* every rank keeps a heartbeat connection ``hb/<rank>`` to it.  A process that dies closes its
  socket without the orderly BYE, which the server records as a *lost* client immediately (no
  timeout needed); a hung process stops pinging and goes stale;
* :class:`~..utils.fault.PeerWatchdog` runs on every rank over this object exactly as over a
  :class:`~.rendezvous.Rendezvous` (same attributes: ``server``, ``store_host``/``store_port``,
  ``layout``, ``dead_peers``) and turns a fault into ``PeerLostError`` at the next execution
  boundary, or ends a rank that is blocked in a collective after a grace period.

Shutdown is ordered: rank 0 keeps its server up until the other ranks' clients have left.
"""
from __future__ import annotations

import os
import socket
import threading
import time
from types import SimpleNamespace
from typing import List, Optional

from .. import ops

_KEY = "tdl/liveness/addr"


def _my_host() -> str:
    h = os.environ.get("TDL_LIVENESS_HOST")
    if h:
        return h
    master = os.environ.get("MASTER_ADDR", "127.0.0.1")
    if master in ("127.0.0.1", "localhost", ""):
        return "127.0.0.1"
    try:
        return socket.gethostbyname(socket.gethostname())
    except OSError:
        return master


def heartbeat_thread(host: str, port: int, name: str, interval: float, stop: threading.Event) -> threading.Thread:
    """Daemon thread keeping one named client connection to the store alive (one ping per
    ``interval``); the server tracks each named client's last contact (heartbeat_ages) and marks
    it lost when its socket drops without BYE."""

    def beat():
        try:
            cli = ops.native().KVClient(host, port, 10000, name)
        except Exception:
            return
        while not stop.wait(interval):
            try:
                cli.ping()
            except Exception:
                break
        try:
            cli.close()
        except Exception:
            pass

    t = threading.Thread(target=beat, name="tdl-heartbeat", daemon=True)
    t.start()
    return t


class Liveness:
    """Failure detector of one job (see module docstring).  ``store``: any torch.distributed-style
    store shared by the ranks (used once, to publish the server address)."""

    def __init__(self, rank: int, world: int, store, heartbeat_interval: float = 2.0, timeout: float = 120.0):
        self.layout = SimpleNamespace(rank=int(rank), world_size=int(world))
        self.heartbeat_interval = float(heartbeat_interval)
        self.server = None
        self._stop = threading.Event()
        if rank == 0:
            self.server = ops.native().KVServer("0.0.0.0", 0)
            addr = f"{_my_host()}:{self.server.port}"
            store.set(_KEY, addr.encode())
        else:
            if hasattr(store, "wait"):
                try:
                    from datetime import timedelta

                    store.wait([_KEY], timedelta(seconds=timeout))
                except TypeError:
                    store.wait([_KEY])
            addr = bytes(store.get(_KEY)).decode()
        host, port = addr.rsplit(":", 1)
        self.store_host, self.store_port = host, int(port)
        self._hb = heartbeat_thread(self.store_host, self.store_port, f"hb/{rank}", self.heartbeat_interval,
                                    self._stop)

    def dead_peers(self, max_age: float) -> List[str]:
        """Rank 0 only: heartbeat clients not heard from within ``max_age`` seconds."""
        if self.server is None:
            return []
        return [k for k, age in self.server.heartbeat_ages().items() if k.startswith("hb/") and age > max_age]

    def shutdown(self, wait: float = 30.0):
        self._stop.set()
        self._hb.join(timeout=2 * self.heartbeat_interval + 1)
        if self.server is not None:
            # keep serving until every other rank's clients have left (a rank still running its
            # watchdog would otherwise see the server vanish and abort a job that finished)
            deadline = time.monotonic() + wait
            while time.monotonic() < deadline:
                if not set(self.server.heartbeat_ages()) - set(self.server.lost_clients()):
                    break
                time.sleep(0.05)
            self.server.stop()
            self.server = None


def start_for_process_group(rank: int, world: int) -> Optional[object]:
    """Liveness + PeerWatchdog for an initialised default process group (None when disabled
    with ``TDL_WATCHDOG=0``, for world 1, or when set-up fails: detection is best effort and never
    fails a job on its own)."""
    if world <= 1 or os.environ.get("TDL_WATCHDOG", "1") != "1" or not ops.native_available():
        return None
    try:
        from torch.distributed import distributed_c10d as c10d

        from ..utils.fault import PeerWatchdog

        store = c10d._get_default_store()
        lv = Liveness(rank, world, store, heartbeat_interval=float(os.environ.get("TDL_HEARTBEAT_INTERVAL", "2")))
        wd = PeerWatchdog(lv, stale_after=float(os.environ.get("TDL_HEARTBEAT_TIMEOUT", "60")),
                          grace=float(os.environ.get("TDL_ABORT_GRACE", "30")))
        wd.liveness = lv
        return wd.start()
    except Exception as e:  # noqa: BLE001
        import sys

        sys.stderr.write(f"[tdl] rank {rank}: job liveness watchdog not started ({type(e).__name__}: {e})\n")
        return None
