"""Cluster bring-up over the native C++ TCP key-value store (csrc/native/store.cpp).

Reference behaviour (README.md:64-68): each task starts a server on its TF_CONFIG ``host:port``,
waits until every peer is up, trains, and shuts down.  Here the chief task's local rank 0 runs a
:class:`KVServer` on the chief's TF_CONFIG address; every replica process connects a client,

1. claims its slot ``member/<type>/<index>/<local_rank>`` with compare-and-set – a second process
   claiming the same slot (tf_dist_example.py:6-10 hard-codes ``index: 1`` on every host, quirk Q1)
   is rejected with a clear error instead of hanging;
2. publishes ``task/<type>/<index>`` = its replica count (one process per GPU);
3. waits until every training task has published, computes the global rank layout
   (chief first, then workers; ranks contiguous per task) and waits for every member;
4. keeps a heartbeat connection so the chief can detect dead peers; ``shutdown()`` is a barrier
   so the chief does not stop the store while peers still need it.

:class:`NativeStore` adapts the same client to ``torch.distributed.Store`` so RCCL (``nccl``)
and gloo process groups bootstrap through the C++ store as well.
"""
from __future__ import annotations

import json
import os
import socket
import threading
import time
import uuid
from dataclasses import dataclass
from datetime import timedelta
from typing import Dict, List, Optional

import torch.distributed as dist

from .. import ops
from .tf_config import ClusterConfigError, TaskSpec, TFConfig


class RendezvousError(RuntimeError):
    pass


def _ms(t: Optional[float]) -> int:
    return -1 if t is None else int(t * 1000)


class NativeStore(dist.Store):
    """torch.distributed.Store backed by the C++ KV client."""

    def __init__(self, host: str, port: int, timeout: float = 300.0, name: str = "", prefix: str = ""):
        super().__init__()
        self._host, self._port, self._name = host, port, name
        self._timeout = timeout
        self._prefix = prefix
        self._client = ops.native().KVClient(host, port, _ms(timeout), name)

    def _k(self, key: str) -> str:
        return self._prefix + key

    # torch.distributed.Store API ------------------------------------------------------------
    def set(self, key, value):
        if isinstance(value, str):
            value = value.encode()
        self._client.set(self._k(key), bytes(value))

    def get(self, key):
        v = self._client.get(self._k(key), _ms(self._timeout))
        if v is None:
            raise RendezvousError(f"store get('{key}') timed out after {self._timeout}s")
        return v

    def add(self, key, amount):
        return self._client.add(self._k(key), int(amount))

    def compare_set(self, key, expected, desired):
        e = expected.encode() if isinstance(expected, str) else bytes(expected)
        d = desired.encode() if isinstance(desired, str) else bytes(desired)
        return self._client.compare_set(self._k(key), e, d)

    def check(self, keys):
        return self._client.check([self._k(k) for k in keys])

    def delete_key(self, key):
        return self._client.delete(self._k(key))

    def num_keys(self):
        return self._client.num_keys()

    def wait(self, keys, timeout=None):
        t = self._timeout if timeout is None else (timeout.total_seconds() if isinstance(timeout, timedelta) else timeout)
        if not self._client.wait([self._k(k) for k in keys], _ms(t)):
            raise RendezvousError(f"store wait({keys}) timed out after {t}s")

    def set_timeout(self, timeout):
        self._timeout = timeout.total_seconds() if isinstance(timeout, timedelta) else float(timeout)

    @property
    def timeout(self):
        return timedelta(seconds=self._timeout)

    def append(self, key, value):
        if isinstance(value, str):
            value = value.encode()
        self._client.append(self._k(key), bytes(value))

    def ping(self) -> bool:
        return self._client.ping()

    def close(self):
        self._client.close()


@dataclass
class RankLayout:
    rank: int
    world_size: int
    local_rank: int
    num_local: int
    task: Optional[TaskSpec]
    task_rank: int
    tasks: List[Dict]

    @property
    def is_chief_process(self) -> bool:
        return self.rank == 0


class Rendezvous:
    """Join a cluster described by TF_CONFIG.  See module docstring."""

    def __init__(self, cfg: TFConfig, local_rank: int = 0, num_local: int = 1, timeout: float = 300.0,
                 heartbeat_interval: float = 5.0, host_for_server: Optional[str] = None):
        if cfg.task is None:
            raise ClusterConfigError("TF_CONFIG has no 'task'; cannot join a multi-worker cluster")
        if not cfg.is_training_task:
            raise ClusterConfigError(
                f"task {cfg.task} is a '{cfg.task.type}' task: ps/evaluator tasks take no part in "
                "MultiWorkerMirroredStrategy all-reduce training (README.md:55-57)")
        self.cfg = cfg
        self.local_rank = int(local_rank)
        self.num_local = int(num_local)
        self.timeout = float(timeout)
        self.heartbeat_interval = heartbeat_interval
        self.server = None
        host, port = cfg.chief_address
        self.store_host = host
        self.store_port = port
        self._uid = uuid.uuid4().hex
        self._hb_stop = threading.Event()
        self._hb_thread = None
        self.layout: Optional[RankLayout] = None
        if cfg.is_chief and self.local_rank == 0:
            bind = host_for_server or os.environ.get("TDL_RENDEZVOUS_BIND", "0.0.0.0")
            try:
                self.server = ops.native().KVServer(bind, port)
            except RuntimeError as e:
                raise RendezvousError(f"chief could not listen on {bind}:{port}: {e}") from e
        name = f"{cfg.task.type}/{cfg.task.index}/{self.local_rank}"
        self.store = NativeStore(host, port, timeout=self.timeout, name=name)

    # ------------------------------------------------------------------------------------------
    def join(self) -> RankLayout:
        cfg, st = self.cfg, self.store
        t = cfg.task
        slot = f"member/{t.type}/{t.index}/{self.local_rank}"
        payload = json.dumps({"uid": self._uid, "pid": os.getpid(), "host": socket.gethostname()}).encode()
        got = st.compare_set(slot, b"", payload)
        if bytes(got) != payload:
            other = json.loads(bytes(got).decode() or "{}")
            raise RendezvousError(
                f"cluster slot {t.type}/{t.index} (local replica {self.local_rank}) is already taken by pid "
                f"{other.get('pid')} on {other.get('host')}: every task needs a distinct TF_CONFIG task "
                "(README.md:59); two processes claimed the same one")
        if self.local_rank == 0:
            st.set(f"task/{t.type}/{t.index}", json.dumps({"num_local": self.num_local}))
        tasks = cfg.cluster.training_tasks()
        keys = [f"task/{x.type}/{x.index}" for x in tasks]
        st.wait(keys, timeout=self.timeout)
        infos = []
        for x in tasks:
            n = int(json.loads(st.get(f"task/{x.type}/{x.index}").decode())["num_local"])
            infos.append({"type": x.type, "index": x.index, "num_local": n})
        offsets, acc = [], 0
        for inf in infos:
            offsets.append(acc)
            acc += inf["num_local"]
        my_task_rank = tasks.index(t)
        if infos[my_task_rank]["num_local"] != self.num_local:
            raise RendezvousError("replica count mismatch between processes of the same task")
        members = [f"member/{x['type']}/{x['index']}/{lr}" for x in infos for lr in range(x["num_local"])]
        st.wait(members, timeout=self.timeout)
        self.layout = RankLayout(rank=offsets[my_task_rank] + self.local_rank, world_size=acc,
                                 local_rank=self.local_rank, num_local=self.num_local, task=t,
                                 task_rank=my_task_rank, tasks=infos)
        self.barrier("joined")
        self._start_heartbeat()
        return self.layout

    def barrier(self, tag: str, timeout: Optional[float] = None):
        lay = self.layout
        if lay is None:
            raise RendezvousError("barrier before join")
        self.store.set(f"barrier/{tag}/{lay.rank}", b"1")
        self.store.wait([f"barrier/{tag}/{r}" for r in range(lay.world_size)],
                        timeout=self.timeout if timeout is None else timeout)

    def _start_heartbeat(self):
        if self.heartbeat_interval <= 0:
            return
        lay = self.layout
        name = f"hb/{lay.rank}"

        def beat():
            try:
                cli = ops.native().KVClient(self.store_host, self.store_port, 10000, name)
            except Exception:
                return
            while not self._hb_stop.wait(self.heartbeat_interval):
                try:
                    cli.ping()
                except Exception:
                    break
            try:
                cli.close()
            except Exception:
                pass

        self._hb_thread = threading.Thread(target=beat, name="tdl-heartbeat", daemon=True)
        self._hb_thread.start()

    def dead_peers(self, max_age: float) -> List[str]:
        """Chief only: heartbeat clients not heard from within ``max_age`` seconds."""
        if self.server is None:
            return []
        return [k for k, age in self.server.heartbeat_ages().items() if k.startswith("hb/") and age > max_age]

    def shutdown(self, timeout: float = 60.0):
        """Orderly teardown (README.md:68): barrier, then the chief stops the store."""
        self._hb_stop.set()
        try:
            if self.layout is not None:
                self.barrier("shutdown", timeout=timeout)
        except Exception:
            pass
        if self._hb_thread is not None:
            self._hb_thread.join(timeout=2 * self.heartbeat_interval + 1)
        if self.server is not None:
            # let the peers leave the shutdown barrier before the store disappears
            deadline = time.time() + 5.0
            while time.time() < deadline:
                ages = self.server.heartbeat_ages()
                if len([k for k in ages if not k.startswith("hb/")]) <= 1:
                    break
                time.sleep(0.02)
        try:
            self.store.close()
        except Exception:
            pass
        if self.server is not None:
            self.server.stop()
            self.server = None
