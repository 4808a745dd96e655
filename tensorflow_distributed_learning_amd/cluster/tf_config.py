"""TF_CONFIG cluster definition (README.md:31-61, tf_dist_example.py:6-10).

``TF_CONFIG`` is a JSON object::

    {"cluster": {"chief": ["host1:port"], "worker": ["host2:port", ...],
                 "ps": [...], "evaluator": [...]},
     "task": {"type": "worker", "index": 0}}

* ``cluster`` must be identical on every task; only ``task`` differs (README.md:59).
* the chief is ``chief/0`` if present, else ``worker/0`` (README.md:51); it does the extra work
  (checkpoints, event logs).
* the collective group is every ``chief`` + ``worker`` task; ``ps`` / ``evaluator`` take no part
  in all-reduce training (README.md:55-57).
* a missing/empty TF_CONFIG, or a cluster with a single training task, degrades to a local
  MirroredStrategy (README.md:34).

Rank layout (ours): training tasks ordered chief first, then workers by index; each task may own
several replicas (one process per GPU); global rank = sum(replicas of earlier tasks) + local rank.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

TRAINING_ROLES = ("chief", "worker")
ALL_ROLES = ("chief", "worker", "ps", "evaluator")


class ClusterConfigError(ValueError):
    pass


def _split_addr(addr: str) -> Tuple[str, int]:
    if not isinstance(addr, str) or ":" not in addr:
        raise ClusterConfigError(f"cluster address must be 'host:port', got {addr!r}")
    host, port = addr.rsplit(":", 1)
    host = host.strip("[]")
    try:
        p = int(port)
    except ValueError:
        raise ClusterConfigError(f"bad port in address {addr!r}") from None
    if not (0 < p < 65536):
        raise ClusterConfigError(f"port out of range in address {addr!r}")
    return host, p


@dataclass(frozen=True)
class TaskSpec:
    type: str
    index: int

    def __str__(self):
        return f"/job:{self.type}/task:{self.index}"


@dataclass
class ClusterSpec:
    """Role -> list of 'host:port' (tf.train.ClusterSpec equivalent)."""

    jobs: Dict[str, List[str]] = field(default_factory=dict)

    def __post_init__(self):
        norm = {}
        for role, addrs in (self.jobs or {}).items():
            if isinstance(addrs, dict):  # {"0": "h:p"} sparse form
                addrs = [addrs[k] for k in sorted(addrs, key=int)]
            if not isinstance(addrs, (list, tuple)):
                raise ClusterConfigError(f"cluster[{role!r}] must be a list of 'host:port'")
            for a in addrs:
                _split_addr(a)
            norm[role] = list(addrs)
        self.jobs = norm
        if len(self.jobs.get("chief", [])) > 1:
            raise ClusterConfigError("a cluster may have at most one chief")
        if len(self.jobs.get("evaluator", [])) > 1:
            raise ClusterConfigError("a cluster may have at most one evaluator")
        seen: Dict[str, str] = {}
        for role, addrs in self.jobs.items():
            for i, a in enumerate(addrs):
                if a in seen:
                    raise ClusterConfigError(f"address {a} used by both {seen[a]} and {role}/{i}")
                seen[a] = f"{role}/{i}"

    @property
    def job_names(self) -> List[str]:
        return list(self.jobs)

    def num_tasks(self, role: str) -> int:
        return len(self.jobs.get(role, []))

    def task_address(self, role: str, index: int) -> str:
        try:
            return self.jobs[role][index]
        except (KeyError, IndexError):
            raise ClusterConfigError(f"task {role}/{index} is not in the cluster {self.jobs}") from None

    def training_tasks(self) -> List[TaskSpec]:
        """Collective-group members in rank order: chief first, then workers by index."""
        out = [TaskSpec("chief", i) for i in range(self.num_tasks("chief"))]
        out += [TaskSpec("worker", i) for i in range(self.num_tasks("worker"))]
        return out

    def as_dict(self) -> Dict[str, List[str]]:
        return {k: list(v) for k, v in self.jobs.items()}


@dataclass
class TFConfig:
    cluster: ClusterSpec
    task: Optional[TaskSpec]
    rpc_layer: str = "grpc"
    environment: str = ""

    # ------------------------------------------------------------------ roles
    @property
    def chief_task(self) -> Optional[TaskSpec]:
        if self.cluster.num_tasks("chief"):
            return TaskSpec("chief", 0)
        if self.cluster.num_tasks("worker"):
            return TaskSpec("worker", 0)
        return None

    @property
    def is_chief(self) -> bool:
        if self.task is None:
            return True
        return self.task == self.chief_task

    @property
    def is_training_task(self) -> bool:
        return self.task is None or self.task.type in TRAINING_ROLES

    @property
    def num_training_tasks(self) -> int:
        return len(self.cluster.training_tasks())

    @property
    def task_rank(self) -> int:
        """Position of this task in the collective group (0 = chief)."""
        if self.task is None:
            return 0
        tasks = self.cluster.training_tasks()
        if self.task not in tasks:
            raise ClusterConfigError(f"{self.task} is not a member of the collective group")
        return tasks.index(self.task)

    @property
    def is_single_worker(self) -> bool:
        return self.num_training_tasks <= 1

    @property
    def chief_address(self) -> Tuple[str, int]:
        c = self.chief_task
        if c is None:
            raise ClusterConfigError("cluster has no chief and no worker")
        return _split_addr(self.cluster.task_address(c.type, c.index))

    @property
    def task_address(self) -> Optional[Tuple[str, int]]:
        if self.task is None:
            return None
        return _split_addr(self.cluster.task_address(self.task.type, self.task.index))

    def to_json(self) -> str:
        d = {"cluster": self.cluster.as_dict()}
        if self.task is not None:
            d["task"] = {"type": self.task.type, "index": self.task.index}
        if self.rpc_layer != "grpc":
            d["rpc_layer"] = self.rpc_layer
        return json.dumps(d)


def parse_tf_config(value=None, *, environ=None) -> Optional[TFConfig]:
    """Parse TF_CONFIG (a JSON string, a dict, or None = read the environment).

    Returns None when TF_CONFIG is absent/empty (local, single-task training)."""
    if value is None:
        env = os.environ if environ is None else environ
        value = env.get("TF_CONFIG", "")
    if isinstance(value, (bytes, str)):
        if not value or not str(value).strip():
            return None
        try:
            value = json.loads(value)
        except json.JSONDecodeError as e:
            raise ClusterConfigError(f"TF_CONFIG is not valid JSON: {e}") from None
    if not isinstance(value, dict):
        raise ClusterConfigError("TF_CONFIG must be a JSON object")
    if not value:
        return None
    unknown = set(value) - {"cluster", "task", "rpc_layer", "environment", "session_master"}
    if unknown:
        raise ClusterConfigError(f"unknown TF_CONFIG keys: {sorted(unknown)}")
    cluster = ClusterSpec(value.get("cluster", {}) or {})
    bad_roles = set(cluster.jobs) - set(ALL_ROLES)
    if bad_roles:
        raise ClusterConfigError(f"unknown cluster roles {sorted(bad_roles)}; expected {ALL_ROLES}")
    task = None
    t = value.get("task")
    if t:
        if "type" not in t:
            raise ClusterConfigError("TF_CONFIG task needs a 'type'")
        ttype = str(t["type"])
        try:
            tidx = int(t.get("index", 0))
        except (TypeError, ValueError):
            raise ClusterConfigError("TF_CONFIG task index must be an integer") from None
        if tidx < 0:
            raise ClusterConfigError("TF_CONFIG task index is 0-based and must be >= 0 (README.md:59)")
        if ttype not in ALL_ROLES:
            raise ClusterConfigError(f"unknown task type {ttype!r}")
        task = TaskSpec(ttype, tidx)
        if cluster.jobs:
            cluster.task_address(ttype, tidx)  # validates membership (README.md:59)
    return TFConfig(cluster=cluster, task=task, rpc_layer=value.get("rpc_layer", "grpc") or "grpc",
                    environment=value.get("environment", ""))


def make_tf_config(workers: List[str], index: int, chief: Optional[str] = None, task_type: str = "worker",
                   ps: Optional[List[str]] = None, evaluator: Optional[str] = None) -> str:
    cluster = {"worker": list(workers)}
    if chief:
        cluster["chief"] = [chief]
    if ps:
        cluster["ps"] = list(ps)
    if evaluator:
        cluster["evaluator"] = [evaluator]
    return json.dumps({"cluster": cluster, "task": {"type": task_type, "index": index}})


class TFConfigClusterResolver:
    """tf.distribute.cluster_resolver.TFConfigClusterResolver equivalent."""

    def __init__(self, task_type: Optional[str] = None, task_id: Optional[int] = None, rpc_layer=None,
                 environment=None, tf_config=None):
        cfg = parse_tf_config(tf_config)
        self._cfg = cfg
        self.task_type = task_type if task_type is not None else (cfg.task.type if cfg and cfg.task else None)
        self.task_id = task_id if task_id is not None else (cfg.task.index if cfg and cfg.task else None)
        self.rpc_layer = rpc_layer or (cfg.rpc_layer if cfg else "grpc")
        self.environment = environment or (cfg.environment if cfg else "")

    @property
    def config(self) -> Optional[TFConfig]:
        if self._cfg is None:
            return None
        if self.task_type is None:
            return self._cfg
        return TFConfig(self._cfg.cluster, TaskSpec(self.task_type, int(self.task_id or 0)), self._cfg.rpc_layer,
                        self._cfg.environment)

    def cluster_spec(self) -> ClusterSpec:
        return self._cfg.cluster if self._cfg else ClusterSpec({})

    def master(self, task_type=None, task_id=None, rpc_layer=None) -> str:
        tt = task_type or self.task_type
        ti = self.task_id if task_id is None else task_id
        if tt is None or self._cfg is None:
            return ""
        addr = self._cfg.cluster.task_address(tt, int(ti))
        layer = rpc_layer or self.rpc_layer
        return f"{layer}://{addr}" if layer else addr

    def num_accelerators(self, task_type=None, task_id=None, config_proto=None) -> Dict[str, int]:
        import torch

        n = torch.cuda.device_count()
        return {"GPU": n} if n else {}
