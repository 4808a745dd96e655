"""Launcher: one process per replica (per GPU), optionally several TF_CONFIG tasks on one node.

    # N replicas of a MirroredStrategy script on one node (torchrun-compatible env):
    python -m tensorflow_distributed_learning_amd.launch --nproc-per-node 8 train.py

    # K TF_CONFIG worker tasks x G GPUs each on one node (MultiWorkerMirroredStrategy, BASELINE
    # config 5; README.md:61 "several cluster tasks on one physical machine"):
    python -m tensorflow_distributed_learning_amd.launch --local-workers 2 --gpus-per-worker 4 train.py

    # one task of a real multi-host cluster (README.md:156-162), G GPUs on this host:
    TF_CONFIG='{"cluster": {...}, "task": {...}}' \\
        python -m tensorflow_distributed_learning_amd.launch --nproc-per-node 4 train.py

Children get RANK / WORLD_SIZE / LOCAL_RANK / LOCAL_WORLD_SIZE (+ MASTER_ADDR/PORT when no
TF_CONFIG is used, + TF_CONFIG and TDL_DEVICE_INDEX -- the node-global GPU of the replica -- for
--local-workers).  If any child fails
the others are terminated and the launcher exits with the failing code.
"""
from __future__ import annotations

import argparse
import atexit
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
import warnings
from typing import Dict, List, Optional


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def free_ports(n: int, host: str = "127.0.0.1") -> List[int]:
    socks, ports = [], []
    try:
        for _ in range(n):
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.bind((host, 0))
            socks.append(s)
            ports.append(s.getsockname()[1])
    finally:
        for s in socks:
            s.close()
    return ports


def _die_with_parent():
    """preexec hook of every replica process: the kernel sends it SIGKILL when the process that
    started it dies (Linux PR_SET_PDEATHSIG), so replicas never outlive a crashed launcher or a
    crashed replica 0 and spin in a collective until their own timeouts."""
    try:
        import ctypes

        libc = ctypes.CDLL("libc.so.6", use_errno=True)
        libc.prctl(1, int(signal.SIGKILL), 0, 0, 0)  # PR_SET_PDEATHSIG
    except Exception:
        pass


class _Group:
    def __init__(self):
        self.procs: List[subprocess.Popen] = []

    def start(self, cmd: List[str], env: Dict[str, str]):
        p = subprocess.Popen(cmd, env=env, start_new_session=True,
                             preexec_fn=_die_with_parent if sys.platform.startswith("linux") else None)
        self.procs.append(p)
        return p

    def first_failure(self) -> Optional[int]:
        """Exit code of the first child that failed, else None."""
        for p in self.procs:
            c = p.poll()
            if c not in (None, 0):
                return c
        return None

    def terminate(self, sig=signal.SIGTERM):
        for p in self.procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, sig)
                except (ProcessLookupError, PermissionError):
                    pass

    def wait(self, poll: float = 0.1) -> int:
        """Wait for all; on the first failure terminate the rest.  Returns the job exit code."""
        try:
            while True:
                codes = [p.poll() for p in self.procs]
                bad = [c for c in codes if c not in (None, 0)]
                if bad:
                    self.terminate()
                    deadline = time.time() + 10
                    while time.time() < deadline and any(p.poll() is None for p in self.procs):
                        time.sleep(0.05)
                    self.terminate(signal.SIGKILL)
                    return bad[0]
                if all(c == 0 for c in codes):
                    return 0
                time.sleep(poll)
        except KeyboardInterrupt:
            self.terminate()
            return 130


# Environment every replica of a job must share, replica 0 included, set before any HIP call.
# HSA_ENABLE_IPC_MODE_LEGACY=0: HIP IPC through dmabuf file descriptors -- the only IPC mode the
# MI355X hosts' kernel driver supports; in legacy mode hipIpcGetMemHandle fails with "invalid
# argument", which breaks RCCL's P2P transport and the xGMI kernel's peer-buffer mapping.  A job
# whose replicas disagree on it cannot map each other's buffers.
REPLICA_SHARED_ENV = {"HSA_ENABLE_IPC_MODE_LEGACY": "0"}


def ipc_mode() -> str:
    """The IPC mode this process runs with ("dmabuf" or "legacy"), for the bench JSON."""
    return "legacy" if os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0") == "1" else "dmabuf"


def _base_env(nprocs: int = 1) -> Dict[str, str]:
    env = dict(os.environ)
    for k, v in REPLICA_SHARED_ENV.items():
        env.setdefault(k, v)
    if "OMP_NUM_THREADS" not in env:
        # one replica process per GPU: do not let every process spawn a thread per core
        env["OMP_NUM_THREADS"] = str(max(1, (os.cpu_count() or 1) // max(1, nprocs)))
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    return env


def launch_replicas(cmd: List[str], nproc: int, master_addr: str = "127.0.0.1", master_port: Optional[int] = None,
                    tf_config: Optional[str] = None) -> int:
    env0 = _base_env(nproc)
    port = master_port or free_port(master_addr)
    g = _Group()
    for lr in range(nproc):
        env = dict(env0)
        env.update(RANK=str(lr), WORLD_SIZE=str(nproc), LOCAL_RANK=str(lr), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR=master_addr, MASTER_PORT=str(port), TDL_LAUNCHED="1")
        if tf_config is not None:
            env["TF_CONFIG"] = tf_config
        g.start(cmd, env)
    return g.wait()


def launch_local_workers(cmd: List[str], workers: int, gpus_per_worker: int, base_port: Optional[int] = None,
                         chief: bool = False) -> int:
    """K TF_CONFIG tasks on this host, each with G replica processes (one per GPU)."""
    env0 = _base_env(workers * max(1, gpus_per_worker))
    ntasks = workers + (1 if chief else 0)
    ports = [base_port + i for i in range(ntasks)] if base_port else free_ports(ntasks)
    addrs = [f"127.0.0.1:{p}" for p in ports]
    cluster = {"worker": addrs[1:] if chief else addrs}
    if chief:
        cluster["chief"] = [addrs[0]]
    tasks = ([("chief", 0)] if chief else []) + [("worker", i) for i in range(workers)]
    world = ntasks * gpus_per_worker
    g = _Group()
    for t_rank, (ttype, tidx) in enumerate(tasks):
        tfc = json.dumps({"cluster": cluster, "task": {"type": ttype, "index": tidx}})
        for lr in range(gpus_per_worker):
            env = dict(env0)
            env.update(TF_CONFIG=tfc, RANK=str(t_rank * gpus_per_worker + lr), WORLD_SIZE=str(world),
                       LOCAL_RANK=str(lr), LOCAL_WORLD_SIZE=str(gpus_per_worker), TDL_LAUNCHED="1")
            env.pop("MASTER_ADDR", None)
            env.pop("MASTER_PORT", None)
            if gpus_per_worker > 0:
                first = t_rank * gpus_per_worker
                if os.environ.get("TDL_GPU_PARTITION") == "1":
                    # opt-in: each task sees only its own GPUs (as on separate hosts); the xGMI
                    # kernel's IPC mapping then fails its self-test and AUTO falls back to RCCL
                    env["HIP_VISIBLE_DEVICES"] = ",".join(str(first + i) for i in range(gpus_per_worker))
                else:
                    # default: every task sees every GPU of the node and pins its replica to a
                    # disjoint device, so peer IPC (xGMI kernel, RCCL P2P) works across tasks
                    env["TDL_DEVICE_INDEX"] = str(first + lr)
            g.start(cmd, env)
    return g.wait()


# ------------------------------------------------------------------------------------------------
_SPAWNED: Optional[_Group] = None


def _relaunch_argv() -> Optional[list]:
    """Command line that re-runs this program: ``python script.py args`` or, for a program started
    with ``python -m pkg.mod``, ``python -m pkg.mod args``; None for ``python -c`` / interactive."""
    main = sys.argv[0] if sys.argv else ""
    if not main or main == "-c" or not os.path.isfile(main):
        return None
    spec = getattr(sys.modules.get("__main__"), "__spec__", None)
    if spec is not None and spec.name and spec.name != "__main__":
        name = spec.name[:-len(".__main__")] if spec.name.endswith(".__main__") else spec.name
        return [sys.executable, "-m", name] + sys.argv[1:]
    return [sys.executable] + sys.argv


def maybe_spawn_local_replicas(n: int, spawn: Optional[bool] = None) -> Optional[dict]:
    """MirroredStrategy started as a plain script with n > 1 devices: re-run the script once per
    extra device (children are replicas 1..n-1, this process is replica 0).  Must run before this
    process touches the GPU.  Returns the placement dict, or None to stay single-replica."""
    global _SPAWNED
    if os.environ.get("TDL_LAUNCHED") == "1":
        return None  # this process already is one of a launched group
    if spawn is None:
        spawn = os.environ.get("TDL_AUTO_SPAWN", "1") == "1"
    main = sys.argv[0] if sys.argv else ""
    argv = _relaunch_argv()
    why = None
    if not spawn:
        why = "TDL_AUTO_SPAWN=0"
    elif argv is None:
        why = "the program is not a script or module file that can be re-run (python -c / interactive)"
    elif "pytest" in sys.modules or os.path.basename(main).startswith("pytest") or \
            os.path.basename(os.path.dirname(main)) in ("pytest", "_pytest"):
        why = "running under pytest"
    if why is not None:
        warnings.warn(f"MirroredStrategy asked for {n} devices but runs as ONE replica: {why}; launch "
                      f"with `python -m tensorflow_distributed_learning_amd.launch --nproc-per-node {n} ...` "
                      f"for {n} replicas", RuntimeWarning, stacklevel=3)
        sys.stderr.write(f"[tdl] WARNING: {n} devices requested, running 1 replica ({why})\n")
        return None
    port = free_port()
    own, children = spawn_envs(n, port)
    g = _Group()
    for env in children:
        g.start(argv, env)
    os.environ.update(own)
    _SPAWNED = g
    _supervise(g)

    def _join():
        code = g.wait()
        if code != 0:
            # a failed replica fails the job: this process exits non-zero as well (the replicas'
            # own output, e.g. a GPU fault report, went to the shared stderr)
            sys.stderr.write(f"[tdl] a spawned replica exited with code {code}\n")
            sys.stderr.flush()
            sys.stdout.flush()
            os._exit(code if 0 < code < 256 else 1)

    atexit.register(_join)
    return {"rank": 0, "world_size": n, "local_rank": 0, "local_world_size": n}


def spawn_envs(n: int, port: int):
    """Environments of a self-spawned group of n replicas: (the updates replica 0 applies to its
    own environment, the full environments of replicas 1 .. n-1).  Every replica-shared variable
    (REPLICA_SHARED_ENV) gets the same value in all n, replica 0 included -- it keeps its own value
    where it has one, and the children inherit that value."""
    env0 = _base_env(n)
    shared = {k: env0[k] for k in REPLICA_SHARED_ENV}
    own = dict(shared, RANK="0", WORLD_SIZE=str(n), LOCAL_RANK="0", LOCAL_WORLD_SIZE=str(n),
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TDL_LAUNCHED="1")
    children = []
    for lr in range(1, n):
        env = dict(env0)
        env.update(RANK=str(lr), WORLD_SIZE=str(n), LOCAL_RANK=str(lr), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TDL_LAUNCHED="1")
        children.append(env)
    return own, children


def _supervise(g: "_Group", poll: float = 0.2) -> threading.Thread:
    """Replica 0 supervises the replicas it spawned: the moment one of them fails, the others are
    terminated and this process exits with the failing code (it may be blocked inside a collective
    with the dead replica, so this cannot wait for the main thread)."""

    def run():
        while True:
            code = g.first_failure()
            if code is not None:
                sys.stderr.write(f"[tdl] a spawned replica exited with code {code}; ending the job\n")
                sys.stderr.flush()
                g.terminate()
                deadline = time.time() + 5
                while time.time() < deadline and any(p.poll() is None for p in g.procs):
                    time.sleep(0.05)
                g.terminate(signal.SIGKILL)
                sys.stdout.flush()
                os._exit(code if 0 < code < 256 else 1)
            if all(p.poll() == 0 for p in g.procs):
                return
            time.sleep(poll)

    t = threading.Thread(target=run, name="tdl-replica-supervisor", daemon=True)
    t.start()
    return t


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m tensorflow_distributed_learning_amd.launch",
                                 description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=None)
    ap.add_argument("--local-workers", type=int, default=None)
    ap.add_argument("--gpus-per-worker", type=int, default=1)
    ap.add_argument("--chief", action="store_true", help="add a separate chief task (with --local-workers)")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=None)
    ap.add_argument("--base-port", type=int, default=None)
    ap.add_argument("-m", dest="module", default=None, help="run a module instead of a script")
    ap.add_argument("script", nargs="?")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if a.module:
        cmd = [sys.executable, "-m", a.module] + ([a.script] if a.script else []) + a.args
    else:
        if not a.script:
            ap.error("a training script is required")
        cmd = [sys.executable, a.script] + a.args
    if a.local_workers:
        return launch_local_workers(cmd, a.local_workers, a.gpus_per_worker, a.base_port, chief=a.chief)
    n = a.nproc_per_node
    if n is None:
        try:
            import torch

            n = max(1, torch.cuda.device_count())
        except Exception:
            n = 1
    tfc = os.environ.get("TF_CONFIG")
    if tfc:
        # one TF_CONFIG task with n local replica processes: rank layout comes from the rendezvous
        env0 = _base_env(n)
        g = _Group()
        port = a.master_port or free_port(a.master_addr)
        for lr in range(n):
            env = dict(env0)
            env.update(RANK=str(lr), WORLD_SIZE=str(n), LOCAL_RANK=str(lr), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR=a.master_addr, MASTER_PORT=str(port), TDL_LAUNCHED="1")
            g.start(cmd, env)
        return g.wait()
    return launch_replicas(cmd, n, a.master_addr, a.master_port)


if __name__ == "__main__":
    sys.exit(main())
