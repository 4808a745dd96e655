"""bench.py as the driver runs it: exactly N replicas for --gpus N, self-launched without a
launcher, with the all-reduce algorithm and the replica-consistency check in the JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _bench(args, **env_extra):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_one_gpu_is_one_replica():
    d = _bench(["--gpus", "1", "--steps", "20", "--warmup", "5"], HIP_VISIBLE_DEVICES="0")
    assert d["n_gpus"] == 1 and d["config"]["global_batch"] == 64
    assert d["config"]["engine"] == "fused" and d["config"]["replicas_identical"] is True
    assert d["value"] > 0 and d["steps"] == 20


def test_bench_two_replicas_self_launched_shared_gpu():
    d = _bench(["--gpus", "2", "--steps", "20", "--warmup", "5"], TDL_SHARE_GPU="1")
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 128
    assert d["config"]["allreduce"] == "xgmi-oneshot+gloo"
    assert d["config"]["allreduce_in_graph"] is True
    assert d["config"]["replicas_identical"] is True
    # per-rank timed regions (the MAX is the reported time) and the fallbacks taken (none here)
    assert len(d["config"]["rank_ms_per_step"]) == 2 and max(d["config"]["rank_ms_per_step"]) == d["ms_per_step"]
    assert d["config"]["rank_spread_pct"] >= 0 and d["config"]["fallbacks"] == [], d["config"]


def test_bench_three_replicas_two_shot_shared_gpu():
    """R >= 3: the 900 KB slab takes the two-shot xGMI all-reduce (reduce-scatter + all-gather, SGD
    applied by each shard's owner); its start-up self-test must pass (it used to compare every
    rank's result with its own random parameters, which the owner-applied update cannot match)."""
    d = _bench(["--gpus", "3", "--steps", "20", "--warmup", "5"], TDL_SHARE_GPU="1")
    assert d["n_gpus"] == 3 and d["config"]["global_batch"] == 192
    assert d["config"]["allreduce"] == "xgmi-twoshot+gloo", d["config"]
    assert d["config"]["allreduce_in_graph"] is True
    assert d["config"]["replicas_identical"] is True


def test_bench_eight_replicas_shared_gpu():
    """bench.py --gpus 8 (BASELINE config 3's replica count) as 8 replica processes on the one GPU,
    8 images each: the two-shot xGMI all-reduce over IPC-mapped buffers of all 8 replicas with SGD
    fused, in the captured graphs; replicas bit-identical, no fallback taken.  (On a shared GPU the
    engine keeps the standalone all-reduce kernel: the in-finalize exchange needs every replica's
    fused kernel fully resident, which 8 concurrent replicas cannot guarantee on one GPU --
    tests/test_mnist_exchange_gpu.py covers it at R = 8 with phases separated.)"""
    d = _bench(["--gpus", "8", "--per-replica-batch", "8", "--steps", "20", "--warmup", "5"], TDL_SHARE_GPU="1")
    assert d["n_gpus"] == 8 and d["config"]["global_batch"] == 64
    assert d["config"]["allreduce"] == "xgmi-twoshot+gloo", d["config"]
    assert d["config"]["allreduce_in_graph"] is True
    assert d["config"]["replicas_identical"] is True
    assert d["config"]["fallbacks"] == [], d["config"]
    assert len(d["config"]["rank_ms_per_step"]) == 8


def test_bench_two_replicas_under_torchrun_shared_gpu():
    """The driver's launch form: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "20", "--warmup", "5"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 128 and d["steps"] == 20
    assert d["config"]["replicas_identical"] is True
