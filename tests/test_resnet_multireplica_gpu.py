"""ResNet-50 (the BASELINE config-4/5 model) with REAL peer replica processes sharing the box's one
GPU: gloo control plane, the xGMI kernel as the device data plane (messages above its channel
limit in chunks), gradient buckets launched from the backward hooks and recorded in the
whole-step hipGraph.  64x64 images keep it short; the layer graph, fusion plan and bucket plan are
those of the 224x224 model.  Replicas must end bit-identical (scripts/bench_resnet50.py checks)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _run(args):
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "TF_CONFIG", "TDL_LAUNCHED", "MASTER_ADDR",
              "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "scripts/bench_resnet50.py", "--image", "64", "--conv-search", "0"] + args,
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "capture failed" not in r.stderr, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


def test_resnet50_two_replicas():
    d = _run(["--gpus", "2", "--batch", "16", "--steps", "4", "--warmup", "3"])
    c = d["config"]
    assert d["n_gpus"] == 2 and c["replicas_identical"] and c["allreduce"].startswith("xgmi"), c
    assert c["buckets"]["n"] > 1 and c["buckets"]["overlapped_with_backward"], c


def test_resnet50_config5_two_workers_two_replicas():
    d = _run(["--strategy", "mwms", "--workers", "2", "--gpus", "4", "--batch", "8", "--steps", "3",
              "--warmup", "3"])
    c = d["config"]
    assert d["n_gpus"] == 4 and c["replicas_identical"] and c["allreduce"].startswith("xgmi"), c
