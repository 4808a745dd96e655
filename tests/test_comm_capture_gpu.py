"""RCCL all-reduce captured inside the fused engine's execution graph (two gradient buckets on a
side stream, the dense bucket overlapping the conv backward kernel).

A one-GPU box cannot host two RCCL ranks, so the job is a world-1 RCCL group with the trainer
forced to R=2: every all-reduce is a real (identity) RCCL collective issued inside the capture,
and the captured/overlapped execution must equal the eager-all-reduce execution bit for bit.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

BODY = """
import json, sys, torch, torch.distributed as dist
import tensorflow_distributed_learning_amd as tdl
from tensorflow_distributed_learning_amd.models.mnist_cnn import build_mnist_cnn
from tensorflow_distributed_learning_amd.data.tfds import synthetic_mnist
from tensorflow_distributed_learning_amd.parallel.communicator import TorchCommunicator

dev = torch.device("cuda:0")
torch.cuda.set_device(dev)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
comm = TorchCommunicator("nccl", 0, 1, dev, init=False)
x, y = synthetic_mnist(2048, 2)

def run(capture, overlap, momentum):
    strategy = tdl.distribute.OneDeviceStrategy("/gpu:0")
    tdl.keras.utils.set_random_seed(3)
    ds = tdl.data.Dataset.from_tensor_slices((x.reshape(-1, 28, 28, 1), y))
    ds = ds.map(lambda i, l: (i.to(torch.float32) / 255, l)).cache().shuffle(2048, seed=1).batch(128).repeat()
    with strategy.scope():
        m = build_mnist_cnn()
        m.compile(loss=tdl.keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=tdl.keras.optimizers.SGD(0.05, momentum=momentum),
                  metrics=["sparse_categorical_accuracy"], steps_per_execution=4)
    tr = m._get_trainer()
    assert tr.kind == "fused", getattr(m, "_fused_reason", "?")
    tr.comm, tr.R, tr.overlap = comm, 2, overlap
    tr._capture_comm = None if capture else False
    h = tr.prepare(ds)
    assert h.b == 64
    tr.warm_graphs(12)
    n = tr.run_train(h, 12)
    torch.cuda.synchronize()
    graph = tr._graphs[(4, 64, 0)][0]
    kind = "list" if isinstance(graph, list) else ("whole" if graph is not None else "none")
    return tr.W.detach().cpu().clone(), n, kind, bool(tr.capture_comm)

out = {}
for mom in (0.0, 0.9):
    w_eager, n0, k0, c0 = run(False, True, mom)
    w_cap, n1, k1, c1 = run(True, True, mom)
    w_cap_serial, n2, k2, c2 = run(True, False, mom)
    out[str(mom)] = dict(n=[n0, n1, n2], kinds=[k0, k1, k2], captured=[c0, c1, c2],
                         eq_cap=bool(torch.equal(w_eager, w_cap)), eq_serial=bool(torch.equal(w_eager, w_cap_serial)),
                         moved=float((w_eager - w_cap).abs().max()))
json.dump(out, open(sys.argv[1], "w"))
dist.destroy_process_group()
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_captured_overlapped_allreduce_matches_eager(tmp_path):
    script = tmp_path / "job.py"
    script.write_text(textwrap.dedent(BODY))
    res = tmp_path / "res.json"
    # (the overlap option splits the step into forward_dense / backward_conv launches; the compared
    # eager and serial paths must use the same unfused kernels to be bit-comparable)
    env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               TDL_MNIST_FUSED_BWD="0")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG", "TDL_CAPTURE_ALLREDUCE"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, str(script), str(res)], env=env, capture_output=True, text=True,
                       timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    out = json.load(open(res))
    for mom, d in out.items():
        assert d["n"] == [12, 12, 12], d
        assert d["kinds"] == ["list", "whole", "whole"], d
        assert d["captured"] == [False, True, True], d
        assert d["eq_cap"] and d["eq_serial"], d
