"""Communicator selection rules that do not need a GPU."""
import torch

from tensorflow_distributed_learning_amd.parallel import xgmi
from tensorflow_distributed_learning_amd.parallel.communicator import Communicator, LocalCommunicator


def test_xgmi_env_defaults(monkeypatch):
    monkeypatch.delenv("TDL_XGMI", raising=False)
    monkeypatch.delenv("TDL_XGMI_MAX_BYTES", raising=False)
    assert xgmi.enabled_by_env()
    assert xgmi.max_bytes() == 4 << 20
    monkeypatch.setenv("TDL_XGMI", "0")
    assert not xgmi.enabled_by_env()


def test_base_communicator_has_no_fused_sgd():
    c = LocalCommunicator(torch.device("cpu"))
    g, w = torch.ones(8), torch.zeros(8)
    assert c.all_reduce_sgd(g, w, torch.tensor([0.1])) is False
    assert torch.equal(w, torch.zeros(8))
    c.prepare_all_reduce(8, 16)  # no-op
    c.check_health()
    assert isinstance(c, Communicator)


def _gloo_worker(rank, port, q):
    import os

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    from tensorflow_distributed_learning_amd.parallel.communicator import TorchCommunicator

    c = TorchCommunicator("gloo", rank, 2, torch.device("cpu"), timeout=60)
    a = c.all_gather(torch.tensor([float(rank + 1)], dtype=torch.float64))  # bench.py's per-rank times
    b = c.all_gather(torch.full((2, 3), rank, dtype=torch.int32))
    t = torch.tensor([1.0 + rank])
    c.all_reduce(t, "max")
    q.put((rank, a.tolist(), b.shape, b[1].tolist(), float(t)))
    c.shutdown()


def test_torch_communicator_all_gather_shapes_gloo():
    """all_gather returns [world, *shape] for any shape (gloo's all-gather-into-tensor wants a flat
    output: a [world, 1] buffer failed, and with it bench.py at N > 1)."""
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gloo_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, a, bshape, b1, t in got:
        assert a == [[1.0], [2.0]]
        assert tuple(bshape) == (2, 2, 3) and b1 == [[1, 1, 1], [1, 1, 1]]
        assert t == 2.0
