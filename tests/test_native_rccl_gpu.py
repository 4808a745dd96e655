"""The framework's own RCCL communicator (csrc/rccl_comm.cpp, parallel/communicator.py
NativeRcclCommunicator) on the box's GPU: world 1 (RCCL refuses two ranks on one device, so the
multi-rank path runs only on a multi-GPU node).  Collectives on the current stream, hipGraph
capture, the async-error query and ncclCommAbort."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    import torch.distributed as dist

    from tensorflow_distributed_learning_amd.parallel.communicator import NativeRcclCommunicator

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    old = {k: os.environ.get(k) for k in ("MASTER_ADDR", "MASTER_PORT")}
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    c = NativeRcclCommunicator(0, 1, torch.device("cuda", 0), timeout=60)
    yield c
    c.shutdown()
    if dist.is_initialized():
        dist.destroy_process_group()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_version_and_collectives(comm):
    assert comm.rccl_version >= 21800 and comm.name == "rccl"
    t = torch.arange(10, dtype=torch.float32, device="cuda")
    comm.all_reduce(t, "sum")
    comm.all_reduce(t, "mean")
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(10, dtype=torch.float32, device="cuda"))
    b = torch.full((5,), 3, dtype=torch.bfloat16, device="cuda")
    comm.broadcast(b, 0)
    g = comm.all_gather(torch.ones(2, 3, device="cuda"))
    assert g.shape == (1, 2, 3) and bool((g == 1).all())
    w = comm.all_reduce_async(torch.ones(7, device="cuda"))
    w.wait()
    comm.check_health()
    assert comm.rccl.async_error() == 0


def test_capture_probe_and_graph_replay(comm):
    assert comm.capture_probe() is True
    x = torch.ones(1 << 16, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        x.mul_(2.0)
        comm.all_reduce(x, "sum")
    torch.cuda.synchronize()
    x.fill_(1.0)
    g.replay()
    torch.cuda.synchronize()
    assert bool((x == 2.0).all())


def test_abort_last():
    """ncclCommAbort on a fresh world-1 communicator: later collectives raise, health reports it."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    c = C.RcclComm(C.RcclComm.unique_id(), 0, 1, 0)
    t = torch.ones(4, device="cuda")
    c.all_reduce(t, 0)
    torch.cuda.synchronize()
    c.abort()
    assert c.aborted and c.async_error() != 0
    with pytest.raises(RuntimeError, match="aborted"):
        c.all_reduce(t, 0)


def test_clique_one_process_grouped_calls():
    """The multi-device-per-process RCCL clique (ncclCommInitAll + ncclGroupStart/End of the
    per-device calls, csrc/rccl_comm.cpp RcclClique) on the box's one device; a duplicate device is
    refused with a clear error (RCCL cannot put two ranks on one GPU)."""
    from tensorflow_distributed_learning_amd.ops import hip

    C = hip()
    cl = C.RcclClique([0])
    assert cl.size == 1 and list(cl.devices) == [0]
    t = torch.arange(8, dtype=torch.float32, device="cuda")
    cl.all_reduce([t], 0)
    cl.broadcast([t], 0)
    torch.cuda.synchronize()
    assert torch.equal(t, torch.arange(8, dtype=torch.float32, device="cuda"))
    assert cl.async_error() == 0
    with pytest.raises(Exception, match="distinct devices"):
        C.RcclClique([0, 0])
    with pytest.raises(Exception, match="one tensor per device"):
        cl.all_reduce([t, t], 0)
    cl.abort()
    assert cl.aborted
