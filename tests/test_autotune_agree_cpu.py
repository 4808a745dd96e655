"""The conv autotuner's decisions are rank 0's on every replica (ops/conv.py ``_agree``): gloo,
world 2, each rank's local timing deliberately disagrees."""
import os
import socket

import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch

    from tensorflow_distributed_learning_amd.ops import conv as CV
    from tensorflow_distributed_learning_amd.parallel.communicator import TorchCommunicator

    comm = TorchCommunicator("gloo", rank, 2, torch.device("cpu"), timeout=60)
    CV.bind_communicator(comm)
    called = []

    def local_bool():
        called.append(1)
        return rank == 0  # rank 0 says "hand-written kernel", rank 1 would say "library"

    # encodings of different lengths (a bool, a [wmw, wnw, nsplit, kind] plan, "library") travel in
    # one fixed-width message: non-deciding ranks must post a buffer of the same size
    b = CV._agree(local_bool, lambda v: [int(v)], lambda a: bool(a[0]))
    plan = CV._agree(lambda: [2, 1, 4 + rank, 1], lambda v: [1] + list(v) if v is not None else [0],
                     lambda a: list(a[1:]) if a[0] else None)
    none = CV._agree(lambda: None if rank == 0 else [1, 1, 1, 0], lambda v: [1] + list(v) if v is not None else [0],
                     lambda a: list(a[1:]) if a[0] else None)
    q.put((rank, b, plan, none, len(called)))
    CV.bind_communicator(None)
    comm.shutdown()


def test_rank0_decides_for_every_replica():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0][1:4] == got[1][1:4] == (True, [2, 1, 4, 1], None)
    assert got[0][4] == 1 and got[1][4] == 0  # only rank 0 timed anything
