"""xGMI one-shot all-reduce kernel (csrc/kernels/xgmi.hip) on one MI355X.

The box has one GPU, so ranks are R processes sharing it: they exchange HIP IPC handles exactly
as the ranks of an 8-GPU node do, and their kernels run concurrently, which exercises the protocol
(flags, parity halves, per-workgroup epochs, graph replay, fused SGD) and the cross-process
mapping; only the fabric hop differs.  (Emulating ranks as streams of ONE process is unreliable:
two streams may share a hardware queue, serialising kernels that wait for each other.)
Expected values are the rank-order sums computed with the same f32 adds (bit-identical)."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _C():
    from tensorflow_distributed_learning_amd import ops

    return ops.hip()


def test_timeout_sets_error_instead_of_hanging(cuda):
    C = _C()
    a = C.XgmiChannel(0, 2, 1024, cuda.index or 0, 0.05)
    b = C.XgmiChannel(1, 2, 1024, cuda.index or 0, 0.05)
    a.connect_local([a, b])
    b.connect_local([a, b])
    x = torch.ones(1024, device=cuda)
    a.all_reduce(x, x.clone(), 1.0)  # rank 1 never arrives
    torch.cuda.synchronize(cuda)
    assert a.error() == 1
    a.reset_error()
    assert a.error() == 0


IPC_BODY = """
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[2])
from tensorflow_distributed_learning_amd import ops
from tensorflow_distributed_learning_amd.parallel.xgmi import choose_algo
rank, R = int(sys.argv[1]), int(sys.argv[4])
dist.init_process_group("gloo", rank=rank, world_size=R, init_method="tcp://127.0.0.1:" + sys.argv[3])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
C = ops.hip()
keep = []  # (freeing an exported buffer a peer still maps, then re-allocating it, breaks IPC export)
for n, algo in [(37, 0), (70000, 0), (70000, 1), (206218, choose_algo(206218, R)), (18816, 1)]:
    ch = C.XgmiChannel(rank, R, n, 0, 20.0, algo)
    assert ch.algo == algo
    mine = (bytes(ch.handle(False)), bytes(ch.handle(True)))
    allh = [None] * R
    dist.all_gather_object(allh, mine)
    ch.open([h[0] for h in allh], [h[1] for h in allh])
    dist.barrier()
    g = torch.Generator().manual_seed(n)
    for it in range(4):
        xs = [torch.randn(n, generator=g) for _ in range(R)]
        want = xs[0].clone()
        for r in range(1, R):
            want += xs[r]
        x = xs[rank].to(dev)
        y = torch.empty_like(x)
        ch.all_reduce(x, y, 1.0)
        torch.cuda.synchronize(dev)
        assert ch.error() == 0, "timeout"
        assert torch.equal(y.cpu(), want), f"mismatch n={n} algo={algo} it={it}"
    # graph replay with two calls per replay, then fused SGD
    s = torch.cuda.Stream(dev)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        ch.all_reduce(x, y, 1.0)
        ch.all_reduce(x, y, 1.0)
    for it in range(3):
        y.zero_()
        gr.replay()
        torch.cuda.synchronize(dev)
        assert torch.equal(y.cpu(), want), f"graph mismatch n={n} it={it}"
    z = x.clone()
    ch.all_reduce(z, z, 0.5)  # in place, scaled
    torch.cuda.synchronize(dev)
    assert torch.equal(z.cpu(), want * 0.5)
    w = torch.ones(n, device=dev)
    ch.all_reduce_sgd(x, w, torch.tensor([0.25], device=dev), 1.0)
    torch.cuda.synchronize(dev)
    torch.testing.assert_close(w.cpu(), 1 - 0.25 * want, rtol=0, atol=1e-6)
    assert ch.error() == 0
    dist.barrier()
    keep.append(ch)
print("ipc ok", rank, flush=True)
"""


@pytest.mark.parametrize("R", [2, 3, 4, 8])
def test_multi_process_ipc(tmp_path, R):
    """R processes on the one GPU exchange HIP IPC handles (the same path as R GPUs of a node,
    minus the fabric) and all-reduce eagerly, in graphs and with the fused SGD.  R = 8 is the
    8-GPU node's world size (two-shot shards of 1/8, all 8 signal slots); its largest message
    (206,218 floats) launches 202 256-thread workgroups per rank, 8 x 202 resident together."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    f = tmp_path / "ipc.py"
    f.write_text(textwrap.dedent(IPC_BODY))
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG"):
        env.pop(k, None)
    procs = [subprocess.Popen([sys.executable, str(f), str(r), ROOT, port, str(R)], env=env, stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(R)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=240)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        assert "ipc ok" in out
