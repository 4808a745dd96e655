"""The fused MNIST step's finalize with the cross-replica all-reduce built in (k_finalize_x with
an xGMI exchange per finalize workgroup; engine/fused.py uses it at R > 1 with plain SGD).

R replica processes share the box's one GPU and exchange HIP IPC handles as the replicas of an
8-GPU node do.  Each runs the fused forward/backward on its own batch slice, then (after a barrier,
so no replica's fused kernel is still running beside the spinning exchange workgroups of another:
the engine never selects the fused kernel on a shared GPU) the exchange finalize.  Expected: every replica ends with bit-identical parameters equal to
W - lr * (sum of the replicas' gradients in rank order), eagerly and in graph replays."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

BODY = """
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, sys.argv[2])
from tensorflow_distributed_learning_amd import ops
from tensorflow_distributed_learning_amd.models import mnist_cnn as M
rank, R, two = int(sys.argv[1]), int(sys.argv[4]), sys.argv[5] == "1"
b = int(sys.argv[6])
dist.init_process_group("gloo", rank=rank, world_size=R, init_method="tcp://127.0.0.1:" + sys.argv[3])
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
C = ops.hip()
N = 512
g = torch.Generator().manual_seed(0)
X = torch.rand(N, 28, 28, 1, generator=g).to(dev)
Y = torch.randint(0, 10, (N,), generator=g, dtype=torch.int32).to(dev)
layout = M.mnist_layout()
W = layout.pack(M.init_mnist_params(0), device=dev)
G = torch.zeros_like(W)
idx = torch.randperm(N, generator=g)[: 4 * b * R].to(torch.int32)
mine = torch.cat([idx[k * b * R + rank * b: k * b * R + (rank + 1) * b] for k in range(4)]).to(dev)
lr = torch.tensor([0.05], device=dev)
st = M.FusedMnistTrainStep(X, Y, mine, W, G, layout, b, R, lr)
assert st.fused_bwd, "fused backward not selected"
ch = C.XgmiChannel(rank, R, W.numel(), 0, 20.0, 0, M.FINALIZE_BLOCKS)
hs = [None] * R
dist.all_gather_object(hs, (bytes(ch.handle(False)), bytes(ch.handle(True))))
ch.open([h[0] for h in hs], [h[1] for h in hs])
st.set_exchange(ch, twoshot=two)
assert st.has_exchange and st.exchange_twoshot == two


def step(k, graph=None):
    W0 = W.clone()
    st.forward_backward(k * b)
    st.finalize(False)  # local gradient into G (the reference), no update
    torch.cuda.synchronize(dev)
    parts = [torch.empty_like(G).cpu() for _ in range(R)]
    dist.all_gather(parts, G.cpu())
    want = parts[0].clone()
    for r in range(1, R):
        want += parts[r]
    dist.barrier()
    # (the replicas share ONE GPU here: a replica's spinning exchange workgroups could keep another
    # replica's fused kernel from being fully resident, which its intra-image hand-offs require; so
    # every fused kernel completes before any exchange starts.  With one GPU per replica the
    # stream order alone guarantees that.)
    if graph is None:
        st.forward_backward(k * b)
    else:
        graph[0].replay()
    torch.cuda.synchronize(dev)
    assert st._impl.error(False) == 0, "fused kernel hand-off timed out"
    dist.barrier()
    if graph is None:
        # (k = 1: the trainer's form -- the exchange applies SGD without writing G)
        st.finalize(True, exchange=True, keep_grad=(k != 1))
    else:
        graph[1].replay()
    torch.cuda.synchronize(dev)
    assert ch.error() == 0 and st._impl.error(False) == 0, "exchange timed out"
    ref = W0.cpu() - 0.05 * want
    bad = (W.cpu() - ref).abs() > 2e-7
    if bad.any():  # diagnose: which slab ranges, and what the applied update corresponds to
        got_g = (W0.cpu() - W.cpu()) / 0.05
        ids = bad.nonzero().flatten()
        print(f"rank {rank} step {k} graph={graph is not None}: {int(bad.sum())} bad, first {ids[:8].tolist()}",
              flush=True)
        for lo, hi, name in [(0, 320, "conv1"), (320, 18816, "conv2"), (18816, 225034, "dense")]:
            m = bad[lo:hi]
            if m.any():
                d = got_g[lo:hi][m]
                cands = {"sum": want[lo:hi][m], **{f"g{r}": parts[r][lo:hi][m] for r in range(R)},
                         **{f"sum-g{r}": (want - parts[r])[lo:hi][m] for r in range(R)}}
                best = min(cands, key=lambda c: float((cands[c] - d).abs().max()))
                print(f"  {name}: {int(m.sum())} bad; applied update closest to {best} "
                      f"(err {float((cands[best] - d).abs().max()):.3g}); blocks "
                      f"{sorted(set(((m.nonzero().flatten() + lo - 18816) // 2048).tolist()))[:20] if name == 'dense' else ''}",
                      flush=True)
    torch.testing.assert_close(W.cpu(), ref, rtol=0, atol=2e-7)
    allw = [torch.empty_like(W).cpu() for _ in range(R)]
    dist.all_gather(allw, W.cpu())
    assert all(torch.equal(allw[0], x) for x in allw[1:]), "replicas differ"
    dist.barrier()


for k in range(2):
    step(k)
s = torch.cuda.Stream(dev)
s.wait_stream(torch.cuda.current_stream(dev))
g_fwd, g_fin = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
with torch.cuda.graph(g_fwd, stream=s):
    st.forward_backward(2 * b)
with torch.cuda.graph(g_fin, stream=s):
    st.finalize(True, exchange=True, keep_grad=False)
torch.cuda.synchronize(dev)
for _ in range(2):
    step(2, (g_fwd, g_fin))
dist.barrier()
print("exchange ok", rank, flush=True)
"""


@pytest.mark.parametrize("two", [False, True], ids=["oneshot", "twoshot"])
@pytest.mark.parametrize("R", [2, 8])
def test_finalize_exchange_multi_process(tmp_path, R, two):
    """R = 2 with the full finalize grid, R = 8 (BASELINE config 3's world size: the two-shot shard
    math, the 8-slot signal words, the largest rank-order sums) with the grid capped (TDL_FX_GRID):
    the exchange needs range j of every replica in flight together, and a one-GPU box holds 768 of
    the finalize's 512-thread workgroups (72 VGPRs: 3 per CU) -- 8 x 269 full grids would let some
    replicas fill the GPU while the peers they wait for have none resident.  At 8 x 48 every
    replica's workgroups are resident together and loop over the 269 ranges in the same order.
    With one GPU per replica the full grid is resident at once.  (b = 4 at R = 8: each replica's
    fused kernel needs its 4b workgroups resident together, 8 x 16 of the 256 CUs.)"""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    f = tmp_path / "xchg.py"
    f.write_text(textwrap.dedent(BODY))
    env = dict(os.environ, TDL_MNIST_DP2_FWD="1", TDL_MNIST_FUSED_BWD="1")
    if R > 2:
        env["TDL_FX_GRID"] = "48"
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG", "TDL_SHARE_GPU"):
        env.pop(k, None)
    b = 16 if R == 2 else 4
    procs = [subprocess.Popen([sys.executable, str(f), str(r), ROOT, port, str(R), "1" if two else "0", str(b)],
                              env=env, stdout=subprocess.PIPE,
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
        assert "exchange ok" in out


def _bench2(extra_env):
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", TDL_MNIST_DP2_FWD="1", TDL_XGMI_TIMEOUT="30",
               **extra_env)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG", "TDL_LAUNCHED", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--per-replica-batch", "16", "--steps", "40",
                        "--warmup", "8"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json as _json

    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return _json.loads(line), r.stderr


def test_bench_exchange_selftest_failure_falls_back(tmp_path):
    """A start-up self-test failure of the exchange-in-finalize path on ONE rank (injected:
    TDL_FAULT_XCHG_SELFTEST=1 makes rank 1 see a wrong result) moves EVERY rank to the serial
    all-reduce, and the run still ends with bit-identical replicas."""
    d, err = _bench2({"TDL_FAULT_XCHG_SELFTEST": "1"})
    cfg = d["config"]
    assert not cfg["allreduce"].startswith("xgmi-in-finalize") and cfg["replicas_identical"], cfg
    assert "self-test failed" in err, err[-3000:]


def test_bench_two_replicas_exchange_in_finalize(tmp_path):
    """bench.py at N=2 end to end on the R > 1 production path: the fused forward/backward kernel
    and the finalize whose workgroups all-reduce over xGMI, captured in the execution graphs.  On
    the shared GPU this needs both replicas' kernels resident beside each other, so the per-replica
    batch is 16 (64 fused workgroups each); on one GPU per replica b = 64 is the default."""
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", TDL_MNIST_DP2_FWD="1", TDL_XGMI_TIMEOUT="30")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG", "TDL_LAUNCHED", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--per-replica-batch", "16", "--steps", "40",
                        "--warmup", "8"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    import json as _json

    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    d = _json.loads(line)
    cfg = d["config"]
    assert d["n_gpus"] == 2 and cfg["allreduce"] == "xgmi-in-finalize", cfg
    assert cfg["kernels_per_step"] == 2 and cfg["allreduce_in_graph"] and cfg["replicas_identical"], cfg


def test_bench_two_replicas_exchange_in_finalize_twoshot(tmp_path):
    """The same with the two-shot exchange (the default from R = 3; forced at R = 2 here): every
    rank reduces and updates half of each finalize range and copies the other half."""
    d, _ = _bench2({"TDL_FX_TWOSHOT_MIN_R": "2"})
    cfg = d["config"]
    assert cfg["allreduce"] == "xgmi-in-finalize-twoshot" and cfg["replicas_identical"], cfg


def test_bench_exchange_selftest_one_rank_raises_fails_every_rank(tmp_path):
    """A rank whose self-test raises BEFORE the exchange (injected: TDL_FAULT_XCHG_SELFTEST_RAISE=1)
    leaves its peer waiting in the xGMI exchange until the bounded wait expires (TDL_XGMI_TIMEOUT=30).
    Both ranks then reach the same agreement collective, see the timeout and fail the job with the
    same diagnosis instead of hanging or reducing garbage (the peer's device carries the sticky error
    word, so no fallback can run there)."""
    env = dict(os.environ, PYTHONPATH=ROOT, TDL_SHARE_GPU="1", TDL_MNIST_DP2_FWD="1", TDL_XGMI_TIMEOUT="30",
               TDL_FAULT_XCHG_SELFTEST_RAISE="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "TF_CONFIG", "TDL_LAUNCHED", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--per-replica-batch", "16", "--steps", "10",
                        "--warmup", "2"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode != 0, r.stdout[-2000:]
    assert "did not arrive at the xGMI exchange" in r.stderr + r.stdout, (r.stdout + r.stderr)[-4000:]
