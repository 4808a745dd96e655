#!/usr/bin/env python3
"""All-reduce latency of the xGMI one-shot kernel vs the process group's own collective.

    python scripts/bench_allreduce.py --procs 2          # R processes (one GPU each if there are
                                                        # enough GPUs, else sharing cuda:0)

Each rank times ``--iters`` back-to-back calls captured in one hipGraph (xGMI) or issued eagerly
(RCCL / gloo), for the MNIST gradient bucket sizes and a few powers of two; rank 0 prints one
JSON line per size.  On a one-GPU box the ranks share the GPU (no fabric hop): the numbers then
bound the kernel's fixed cost (flags, fences, launch), not xGMI bandwidth.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [18816, 206218, 225034, 1 << 16, 1 << 20]


def worker(rank: int, R: int, port: str, iters: int):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from tensorflow_distributed_learning_amd import ops

    ngpu = torch.cuda.device_count()
    dev = torch.device("cuda", rank if ngpu >= R else 0)
    torch.cuda.set_device(dev)
    backend = "nccl" if ngpu >= R else "gloo"
    dist.init_process_group(backend, rank=rank, world_size=R, init_method=f"tcp://127.0.0.1:{port}")
    C = ops.hip()
    out = []
    keep = []  # channels live to the end: freeing an exported buffer while a peer still maps it
    # and re-allocating at the same address makes the next hipIpcGetMemHandle fail
    for n, algo in [(n, a) for n in SIZES for a in (0, 1)]:
        ch = C.XgmiChannel(rank, R, n, dev.index, 60.0, algo)
        mine = (bytes(ch.handle(False)), bytes(ch.handle(True)))
        allh = [None] * R
        dist.all_gather_object(allh, mine)
        ch.open([h[0] for h in allh], [h[1] for h in allh])
        x = torch.randn(n, device=dev)
        y = torch.empty_like(x)
        for _ in range(5):
            ch.all_reduce(x, y, 1.0)
        torch.cuda.synchronize(dev)
        s = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                ch.all_reduce(x, y, 1.0)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        t_x = (time.perf_counter() - t0) / iters
        assert ch.error() == 0
        # the process group's own all-reduce
        z = x.clone() if backend == "nccl" else x.cpu()
        for _ in range(3):
            dist.all_reduce(z)
        dist.barrier()
        if backend == "nccl":
            torch.cuda.synchronize(dev)
        k = max(1, iters // 10) if backend == "gloo" else iters
        t0 = time.perf_counter()
        for _ in range(k):
            dist.all_reduce(z)
        if backend == "nccl":
            torch.cuda.synchronize(dev)
        t_pg = (time.perf_counter() - t0) / k
        tt = torch.tensor([t_x, t_pg], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t_x, t_pg = (float(v) for v in tt.cpu())
        out.append({"numel": n, "bytes": 4 * n, "ranks": R, "shared_gpu": ngpu < R,
                    "algo": ("one-shot", "two-shot")[algo], "xgmi_us": round(t_x * 1e6, 2),
                    f"{backend}_us": round(t_pg * 1e6, 2)})
        dist.barrier()
        keep.append((g, ch))
    if rank == 0:
        for o in out:
            print(json.dumps(o), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rank", type=int, default=-1, help=argparse.SUPPRESS)
    ap.add_argument("--port", default="", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.rank >= 0:
        worker(a.rank, a.procs, a.port, a.iters)
        return
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = str(s.getsockname()[1])
    s.close()
    procs = [subprocess.Popen([sys.executable, __file__, "--procs", str(a.procs), "--iters", str(a.iters),
                               "--rank", str(r), "--port", port]) for r in range(a.procs)]
    rc = 0
    for p in procs:
        rc |= p.wait(timeout=600)
    sys.exit(rc)


if __name__ == "__main__":
    main()
