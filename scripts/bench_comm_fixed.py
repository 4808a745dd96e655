#!/usr/bin/env python3
"""Fixed costs of the gradient all-reduce paths on ONE MI355X (replace guessed
constants in parallel/bucketing.py with measured ones).

    python scripts/bench_comm_fixed.py > profiles/comm_fixed_costs_r3.jsonl

* ``rccl_world1``: RCCL all-reduce in a world-1 process group (``nccl`` backend), 50 calls captured
  in one hipGraph: the per-call cost of launch + RCCL's kernel without any fabric hop.
* ``xgmi_oneshot`` / ``xgmi_twoshot`` at R = 2 and 4: the xGMI all-reduce kernel between R
  processes that share the one GPU (IPC-mapped exchange buffers, flags, fences, rank-order sums):
  its fixed cost and its local memory traffic, again without a fabric hop.

Sizes 64 KiB .. 32 MiB of f32.  One JSON line per (path, R, bytes).  The xGMI link term of the
bucket cost model (153.6 GB/s per link, ring hops) stays modelled: this box has one GPU.
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20, 32 << 20]
ITERS = 50


def _time_graph(fn, dev, iters=ITERS):
    import torch

    for _ in range(3):
        fn()
    torch.cuda.synchronize(dev)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(iters):
            fn()
    torch.cuda.synchronize(dev)
    best = float("inf")
    for _ in range(3):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize(dev)
        best = min(best, (time.perf_counter() - t0) / iters * 1e6)
    return best


def rccl_world1():
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, init_method=f"tcp://127.0.0.1:{port}", device_id=dev)
    for nbytes in SIZES:
        x = torch.randn(nbytes // 4, device=dev)
        us = _time_graph(lambda: dist.all_reduce(x), dev)
        print(json.dumps({"path": "rccl_world1", "R": 1, "bytes": nbytes, "us_per_call": round(us, 2),
                          "note": "launch + RCCL kernel, no fabric hop"}), flush=True)
    dist.destroy_process_group()


def xgmi_worker(rank: int, R: int, port: str):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from tensorflow_distributed_learning_amd import ops

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=R, init_method=f"tcp://127.0.0.1:{port}")
    C = ops.hip()
    keep = []
    for nbytes in SIZES:
        n = nbytes // 4
        for algo in (0, 1):
            ch = C.XgmiChannel(rank, R, n, 0, 60.0, algo)
            hs = [None] * R
            dist.all_gather_object(hs, (bytes(ch.handle(False)), bytes(ch.handle(True))))
            ch.open([h[0] for h in hs], [h[1] for h in hs])
            x = torch.randn(n, device=dev)
            y = torch.empty_like(x)
            dist.barrier()
            us = _time_graph(lambda: ch.all_reduce(x, y, 1.0), dev)
            assert ch.error() == 0
            t = torch.tensor([us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            if rank == 0:
                print(json.dumps({"path": "xgmi_oneshot" if algo == 0 else "xgmi_twoshot", "R": R, "bytes": nbytes,
                                  "us_per_call": round(float(t), 2),
                                  "note": f"{R} processes sharing one GPU: fixed cost + local traffic, no fabric hop"}),
                      flush=True)
            keep.append(ch)
            dist.barrier()
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--xgmi-worker":
        xgmi_worker(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        return
    if len(sys.argv) > 1 and sys.argv[1] == "--rccl":
        rccl_world1()
        return
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, __file__, "--rccl"], env=env, timeout=300)
    if r.returncode:
        sys.exit(r.returncode)
    for R in (2, 4):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = str(s.getsockname()[1])
        s.close()
        ps = [subprocess.Popen([sys.executable, __file__, "--xgmi-worker", str(rk), str(R), port], env=env)
              for rk in range(R)]
        codes = [p.wait(timeout=300) for p in ps]
        if any(codes):
            sys.exit(max(codes))


if __name__ == "__main__":
    main()
