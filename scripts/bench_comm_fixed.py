#!/usr/bin/env python3
"""Fixed costs of the gradient all-reduce paths on ONE MI355X (replace guessed
constants in parallel/bucketing.py with measured ones).

    python scripts/bench_comm_fixed.py > profiles/comm_fixed_costs_r4.jsonl

(A world-1 RCCL "all-reduce" launches nothing and measures nothing: no such rows.)  The round-3
single-sample 28.5 us for the 64 KiB two-shot was a cold first call: with interleaved repeats its
median is 6.8 us and that sample shows up as the max (profiles/comm_fixed_costs_r4.jsonl).

* ``xgmi_oneshot`` / ``xgmi_twoshot`` at R = 2 and 4: the xGMI all-reduce kernel between R
  processes that share the one GPU (IPC-mapped exchange buffers, flags, fences, rank-order sums):
  its fixed cost and its local memory traffic, again without a fabric hop.

Sizes 64 KiB .. 4 MiB of f32 (one channel), REPEATS interleaved rounds: median / min / max per
(path, R, bytes), one JSON line each.  The xGMI link term of the
bucket cost model (153.6 GB/s per link, ring hops) stays modelled: this box has one GPU.
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIZES = [64 << 10, 256 << 10, 1 << 20, 4 << 20]  # up to one channel's limit (TDL_XGMI_MAX_BYTES)
ITERS = 50
REPEATS = 7


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


def xgmi_worker(rank: int, R: int, port: str):
    """Every (size, algorithm) channel is set up first; then REPEATS rounds time each channel once,
    in a rotated order per round (interleaved repeats: a drift of the box or a cold first call shows
    up as spread instead of biasing one row)."""
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist

    from tensorflow_distributed_learning_amd import ops

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=R, init_method=f"tcp://127.0.0.1:{port}")
    C = ops.hip()
    cases = []
    # R replica processes share the ONE GPU: every launch's workgroups spin until the same workgroup
    # of each peer arrives, so all R launches must be resident at once -- at R = 4 only the small
    # channels fit (the 1-4 MiB ones time out: 256-1024 spinning workgroups per process)
    for nbytes in (SIZES if R <= 2 else [b for b in SIZES if b <= (256 << 10)]):
        n = nbytes // 4
        for algo in (0, 1):
            ch = C.XgmiChannel(rank, R, n, 0, 60.0, algo)
            hs = [None] * R
            dist.all_gather_object(hs, (bytes(ch.handle(False)), bytes(ch.handle(True))))
            ch.open([h[0] for h in hs], [h[1] for h in hs])
            x = torch.randn(n, device=dev)
            cases.append((nbytes, algo, ch, x, torch.empty_like(x)))
    times = {(c[0], c[1]): [] for c in cases}
    for rep in range(REPEATS):
        k = rep % len(cases)
        for nbytes, algo, ch, x, y in cases[k:] + cases[:k]:
            dist.barrier()
            us = _time_graph(lambda: ch.all_reduce(x, y, 1.0), dev)
            assert ch.error() == 0
            t = torch.tensor([us])
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            times[(nbytes, algo)].append(float(t))
    if rank == 0:
        for (nbytes, algo), ts in times.items():
            ts = sorted(ts)
            print(json.dumps({"path": "xgmi_oneshot" if algo == 0 else "xgmi_twoshot", "R": R, "bytes": nbytes,
                              "us_per_call_median": round(ts[len(ts) // 2], 2), "us_min": round(ts[0], 2),
                              "us_max": round(ts[-1], 2), "repeats": len(ts),
                              "note": f"{R} processes sharing one GPU: fixed cost + local traffic, no fabric hop"}),
                  flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--xgmi-worker":
        xgmi_worker(int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
        return
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
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
