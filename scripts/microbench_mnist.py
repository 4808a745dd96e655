"""Microbenchmark of the fused MNIST step on one GPU (graph-captured, K steps per graph).

    python scripts/microbench_mnist.py [--b 64] [--k 20] [--iters 50]
Prints per-step time for eager launches and graph replay, plus per-stage device times.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from tensorflow_distributed_learning_amd.models import mnist_cnn as M  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=64)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    N = 60000
    X = torch.rand(N, 28, 28, 1, device=dev)
    Y = torch.randint(0, 10, (N,), device=dev, dtype=torch.int32)
    layout = M.mnist_layout()
    W = layout.pack(M.init_mnist_params(0), device=dev)
    G = torch.zeros_like(W)
    idx = torch.randperm(N, device=dev)[: a.k * a.b].to(torch.int32)
    lr = torch.tensor([1e-3], device=dev)
    step = M.FusedMnistTrainStep(X, Y, idx, W, G, layout, a.b, 1, lr)

    def run_k():
        for k in range(a.k):
            step.forward_backward(k * a.b)
            step.finalize(True)

    for _ in range(3):
        run_k()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(a.iters):
        run_k()
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t) / (a.iters * a.k)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        run_k()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    reps = []
    for _ in range(5):
        t = time.perf_counter()
        for _ in range(a.iters):
            g.replay()
        torch.cuda.synchronize()
        reps.append((time.perf_counter() - t) / (a.iters * a.k))
    graph = sorted(reps)[len(reps) // 2]

    # per-stage device time (events around many launches of one stage)
    stages = {}
    for k in (8, 5, 6, 9):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(5):
            step.stage(k)
        e0.record()
        for _ in range(200):
            step.stage(k)
        e1.record()
        torch.cuda.synchronize()
        stages[k] = e0.elapsed_time(e1) * 1000 / 200
    print(f"b={a.b} eager {eager*1e6:.1f} us/step  graph {graph*1e6:.1f} us/step  "
          f"-> {a.b/graph:,.0f} img/s/GPU")
    print("stage us (back-to-back same-kernel launches):", {k: round(v, 2) for k, v in stages.items()})


if __name__ == "__main__":
    main()
