"""Where the K=20 overhead of the MNIST bench goes: device time and host wall of ONE replay of a
K-step graph (the engine's whole-execution graph), for several K, (a) right after the previous
replay finished ("warm") and (b) after the GPU sat idle for 2 ms ("cold")."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_learning_amd.models import mnist_cnn as M  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    b, N = 64, 60000
    X = torch.rand(N, 28, 28, 1, device=dev)
    Y = torch.randint(0, 10, (N,), device=dev, dtype=torch.int32)
    layout = M.mnist_layout()
    W = layout.pack(M.init_mnist_params(0), device=dev)
    G = torch.zeros_like(W)
    lr = torch.tensor([1e-3], device=dev)
    for K in (1, 2, 5, 10, 20, 50):
        idx = torch.randperm(N, device=dev)[: K * b].to(torch.int32)
        st = M.FusedMnistTrainStep(X, Y, idx, W, G, layout, b, 1, lr)
        for k in range(K):
            st.forward_backward(k * b)
            st.finalize(True)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for k in range(K):
                st.forward_backward(k * b)
                st.finalize(True)
        # the same K steps as one eager lead step + a graph of the other K - 1 (the graph launch's
        # host latency then overlaps the lead step on the GPU)
        gl = None
        if K > 1:
            gl = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gl, stream=s):
                for k in range(1, K):
                    st.forward_backward(k * b)
                    st.finalize(True)
        torch.cuda.synchronize(dev)
        res = {"warm": [], "cold": [], "lead-cold": []}
        for rep in range(30):
            for mode in res:
                if mode != "warm":
                    time.sleep(0.002)
                if mode == "lead-cold" and gl is None:
                    continue
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                t0 = time.perf_counter()
                e0.record()
                if mode == "lead-cold":
                    st.forward_backward(0)
                    st.finalize(True)
                    gl.replay()
                else:
                    g.replay()
                e1.record()
                torch.cuda.synchronize(dev)
                res[mode].append((e0.elapsed_time(e1) * 1e3, (time.perf_counter() - t0) * 1e6))
        for mode, v in res.items():
            if not v:
                continue
            a = np.array(v)
            print(f"K={K:3d} {mode}: device {np.median(a[:, 0]):8.1f} us ({np.median(a[:, 0]) / K:6.2f}/step)  "
                  f"wall {np.median(a[:, 1]):8.1f} us ({np.median(a[:, 1]) / K:6.2f}/step)", flush=True)


if __name__ == "__main__":
    main()
