"""Phase timestamps (s_memrealtime, 10 ns ticks) of the per-image kernels: median over workgroups
of each phase duration and of the kernel span, after warm-up."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_learning_amd.models import mnist_cnn as M

dev = torch.device("cuda:0")
b, N = 64, 60000
X = torch.rand(N, 28, 28, 1, device=dev)
Y = torch.randint(0, 10, (N,), device=dev, dtype=torch.int32)
layout = M.mnist_layout()
W = layout.pack(M.init_mnist_params(0), device=dev)
G = torch.zeros_like(W)
idx = torch.randperm(N, device=dev)[:b].to(torch.int32)
lr = torch.tensor([1e-3], device=dev)
st = M.FusedMnistTrainStep(X, Y, idx, W, G, layout, b, 1, lr)
for _ in range(20):
    st.forward_backward(0); st.finalize(True)
for name, k, grid, phases in (("fwd_conv", 8, b * 4, ["stage-issue", "stage-barrier", "conv1", "barrier2", "conv2-mfma", "epilogue"]),
                               ("conv_bwd", 6, b * 4, ["stage-issue", "stage-barrier", "wgrad", "dgrad+epi", "final-barrier"])):
    buf = torch.zeros(grid * 8, dtype=torch.int64, device=dev)
    res = []
    for rep in range(5):
        st.forward_backward(0); st.finalize(True)
        buf.zero_()
        st._impl.set_stamps(buf)
        st.stage(k)
        st._impl.set_stamps(None)
        torch.cuda.synchronize()
        res.append(buf.view(grid, 8).cpu().numpy().astype(np.int64))
    r = res[-1]
    n = len(phases) + 1
    d = np.diff(r[:, :n], axis=1) * 10 / 1000.0  # us
    span = (r[:, n - 1].max() - r[:, 0].min()) * 10 / 1000.0
    starts = (r[:, 0] - r[:, 0].min()) * 10 / 1000.0
    print(f"{name}: kernel span {span:.2f} us; WG start spread {starts.max():.2f} us")
    for j, ph in enumerate(phases):
        print(f"   {ph:14s} median {np.median(d[:, j]):6.2f}  max {d[:, j].max():6.2f} us")
