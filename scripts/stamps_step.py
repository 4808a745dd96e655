"""Whole-step timeline of the fused MNIST step (fused kernel + KF-X finalize) from per-wave
s_memrealtime stamps (10 ns ticks): span of each launch and the gap between them."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_learning_amd.models import mnist_cnn as M  # noqa: E402


def _cats(nfx):
    """KF-X block ranges (dW3 / small dense / conv2 / conv1) for a finalize of nfx workgroups."""
    d = nfx - 146 - 20  # kFxDense (= kFxW3 + 9 small dense blocks)
    return {f"dW3 rows (0-{d - 10})": (0, d - 9), f"db3/dW4/db4 ({d - 9}-{d - 1})": (d - 9, d),
            f"conv2 pieces ({d}-{d + 145})": (d, d + 146), f"conv1 ({d + 146}-{nfx - 1})": (d + 146, nfx)}


def main():
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
        st.forward_backward(0)
        st.finalize(True)
    grid, nfx = 4 * b, M.FINALIZE_BLOCKS
    CATS = _cats(nfx)
    rows, cats, lasts = [], [], []
    for rep in range(int(os.environ.get("REPS", "20"))):
        buf = torch.zeros(grid * 104 + nfx * 16, dtype=torch.int64, device=dev)
        st._impl.set_stamps(buf)
        st.forward_backward(0)
        st.finalize(True)
        st._impl.set_stamps(None)
        torch.cuda.synchronize()
        f = buf[:grid * 104].cpu().numpy().astype(np.int64)
        f = f[f > (1 << 32)]  # (time stamps only: the head's slot 4 holds a poll count)
        x = buf[grid * 104:].view(nfx, 8, 2).cpu().numpy().astype(np.int64)
        t0 = f.min()
        xs0 = x[:, :, 0].min()
        cats.append([((x[lo:hi, :, 0].min() - xs0) / 100, (np.median(x[lo:hi, :, 0]) - xs0) / 100,
                      (np.median(x[lo:hi, :, 1]) - xs0) / 100, (x[lo:hi, :, 1].max() - xs0) / 100)
                     for lo, hi in CATS.values()])
        lasts.append((x[:, :, 1].max(axis=1) - xs0) / 100)  # per-block last wave end
        rows.append([(f.max() - t0) / 100, (x[:, :, 0].min() - f.max()) / 100, (x[:, :, 1].max() - x[:, :, 0].min()) / 100,
                     (np.median(x[:, :, 1] - x[:, :, 0])) / 100, (x[:, :, 0].max() - x[:, :, 0].min()) / 100,
                     (x[:, :, 1].max() - t0) / 100])
        for _ in range(3):
            st.forward_backward(0)
            st.finalize(True)
    a = np.array(rows)
    names = ["fused span", "gap fused->KF-X", "KF-X span", "KF-X median wave life", "KF-X wave start spread", "step span"]
    for k, nm in enumerate(names):
        print(f"{nm:24s} median {np.median(a[:, k]):6.2f} us  min {a[:, k].min():6.2f}  max {a[:, k].max():6.2f}")
    c = np.median(np.array(cats), axis=0)
    print("KF-X blocks, us since KF-X first wave (median over reps): first start / median start / median end / last end")
    for (nm, _), v in zip(CATS.items(), c):
        print(f"  {nm:22s} " + " ".join(f"{t:6.2f}" for t in v))
    ml = np.median(np.array(lasts), axis=0)
    late = np.argsort(ml)[::-1][:12]
    print("latest KF-X blocks (median last-wave end, us): " + ", ".join(f"{j}:{ml[j]:.2f}" for j in late))


if __name__ == "__main__":
    main()
