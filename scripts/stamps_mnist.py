"""Per-wave phase timestamps (s_memrealtime, 10 ns ticks) of the per-image MNIST kernels.

For every wave slot, prints the median (over workgroups) time from the kernel's first wave start
to each stamped point, so phases of different waves can be compared on one clock."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_learning_amd.models import mnist_cnn as M  # noqa: E402

KERNELS = {
    "fwd_conv": (8, 8, {0: "start", 1: "stage-issued", 2: "stage-barrier", 3: "conv1-done", 4: "barrier2",
                        5: "conv2-mfma", 6: "dense1-partial", 7: "dP2-done|fused: dP2-start"}, 256),
    "conv_bwd": (6, 8, {0: "start", 1: "stage-issued", 2: "stage-barrier", 3: "wgrad-done", 6: "dgrad-mfma",
                        4: "dgrad-epi", 5: "final-barrier"}, 256),
}


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
    fused = bool(st.fused_bwd)
    print(f"fused_bwd={fused}")
    for name, (k, waves, slots, grid) in KERNELS.items():
        if fused and name == "conv_bwd":
            continue
        buf = torch.zeros(grid * 104, dtype=torch.int64, device=dev)
        st.forward_backward(0)
        st.finalize(True)
        st._impl.set_stamps(buf)
        st.stage(k)
        st._impl.set_stamps(None)
        torch.cuda.synchronize()
        r = buf[:grid * 64].view(grid, 8, 8).cpu().numpy().astype(np.int64)
        hs = buf[grid * 64:grid * 72].view(grid, 8).cpu().numpy().astype(np.int64)
        t0 = r[:, :waves, 0].min(axis=1, keepdims=True)
        rel = (r - t0[:, :, None]) * 10 / 1000.0  # us since the workgroup's first wave started
        span = (r[:, :waves][r[:, :waves] > 0].max() - r[:, :waves, 0].min()) * 10 / 1000.0
        starts = r[:, 0, 0]
        print(f"{name}: kernel span {span:.2f} us; workgroup start spread {(starts.max() - starts.min()) / 100:.2f} us"
              "  (median us since workgroup start, per wave)")
        if name == "fwd_conv":
            # the loss head ran in the last quarter workgroup of each image: its phases
            # (0 hand-off won, 1 partials loaded, 2 logits/softmax, 3 end) follow the wave stamps
            last = hs[:, 0] > 0
            g0 = r[:, :waves, 0][r[:, :waves, 0] > 0].min()
            h = (hs[last][:, :4] - g0) / 100.0
            p6 = (r[:, 0, 6] - g0) / 100.0
            print(f"  head in {last.sum()} workgroups; us since kernel start (median / max): dense1 partial stored "
                  f"{np.median(p6):.2f}/{p6.max():.2f}; head won {np.median(h[:, 0]):.2f}/{h[:, 0].max():.2f}; "
                  f"partials loaded {np.median(h[:, 1]):.2f}/{h[:, 1].max():.2f}; softmax {np.median(h[:, 2]):.2f}/"
                  f"{h[:, 2].max():.2f}; dH published {np.median(h[:, 3]):.2f}/{h[:, 3].max():.2f}")
            if last.all() and grid % 4 == 0:
                # every quarter ran the head: its wait is set by the LAST of the image's other three
                # quarters to store its partial (p6 of wave 0); loaded - that = visibility + detection
                p6i = p6.reshape(-1, 4)
                other = np.stack([np.delete(p6i, c, axis=1).max(axis=1) for c in range(4)], axis=1).reshape(-1)
                lat = h[:, 1] - other
                polls = hs[:, 4]
                print(f"  partial hand-off: last partner store -> partials loaded median {np.median(lat):.2f} "
                      f"us (p10 {np.percentile(lat, 10):.2f}, p90 {np.percentile(lat, 90):.2f}); poll rounds "
                      f"median {np.median(polls):.0f} (min {polls.min()}, max {polls.max()})")
        if name == "fwd_conv" and fused:
            bs = buf[grid * 72:].view(grid, 8, 4).cpu().numpy().astype(np.int64)
            t0w = r[:, :waves, 0].min(axis=1)
            relb = (bs - t0w[:, None, None]) * 10 / 1000.0
            for k2, label in enumerate(["bwd dC2 ready", "bwd wgrad done", "bwd dgrad done", "bwd reduced"]):
                vals = [np.median(relb[:, w, k2]) for w in range(waves)]
                print(f"  {label:14s}" + " ".join(f"{v:6.2f}" for v in vals))
        print("  slot/wave " + " ".join(f"{w:>6d}" for w in range(waves)))
        for s, label in sorted(slots.items(), key=lambda kv: np.median(rel[:, 0, kv[0]])):
            vals = [np.median(rel[:, w, s]) if (r[:, w, s] > 0).all() else float("nan") for w in range(waves)]
            print(f"  {label:14s}" + " ".join(f"{v:6.2f}" for v in vals))


if __name__ == "__main__":
    main()
