"""One hand-written conv forward shape, launched `reps` times (for rocprofv3 PMC passes / A-B builds).

    python scripts/conv_one.py H W C K KH STRIDE PAD [batch] [reps]
Prints the mean kernel time and TFLOP/s."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402


def main():
    H, W, C, K, KH, S, P = (int(v) for v in sys.argv[1:8])
    B = int(sys.argv[8]) if len(sys.argv) > 8 else 256
    reps = int(sys.argv[9]) if len(sys.argv) > 9 else 50
    dev = torch.device("cuda:0")
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.rand(B, H, W, C, generator=g) * 2 - 1).to(dev, torch.bfloat16)
    w = ((torch.rand(K, KH, KH, C, generator=g) * 2 - 1) * 0.05).to(dev, torch.bfloat16)
    OH, OW = (H + 2 * P - KH) // S + 1, (W + 2 * P - KH) // S + 1
    Cx = hip()
    for _ in range(3):
        Cx.conv_fwd(x, w, OH, OW, S, S, P, P)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        Cx.conv_fwd(x, w, OH, OW, S, S, P, P)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    fl = 2.0 * B * OH * OW * K * KH * KH * C
    print(f"conv fwd {B}x{H}x{W}x{C} -> {K} k{KH} s{S}: {us:.1f} us  {fl / us / 1e6:.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
