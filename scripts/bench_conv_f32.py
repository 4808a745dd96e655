"""Generic f32 conv / Dense kernels (csrc/kernels/gemm_f32.hip) vs the library (MIOpen / hipBLASLt
through torch) on the reference CNN's layer shapes and a few larger f32 shapes: median us per call
of forward, input gradient and weight gradient.  Usage: python scripts/bench_conv_f32.py"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensorflow_distributed_learning_amd.ops import conv_f32 as CF  # noqa: E402

SHAPES = [
    # N, H, W, C, K, R, stride, pad(same)
    (64, 28, 28, 1, 32, 3, 1, 0),
    (64, 13, 13, 32, 64, 3, 1, 0),
    (64, 28, 28, 1, 32, 3, 1, 1),
    (256, 28, 28, 32, 64, 3, 1, 1),
    (256, 14, 14, 64, 128, 3, 2, 1),
    (128, 56, 56, 64, 64, 3, 1, 1),
]


def med(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    return sorted(ts)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    torch.backends.cudnn.benchmark = False
    for (N, H, W, C, K, R, s, p) in SHAPES:
        x = torch.randn(N, H, W, C, device=dev)
        w = torch.randn(R, R, C, K, device=dev) / (R * R * C) ** 0.5
        pads = (p, p, p, p)
        y = CF.fwd(x, w, None, (s, s), pads)
        dy = torch.randn_like(y)
        xn, wn, dyn = x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1).contiguous(), dy.permute(0, 3, 1, 2)
        mask = [True, True, False]
        r = {"shape": [N, H, W, C, K, R, s, p]}
        r["hip_fwd_us"] = med(lambda: CF.fwd(x, w, None, (s, s), pads))
        r["lib_fwd_us"] = med(lambda: F.conv2d(xn, wn, None, s, p))
        r["hip_dgrad_us"] = med(lambda: CF.dgrad(dy, w, (H, W), (s, s), pads))
        r["hip_wgrad_us"] = med(lambda: CF.wgrad(x, dy, (R, R), (s, s), pads))
        r["lib_bwd_us"] = med(lambda: torch.ops.aten.convolution_backward(dyn, xn, wn, None, [s, s], [p, p], [1, 1],
                                                                          False, [0, 0], 1, mask))
        flop = 2.0 * N * y.shape[1] * y.shape[2] * K * R * R * C
        r["hip_fwd_tflops"] = round(flop / r["hip_fwd_us"] / 1e6, 2)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
    for (M, D, U) in [(64, 1600, 128), (64, 128, 10), (4096, 4096, 4096)]:
        a = torch.randn(M, D, device=dev)
        b = torch.randn(D, U, device=dev)
        from tensorflow_distributed_learning_amd.ops import hip

        r = {"gemm": [M, D, U], "hip_us": med(lambda: hip().gemm_f32(a, 0, b, 1)), "lib_us": med(lambda: a @ b)}
        r["hip_tflops"] = round(2.0 * M * D * U / r["hip_us"] / 1e6, 2)
        print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)


if __name__ == "__main__":
    main()
