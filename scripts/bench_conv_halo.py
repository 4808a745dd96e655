"""A/B of the halo (input-reuse) conv main loop (k_conv_halo) against the default selection (dma1 for
the 3x3 shapes) on the Keras ResNet-50 b=256 stride-1 3x3 convolutions: forward and input gradient,
interleaved repeats, plus the max relative difference of the two outputs and of each against a float32
reference.  One JSON line per (shape, direction)."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
HALO_ARM = int(sys.argv[2]) if len(sys.argv) > 2 else 1  # conv_force_halo value of the halo arm
# (H, W, C, K, calls per ResNet-50 step)
SHAPES = [(56, 56, 64, 64, 3), (28, 28, 128, 128, 4), (14, 14, 256, 256, 6), (7, 7, 512, 512, 3)]


def t(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-30)).item()


def main():
    C = hip()
    dev = "cuda:0"
    tot = {"default": 0.0, "halo": 0.0}
    for H, W, Ci, K, calls in SHAPES:
        g = torch.Generator(device="cpu").manual_seed(H * 1000 + Ci)
        x = torch.randn(B, H, W, Ci, generator=g).to(dev).bfloat16()
        k = (torch.randn(3, 3, Ci, K, generator=g) / (9 * Ci) ** 0.5).to(dev).bfloat16()
        dy = torch.randn(B, H, W, K, generator=g).to(dev).bfloat16()
        w_ohwi = k.permute(3, 0, 1, 2).contiguous()
        kc = k.contiguous()
        fns = {"fwd": lambda: C.conv_fwd(x, w_ohwi, H, W, 1, 1, 1, 1),
               "dgrad": lambda: C.conv_dgrad(dy, kc, H, W, 1, 1)}
        for d, fn in fns.items():
            C.conv_force_halo(0)
            y0 = fn()
            C.conv_force_halo(HALO_ARM)
            y1 = fn()
            if d == "fwd":
                ref = F.conv2d(x.float().permute(0, 3, 1, 2), k.float().permute(3, 2, 0, 1), None, 1, 1).permute(0, 2, 3, 1)
            else:
                ref = F.conv_transpose2d(dy.float().permute(0, 3, 1, 2), k.float().permute(3, 2, 0, 1), None, 1, 1
                                         ).permute(0, 2, 3, 1)
            ts = {"default": [], "halo": []}
            for _ in range(3):
                for arm, on in (("default", 0), ("halo", HALO_ARM)):
                    C.conv_force_halo(on)
                    ts[arm].append(t(fn))
            C.conv_force_halo(2)
            med = {a: sorted(v)[1] for a, v in ts.items()}
            for a in tot:
                tot[a] += med[a] * calls
            fl = 2.0 * B * H * W * K * 9 * Ci
            print(json.dumps({"dir": d, "shape": [B, H, W, Ci, K, 3], "default_us": round(med["default"], 1),
                              "halo_us": round(med["halo"], 1), "halo_tflops": round(fl / med["halo"] / 1e6, 1),
                              "default_tflops": round(fl / med["default"] / 1e6, 1),
                              "rel_halo_vs_default": rel(y1, y0), "rel_default_vs_f32": rel(y0, ref),
                              "rel_halo_vs_f32": rel(y1, ref)}), flush=True)
            del y0, y1, ref
    print(json.dumps({"step_weighted_us": {a: round(v, 1) for a, v in tot.items()}}))


if __name__ == "__main__":
    main()
