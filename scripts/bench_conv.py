"""Per-shape timing of the hand-written implicit-GEMM conv kernels vs MIOpen (F.conv2d, channels_last
bf16) on the ResNet-50 b=256 convolutions: forward and stride-1 input gradient.  Prints one JSON line
per (shape, direction) with both times and the TFLOP/s of the hand-written kernel."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
KERAS = len(sys.argv) > 2 and sys.argv[2] == "keras"
# (H, W, C, K, KH, stride, pad) of ResNet-50 v1.5 (C % 64 == 0 ones; the 7x7 stem stays on MIOpen)
SHAPES_V15 = [
    (56, 56, 64, 64, 1, 1, 0), (56, 56, 64, 64, 3, 1, 1), (56, 56, 64, 256, 1, 1, 0), (56, 56, 256, 64, 1, 1, 0),
    (56, 56, 256, 128, 1, 1, 0), (56, 56, 128, 128, 3, 2, 1), (28, 28, 128, 128, 3, 1, 1),
    (28, 28, 128, 512, 1, 1, 0), (28, 28, 512, 128, 1, 1, 0), (56, 56, 256, 512, 1, 2, 0),
    (28, 28, 512, 256, 1, 1, 0), (14, 14, 256, 256, 3, 1, 1), (14, 14, 256, 1024, 1, 1, 0),
    (14, 14, 1024, 256, 1, 1, 0), (14, 14, 1024, 512, 1, 1, 0), (7, 7, 512, 512, 3, 1, 1),
    (7, 7, 512, 2048, 1, 1, 0), (7, 7, 2048, 512, 1, 1, 0),
]
# the Keras ResNet50 of models/resnet50.py (stride on the 1x1 convs), with the per-step call count
SHAPES_KERAS = {
    (56, 56, 64, 64, 1, 1, 0): 1, (56, 56, 64, 64, 3, 1, 1): 3, (56, 56, 64, 256, 1, 1, 0): 4,
    (56, 56, 256, 64, 1, 1, 0): 2, (56, 56, 256, 128, 1, 2, 0): 1, (56, 56, 256, 512, 1, 2, 0): 1,
    (28, 28, 128, 128, 3, 1, 1): 4, (28, 28, 128, 512, 1, 1, 0): 4, (28, 28, 512, 128, 1, 1, 0): 3,
    (28, 28, 512, 256, 1, 2, 0): 1, (28, 28, 512, 1024, 1, 2, 0): 1, (14, 14, 256, 256, 3, 1, 1): 6,
    (14, 14, 256, 1024, 1, 1, 0): 6, (14, 14, 1024, 256, 1, 1, 0): 5, (14, 14, 1024, 512, 1, 2, 0): 1,
    (14, 14, 1024, 2048, 1, 2, 0): 1, (7, 7, 512, 512, 3, 1, 1): 3, (7, 7, 512, 2048, 1, 1, 0): 3,
    (7, 7, 2048, 512, 1, 1, 0): 2,
}
SHAPES = list(SHAPES_KERAS) if KERAS else SHAPES_V15


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


def sweep(C, fn):
    """Times of the v1 (register-staged, 128-row tiles), v2 (LDS-DMA ring, 256-row tiles where
    the grid fills the chip) and dma1 (single-stage LDS-DMA, 128-row tiles, at 4 and 3 waves per
    SIMD) main loops, and of the default selection without the single-stage
    variant for 1-2 k-tile reductions (conv_force_depth(3)), of the single stage everywhere
    (conv_force_depth(0), plain epilogues) and of the single LDS stage with register prefetch at 3
    workgroups per CU everywhere (conv_force_depth(4))."""
    out = []
    for impl in (1, 3, 4, 5):
        C.conv_force_impl(impl)
        out.append(round(t(fn), 1))
    C.conv_force_impl(2)
    for d in (3, 0, 4):  # d3: the pre-round-4 default selection; d0 / d4: v1 variants everywhere
        C.conv_force_impl(2 if d == 3 else 1)
        C.conv_force_depth(d)
        out.append(round(t(fn), 1))
    C.conv_force_depth(2)
    C.conv_force_impl(2)
    return out


def main():
    C = hip()
    dev = "cuda:0"
    torch.backends.cudnn.benchmark = True
    for H, W, Ci, K, KH, s, p in SHAPES:
        x = torch.randn(B, H, W, Ci, device=dev).bfloat16()
        k = (torch.randn(KH, KH, Ci, K, device=dev) * 0.05).bfloat16()
        OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KH) // s + 1
        w_oihw = k.permute(3, 2, 0, 1)
        w_ohwi = k.permute(3, 0, 1, 2).contiguous()
        xc = x.permute(0, 3, 1, 2)
        flop = 2.0 * B * OH * OW * K * KH * KH * Ci
        y_h, y_m = C.conv_fwd(x, w_ohwi, OH, OW, s, s, p, p), F.conv2d(xc, w_oihw, None, s, p).permute(0, 2, 3, 1)
        err = float((y_h.float() - y_m.float()).abs().max() / y_m.float().abs().max())
        t_h = t(lambda: C.conv_fwd(x, w_ohwi, OH, OW, s, s, p, p))
        tiles = sweep(C, lambda: C.conv_fwd(x, w_ohwi, OH, OW, s, s, p, p))
        t_m = t(lambda: F.conv2d(xc, w_oihw, None, s, p))
        byt = 2.0 * B * (H * W * Ci + OH * OW * K)
        floor = max(flop / 1.2e15, byt / 5e12) * 1e6
        print(json.dumps({"dir": "fwd", "shape": [B, H, W, Ci, K, KH, s, p], "rel_err": round(err, 5), "hip_us": round(t_h, 1), "v1_v2_dma4_dma3_d3_d0_d4_us": tiles,
                          "miopen_us": round(t_m, 1), "hip_tflops": round(flop / t_h / 1e6, 1),
                          "speedup": round(t_m / t_h, 3), "floor_us": round(floor, 1),
                          "calls": SHAPES_KERAS.get((H, W, Ci, K, KH, s, p), 0)}), flush=True)
        if s == 1:
            dy = torch.randn(B, OH, OW, K, device=dev).bfloat16()
            kc = k.contiguous()
            dyc = dy.permute(0, 3, 1, 2)
            d_h = C.conv_dgrad(dy, kc, H, W, p, p)
            d_m = torch.ops.aten.convolution_backward(dyc, xc, w_oihw, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                      [True, False, False])[0].permute(0, 2, 3, 1)
            err = float((d_h.float() - d_m.float()).abs().max() / d_m.float().abs().max())
            t_h = t(lambda: C.conv_dgrad(dy, kc, H, W, p, p))
            tiles = sweep(C, lambda: C.conv_dgrad(dy, kc, H, W, p, p))
            t_m = t(lambda: torch.ops.aten.convolution_backward(dyc, xc, w_oihw, None, [s, s], [p, p], [1, 1], False,
                                                                [0, 0], 1, [True, False, False]))
            print(json.dumps({"dir": "dgrad", "shape": [B, H, W, Ci, K, KH, s, p], "rel_err": round(err, 5), "hip_us": round(t_h, 1), "v1_v2_dma4_dma3_d3_d0_d4_us": tiles,
                              "miopen_us": round(t_m, 1), "hip_tflops": round(flop / t_h / 1e6, 1),
                              "speedup": round(t_m / t_h, 3), "floor_us": round(floor, 1),
                              "calls": SHAPES_KERAS.get((H, W, Ci, K, KH, s, p), 0)}), flush=True)


if __name__ == "__main__":
    main()
