"""The dma1 conv main loop (single LDS stage, LDS-DMA operands, 128x128 tiles of 4 waves x 64x64) on
v_mfma_f32_16x16x32_bf16 (conv_force_impl(4)) vs v_mfma_f32_32x32x16_bf16 (conv_force_impl(6)), on the
Keras ResNet-50 b=256 convolutions dma1 serves (3x3, and every shape when forced): median us per
call, interleaved repeats, and the max relative difference of the two outputs."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

B = 256
SHAPES = [  # H, W, C, K, KH, stride, pad
    (56, 56, 64, 64, 3, 1, 1), (28, 28, 128, 128, 3, 1, 1), (14, 14, 256, 256, 3, 1, 1), (7, 7, 512, 512, 3, 1, 1),
    (28, 28, 512, 128, 1, 1, 0), (14, 14, 1024, 256, 1, 1, 0), (7, 7, 2048, 512, 1, 1, 0), (14, 14, 256, 1024, 1, 1, 0),
]


def med(fn, reps=15):
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
    C = hip()
    dev = "cuda:0"
    tot = {4: 0.0, 6: 0.0}
    for H, W, Ci, K, KH, s, p in SHAPES:
        x = torch.randn(B, H, W, Ci, device=dev).bfloat16()
        k = (torch.randn(KH, KH, Ci, K, device=dev) * 0.05).bfloat16()
        OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KH) // s + 1
        w_ohwi = k.permute(3, 0, 1, 2).contiguous()
        dy = torch.randn(B, OH, OW, K, device=dev).bfloat16()
        kc = k.contiguous()
        flop = 2.0 * B * OH * OW * K * KH * KH * Ci
        for d, fn in (("fwd", lambda: C.conv_fwd(x, w_ohwi, OH, OW, s, s, p, p)),
                      ("dgrad", lambda: C.conv_dgrad(dy, kc, H, W, p, p))):
            outs, ts = {}, {4: [], 6: []}
            for impl in (4, 6):
                C.conv_force_impl(impl)
                outs[impl] = fn().float()
            for _ in range(3):  # interleaved
                for impl in (4, 6):
                    C.conv_force_impl(impl)
                    ts[impl].append(med(fn))
            C.conv_force_impl(2)
            t4, t6 = sorted(ts[4])[1], sorted(ts[6])[1]
            tot[4] += t4
            tot[6] += t6
            diff = float((outs[4] - outs[6]).abs().max() / outs[4].abs().max())
            print(json.dumps({"dir": d, "shape": [B, H, W, Ci, K, KH, s, p], "mfma16x16x32_us": round(t4, 1),
                              "mfma32x32x16_us": round(t6, 1), "tflops16": round(flop / t4 / 1e6, 1),
                              "tflops32": round(flop / t6 / 1e6, 1), "max_rel_diff": round(diff, 5)}), flush=True)
    print(json.dumps({"sum_us": {"16x16x32": round(tot[4], 1), "32x32x16": round(tot[6], 1)}}))


if __name__ == "__main__":
    main()
