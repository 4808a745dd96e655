"""Per-shape timing of the hand-written weight-gradient kernel (csrc/kernels/conv_wgrad.hip) and the
1x1 stride-2 input gradient vs MIOpen on the convolutions of the Keras ResNet-50 (stride on the 1x1
convs) at b=256.  One JSON line per (shape, direction): times, TFLOP/s, the split plan and, with
the time of the cost model's first --candidates plans (checks the model's ranking)."""
import argparse
import json
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

# (H, W, C, K, KH, stride, pad): input size of the conv
SHAPES = [
    (56, 56, 64, 64, 1, 1, 0), (56, 56, 64, 64, 3, 1, 1), (56, 56, 64, 256, 1, 1, 0), (56, 56, 256, 64, 1, 1, 0),
    (56, 56, 256, 128, 1, 2, 0), (56, 56, 256, 512, 1, 2, 0), (28, 28, 128, 128, 3, 1, 1),
    (28, 28, 128, 512, 1, 1, 0), (28, 28, 512, 128, 1, 1, 0), (28, 28, 512, 256, 1, 2, 0),
    (28, 28, 512, 1024, 1, 2, 0), (14, 14, 256, 256, 3, 1, 1), (14, 14, 256, 1024, 1, 1, 0),
    (14, 14, 1024, 256, 1, 1, 0), (14, 14, 1024, 512, 1, 2, 0), (14, 14, 1024, 2048, 1, 2, 0),
    (7, 7, 512, 512, 3, 1, 1), (7, 7, 512, 2048, 1, 1, 0), (7, 7, 2048, 512, 1, 1, 0),
]


def t(fn, reps=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--candidates", type=int, default=8, help="model plans timed per shape")
    ap.add_argument("--single", type=int, default=0, help="register-staged kernel: 1 single LDS stage, 0 double-buffered")
    a = ap.parse_args()
    C = hip()
    C.conv_wgrad_force_single(bool(a.single))
    dev = "cuda:0"
    B = a.batch
    torch.backends.cudnn.benchmark = True
    tot_h = tot_m = 0.0
    for H, W, Ci, K, KH, s, p in SHAPES:
        x = torch.randn(B, H, W, Ci, device=dev).bfloat16()
        OH, OW = (H + 2 * p - KH) // s + 1, (W + 2 * p - KH) // s + 1
        dy = torch.randn(B, OH, OW, K, device=dev).bfloat16()
        k = (torch.randn(KH, KH, Ci, K, device=dev) * 0.05).bfloat16()
        w_oihw = k.permute(3, 2, 0, 1)
        xc, dyc = x.permute(0, 3, 1, 2), dy.permute(0, 3, 1, 2)
        flop = 2.0 * B * OH * OW * K * KH * KH * Ci

        def mi(mask):
            return torch.ops.aten.convolution_backward(dyc, xc, w_oihw, None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
                                                       mask)

        plans = C.conv_wgrad_plans(list(x.shape), list(dy.shape), KH, KH, s, s, p, p, a.candidates)
        ref = mi([False, True, False])[1].permute(2, 3, 1, 0).float()
        times, errs = [], []
        for pl in plans:
            hw = lambda: C.conv_wgrad(x, dy, KH, KH, s, s, p, p, plan=[pl[0], pl[1], pl[3], pl[4]])  # noqa: E731
            errs.append(float((hw().float() - ref).abs().max() / ref.abs().max()))
            times.append(round(t(hw), 1))
        err = max(errs)
        t_m = t(lambda: mi([False, True, False]))
        i = min(range(len(times)), key=times.__getitem__)
        t_h = times[i]
        tot_h += min(t_h, t_m)
        tot_m += t_m
        print(json.dumps({"dir": "wgrad", "shape": [B, H, W, Ci, K, KH, s, p], "rel_err": round(err, 5),
                          "hip_us": t_h, "miopen_us": round(t_m, 1), "hip_tflops": round(flop / t_h / 1e6, 1),
                          "speedup": round(t_m / t_h, 3), "best_plan": plans[i], "model_rank_of_best": i,
                          "candidates_us": {str(pl): tt for pl, tt in zip(plans, times)}}), flush=True)
        if s == 2 and KH == 1:
            kc = k.contiguous()
            hd = lambda: C.conv_dgrad_s2(dy, kc, H, W)  # noqa: E731
            ref = mi([True, False, False])[0].permute(0, 2, 3, 1).float()
            err = float((hd().float() - ref).abs().max() / ref.abs().max())
            t_h, t_m = t(hd), t(lambda: mi([True, False, False]))
            print(json.dumps({"dir": "dgrad_s2", "shape": [B, H, W, Ci, K, KH, s, p], "rel_err": round(err, 5),
                              "hip_us": round(t_h, 1), "miopen_us": round(t_m, 1),
                              "hip_tflops": round(flop / t_h / 1e6, 1), "speedup": round(t_m / t_h, 3)}), flush=True)
    print(json.dumps({"wgrad_total_us_best_of": round(tot_h, 1), "wgrad_total_us_miopen": round(tot_m, 1),
                      "single": a.single}))


if __name__ == "__main__":
    main()
