"""Input-side BN -> ReLU (conv_fwd_stats / conv_wgrad in_bn) vs the BN apply pass + plain kernels on the
ResNet-50 bottleneck's last 1x1 convs at b=256: per shape, microseconds of (apply + fwd) vs fused fwd,
and of the weight gradient over the materialised tensor vs with in_bn (each best of the in_bn plans)."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

SHAPES = [(56, 64, 256), (28, 128, 512), (14, 256, 1024), (7, 512, 2048)]


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


def main():
    C = hip()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    for H, Ci, K in SHAPES:
        x = (torch.randn(B, H, H, Ci, device="cuda") * 2 + 0.3).bfloat16()
        g, b = torch.rand(Ci, device="cuda") + 0.5, torch.randn(Ci, device="cuda")
        mm, mv = torch.zeros(Ci, device="cuda"), torch.ones(Ci, device="cuda")
        y, st = C.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, True, None, None)
        w = (torch.randn(K, 1, 1, Ci, device="cuda") / Ci ** 0.5).bfloat16()
        dy = torch.randn(B, H, H, K, device="cuda").bfloat16()
        t_apply = t(lambda: C.bn_forward_train(x, g, b, mm, mv, 0.9, 1e-3, True, None, None))
        t_stats = t(lambda: C.bn_stats_train(x, g, b, mm, mv, 0.9, 1e-3))
        t_fwd = t(lambda: C.conv_fwd_stats(y, w, H, H, 1, 1, 0, 0))
        t_pro = t(lambda: C.conv_fwd_stats(x, w, H, H, 1, 1, 0, 0, in_bn=st))

        def best(plans, **kw):
            return min(t(lambda: C.conv_wgrad(kw.get("src", y), dy, 1, 1, 1, 1, 0, 0,
                                              plan=[p[0], p[1], p[3], p[4]], in_bn=kw.get("st")))
                       for p in plans)

        t_wg = best(C.conv_wgrad_plans(list(x.shape), list(dy.shape), 1, 1, 1, 1, 0, 0, 6))
        t_wg_pro = best(C.conv_wgrad_plans(list(x.shape), list(dy.shape), 1, 1, 1, 1, 0, 0, 6, in_bn=True), src=x, st=st)
        print(json.dumps({"shape": [B, H, H, Ci, K], "bn_apply_us": round(t_apply - t_stats, 1),
                          "fwd_us": round(t_fwd, 1), "fwd_in_bn_us": round(t_pro, 1), "wgrad_us": round(t_wg, 1),
                          "wgrad_in_bn_us": round(t_wg_pro, 1)}), flush=True)


if __name__ == "__main__":
    main()
