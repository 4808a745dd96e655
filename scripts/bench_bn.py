"""Effective HBM bandwidth of the NHWC batch-norm kernels (csrc/kernels/bn.hip) on the ResNet-50
b=256 shapes, over a sweep of the tuning knobs (partial-pass workgroups, elementwise grid, vectors per
thread, elementwise kernel family: 0 grid-stride, 1 blocked), with a plain device copy as the reference
ceiling.  One JSON line per shape."""
import json
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

SHAPES = [(802816, 64), (802816, 256), (200704, 128), (200704, 512), (50176, 256), (50176, 1024), (12544, 512),
          (12544, 2048), (3211264, 64)]
# (max_parts, elem_blocks, elem_unroll, kind, vectors per thread)
CONFIGS = [(512, 4096, 1, 0, 4), (512, 4096, 1, 1, 2), (512, 4096, 1, 1, 4), (512, 4096, 1, 1, 8),
           (512, 8192, 1, 1, 4), (512, 2048, 1, 1, 4), (512, 1024, 1, 1, 8)]


def t(fn, reps=10):
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
    dev = "cuda:0"
    tot = {}
    for M, Ch in SHAPES:
        x = torch.randn(M, Ch, device=dev).bfloat16()
        dy = torch.randn(M, Ch, device=dev).bfloat16()
        r = torch.randn(M, Ch, device=dev).bfloat16()
        y = torch.empty_like(x)
        g, b = torch.rand(Ch, device=dev) + 0.5, torch.randn(Ch, device=dev)
        mm, mv = torch.zeros(Ch, device=dev), torch.ones(Ch, device=dev)
        nb = M * Ch * 2
        tc = t(lambda: y.copy_(x))
        rec = {"shape": [M, Ch], "copy_TBps": round(2 * nb / tc / 1e6, 2)}
        for cfg in CONFIGS:
            C.bn_set_tuning(*cfg[:3])
            C.bn_set_elementwise(*cfg[3:])
            yf, st = C.bn_forward_train(x, g, b, mm, mv, 0.99, 1e-3, True, None, None)
            t_f = t(lambda: C.bn_forward_train(x, g, b, mm, mv, 0.99, 1e-3, True, None, None))
            t_fr = t(lambda: C.bn_forward_train(x, g, b, mm, mv, 0.99, 1e-3, True, r, None))
            t_b1 = t(lambda: C.bn_backward(dy, x, None, g, st, 1))
            t_b2 = t(lambda: C.bn_backward(dy, x, yf, g, st, 2))
            key = str(cfg)
            rec[key] = {"fwd_us": round(t_f, 1), "fwd_TBps": round(3 * nb / t_f / 1e6, 2),
                        "fwd_res_us": round(t_fr, 1), "bwd_relu_us": round(t_b1, 1),
                        "bwd_relu_TBps": round(5 * nb / t_b1 / 1e6, 2), "bwd_res_us": round(t_b2, 1),
                        "bwd_res_TBps": round(8 * nb / t_b2 / 1e6, 2)}
            tot[key] = tot.get(key, 0.0) + t_f + t_fr + t_b1 + t_b2
        print(json.dumps(rec), flush=True)
    print(json.dumps({"total_us_per_config": {k: round(v, 1) for k, v in tot.items()}}))
    C.bn_set_tuning(512, 4096, 1)  # the defaults (the blocked kernels' grid cap back to 8192 below)
    C.bn_set_elementwise(1, 4)
    C.bn_set_tuning(0, 8192, 0)


if __name__ == "__main__":
    main()
