"""Bitwise run-to-run determinism of every hand-written ResNet-path kernel (diagnostic).

Each op runs REPS times on identical inputs; between repetitions a different kernel streams a
large buffer (cache / LDS state changes) and, every other time, the host sleeps (the GPU drains:
the launch-blocking pattern).  Any output that is not bit-identical to the first repetition is
reported with its largest difference.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

REPS = int(os.environ.get("REPS", "6"))
C = hip()
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(0)
junk = torch.empty(64 << 20, dtype=torch.float32, device=dev)


def rnd(*s, scale=1.0, dtype=torch.bfloat16):
    return (torch.randn(*s, generator=g) * scale).to(dev, dtype)


def perturb(i):
    junk.uniform_()  # streams 256 MB: evicts L2 / MALL
    if i % 2:
        torch.cuda.synchronize()
        time.sleep(0.01)


def _data_rows(t):
    """A BN partial-sum buffer [P + ceil(P/64)][2][C] from a conv epilogue: only its first P rows
    are outputs; the rest is scratch for the BN's pre-reduction (written only when P > 1024)."""
    if t.dim() == 3 and t.size(1) == 2 and t.dtype == torch.float32:
        P = t.size(0)
        while P > 1 and (P - 1) + (P - 1 + 63) // 64 >= t.size(0):
            P -= 1
        return t[:P]
    return t


def outs(r):
    if isinstance(r, (list, tuple)):
        return [_data_rows(t).clone() for t in r if isinstance(t, torch.Tensor)]
    return [_data_rows(r).clone()]


bad = []


def check(name, fn):
    ref = None
    for i in range(REPS):
        perturb(i)
        o = outs(fn())
        if ref is None:
            ref = o
            continue
        for j, (a, b) in enumerate(zip(ref, o)):
            if not torch.equal(a.view(torch.uint8) if a.dtype != torch.bool else a,
                               b.view(torch.uint8) if b.dtype != torch.bool else b):
                d = (a.double() - b.double()).abs()
                m = float(d.max()) if d.numel() else 0.0
                n = int((d > 0).sum())
                bad.append((name, j, i, m, n))
                print(f"NONDETERMINISTIC {name} out{j} rep{i}: {n} elems differ, max |d| {m:.3e}", flush=True)
                return
    print(f"ok {name}", flush=True)


def conv_cases():
    # (N, H, C, K, kh, stride): the diag model's shapes and a few ResNet-50 ones
    for (N, H, Ci, K, kh, s) in [(32, 8, 64, 64, 3, 1), (32, 8, 64, 128, 1, 1), (32, 8, 128, 64, 1, 1),
                                 (32, 8, 64, 128, 1, 2), (32, 4, 128, 64, 1, 1), (256, 56, 64, 64, 3, 1),
                                 (256, 28, 128, 128, 3, 1), (256, 14, 1024, 256, 1, 1), (256, 7, 512, 2048, 1, 1),
                                 (256, 56, 256, 512, 1, 2)]:
        p = kh // 2
        OH = (H + 2 * p - kh) // s + 1
        x = rnd(N, H, H, Ci)
        w = rnd(kh, kh, Ci, K, scale=0.05)
        wo = w.permute(3, 0, 1, 2).contiguous()
        dy = rnd(N, OH, OH, K)
        tag = f"N{N} H{H} {Ci}->{K} k{kh} s{s}"
        check(f"conv_fwd {tag}", lambda: C.conv_fwd(x, wo, OH, OH, s, s, p, p))
        check(f"conv_fwd_stats {tag}", lambda: C.conv_fwd_stats(x, wo, OH, OH, s, s, p, p))
        r = rnd(N, H, H, Ci)
        by = rnd(N, H, H, Ci)
        bx = rnd(N, H, H, Ci)
        if s == 1:
            check(f"conv_dgrad {tag}", lambda: C.conv_dgrad(dy, w, H, H, p, p, r))
            check(f"conv_dgrad_bn {tag}", lambda: C.conv_dgrad_bn(dy, w, H, H, p, p, r, by, bx, bx))
        elif kh == 1:
            check(f"conv_dgrad_s2 {tag}", lambda: C.conv_dgrad_s2(dy, w, H, H, r))
            check(f"conv_dgrad_s2_bn {tag}", lambda: C.conv_dgrad_s2_bn(dy, w, H, H, r, by, bx, bx))
        plans = C.conv_wgrad_plans(list(x.shape), list(dy.shape), kh, kh, s, s, p, p, 6)
        for pl in plans:
            plan = [pl[0], pl[1], pl[3], pl[4]]
            if N * OH * OH >= (1 << 24):
                continue
            check(f"conv_wgrad {tag} plan {plan}", lambda: C.conv_wgrad(x, dy, kh, kh, s, s, p, p, plan=plan))
            o = torch.zeros(kh * kh * Ci * K, device=dev)

            def acc(plan=plan, o=o):
                o.zero_()
                C.conv_wgrad(x, dy, kh, kh, s, s, p, p, out=o, accumulate=True, plan=plan)
                return o
            check(f"conv_wgrad_acc {tag} plan {plan}", acc)


def bn_cases():
    for (M, Cc) in [(32 * 64, 64), (32 * 64, 128), (32 * 16, 128), (256 * 3136, 64), (256 * 196, 1024), (256 * 49, 2048)]:
        x = rnd(M, Cc)
        r = rnd(M, Cc)
        ga = torch.rand(Cc, generator=g).to(dev) + 0.5
        be = torch.randn(Cc, generator=g).to(dev) * 0.1
        for relu, res in ((False, None), (True, None), (True, r)):
            mm, mv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
            tag = f"M{M} C{Cc} relu{int(relu)} res{int(res is not None)}"

            def fwd(relu=relu, res=res, mm=mm, mv=mv):
                y, st = C.bn_forward_train(x, ga, be, mm, mv, 0.99, 1e-3, relu, res, None, None)
                return [y, st]
            check(f"bn_fwd {tag}", fwd)
            y, st = C.bn_forward_train(x, ga, be, mm, mv, 0.99, 1e-3, relu, res, None, None)
            dy = rnd(M, Cc)
            mode = 2 if res is not None else (1 if relu else 0)
            check(f"bn_bwd {tag}", lambda mode=mode, y=y, st=st: C.bn_backward(dy, x, y if mode == 2 else None, ga, st,
                                                                                 mode, None, None, None))
            dg, db = torch.zeros(Cc, device=dev), torch.zeros(Cc, device=dev)

            def bwd_acc(mode=mode, y=y, st=st, dg=dg, db=db):
                dg.zero_()
                db.zero_()
                out = C.bn_backward(dy, x, y if mode == 2 else None, ga, st, mode, dg, db, None)
                return [out[0], dg, db]
            check(f"bn_bwd_acc {tag}", bwd_acc)


def misc_cases():
    for (M, N, K) in [(32, 16, 128), (256, 1000, 2048), (64, 128, 1600)]:
        a, b = rnd(M, K), rnd(N, K, scale=0.05)
        check(f"gemm_nt {M}x{N}x{K}", lambda: C.gemm_bf16(a, 0, b, 0))
        o = torch.zeros(N, K, device=dev)
        dy = rnd(M, N)

        def wg(o=o, dy=dy, a=a):
            o.zero_()
            C.gemm_bf16(dy, 1, a, 1, None, o, True)
            return o
        check(f"gemm_wgrad {M}x{N}x{K}", wg)
    x = rnd(32, 4, 4, 128)
    check("gap_fwd", lambda: C.gap_fwd(x))
    check("gap_bwd", lambda: C.gap_bwd(rnd(32, 128) * 0 + x[:, 0, 0, :], 4, 4))
    z = torch.randn(256, 1000, generator=g).to(dev)
    lab = torch.randint(0, 1000, (256,), generator=g).to(dev)
    check("xent_fwd", lambda: C.xent_fwd(z, lab))
    gg = torch.rand(256, generator=g).to(dev)
    check("xent_bwd", lambda: C.xent_bwd(z, lab, gg))
    xp = rnd(64, 112, 112, 64)
    check("maxpool_fwd", lambda: C.maxpool_fwd(xp, 3, 3, 2, 2, 1, 1, 56, 56, True))
    y, arg = C.maxpool_fwd(xp, 3, 3, 2, 2, 1, 1, 56, 56, True)
    dyp = rnd(64, 56, 56, 64)
    check("maxpool_bwd", lambda: C.maxpool_bwd(dyp, arg, [64, 112, 112, 64], 3, 3, 2, 2, 1, 1))
    W = torch.randn(1 << 20, generator=g).to(dev)
    Wc = torch.empty(1 << 20, dtype=torch.bfloat16, device=dev)
    check("slab_cast", lambda: (C.slab_cast_bf16(W, Wc), Wc)[1])
    xs = rnd(32, 224, 224, 3, dtype=torch.float32)
    ws = rnd(7, 7, 3, 64, scale=0.05)
    check("stem_fwd", lambda: C.stem_fwd(xs, ws, 3, 3, 3, 3, 2, 2, True))
    y, xpk, part = C.stem_fwd(xs, ws, 3, 3, 3, 3, 2, 2, True)
    dys = rnd(32, 112, 112, 64)
    check("stem_wgrad", lambda: C.stem_wgrad(xpk, dys, 7, 7, 3, 2))


if __name__ == "__main__":
    which = sys.argv[1:] or ["conv", "bn", "misc"]
    for w in which:
        {"conv": conv_cases, "bn": bn_cases, "misc": misc_cases}[w]()
    torch.cuda.synchronize()
    print(f"SUMMARY: {len(bad)} non-deterministic outputs", flush=True)
    for b in bad:
        print("  ", b)
