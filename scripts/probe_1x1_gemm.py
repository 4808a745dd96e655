# compare MIOpen 1x1 conv vs hipBLASLt matmul for ResNet-50 1x1 shapes (bf16, b=256): fwd+bwd time
import torch, time, torch.nn.functional as F
dev = "cuda"
shapes = [(56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (14, 1024, 256), (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]
N = 256
def bench(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e3
for H, Ci, Co in shapes:
    x = torch.randn(N, H, H, Ci, device=dev, dtype=torch.bfloat16, requires_grad=True)
    w = torch.randn(Ci, Co, device=dev, dtype=torch.bfloat16, requires_grad=True)
    wc = w.detach().t().contiguous().view(Co, Ci, 1, 1).requires_grad_(True)
    def mm():
        y = x.reshape(-1, Ci) @ w
        y.sum().backward()
    def cv():
        y = F.conv2d(x.permute(0, 3, 1, 2), wc)
        y.sum().backward()
    tm, tc = bench(mm), bench(cv)
    fl = 3 * 2 * N * H * H * Ci * Co / 1e12
    print(f"H={H} {Ci}->{Co}: matmul {tm:.3f} ms ({fl/tm*1e3:.0f} TF/s)  conv {tc:.3f} ms ({fl/tc*1e3:.0f} TF/s)")
