"""PMC target: the 56x56 64->256 1x1 forward of the ResNet-50 bottleneck, plain over the BN -> ReLU
output and with the input-side BN (in_bn), 10 calls each."""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

C = hip()
B, H, Ci, K = 256, 56, 64, 256
x = (torch.randn(B, H, H, Ci, device="cuda") * 2 + 0.3).bfloat16()
g, b = torch.rand(Ci, device="cuda") + 0.5, torch.randn(Ci, device="cuda")
y, st = C.bn_forward_train(x, g, b, torch.zeros(Ci, device="cuda"), torch.ones(Ci, device="cuda"), 0.9, 1e-3, True,
                           None, None)
w = (torch.randn(K, 1, 1, Ci, device="cuda") / Ci ** 0.5).bfloat16()
for _ in range(10):
    C.conv_fwd_stats(y, w, H, H, 1, 1, 0, 0)
    C.conv_fwd_stats(x, w, H, H, 1, 1, 0, 0, in_bn=st)
torch.cuda.synchronize()
