"""One ResNet-50 convolution (default: b=256 28x28 3x3 128->128) on the hand-written forward kernel,
a few launches, for rocprofv3 PMC passes (scripts/pmc_conv.sh).

    python scripts/microbench_conv.py [B H Cin K KH [impl]]"""
import sys

import torch

sys.path.insert(0, ".")
from tensorflow_distributed_learning_amd.ops import hip  # noqa: E402

B, H, Ci, K, KH = (int(v) for v in (sys.argv[1:6] if len(sys.argv) > 5 else (256, 28, 128, 128, 3)))
IMPL = int(sys.argv[6]) if len(sys.argv) > 6 else 2  # conv_force_impl: 1 v1 only, 2 default, 4 dma1
C = hip()
C.conv_force_impl(IMPL)
x = torch.randn(B, H, H, Ci, device="cuda:0").bfloat16()
w = (torch.randn(K, KH, KH, Ci, device="cuda:0") * 0.05).bfloat16()
for _ in range(5):
    C.conv_fwd(x, w, H, H, 1, 1, KH // 2, KH // 2)
torch.cuda.synchronize()
