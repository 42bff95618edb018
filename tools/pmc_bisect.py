"""Bisect the rocprofv3 --pmc segfault: libfedhip launches in isolation.
usage: python tools/pmc_bisect.py fedavg|conv|bn  (each ~2k dispatches, progress printed)"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."),
                os.path.join(HERE, "..", "federated-learning-for-privacy-preserving-image-classification_amd")]
import torch  # noqa: E402

from fedhip import ops  # noqa: E402

what = sys.argv[1]
dev = torch.device("cuda", 0)
if what == "fedavg":
    rows = torch.randn(8, 1 << 16, device=dev)
    w = torch.full((8,), 0.125, device=dev)
    out = torch.empty(1 << 16, device=dev)
    for i in range(2000):
        ops.fedavg_weighted_sum(rows, w, out)
        if i % 500 == 0:
            torch.cuda.synchronize()
            print(what, i, flush=True)
elif what == "conv":  # direct conv fwd + dgrad (split-K epilogue at 1 client)
    B, C, hw = 32, 32, 32
    x = torch.randn(1, B, C, hw, hw, device=dev)
    wt = torch.randn(1, C, C, 3, 3, device=dev) * 0.05
    b = torch.zeros(1, C, device=dev)
    y = torch.empty_like(x)
    for i in range(1000):
        ops.conv2d_fwd(x, wt, b, y, 1, B, C, hw, hw, C, 3, 1, 1)
        ops.conv2d_dgrad(y, wt, x, 1, B, C, hw, hw, C, 3, 1, 1)
        if i % 250 == 0:
            torch.cuda.synchronize()
            print(what, i, flush=True)
torch.cuda.synchronize()
print("done", flush=True)
