"""Diagnostic: FWD conv timed against the same product run by the DGRAD kernel on
transposed + flipped weights (W'[ci][co][2-kh][2-kw] = W[co][ci][kh][kw]); the two differ
only in weight staging layout and epilogue.  Also checks the two outputs agree."""
import sys
import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "federated-learning-for-privacy-preserving-image-classification_amd"))
import torch
from fedhip import ops
from conv_bench import timeit, LAYERS


def main():
    dev = torch.device("cuda")
    B, C = 32, 32
    for cin, cout, hw in LAYERS[1:]:
        x = torch.randn(C, B, cin, hw, hw, device=dev)
        w = torch.randn(C, cout, cin, 3, 3, device=dev) * 0.1
        wt = w.transpose(1, 2).flip(-1, -2).contiguous()
        y = torch.empty(C, B, cout, hw, hw, device=dev)
        y2 = torch.empty_like(y)
        fl = 2.0 * C * B * hw * hw * cout * cin * 9
        t1 = timeit(lambda: ops.conv2d_fwd(x, w, None, y, C, B, cin, hw, hw, cout, 3, 1, 1))
        t2 = timeit(lambda: ops.conv2d_dgrad(x, wt, y2, C, B, cout, hw, hw, cin, 3, 1, 1))
        torch.cuda.synchronize()
        err = (y - y2).abs().max().item()
        print(f"{cin:3d}->{cout:3d} {hw:2d}x{hw:<2d} fwd {t1*1e3:7.1f}us {fl/t1/1e9:6.1f}TF  "
              f"fwd-as-dgrad {t2*1e3:7.1f}us {fl/t2/1e9:6.1f}TF  max|diff| {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
