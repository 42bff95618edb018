"""Linear-layer (classifier) launch costs per client count: fwd / dgrad / wgrad of
CIFAR10CNN's fc1-fc3 on packed clients (32 images each), HIP-event timed.
[--lib path/libfedhip.so] times another build."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "federated-learning-for-privacy-preserving-image-classification_amd"))
from fedhip import _lib, ops  # noqa: E402

if "--lib" in sys.argv:  # A/B: time another libfedhip.so (tools/build_base_lib.sh)
    _lib.load.__defaults__ = (sys.argv[sys.argv.index("--lib") + 1],)

LAYERS = [(2048, 512), (512, 256), (256, 10)]
if os.environ.get("FH_BENCH_LAYERS"):  # e.g. "3136x128,128x10" (SimpleCNN)
    LAYERS = [tuple(int(v) for v in t.split("x")) for t in os.environ["FH_BENCH_LAYERS"].split(",")]
FWD_ONLY = os.environ.get("FH_BENCH_FWD_ONLY") == "1"


def timeit(fn, it=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    dev = torch.device("cuda")
    if os.environ.get("FH_BENCH_FILL"):  # a lane's split-K fill fraction (fedhip/lanes.py)
        ops.set_fill_fraction(float(os.environ["FH_BENCH_FILL"]))
    B = 32
    for C in [int(v) for v in os.environ.get("FH_BENCH_CLIENTS", "32,23,8,1").split(",")]:
        tot = 0.0
        line = f"C={C:2d}"
        for fi, fo in LAYERS:
            x = torch.randn(C, B, fi, device=dev)
            w = torch.randn(C, fo, fi, device=dev) * 0.05
            b = torch.randn(C, fo, device=dev)
            y = torch.empty(C, B, fo, device=dev)
            dy = torch.randn_like(y)
            dx = torch.empty_like(x)
            dw, db = torch.empty_like(w), torch.empty_like(b)
            t1 = timeit(lambda: ops.linear_fwd(x, w, b, y, C, B, fi, fo, relu=True))
            if FWD_ONLY:  # kernel-trace sweeps of the forward (tools/lf_trace.py)
                t2 = t3 = 0.0
            else:
                t2 = timeit(lambda: ops.linear_dgrad(dy, w, dx, C, B, fi, fo))
                t3 = timeit(lambda: ops.linear_wgrad(x, dy, dw, db, C, B, fi, fo))
            tot += t1 + t2 + t3
            gbs = 4.0 * C * (B * fi + B * fo + fi * fo) / (t1 * 1e-6) / 1e9  # fwd algorithmic
            line += f" | {fi}->{fo} {t1:6.1f} {t2:6.1f} {t3:6.1f} (fwd {gbs:5.0f} GB/s)"
        print(line + f" | total {tot:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
