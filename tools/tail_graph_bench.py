"""Few-client conv costs as they occur inside a replayed step graph: each op captured
20x in a HIP graph and replayed, per (clients, fill fraction).  Prints us per op."""
import os
import sys
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..",
                                "federated-learning-for-privacy-preserving-image-classification_amd"))
from fedhip import ops  # noqa: E402

LAYERS = [(3, 32, 32), (32, 32, 32), (32, 64, 16), (64, 64, 16), (64, 128, 8), (128, 128, 8)]
REP = 20


def graph_time(fn):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        fn()
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(REP):
                fn()
    torch.cuda.synchronize()
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(5):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / (5 * REP) * 1e3


def main():
    dev = torch.device("cuda")
    B = 32
    fills = [float(v) for v in os.environ.get("FH_FILLS", "1,0.25,0.06").split(",")]
    for C in [int(v) for v in os.environ.get("FH_BENCH_CLIENTS", "1,2,4").split(",")]:
        for cin, cout, hw in LAYERS:
            x = torch.randn(C, B, cin, hw, hw, device=dev)
            w = torch.randn(C, cout, cin, 3, 3, device=dev) * 0.1
            b = torch.randn(C, cout, device=dev)
            y = torch.empty(C, B, cout, hw, hw, device=dev)
            dy = torch.randn_like(y)
            dx = torch.empty_like(x)
            dw = torch.empty_like(w)
            db = torch.empty_like(b)
            row = f"C={C:2d} {cin:3d}->{cout:3d} {hw:2d}x{hw:<2d}"
            for f in fills:
                ops.set_fill_fraction(f)
                t1 = graph_time(lambda: ops.conv2d_fwd(x, w, b, y, C, B, cin, hw, hw, cout, 3, 1, 1))
                t2 = graph_time(lambda: ops.conv2d_dgrad(dy, w, dx, C, B, cin, hw, hw, cout, 3, 1, 1))
                t3 = graph_time(lambda: ops.conv2d_wgrad(x, dy, dw, db, C, B, cin, hw, hw, cout, 3, 1, 1))
                row += f" | f{f:g} {t1:5.1f} {t2:5.1f} {t3:5.1f}"
            print(row, flush=True)
    ops.set_fill_fraction(1.0)


if __name__ == "__main__":
    main()
