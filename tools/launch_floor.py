"""Per-kernel floor on MI355X: tiny kernels back to back, eager vs HIP graph replay."""
import time
import torch

dev = torch.device("cuda:0")
x = torch.zeros(256, device=dev)


def body(n):
    for _ in range(n):
        x.add_(1.0)


for n in (1, 80):
    body(n)
torch.cuda.synchronize()
N = 2000
t = time.perf_counter()
body(N)
torch.cuda.synchronize()
print(f"eager: {(time.perf_counter() - t) / N * 1e6:.2f} us/kernel")

for n in (10, 80, 200):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        body(3)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            body(n)
    torch.cuda.synchronize()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    R = 50
    t = time.perf_counter()
    for _ in range(R):
        g.replay()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / R
    print(f"graph n={n}: {dt * 1e6:.1f} us/replay, {dt / n * 1e6:.2f} us/kernel")
