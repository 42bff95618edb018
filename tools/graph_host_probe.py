"""Host-side cost of HIP graph replay on MI355X, and whether replays of one graph exec
serialise the host: per-replay host time (no sync) vs wall, single exec vs two
alternating execs, and three streams issued from one thread vs one thread each.
Work per kernel: a small add on a 4 MB tensor (~2-3 us of GPU time)."""
import threading
import time

import torch

dev = torch.device("cuda:0")
NK = 80


def make_graph(stream, x, n=NK):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        for _ in range(2):
            x.add_(1.0)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=stream):
            for _ in range(n):
                x.add_(1.0)
    torch.cuda.synchronize()
    return g


def timed(fn, R):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn(R)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return (t1 - t0) / R * 1e6, (t2 - t0) / R * 1e6


s = [torch.cuda.Stream() for _ in range(3)]
xs = [torch.zeros(1 << 20, device=dev) for _ in range(3)]
g1 = make_graph(s[0], xs[0])
g1b = make_graph(s[0], xs[0])
R = 60


def one(R):
    with torch.cuda.stream(s[0]):
        for _ in range(R):
            g1.replay()


def alt(R):
    with torch.cuda.stream(s[0]):
        for i in range(R):
            (g1 if i % 2 == 0 else g1b).replay()


for name, fn in (("single exec", one), ("two alternating execs", alt)):
    fn(3)
    h, w = timed(fn, R)
    print(f"{name}: host {h:8.1f} us/replay, wall {w:8.1f} us/replay ({NK} kernels)")

gs = [make_graph(s[i], xs[i]) for i in range(3)]


def three_one_thread(R):
    for _ in range(R):
        for i in range(3):
            with torch.cuda.stream(s[i]):
                gs[i].replay()


def three_threads(R):
    def worker(i):
        with torch.cuda.stream(s[i]):
            for _ in range(R):
                gs[i].replay()
    th = [threading.Thread(target=worker, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()


for name, fn in (("3 streams, 1 thread", three_one_thread), ("3 streams, 3 threads", three_threads)):
    fn(2)
    h, w = timed(fn, R)
    print(f"{name}: host {h:8.1f} us/round of 3 replays, wall {w:8.1f} us")

# eager launches of the same kernel
def eager(R):
    with torch.cuda.stream(s[0]):
        for _ in range(R * NK):
            xs[0].add_(1.0)


eager(1)
h, w = timed(eager, R)
print(f"eager: host {h / NK:6.2f} us/kernel, wall {w / NK:6.2f} us/kernel")
