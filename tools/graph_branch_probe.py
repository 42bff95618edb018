"""Does a replayed HIP graph run captured fork/join branches concurrently?  Three GPU spins
(A on the capture stream, B on a forked stream, C on the capture stream after A): ~2 spins of
wall time = branches overlap, ~3 = serialised.  Also the same pattern issued eagerly."""
import torch

N = 2_000_000  # spin cycles


def run(mode):
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    def body():
        torch.cuda._sleep(N)
        s1.wait_stream(s0)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(N)
        torch.cuda._sleep(N)
        s0.wait_stream(s1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s0):
        if mode == "graph":
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s0):
                body()
            g.replay()
            torch.cuda.synchronize()
            e0.record(s0); g.replay(); e1.record(s0)
        else:
            body()
            torch.cuda.synchronize()
            e0.record(s0); body(); e1.record(s0)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


one = None
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(N); torch.cuda.synchronize()
    a.record(); torch.cuda._sleep(N); b.record()
torch.cuda.synchronize()
one = a.elapsed_time(b)
print(f"one spin {one:.3f} ms; eager fork/join {run('eager'):.3f} ms; graph replay {run('graph'):.3f} ms")
