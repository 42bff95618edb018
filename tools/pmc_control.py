"""Control workloads for rocprofv3 --pmc runs.
usage: python tools/pmc_control.py [default|stream|stream_prio]
torch only (libfedhip is not loaded): 40k small dispatches on the default stream, on a
torch.cuda.Stream(), or on a torch.cuda.Stream(priority=-1); progress printed every 5k."""
import sys

import torch

mode = sys.argv[1] if len(sys.argv) > 1 else "default"
x = torch.randn(1 << 20, device="cuda")
y = torch.empty_like(x)
s = None
if mode == "stream":
    s = torch.cuda.Stream()
elif mode == "stream_prio":
    s = torch.cuda.Stream(priority=-1)
ctx = torch.cuda.stream(s) if s is not None else torch.cuda.stream(torch.cuda.current_stream())
with ctx:
    for i in range(40000):
        y.copy_(x) if i % 2 else x.add_(1.0)
        if i % 5000 == 0:
            torch.cuda.synchronize()
            print(mode, "dispatches", i, flush=True)
torch.cuda.synchronize()
print("done", flush=True)
