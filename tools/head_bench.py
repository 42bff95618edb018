"""Classifier-head launch cost (fh_linear_head_ce) per client count, alone on the chip and
HIP-event timed: SimpleCNN fc2 128->10 and CIFAR10CNN fc3 256->10, dropout keep-mask in front.
usage (GPU box): python tools/head_bench.py [clients,...] [--lib path/libfedhip.so]
[--save out.npz]: the outputs of one launch per case, to compare two builds bit for bit"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "federated-learning-for-privacy-preserving-image-classification_amd"))
from fedhip import _lib, ops  # noqa: E402

if "--lib" in sys.argv:  # time another build (e.g. a phase-stop variant of the kernel)
    _lib.load.__defaults__ = (sys.argv[sys.argv.index("--lib") + 1],)
    del sys.argv[sys.argv.index("--lib"):sys.argv.index("--lib") + 2]
SAVE = None
if "--save" in sys.argv:
    SAVE = sys.argv[sys.argv.index("--save") + 1]
    del sys.argv[sys.argv.index("--save"):sys.argv.index("--save") + 2]


def timeit(fn, it=50):
    for _ in range(5):
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
    B, K = 32, 10
    clients = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "1,10,21,32").split(",")]
    out = {}
    for F in (128, 256):
        for C in clients:
            g = torch.Generator().manual_seed(C)
            x = torch.relu(torch.randn(C, B, F, generator=g)).to(dev)
            w = (torch.randn(C, K, F, generator=g) * 0.1).to(dev)
            b = torch.randn(C, K, generator=g).to(dev)
            y = torch.randint(0, K, (C, B), generator=g).to(dev)
            m = (torch.rand(C, B, F, generator=g) > 0.5).to(torch.uint8).to(dev)
            lg, dl = torch.zeros(C, B, K, device=dev), torch.zeros(C, B, K, device=dev)
            dw, db = torch.zeros(C, K, F, device=dev), torch.zeros(C, K, device=dev)
            dx = torch.zeros(C, B, F, device=dev)
            lo = torch.zeros(C, device=dev)
            al = torch.zeros(C, dtype=torch.float64, device=dev)
            ac, asn = (torch.zeros(C, dtype=torch.int64, device=dev) for _ in range(2))
            cnt = torch.full((C,), B, dtype=torch.int32, device=dev)

            def run():
                ops.linear_head_ce(x, w, b, y, lg, dl, dw, db, dx, C, B, F, K, loss_out=lo,
                                   acc_loss=al, acc_correct=ac, acc_seen=asn, mask=m, p_drop=0.5,
                                   relu_in=True, counts=cnt)
            print(f"F={F} clients={C}: {timeit(run):.1f} us per launch", flush=True)
            if SAVE:
                al.zero_()
                ac.zero_()
                asn.zero_()
                cnt[1::3] = 17  # ragged clients too
                run()
                torch.cuda.synchronize()
                for nm, t in (("lg", lg), ("dl", dl), ("dw", dw), ("db", db), ("dx", dx),
                              ("lo", lo), ("al", al), ("ac", ac), ("as", asn)):
                    out[f"{F}_{C}_{nm}"] = t.cpu().numpy()
    if SAVE:
        import numpy as np
        np.savez(SAVE, **out)


if __name__ == "__main__":
    main()
