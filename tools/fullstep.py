"""Full-width training steps of one packed lane (every client at every step: equal shards), for
a kernel trace of the marginal cost of a client-step.

usage (GPU box):
  python tools/fullstep.py [model] [clients] [steps]              # plain run: ms per step
  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/fullstep.py ...
  python tools/fullstep.py --breakdown DIR                         # per-step kernel table
model: cifar10_cnn (default) | simple_cnn | federated_resnet; the steps are graph-replayed
(program launch mode), as the bench's lanes issue them."""
import collections
import csv
import glob
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "federated-learning-for-privacy-preserving-image-classification_amd"))


def breakdown(d, top=40):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"].split("(")[0].replace("void ", "")
    opt = [i for i, r in enumerate(rows) if any(k in name(r) for k in ("sgd", "adam", "opt_slabs"))]
    sub = rows[opt[4] + 1: opt[-1] + 1]  # whole steps after the first five
    n = len(opt) - 5
    t0, t1 = int(sub[0]["Start_Timestamp"]), int(sub[-1]["End_Timestamp"])
    dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    busy = sum(dur(r) for r in sub)
    print(f"steps {n}  {(t1 - t0) / 1e3 / n:.1f} us/step wall  {busy / 1e3 / n:.1f} us/step "
          f"kernel-busy  {len(sub) / n:.1f} launches/step")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in sub:
        k = name(r)[:110]
        agg[k][0] += 1
        agg[k][1] += dur(r)
    for k, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t / 1e3 / n:8.1f} us/step {100 * t / busy:5.1f}% {c / n:5.1f}x {t / c / 1e3:7.1f} us  {k}")


def run(model_name="cifar10_cnn", clients=32, steps=12, u8=False, fill=None, dpsgd=False):
    import torch
    from fedhip import ops
    from fedhip.engine import DPSGDConfig, PackedTrainer
    from src.shared import models_pytorch as hm
    dev = torch.device("cuda")
    shape = (1, 28, 28) if model_name == "simple_cnn" else (3, 32, 32)
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(model_name).to(dev)
    eng = PackedTrainer(model, capacity=clients, batch=32, device=dev,
                        dpsgd=DPSGDConfig(max_grad_norm=1.0, noise_multiplier=1.0) if dpsgd else None)
    eng.launch_mode = "program"
    if fill:
        ops.set_fill_fraction(fill)
    if u8:  # raw uint8 images with the MNIST / CIFAR transform on the chip, as the bench
        eng.transform = ops.DataTransform.mnist() if model_name == "simple_cnn" else \
            ops.DataTransform.cifar10()
    for k in range(clients):
        eng.load_module_state(k, model)
    per = 32 * steps
    g = torch.Generator().manual_seed(1)
    if u8:
        data = torch.randint(0, 256, (clients * per, *shape[1:], shape[0]) if shape[0] == 3
                             else (clients * per, *shape[1:]), generator=g,
                             dtype=torch.uint8).to(dev)
    else:
        data = torch.randn(clients * per, *shape, generator=g).to(dev)
    labels = torch.randint(0, 10, (clients * per,), generator=g).to(dev)
    offs = [k * per for k in range(clients)]
    gen = torch.Generator().manual_seed(2)
    for r in range(3):
        plan = eng.make_plan([per] * clients, 1, generator=gen)
        torch.cuda.synchronize()
        t = time.perf_counter()
        eng.run_round(data, labels, offs, plan, lr=0.01, seed=r)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) * 1e3
        print(f"round {r}: {steps} full-width steps of {clients} clients, {ms / steps:.3f} ms/step")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--breakdown":
        breakdown(sys.argv[2])
    else:  # [--u8] [--dpsgd] [--lib PATH] [--fill F] model clients steps
        a = sys.argv[1:]
        u8 = "--u8" in a
        dp = "--dpsgd" in a
        a = [x for x in a if x not in ("--u8", "--dpsgd")]
        fill = None
        if "--lib" in a:
            i = a.index("--lib")
            from fedhip import _lib
            _lib.load.__defaults__ = (a[i + 1],)
            del a[i:i + 2]
        if "--separate" in a:  # each layer's WGRAD and DGRAD as two launches
            from fedhip import ops as _ops
            _ops.set_conv_pairing(False)
            a.remove("--separate")
        if "--fill" in a:
            i = a.index("--fill")
            fill = float(a[i + 1])
            del a[i:i + 2]
        run(a[0] if a else "cifar10_cnn", int(a[1]) if len(a) > 1 else 32,
            int(a[2]) if len(a) > 2 else 12, u8=u8, fill=fill, dpsgd=dp)
