"""Accuracy diagnostic: one client, T packed SGD steps on GPU vs the fp32 CPU oracle and
its fp64 twin (HIP ReLU/pool decisions replayed); per-parameter errors vs fp64.
usage: python tools/diag_acc.py <model> <num_blocks e.g. 2,2,2> <steps> [batch]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
import conftest  # noqa: F401,E402
import torch  # noqa: E402
from fedhip.engine import PackedTrainer  # noqa: E402
from oracle import train_ref  # noqa: E402
from src.shared import models_pytorch as hm  # noqa: E402
from test_train_gpu import pool_snapshot, rsliced, sliced, twin  # noqa: E402

name = sys.argv[1]
kw = {"num_blocks": [int(v) for v in sys.argv[2].split(",")]} if name == "federated_resnet" else {}
T = int(sys.argv[3])
B = int(sys.argv[4]) if len(sys.argv) > 4 else 32
DEV = torch.device("cuda")
shape = (1, 28, 28) if name == "simple_cnn" else (3, 32, 32)
ref, ref64 = twin(name, 3, **kw)
init = {k: p.detach().clone() for k, p in ref.named_parameters()}
torch.manual_seed(3)
model = hm.ModelFactory.create_model(name, **kw).to(DEV)
eng = PackedTrainer(model, capacity=1, batch=32, device=DEV)
eng.load_module_state(0, model)
eng.begin_round("sgd", 0.01)
o32, o64 = train_ref.make_optimizer(ref, "sgd", 0.01), train_ref.make_optimizer(ref64, "sgd", 0.01)
g = torch.Generator().manual_seed(4)
for t in range(T):
    x, y = torch.randn(B, *shape, generator=g), torch.randint(0, 10, (B,), generator=g)
    eng.net.x[0, :B].copy_(x)
    eng.net.y[0, :B].copy_(y)
    eng.step(1, torch.tensor([B], dtype=torch.int32, device=DEV))
    snap = pool_snapshot(eng, 1)[0]
    l32, _, _, _ = train_ref.train_step(ref, o32, x, y)
    l64, _, _, _ = train_ref.train_step(ref64, o64, x.double(), y, pools=sliced(snap, B),
                                        relus=rsliced(snap, B))
    lg = eng.loss_out[0].item()
    print(f"step {t}: loss hip {lg:.9f} cpu32 {l32:.9f} fp64 {l64:.9f}  "
          f"|hip-64| {abs(lg-l64):.2e} |cpu-64| {abs(l32-l64):.2e}")
got = eng.weights_dict(0)
p64s = dict(ref64.named_parameters())
worst = []
for n, p32 in ref.named_parameters():
    p64 = p64s[n].detach().double()
    pg = got[n].cpu().double()
    upd = (p64 - init[n].double()).norm().item()
    eh, ec = (pg - p64).norm().item(), (p32.detach().double() - p64).norm().item()
    worst.append((eh / max(upd, 1e-30), n, eh, ec, upd))
for r, n, eh, ec, upd in sorted(worst, reverse=True)[:12]:
    print(f"{n:34s} e_hip {eh:.2e} e_cpu {ec:.2e} upd {upd:.2e}  hip/upd {r:.2e} cpu/upd {ec/max(upd,1e-30):.2e}")
