"""Per-layer accuracy of one ResNet training step: GPU activations / weight gradients vs
the fp64 twin (HIP ReLU decisions replayed) and vs the fp32 CPU oracle.
usage: python tools/diag_layers.py <num_blocks e.g. 1,1,1> [batch]"""
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

nb = [int(v) for v in sys.argv[1].split(",")]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
kw = {"num_blocks": nb}
DEV = torch.device("cuda")
ref, ref64 = twin("federated_resnet", 3, **kw)
torch.manual_seed(3)
model = hm.ModelFactory.create_model("federated_resnet", **kw).to(DEV)
eng = PackedTrainer(model, capacity=1, batch=32, device=DEV)
eng.load_module_state(0, model)
init0 = {n: p.detach().float().cpu().clone() for n, p in model.named_parameters()}
eng.begin_round("sgd", 0.01)
g = torch.Generator().manual_seed(4)
x, y = torch.randn(B, 3, 32, 32, generator=g), torch.randint(0, 10, (B,), generator=g)
eng.net.x[0, :B].copy_(x)
eng.net.y[0, :B].copy_(y)
eng.step(1, torch.tensor([B], dtype=torch.int32, device=DEV))
torch.cuda.synchronize()
snap = pool_snapshot(eng, 1)[0]

acts = {}


def hook(tag, store):
    def f(mod, inp, out):
        store[tag] = out.detach().double().clone()
    return f


def attach(m, store):
    hs = [m.conv1.register_forward_hook(hook("c_stem", store))]
    blocks = []
    for li, layer in enumerate((m.layer1, m.layer2, m.layer3), 1):
        for bi, blk in enumerate(layer):
            pf = f"layer{li}.{bi}"
            hs.append(blk.conv1.register_forward_hook(hook(f"{pf}.a", store)))
            hs.append(blk.conv2.register_forward_hook(hook(f"{pf}.b", store)))
            hs.append(blk.register_forward_hook(hook(f"{pf}.out", store)))
            if len(blk.shortcut):
                hs.append(blk.shortcut[0].register_forward_hook(hook(f"{pf}.sc", store)))
    hs.append(m.fc.register_forward_hook(hook("logits", store)))
    return hs


a32, a64 = {}, {}
attach(ref, a32)
attach(ref64, a64)
gr64 = {}


def ghook(tag):
    def f(mod, gin, gout):
        if tag.endswith(".dar") or tag.endswith(".dsc_in"):
            gr64[tag] = gin[0].detach().clone()
        else:
            gr64[tag] = gout[0].detach().clone()
    return f


for li, layer in enumerate((ref64.layer1, ref64.layer2, ref64.layer3), 1):
    for bi, blk in enumerate(layer):
        pf = f"layer{li}.{bi}"
        blk.conv2.register_full_backward_hook(ghook(f"{pf}.dar"))   # grad wrt conv2 input
        blk.conv2.register_full_backward_hook(ghook(f"{pf}.db"))    # grad wrt conv2 output
        blk.conv1.register_full_backward_hook(ghook(f"{pf}.da"))    # grad wrt conv1 output
o32, o64 = train_ref.make_optimizer(ref, "sgd", 0.01), train_ref.make_optimizer(ref64, "sgd", 0.01)
train_ref.train_step(ref, o32, x, y)
train_ref.train_step(ref64, o64, x.double(), y, pools=sliced(snap, B), relus=rsliced(snap, B))
A = eng.net.A.t
print("activation                 |gpu-64|/|64|   |cpu-64|/|64|")
for k, v64 in a64.items():
    gk = "logits" if k == "logits" else k
    if gk == "logits":
        gv = eng.net.logits[0, :B].double().cpu()
    elif gk in A:
        gv = A[gk][0, :B].double().cpu()
    else:
        continue
    n = v64.norm().item()
    print(f"{k:26s} {((gv - v64).norm().item() / n):.2e}       {((a32[k] - v64).norm().item() / n):.2e}")
print("activation grads           |gpu-64|/|64|   per-channel-mean part of the error")
for k, v64 in gr64.items():
    if k not in A:
        continue
    gv = A[k][0, :B].double().cpu()
    e = gv - v64
    cm = e.mean(dim=(0, 2, 3), keepdim=True)
    print(f"{k:26s} {(e.norm().item() / v64.norm().item()):.2e}       "
          f"{(cm.expand_as(e).norm().item() / max(e.norm().item(), 1e-300)):.3f}")
# layer3.0 bn1: recompute the backward's ReLU mask on the host and compare with ar > 0
for pf in [f"layer{li}.{bi}" for li, layer in enumerate((ref64.layer1, ref64.layer2, ref64.layer3), 1)
           for bi in range(len(layer))]:
    a_ = A[f"{pf}.a"][0, :B].cpu()
    ar_ = A[f"{pf}.ar"][0, :B].cpu()
    sm, si = A[f"{pf}.bn1.save"]
    gam = init0[f"{pf}.bn1.weight"]  # the values the step's forward/backward used
    bet = init0[f"{pf}.bn1.bias"]
    alpha = si[0].cpu() * gam
    bconst = bet - sm[0].cpu() * alpha
    v = a_ * alpha.view(1, -1, 1, 1) + bconst.view(1, -1, 1, 1)
    mism = ((v > 0) != (ar_ > 0))
    print(f"{pf}.bn1 mask: recomputed vs ar>0 mismatches {int(mism.sum())} of {mism.numel()}, "
          f"ar==0 {int((ar_ == 0).sum())}, exact-zero v {int((v == 0).sum())}, "
          f"|v|<1e-6: {int((v.abs() < 1e-6).sum())}")
    if int(mism.sum()):
        idx = mism.nonzero()[0].tolist()
        i0, c0, h0, w0 = idx
        xa, al, bc = a_[i0, c0, h0, w0], alpha[c0], bconst[c0]
        fma = (xa.double() * al.double() + bc.double()).float()
        print(f"   first mismatch at {idx}: x={xa.item()!r} alpha={al.item()!r} bconst={bc.item()!r} "
              f"gpu_ar={ar_[i0, c0, h0, w0].item()!r} host_muladd={v[i0, c0, h0, w0].item()!r} "
              f"fma={fma.item()!r} prod={(xa * al).item()!r}")
    if f"{pf}.dar" in gr64:
        dar_g = A[f"{pf}.dar"][0, :B].double().cpu()
        dar_64 = gr64[f"{pf}.dar"]
        m = (ar_ > 0).double()
        sg_g = (m * dar_g).sum(dim=(0, 2, 3))
        sg_6 = (m * dar_64).sum(dim=(0, 2, 3))
        db_gpu = eng.layout.view(eng.grads, f"{pf}.bn1.bias")[0].double().cpu()
        db_64 = dict(ref64.named_parameters())[f"{pf}.bn1.bias"].grad
        c = int((db_gpu - db_64).abs().argmax())
        print(f"   bn1.bias grad worst channel {c}: gpu {db_gpu[c].item():.9e} fp64 {db_64[c].item():.9e} "
              f"host-sum(gpu dar, gpu mask) {sg_g[c].item():.9e} host-sum(fp64 dar) {sg_6[c].item():.9e}")
        e = (dar_g - dar_64)[:, c]
        print(f"   dar error in that channel: max {e.abs().max().item():.3e} at "
              f"{(e.abs() == e.abs().max()).nonzero()[0].tolist()}, dar scale {dar_64[:, c].abs().max().item():.3e}")
    if f"{pf}.da" in gr64:
        e = (A[f"{pf}.da"][0, :B].double().cpu() - gr64[f"{pf}.da"])
        per_c = e.pow(2).sum(dim=(0, 2, 3)).sqrt()
        top = per_c.topk(3)
        print(f"   da error by channel: top {top.values.tolist()} at {top.indices.tolist()}, "
              f"median {per_c.median().item():.2e}")
print("weight gradient            |gpu-64|/|64|   |cpu-64|/|64|")
L = eng.layout
g64 = {n: p.grad.double() for n, p in ref64.named_parameters()}
g32 = {n: p.grad.double() for n, p in ref.named_parameters()}
for n in L.names:
    gg = L.view(eng.grads, n)[0].reshape(g64[n].shape).double().cpu()
    d = g64[n].norm().item()
    print(f"{n:34s} {((gg - g64[n]).norm().item() / d):.2e}  {((g32[n] - g64[n]).norm().item() / d):.2e}")
