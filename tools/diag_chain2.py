"""Layer-by-layer fwd/bwd accuracy vs fp64 for a given init/data seed (CIFAR10CNN)."""
import sys, torch, torch.nn.functional as F
sys.path[:0] = ["/root/repo", "/root/repo/federated-learning-for-privacy-preserving-image-classification_amd"]
from fedhip.engine import PackedTrainer
from fedhip import ops
from src.shared import models_pytorch as hm
from oracle import train_ref
DEV = torch.device("cuda")
iseed, dseed, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
torch.manual_seed(iseed)
model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.0)
sd0 = {k: v.clone() for k, v in model.state_dict().items()}
model = model.to(DEV)
g = torch.Generator().manual_seed(dseed)
x = torch.randn(n, 3, 32, 32, generator=g); y = torch.randint(0, 10, (n,), generator=g)
x, y = x[:32], y[:32]
eng = PackedTrainer(model, capacity=1, batch=32, device=DEV)
eng.load_module_state(0, model); eng.begin_round("sgd", 0.01)
eng.net.x[0].copy_(x); eng.net.y[0].copy_(y)
cnt = torch.tensor([32], dtype=torch.int32, device=DEV)
net = eng.net
net.forward(eng.params, eng.bufs, 1, cnt, True)
ops.ce_fwd_bwd(net.logits, net.y, net.dlogits, 1, 32, 10, counts=cnt)
net.backward(eng.params, eng.grads, 1, cnt)
torch.cuda.synchronize()
A = {k: v[0].double().cpu() for k, v in net.A.t.items() if torch.is_tensor(v)}
def run(ref, xx):
    acts = {}
    def hook(name):
        def f(m, i, o):
            o.retain_grad(); acts[name] = o
        return f
    for i in range(1, 7):
        getattr(ref, f"conv{i}").register_forward_hook(hook(f"c{i}"))
        getattr(ref, f"bn{i}").register_forward_hook(hook(f"b{i}"))
    ref.train(); out = ref(xx); F.cross_entropy(out, y).backward()
    return acts, out
def mk(dt):
    m = train_ref.make_model("cifar10_cnn", None, dropout_rate=0.0)
    m.load_state_dict(sd0); return m.to(dt)
r64 = mk(torch.float64); a64, o64 = run(r64, x.double())
r32 = mk(torch.float32); a32, o32 = run(r32, x)
def rel(a, b): return ((a.double() - b.double()).norm() / b.double().norm()).item()
print("logits gpu", rel(net.logits[0].cpu(), o64.detach()), "cpu", rel(o32.detach(), o64.detach()))
for i in range(1, 7):
    cv = f"conv{i}"
    rr64 = F.relu(a64[f"b{i}"]).detach(); rr32 = F.relu(a32[f"b{i}"]).detach()
    print(f"{cv}: c gpu {rel(A['c_'+cv], a64[f'c{i}'].detach()):.1e} cpu {rel(a32[f'c{i}'].detach(), a64[f'c{i}'].detach()):.1e}"
          f" | r gpu {rel(A['r_'+cv], rr64):.1e} cpu {rel(rr32, rr64):.1e}"
          f" | dc gpu {rel(A['dc_'+cv], a64[f'c{i}'].grad):.1e} cpu {rel(a32[f'c{i}'].grad, a64[f'c{i}'].grad):.1e}")
for i in range(1, 7):
    gb = eng.layout.view(eng.grads, f"bn{i}.bias")[0].double().cpu()
    print(f"bn{i}.bias grad gpu {rel(gb, r64.__getattr__(f'bn{i}').bias.grad):.1e} cpu {rel(r32.__getattr__(f'bn{i}').bias.grad, r64.__getattr__(f'bn{i}').bias.grad):.1e}")
c1 = a64["c1"].detach()
print("conv1 out mean/std per channel (first 4):", c1.mean((0,2,3))[:4].tolist(), c1.std((0,2,3))[:4].tolist())
