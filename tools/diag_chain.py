"""Diagnostic: per-intermediate accuracy of the CIFAR10CNN backward chain vs fp64."""
import sys, torch, torch.nn.functional as F
sys.path[:0] = ["/root/repo", "/root/repo/federated-learning-for-privacy-preserving-image-classification_amd"]
from fedhip.engine import PackedTrainer
from fedhip import ops
from src.shared import models_pytorch as hm
from oracle import train_ref
DEV = torch.device("cuda")
torch.manual_seed(0)
model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.0).to(DEV)
g = torch.Generator().manual_seed(2)
x = torch.randn(32, 3, 32, 32, generator=g); y = torch.randint(0, 10, (32,), generator=g)
eng = PackedTrainer(model, capacity=1, batch=32, device=DEV)
eng.load_module_state(0, model); eng.begin_round("sgd", 0.01)
eng.net.x[0].copy_(x); eng.net.y[0].copy_(y)
cnt = torch.tensor([32], dtype=torch.int32, device=DEV)
net = eng.net
net.forward(eng.params, eng.bufs, 1, cnt, True)
ops.ce_fwd_bwd(net.logits, net.y, net.dlogits, 1, 32, 10, counts=cnt)
net.backward(eng.params, eng.grads, 1, cnt)
torch.cuda.synchronize()
A = {k: (v[0].double().cpu() if torch.is_tensor(v) else None) for k, v in net.A.t.items()}
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
    return acts
r64 = train_ref.make_model("cifar10_cnn", 0, dropout_rate=0.0).double()
a64 = run(r64, x.double())
r32 = train_ref.make_model("cifar10_cnn", 0, dropout_rate=0.0)
a32 = run(r32, x)
def rel(a, b): return ((a.double() - b.double()).norm() / b.double().norm()).item()
for i in range(6, 0, -1):
    cv = f"conv{i}"
    print(f"{cv}: fwd c gpu {rel(A['c_'+cv], a64[f'c{i}'].detach()):.2e} cpu {rel(a32[f'c{i}'].detach(), a64[f'c{i}'].detach()):.2e} | "
          f"d(bn out) gpu {rel(A['dr_'+cv], a64[f'b{i}'].grad):.2e}? | d(conv out) gpu {rel(A['dc_'+cv], a64[f'c{i}'].grad):.2e} cpu {rel(a32[f'c{i}'].grad, a64[f'c{i}'].grad):.2e}")
# the relu-masked grad wrt bn output: b_i.grad is grad wrt BN output (pre-relu)
print("---- local step checks (fp64 recompute from GPU inputs)")
W5 = eng.layout.view(eng.params, "conv5.weight")[0].double().cpu().view(128, 64, 3, 3)
dc5 = A["dc_conv5"]
dq4 = torch.nn.grad.conv2d_input((32, 64, 8, 8), W5, dc5, 1, 1)
print("conv5 dgrad: rel", rel(A["dq_conv4"], dq4))
r4 = A["r_conv4"]
r4v = r4.clone().requires_grad_(True)
pooled = F.max_pool2d(r4v, 2, 2)
pooled.backward(A["dq_conv4"])
print("pool4 bwd: rel", rel(A["dr_conv4"], r4v.grad))
# bn4 backward in fp64 from GPU dr_conv4, c_conv4, gamma
c4 = A["c_conv4"].clone().requires_grad_(True)
gam = eng.layout.view(eng.params, "bn4.weight")[0].double().cpu()
bet = eng.layout.view(eng.params, "bn4.bias")[0].double().cpu()
o = F.relu(F.batch_norm(c4, None, None, gam, bet, True, 0.1, 1e-5))
o.backward(A["dr_conv4"])
print("bn4 bwd: rel", rel(A["dc_conv4"], c4.grad))
print("r_conv4 zeros frac", (r4 == 0).double().mean().item())
# tie statistics in pool windows
win = r4.view(32, 64, 8, 2, 8, 2).permute(0, 1, 2, 4, 3, 5).reshape(32, 64, 8, 8, 4)
mx = win.max(-1).values
ties = ((win == mx.unsqueeze(-1)).sum(-1) > 1) & (mx > 0)
print("positive ties in pool4 windows:", int(ties.sum()))
print("---- argmax comparison")
r64b = train_ref.make_model("cifar10_cnn", 0, dropout_rate=0.0).double(); r64b.train()
store = {}
def hin(name):
    def f(m, i, o):
        i[0].retain_grad(); store[name] = i[0]
    return f
r64b.conv5.register_forward_hook(hin("q4"))
r64b.bn4.register_forward_hook(lambda m, i, o: store.__setitem__("b4", o))
out = r64b(x.double()); F.cross_entropy(out, y).backward()
print("dq_conv4 (grad wrt pool4 out) gpu vs fp64:", rel(A["dq_conv4"], store["q4"].grad))
rr = F.relu(store["b4"]).detach()
_, idx64 = F.max_pool2d(rr, 2, 2, return_indices=True)
gw = r4.view(32, 64, 8, 2, 8, 2).permute(0, 1, 2, 4, 3, 5).reshape(32, 64, 8, 8, 4).argmax(-1)
_, idxg = F.max_pool2d(r4, 2, 2, return_indices=True)
gpu_idx = net.A.t["i_conv4"][0].long().cpu()
# convert gpu window code (0..3) to flat index like torch
oh = torch.arange(8).view(1, 1, 8, 1); ow = torch.arange(8).view(1, 1, 1, 8)
flat = (2 * oh + gpu_idx // 2) * 16 + (2 * ow + gpu_idx % 2)
print("gpu idx vs torch-on-gpu-data mismatches:", int((flat != idxg).sum()))
print("gpu idx vs fp64-ref mismatches:", int((flat != idx64).sum()), "of", flat.numel())
mm = (flat != idx64)
print("r4 at mismatches (gpu vals):", r4.flatten(2).gather(2, flat.flatten(2))[mm.flatten(2)][:8])
