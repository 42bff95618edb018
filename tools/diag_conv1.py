"""Diagnostic: isolate the accuracy of CIFAR10CNN conv1 weight gradient on HIP."""
import sys, os, math, torch
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
dc = net.A.t["dc_conv1"][0].double().cpu()       # [32,32,32,32]
xs = net.x[0].double().cpu()
dw_gpu = eng.layout.view(eng.grads, "conv1.weight")[0].double().cpu().view(32, 3, 3, 3)
# fp64 wgrad from the GPU's own dc
xr = xs.clone().requires_grad_(True)
w0 = torch.zeros(32, 3, 3, 3, dtype=torch.float64, requires_grad=True)
out = torch.nn.functional.conv2d(xr, w0, None, 1, 1)
out.backward(dc)
dw64 = w0.grad
print("wgrad(gpu) vs fp64 wgrad on same dc: rel", ((dw_gpu - dw64).norm() / dw64.norm()).item())
# fp32 CPU wgrad on same dc
w1 = torch.zeros(32, 3, 3, 3, requires_grad=True)
out = torch.nn.functional.conv2d(xs.float(), w1, None, 1, 1); out.backward(dc.float())
print("wgrad(cpu32) vs fp64 on same dc: rel", ((w1.grad.double() - dw64).norm() / dw64.norm()).item())
print("|dw|", dw64.norm().item(), " sum|dc|*|x| scale", (dc.abs().sum() * xs.abs().mean()).item())
# compare dc against the oracle in fp64
ref = train_ref.make_model("cifar10_cnn", 0, dropout_rate=0.0).double()
ref.train()
xd = x.double().requires_grad_(False)
acts = {}
h = ref.conv1.register_forward_hook(lambda m, i, o: o.retain_grad() or acts.__setitem__("c1", o))
out = ref(xd); loss = torch.nn.functional.cross_entropy(out, y); loss.backward()
dc64 = acts["c1"].grad
print("dc(gpu) vs dc(fp64): rel", ((dc - dc64).norm() / dc64.norm()).item())
ref32 = train_ref.make_model("cifar10_cnn", 0, dropout_rate=0.0); ref32.train(); acts.clear()
ref32.conv1.register_forward_hook(lambda m, i, o: o.retain_grad() or acts.__setitem__("c1", o))
out = ref32(x); torch.nn.functional.cross_entropy(out, y).backward()
print("dc(cpu32) vs dc(fp64): rel", ((acts["c1"].grad.double() - dc64).norm() / dc64.norm()).item())
print("conv1.weight grad: gpu vs fp64 rel", ((dw_gpu - ref.conv1.weight.grad).norm()/ref.conv1.weight.grad.norm()).item(),
      " cpu32 vs fp64 rel", ((ref32.conv1.weight.grad.double() - ref.conv1.weight.grad).norm()/ref.conv1.weight.grad.norm()).item())
