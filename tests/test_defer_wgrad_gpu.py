"""Split weight-gradient reductions finished by the optimizer step (r03, ops.GradSlabs).

fh_conv2d_wgrad_deferred leaves a split plan's per-split partial sums in a slab and
fh_sgd_step_slabs / fh_adam_step_slabs sum them (conv.hip splitk_sum's order) as the update's
first operation.  The contract is bit-identity with the reducing path: conv2d_wgrad (its own
reduction launch) followed by sgd_step / adam_step — per layer for every WGRAD path that
splits, and for whole training rounds (SGD, Adam, AdamW; graph replay and lanes included)."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _layer_case(n, batch, cin, h, cout, k, stride, pad, affine, bias, opt, seed=0):
    """One WGRAD layer inside packed gradient rows: reducing path vs deferred path."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    oh = (h + 2 * pad - k) // stride + 1
    x = torch.randn(n, batch, cin, h, h, generator=g).to(DEV)
    dy = torch.randn(n, batch, cout, oh, oh, generator=g).to(DEV)
    counts = torch.tensor([batch - (i % 3) * 5 for i in range(n)], dtype=torch.int32, device=DEV)
    aff = None
    if affine:
        aff = (torch.rand(n, cin, generator=g).to(DEV) + 0.5, torch.randn(n, cin, generator=g).to(DEV))
    nw = cout * cin * k * k
    off_w = 36  # rows with other parameters around the layer (float4-aligned offsets)
    off_b = off_w + nw + 8
    Ppad = ((off_b + cout + 100) + 63) // 64 * 64
    out = []
    for deferred in (False, True):
        params = torch.randn(n, Ppad, generator=torch.Generator().manual_seed(3)).to(DEV)
        grads = torch.randn(n, Ppad, generator=torch.Generator().manual_seed(4)).to(DEV)
        st1 = torch.randn(n, Ppad, generator=torch.Generator().manual_seed(5)).to(DEV).abs()
        st2 = torch.randn(n, Ppad, generator=torch.Generator().manual_seed(6)).to(DEV).abs()
        dw = grads[:, off_w:off_w + nw]
        db = grads[:, off_b:off_b + cout] if bias else None
        slabs = ops.GradSlabs(DEV)
        if deferred:
            with slabs.collect(grads):
                ops.conv2d_wgrad(x, dy, dw, db, n, batch, cin, h, h, cout, k, stride, pad,
                                 counts=counts, in_affine=aff)
            ranges = list(slabs.ranges)
        else:
            ops.conv2d_wgrad(x, dy, dw, db, n, batch, cin, h, h, cout, k, stride, pad,
                             counts=counts, in_affine=aff)
        if opt == "sgd":
            if deferred:
                ops.sgd_step_slabs(params, grads, st1, 0.01, 0.9, n, ranges, first_step=False)
            else:
                ops.sgd_step(params, grads, st1, 0.01, 0.9, first_step=False)
        else:
            if deferred:
                ops.adam_step_slabs(params, grads, st1, st2, 3, 1e-3, n, ranges,
                                    weight_decay=0.01, decoupled=True)
            else:
                ops.adam_step(params, grads, st1, st2, 3, 1e-3, weight_decay=0.01,
                              decoupled=True)
        torch.cuda.synchronize()
        out.append((params, grads, st1, st2, ranges if deferred else None))
    return out


@pytest.mark.parametrize("n,batch,cin,h,cout,k,stride,pad,affine,bias", [
    (1, 32, 32, 32, 32, 3, 1, 1, False, True),     # quadrant-wave WGRAD, many splits (G > 1)
    (3, 32, 32, 32, 32, 3, 1, 1, True, True),      # + BN affine on load
    (2, 32, 128, 8, 128, 3, 1, 1, False, True),    # 8x8 maps
    (5, 20, 64, 16, 64, 3, 1, 1, False, False),    # no bias (ResNet)
    (2, 32, 3, 32, 32, 3, 1, 1, False, True),      # RGB first layer (small-cin kernel)
    (3, 32, 1, 28, 32, 3, 1, 1, False, True),      # MNIST conv1 (single-channel MFMA kernel)
    (2, 32, 64, 32, 128, 3, 2, 1, False, False),   # stride-2 direct WGRAD
    (2, 32, 64, 32, 128, 1, 2, 0, False, False),   # 1x1/s2 shortcut (implicit GEMM)
    # r06: stride-2 direct WGRAD whose plan is ONE split (ResNet layer3.0.conv1 at 32 clients):
    # the kernel still writes the slab, and the optimizer must copy it (it used to be reported
    # as "written directly" and the layer's gradient was dropped — K5's full-plan test)
    (32, 32, 128, 16, 256, 3, 2, 1, False, False),
])
@pytest.mark.parametrize("opt", ["sgd", "adamw"])
def test_deferred_layer_bit_identical(n, batch, cin, h, cout, k, stride, pad, affine, bias, opt):
    (p0, g0, a0, b0, _), (p1, g1, a1, b1, ranges) = _layer_case(n, batch, cin, h, cout, k, stride,
                                                                pad, affine, bias, opt)
    assert torch.equal(g0, g1)  # the optimizer stored the summed gradient
    assert torch.equal(p0, p1) and torch.equal(a0, a1) and torch.equal(b0, b1)
    if n == 1 and cin == 32:
        assert ranges and ranges[0][3] >= 16  # the G > 1 range-split path was exercised
    if n == 32:
        assert ranges and all(r[3] == 1 for r in ranges), ranges  # the one-split slab


def test_slab_ranges_rejected_when_misaligned():
    params = torch.zeros(1, 64, device=DEV)
    with pytest.raises(ops.FedHipError, match="bad slab range"):
        ops.sgd_step_slabs(params, params.clone(), params.clone(), 0.1, 0.9, 1,
                           [(2, 8, params.data_ptr(), 2)])


def _round(model_name, kw, shape, sizes, opt, defer, graphs=True, rounds=2):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(model_name, **kw).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.defer_wgrad_reduce = defer
    eng.use_graphs = graphs
    for k in range(S):
        eng.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), *shape, generator=g).to(DEV)
    labels = torch.randint(0, kw.get("num_classes", 10), (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(S)]
    gen = torch.Generator().manual_seed(11)
    for r in range(rounds):
        plan = eng.make_plan(sizes, 1, generator=gen)
        eng.run_round(data, labels, offs, plan, optimizer_type=opt, lr=1e-3, seed=r)
    torch.cuda.synchronize()
    return eng


@pytest.mark.parametrize("model_name,kw,shape,opt", [
    ("cifar10_cnn", {"dropout_rate": 0.5}, (3, 32, 32), "sgd"),
    ("cifar10_cnn", {"dropout_rate": 0.5}, (3, 32, 32), "adam"),
    ("simple_cnn", {"dropout_rate": 0.5}, (1, 28, 28), "adamw"),
    ("federated_resnet", {"num_blocks": [1, 1, 1]}, (3, 32, 32), "sgd"),
])
def test_deferred_rounds_bit_identical(model_name, kw, shape, opt):
    sizes = [100, 70, 40, 9]
    a = _round(model_name, kw, shape, sizes, opt, defer=True)
    b = _round(model_name, kw, shape, sizes, opt, defer=False)
    assert a._slabs is not None and b._slabs is None
    for f in ("params", "grads", "state1", "state2", "bufs"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def _laned_round(defer, sizes, cut, opt="sgd"):
    from fedhip.lanes import LanedTrainer
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.3).to(DEV)
    steps = [-(-n // 32) for n in sizes]
    lt = LanedTrainer(model, steps, batch=32, device=DEV, cut=cut)
    for ln in lt.lanes:
        ln.defer_wgrad_reduce = defer
    for k in range(len(sizes)):
        lt.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    gen = torch.Generator().manual_seed(11)
    for r in range(2):
        lt.run_round(data, labels, offs, lt.make_plan(sizes, 1, generator=gen),
                     optimizer_type=opt, lr=1e-3, seed=r)
    torch.cuda.synchronize()
    return lt


def test_deferred_laned_program_rounds_bit_identical():
    """The default KT / K2 path: a LanedTrainer (3 lanes on their own streams, step programs,
    shared lane streams), deferral on vs off."""
    sizes, cut = [300, 120, 100, 64, 33, 9], [0, 1, 4, 6]
    a = _laned_round(True, sizes, cut)
    b = _laned_round(False, sizes, cut)
    assert all(ln.launch_mode == "program" for ln in a.lanes)
    assert all(ln._slabs is not None for ln in a.lanes)
    for f in ("params", "grads", "state1", "state2", "bufs"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_deferred_arena_growth_and_range_cap(monkeypatch):
    """A deeper ResNet ([2,2,2]) with a 1 KB first arena (it grows mid-step, superseded
    buffers kept alive for the captured steps) and a range cap of 6 (the layers past it fall
    back to their own reduction launches): still bit-identical to deferral off."""
    monkeypatch.setattr(ops.GradSlabs, "MIN_ARENA", 1 << 10)
    monkeypatch.setattr(ops, "MAX_GRAD_SLABS", 6)
    sizes = [70, 40, 9]
    a = _round("federated_resnet", {}, (3, 32, 32), sizes, "sgd", defer=True)
    b = _round("federated_resnet", {}, (3, 32, 32), sizes, "sgd", defer=False)
    assert a._slabs.retired, "the arena never grew"
    assert 0 < len(a._slabs.ranges) <= 6
    for f in ("params", "grads", "state1", "bufs"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f
