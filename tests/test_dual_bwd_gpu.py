"""A layer's WGRAD and DGRAD in one dual-role launch (fh_conv_pair, dconv_wgrad_dual_kernel,
r04): the held quadrant-wave WGRAD and the direct DGRAD run as two workgroup roles of one grid,
each on the same code as its own launch, so results are bit-identical to two launches.
Reference: the per-layer input / weight gradients of the autograd backward of
models_pytorch.py's CIFAR10CNN (:112-141) and FederatedResNet (:230-246)."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _layer(hw, mode, nc=3, B=32, ci=64, co=64, flush_only=False):
    g = torch.Generator().manual_seed(hw)
    x = torch.randn(nc, B * ci * hw * hw, generator=g).to(DEV)
    dy = torch.randn(nc, B * co * hw * hw, generator=g).to(DEV)
    w = (0.05 * torch.randn(nc, co * ci * 9, generator=g)).to(DEV)
    dw = torch.full((nc, co * ci * 9), 7.0, device=DEV)
    db = torch.full((nc, co), 7.0, device=DEV)
    dx = torch.full((nc, B * ci * hw * hw), 7.0, device=DEV)
    cnt = torch.tensor([B, B - 5, 9][:nc], dtype=torch.int32, device=DEV)
    ops.set_fill_fraction(0.001)  # one split per WGRAD tile: dW written by the kernel (held)
    try:
        h = ops.Program.record_begin()
        ops.conv_pair(mode)
        ops.conv2d_wgrad(x, dy, dw, db, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt)
        if not flush_only:
            ops.conv2d_dgrad(dy, w, dx, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt)
        ops.conv_pair(0)
        if flush_only:
            ops.conv2d_dgrad(dy, w, dx, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt)
        prog = ops.Program.record_end(h)
    finally:
        ops.set_fill_fraction(1.0)
    torch.cuda.synchronize()
    k = prog.kernels
    prog.release()
    return dw, db, dx, k


@pytest.mark.parametrize("hw", [32, 16, 8])
@pytest.mark.parametrize("mode", [1, 2])
def test_dual_launch_matches_two_launches(hw, mode):
    a = _layer(hw, mode)
    b = _layer(hw, 0)
    assert a[3] == 1 and b[3] == 2, (a[3], b[3])
    for u, v in zip(a[:3], b[:3]):
        assert torch.equal(u, v)


def test_held_wgrad_flushed_without_dgrad():
    """Armed, then no DGRAD before fh_conv_pair(0): the held WGRAD is issued by the flush."""
    a = _layer(16, 1, flush_only=True)
    b = _layer(16, 0)
    assert a[3] == 2
    for u, v in zip(a[:3], b[:3]):
        assert torch.equal(u, v)


def _round(model_name, kw, sizes, opt, mode, defer=True, rounds=2, shape=(3, 32, 32)):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(model_name, **kw).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.defer_wgrad_reduce = defer
    eng.net.dual_bwd = mode
    for k in range(S):
        eng.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), *shape, generator=g).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(S)]
    gen = torch.Generator().manual_seed(11)
    for r in range(rounds):
        plan = eng.make_plan(sizes, 1, generator=gen)
        eng.run_round(data, labels, offs, plan, optimizer_type=opt, lr=1e-3, seed=r)
    torch.cuda.synchronize()
    return eng


@pytest.mark.parametrize("model_name,kw,opt,defer", [
    ("cifar10_cnn", {"dropout_rate": 0.5}, "sgd", True),
    ("cifar10_cnn", {"dropout_rate": 0.5}, "adam", True),
    ("cifar10_cnn", {"dropout_rate": 0.5}, "sgd", False),
    ("federated_resnet", {"num_blocks": [1, 1, 1]}, "sgd", True),
    ("simple_cnn", {"dropout_rate": 0.25}, "adam", True),
])
def test_dual_rounds_bit_identical(model_name, kw, opt, defer):
    sizes = [100, 70, 40, 9]
    shape = (1, 28, 28) if model_name == "simple_cnn" else (3, 32, 32)
    b = _round(model_name, kw, sizes, opt, 0, defer, shape=shape)
    for mode in (1, 2):
        a = _round(model_name, kw, sizes, opt, mode, defer, shape=shape)
        for f in ("params", "grads", "state1", "state2", "bufs"):
            assert torch.equal(getattr(a, f), getattr(b, f)), (mode, f)


def test_dual_laned_program_rounds_bit_identical():
    """The default KT path: a LanedTrainer (3 lanes, step programs), dual launches on vs off."""
    from fedhip.lanes import LanedTrainer

    def run(mode):
        torch.manual_seed(0)
        model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.3).to(DEV)
        sizes, cut = [300, 120, 100, 64, 33, 9], [0, 1, 4, 6]
        lt = LanedTrainer(model, [-(-n // 32) for n in sizes], batch=32, device=DEV, cut=cut)
        for ln in lt.lanes:
            ln.net.dual_bwd = mode
        for k in range(len(sizes)):
            lt.load_module_state(k, model)
        g = torch.Generator().manual_seed(5)
        data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
        labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
        offs = [sum(sizes[:k]) for k in range(len(sizes))]
        gen = torch.Generator().manual_seed(11)
        for r in range(2):
            lt.run_round(data, labels, offs, lt.make_plan(sizes, 1, generator=gen),
                         optimizer_type="sgd", lr=1e-3, seed=r)
        torch.cuda.synchronize()
        return lt

    a, b = run(1), run(0)
    assert all(ln.launch_mode == "program" for ln in a.lanes)
    for f in ("params", "grads", "state1", "state2", "bufs"):
        assert torch.equal(getattr(a, f), getattr(b, f)), f


def test_reset_drops_held_wgrad():
    """fh_conv_pair(-1) (a step's error path) drops the held WGRAD unissued and disarms."""
    nc, B, c, hw = 2, 32, 64, 16
    x = torch.randn(nc, B * c * hw * hw, device=DEV)
    dy = torch.randn(nc, B * c * hw * hw, device=DEV)
    dw = torch.full((nc, c * c * 9), 7.0, device=DEV)
    db = torch.full((nc, c), 7.0, device=DEV)
    ops.set_fill_fraction(0.001)
    try:
        h = ops.Program.record_begin()
        ops.conv_pair(2)
        ops.conv2d_wgrad(x, dy, dw, db, nc, B, c, hw, hw, c, 3, 1, 1)
        ops.conv_pair_reset()
        ops.conv_pair(0)
        prog = ops.Program.record_end(h)
    finally:
        ops.set_fill_fraction(1.0)
    torch.cuda.synchronize()
    assert prog.kernels == 0
    prog.release()
    assert bool((dw == 7.0).all()) and bool((db == 7.0).all())
