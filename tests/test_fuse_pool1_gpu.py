"""SimpleCNN conv1 -> ReLU -> pool1 in one launch (fh_conv2d_c1_pool_fwd) and its weight
gradient straight from the pooled gradient (fh_conv2d_c1_pool_wgrad): the same fp32
operations as conv2d_fwd(relu) + maxpool2_fwd and maxpool2_bwd + conv2d_wgrad, so whole
rounds (graph replay, dropout, ragged batches, SGD and Adam) are bit-identical to the
three-launch path; the single ops on ragged client counts, dense and pitched pooled planes."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round(fuse, opt, sizes, rounds=2, fuse_bwd=None):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.25).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.net.fuse_pool1 = fuse
    eng.net.fuse_pool1_bwd = fuse if fuse_bwd is None else fuse_bwd
    for k in range(S):
        eng.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), 1, 28, 28, generator=g).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(S)]
    gen = torch.Generator().manual_seed(11)
    metrics = []
    for r in range(rounds):
        plan = eng.make_plan(sizes, 1, generator=gen)
        metrics.append(eng.run_round(data, labels, offs, plan, optimizer_type=opt, lr=1e-2,
                                     seed=r))
    torch.cuda.synchronize()
    return eng, metrics


@pytest.mark.parametrize("opt,fwd,bwd", [("sgd", True, False), ("adam", True, False),
                                         ("sgd", True, True), ("sgd", False, True)])
def test_fused_pool1_rounds_bit_identical(opt, fwd, bwd):
    """fwd: conv1+ReLU+pool1 in one launch (the backward then masks by the pooled output,
    maxpool2_bwd_ymask); bwd: conv1's weight gradient straight from pool1's gradient."""
    sizes = [130, 70, 33, 9]
    a, ma = _round(fwd, opt, sizes, fuse_bwd=bwd)
    b, mb = _round(False, opt, sizes, fuse_bwd=False)
    assert a.net._pool1_fused == fwd and not b.net._pool1_fused
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)


@pytest.mark.parametrize("nc,cout,plane", [(1, 32, 14), (3, 32, 16), (5, 64, 16)])
def test_c1_pool_ops_match_separate_launches(nc, cout, plane):
    B, H = 32, 28
    torch.manual_seed(nc + cout)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, 1, H, H, device=DEV)
    w = torch.randn(nc, cout, 1, 3, 3, device=DEV) * 0.5
    bias = torch.randn(nc, cout, device=DEV) * 0.1
    # separate: conv + relu, pool into the planes
    a1 = torch.zeros(nc, B, cout, H, H, device=DEV)
    ops.conv2d_fwd(x, w, bias, a1, nc, B, 1, H, H, cout, 3, 1, 1, relu=True, counts=cnt)
    p_ref = torch.zeros(nc, B, cout, plane, plane, device=DEV)
    i_ref = torch.zeros(nc, B, cout, H // 2, H // 2, dtype=torch.uint8, device=DEV)
    ops.maxpool2_fwd(a1, p_ref, i_ref, nc, B, cout, H, H, counts=cnt)
    p = torch.zeros_like(p_ref)
    i = torch.zeros_like(i_ref)
    ops.conv2d_c1_pool_fwd(x, w, bias, p, i, nc, B, H, H, cout, counts=cnt)
    torch.cuda.synchronize()
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(p[z, :n], p_ref[z, :n]) and torch.equal(i[z, :n], i_ref[z, :n])
    # backward: the pooled gradient through the pool and the ReLU, then the weight gradient
    dp = torch.randn(nc, B, cout, plane, plane, device=DEV)
    da1 = torch.zeros_like(a1)
    ops.maxpool2_bwd(dp, i_ref, da1, nc, B, cout, H, H, xin=a1, counts=cnt)
    dw1, db1 = torch.zeros_like(w), torch.zeros_like(bias)
    ops.conv2d_wgrad(x, da1, dw1, db1, nc, B, 1, H, H, cout, 3, 1, 1, counts=cnt)
    dw2, db2 = torch.zeros_like(w), torch.zeros_like(bias)
    ops.conv2d_c1_pool_wgrad(x, dp, i, p, dw2, db2, nc, B, H, H, cout, counts=cnt)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)


def _u8_round(fuse_input, opt, sizes, rounds=2, graphs=True):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.25).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.net.fuse_input = fuse_input
    eng.use_graphs = graphs
    eng.transform = ops.DataTransform.mnist()
    for k in range(S):
        eng.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randint(0, 256, (sum(sizes), 28, 28), generator=g, dtype=torch.uint8).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(S)]
    gen = torch.Generator().manual_seed(11)
    metrics = []
    for r in range(rounds):
        plan = eng.make_plan(sizes, 1, generator=gen)
        metrics.append(eng.run_round(data, labels, offs, plan, optimizer_type=opt, lr=1e-2,
                                     seed=r))
    torch.cuda.synchronize()
    return eng, metrics


@pytest.mark.parametrize("opt,graphs", [("sgd", True), ("adam", True), ("sgd", False)])
def test_gather_in_conv1_rounds_bit_identical(opt, graphs):
    """r04: the uint8 batch gather inside conv1's launch (fh_conv2d_c1_pool_fwd_u8) leaves the
    same x / labels as fh_gather_u8 and the same rounds (graph replay and eager)."""
    sizes = [130, 70, 33, 9]
    a, ma = _u8_round(True, opt, sizes, graphs=graphs)
    b, mb = _u8_round(False, opt, sizes, graphs=graphs)
    assert a.net._src is None and b.net._src is None
    assert torch.equal(a.net.x, b.net.x) and torch.equal(a.net.y, b.net.y)
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)
