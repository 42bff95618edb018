"""SimpleCNN conv2 -> ReLU -> pool2 in one launch (fh_conv2d_fwd_relu_pool, r04): the pool is
taken in the direct conv's epilogue from the tile image in LDS when the launch is unsplit, and
in the split reduction otherwise; the pool's backward masks by p2 (maxpool2_bwd_ymask).  The
same fp32 values and first-max argmax as conv2d_fwd(relu) + maxpool2_fwd, so whole rounds are
bit-identical to the two-launch path.  Reference: models_pytorch.py:88-89 (conv2 -> relu ->
pool)."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("nc", [1, 3, 9, 20])
def test_conv_relu_pool_op_matches_separate_launches(nc):
    """nc = 1 / 3: the planner splits over input channels (pool in the split reduction);
    9 / 20: unsplit BM = 32 / 64 launches (pool in the conv's epilogue)."""
    B, H, cin, cout = 32, 16, 32, 64
    torch.manual_seed(nc)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    x = torch.zeros(nc, B, cin, H, H, device=DEV)
    x[..., :14, :14] = torch.randn(nc, B, cin, 14, 14, device=DEV)  # the 14x14 map, zero ring
    w = torch.randn(nc, cout, cin, 3, 3, device=DEV) * 0.1
    bias = torch.randn(nc, cout, device=DEV) * 0.1
    a2 = torch.zeros(nc, B, cout, H, H, device=DEV)
    ops.conv2d_fwd(x, w, bias, a2, nc, B, cin, H, H, cout, 3, 1, 1, relu=True, counts=cnt)
    p_ref = torch.zeros(nc, B, cout, 7, 7, device=DEV)
    i_ref = torch.zeros(nc, B, cout, 7, 7, dtype=torch.uint8, device=DEV)
    ops.maxpool2_fwd(a2, p_ref, i_ref, nc, B, cout, 14, 14, counts=cnt)
    y = torch.zeros_like(a2)
    p = torch.full_like(p_ref, -1.0)
    i = torch.full_like(i_ref, 9)
    ops.conv2d_fwd_relu_pool(x, w, bias, y, p, i, nc, B, cin, H, cout, 14, counts=cnt)
    torch.cuda.synchronize()
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(p[z, :n], p_ref[z, :n]), z
        assert torch.equal(i[z, :n], i_ref[z, :n]), z
        assert (p[z, n:] == -1.0).all() and (i[z, n:] == 9).all()  # past the count: untouched
    # the pool's backward masked by p2 equals the one masked by the full-resolution a2
    dp = torch.randn(nc, B, cout, 7, 7, device=DEV)
    da_x = torch.zeros_like(a2)
    ops.maxpool2_bwd(dp, i_ref, da_x, nc, B, cout, 14, 14, xin=a2, counts=cnt)
    da_y = torch.zeros_like(a2)
    ops.maxpool2_bwd_ymask(dp, i, p, da_y, nc, B, cout, 14, 14, counts=cnt)
    torch.cuda.synchronize()
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(da_x[z, :n], da_y[z, :n])


def _round(fuse, opt, sizes, rounds=2):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.25).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.net.fuse_pool2 = fuse
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


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_fused_pool2_rounds_bit_identical(opt):
    """12 ragged clients: the early steps run unsplit (pool in the epilogue), the tail steps
    with few clients split (pool in the reduction) — both against the two-launch path."""
    sizes = [130, 100, 96, 75, 70, 64, 64, 50, 40, 33, 32, 9]
    a, ma = _round(True, opt, sizes)
    b, mb = _round(False, opt, sizes)
    assert a.net._pool2_fused and not b.net._pool2_fused
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)
