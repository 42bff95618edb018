"""SimpleCNN pool2's backward inside conv2's dual-role backward launch (fh_conv_pooled_dy, r05):
both roles of dconv_wgrad_dual_kernel route the output gradient from the pooled gradient, the
window argmax and the pooled ReLU output as they stage it (maxpool2_bwd_ymask's values), the
WGRAD role skips the plane rows past the 14x14 map (their gradient is exactly zero), and the
16x16 gradient tensor is never written.  Rounds are bit-identical to the path with the separate
maxpool2_bwd launch; a pair that cannot form the dual launch gets the gradient materialised by
the library first.  Reference: models_pytorch.py:88-90 (conv2 -> relu -> pool2), training.py:196
(loss.backward)."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round(pooled, opt, sizes, rounds=2, dual=2, defer=True):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.25).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.net.pooled_dy_bwd = pooled
    eng.net.dual_bwd = dual
    eng.net.defer_dgrad = defer
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
def test_pooled_dy_rounds_bit_identical(opt):
    """12 ragged clients (full, partial and one-client steps; split and unsplit WGRAD plans)
    against the separate maxpool2_bwd launch."""
    sizes = [130, 100, 96, 75, 70, 64, 64, 50, 40, 33, 32, 9]
    a, ma = _round(True, opt, sizes)
    b, mb = _round(False, opt, sizes)
    # the pooled route ran inside the dual launches: the 16x16 gradient was never written
    assert not a.net.A("da2_16", 64, 16, 16).any() and b.net.A("da2_16", 64, 16, 16).any()
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)


def test_pooled_dy_without_dual_launch_materialises():
    """dual_bwd = 0 (two launches): the armed pooled gradient is materialised by the library
    before the WGRAD reads it — the same rounds again."""
    sizes = [70, 33, 9]
    a, _ = _round(True, "sgd", sizes, dual=0)
    b, _ = _round(False, "sgd", sizes, dual=0)
    c, _ = _round(True, "sgd", sizes, dual=2)
    assert torch.equal(a.params, b.params) and torch.equal(a.params, c.params)


def test_pooled_dy_op_level():
    """One pair on random operands with the pooled gradient armed, outside a training step (the
    WGRAD's pixel splits need their own reduction launch, so the pair stays two launches): the
    library materialises dY exactly as maxpool2_bwd_ymask, and dW, db, dX equal the unarmed
    pair's bit for bit, for 1, 7 and 23 clients, ragged counts.  The dual-launch route is the
    training step's (test_pooled_dy_rounds_bit_identical)."""
    for nc in (1, 7, 23):
        torch.manual_seed(nc)
        B, cin, cout = 32, 32, 64
        cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                           dtype=torch.int32, device=DEV)
        x = torch.zeros(nc, B, cin, 16, 16, device=DEV)
        x[..., :14, :14] = torch.randn(nc, B, cin, 14, 14, device=DEV)
        w = torch.randn(nc, cout, cin, 3, 3, device=DEV) * 0.1
        dp = torch.randn(nc, B, cout, 7, 7, device=DEV)
        pi = torch.randint(0, 4, (nc, B, cout, 7, 7), dtype=torch.uint8, device=DEV)
        py = torch.randn(nc, B, cout, 7, 7, device=DEV)  # the pooled ReLU output's sign masks
        outs = []
        for pooled in (False, True):
            dy = torch.zeros(nc, B, cout, 16, 16, device=DEV)
            if not pooled:
                ops.maxpool2_bwd_ymask(dp, pi, py, dy, nc, B, cout, 14, 14, counts=cnt)
            dw = torch.zeros(nc, cout, cin, 3, 3, device=DEV)
            db = torch.zeros(nc, cout, device=DEV)
            dx = torch.zeros(nc, B, cin, 16, 16, device=DEV)
            duals0 = ops._pair_status()[1]
            ops.conv_pair(2)
            if pooled:
                ops.conv_pooled_dy(dp, pi, py)
            ops.conv2d_wgrad(x, dy, dw, db, nc, B, cin, 16, 16, cout, 3, 1, 1, counts=cnt)
            ops.conv2d_dgrad(dy, w, dx, nc, B, cin, 16, 16, cout, 3, 1, 1, counts=cnt)
            ops.conv_pair(0)
            torch.cuda.synchronize()
            outs.append((dw, db, dx, dy, ops._pair_status()[1] > duals0))
        (dw0, db0, dx0, _, _), (dw1, db1, dx1, dy1, dual) = outs
        assert torch.equal(dw0, dw1) and torch.equal(db0, db1), nc
        for z in range(nc):
            n = int(cnt[z])
            assert torch.equal(dx0[z, :n], dx1[z, :n]), (nc, z)
        # outside a training step's GradSlabs scope a WGRAD that splits over pixels has its own
        # reduction launch, so it is not held for the pair: the library filled dY first
        assert not dual and torch.equal(dy1, outs[0][3]), nc


@pytest.mark.parametrize("opt,sizes", [("sgd", [70, 33, 9]), ("adam", [40]),
                                       ("sgd", [130, 64, 64, 50, 9])])
def test_deferred_dgrad_reduction_bit_identical(opt, sizes):
    """r05 fh_conv_defer_dgrad: conv2's split DGRAD (narrow grids) leaves its partials and
    conv1's weight gradient sums them while staging dp1 — the same rounds as with the split-K
    epilogue launch, bit for bit."""
    d0 = ops.defer_status()
    a, ma = _round(True, opt, sizes, defer=True)
    d1 = ops.defer_status()
    b, mb = _round(True, opt, sizes, defer=False)
    d2 = ops.defer_status()
    # the deferral really happened: DGRADs were left unreduced and conv1's weight
    # gradient summed their partials; the defer=False round deferred nothing
    assert d1[0] > d0[0] and d1[1] > d0[1], (d0, d1)
    assert d2 == d1, (d1, d2)
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)
