"""r06 in-launch split-K reduction (fh_set_split_tickets, dconv_kernels.h dconv_body): a split
direct 3x3 FWD / DGRAD stores each split's partial tile write-through, takes a ticket, and the
tile's last arriving workgroup sums the partials in split order and runs the unsplit epilogue —
no splitk_epilogue_kernel launch.  Off by default: measured slower than
the epilogue launches it removes (ops.SPLIT_TICKETS, profiles/r06_inlaunch/); kept as a tested
option.

Against the split-K epilogue launch (ops.SPLIT_TICKETS off) on the same plans: every stored
tensor (y, dX, pooled maps and argmax) bit for bit — the partial sums are added in the same
order; the BatchNorm statistics tiles (fp64) within 1e-12 of them — the last arriver takes them
from its tile image in LDS as an unsplit launch does, a different fp64 summation order.  The
launches really reduced in-launch (fh_split_tickets_status) and left every ticket at zero."""
import pytest
import torch

from fedhip import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _both(fn):
    """fn() with in-launch reductions, then with epilogue launches: (results_on, results_off)."""
    out, prev = [], ops.SPLIT_TICKETS[0]
    for on in (True, False):
        ops.SPLIT_TICKETS[0] = on
        try:
            n0 = ops.split_tickets_status()
            r = fn()
            torch.cuda.synchronize()
            n1 = ops.split_tickets_status()
        finally:
            ops.SPLIT_TICKETS[0] = prev
        assert (n1 > n0) == on, (on, n0, n1)  # on: reduced in-launch; off: never
        out.append(r)
    for tk in ops._TK_DEFAULT.values():  # every launch left its counters at zero
        assert int(tk.t.abs().sum()) == 0
    return out


def _data(C, B, cin, h, cout, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(C, B, cin, h, h, generator=g).to(DEV)
    w = (torch.randn(C, cout, cin, 3, 3, generator=g) / (3.0 * cin ** 0.5)).to(DEV)
    b = torch.randn(C, cout, generator=g).to(DEV)
    dy = torch.randn(C, B, cout, h, h, generator=g).to(DEV)
    counts = torch.tensor([B - (3 * i) % 7 for i in range(C)], dtype=torch.int32, device=DEV)
    return x, w, b, dy, counts


def _eq_valid(a, b, counts):
    for z in range(a.shape[0]):
        n = int(counts[z])
        assert torch.equal(a[z, :n], b[z, :n]), z


@pytest.mark.parametrize("C,cin,h,cout", [(1, 32, 32, 32), (1, 32, 16, 64), (2, 64, 16, 64),
                                          (1, 64, 8, 128), (1, 128, 8, 128), (2, 128, 8, 128)])
def test_fwd_dgrad_inlaunch_bitwise(C, cin, h, cout):
    B = 32
    x, w, b, dy, counts = _data(C, B, cin, h, cout, cin + h + C)
    tiles = ops.bnstats_tiles(B, h, h)

    def run():
        y = torch.zeros(C, B, cout, h, h, device=DEV)
        yr = torch.zeros_like(y)
        part = torch.zeros(C, cout, tiles, 2, dtype=torch.float64, device=DEV)
        ys = torch.zeros_like(y)
        dx = torch.zeros(C, B, cin, h, h, device=DEV)
        dxa = torch.ones_like(dx)
        ops.conv2d_fwd(x, w, b, y, C, B, cin, h, h, cout, 3, 1, 1, counts=counts)
        ops.conv2d_fwd(x, w, b, yr, C, B, cin, h, h, cout, 3, 1, 1, relu=True, counts=counts)
        ops.conv2d_fwd(x, w, b, ys, C, B, cin, h, h, cout, 3, 1, 1, counts=counts, bn_stats=part)
        ops.conv2d_dgrad(dy, w, dx, C, B, cin, h, h, cout, 3, 1, 1, counts=counts)
        ops.conv2d_dgrad(dy, w, dxa, C, B, cin, h, h, cout, 3, 1, 1, counts=counts,
                         accumulate=True)
        return y, yr, ys, part, dx, dxa

    on, off = _both(run)
    for i in (0, 1, 2, 4, 5):
        _eq_valid(on[i], off[i], counts)
    assert torch.allclose(on[3], off[3], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("pooled", [False, True])
def test_dgrad_bn_backward_stats_inlaunch(pooled):
    """The DGRAD epilogue with BN-backward statistics (CIFAR10CNN conv k+1 -> BN k), unpooled
    and routed through a 2x2 max-pool + dropout keep-mask, one client (a split plan)."""
    C, B, cin, h, cout = 1, 32, 64, 16, 64
    x, w, b, dy, counts = _data(C, B, cin, h, cout, 7 + pooled)
    g = torch.Generator().manual_seed(3)
    H = 2 * h if pooled else h
    bx = torch.randn(C, B, cin, H, H, generator=g).to(DEV)
    sc = (torch.rand(C, cin, generator=g) + 0.5).to(DEV)
    sh = torch.randn(C, cin, generator=g).to(DEV)
    mean = torch.randn(C, cin, generator=g).to(DEV)
    pidx = torch.randint(0, 4, (C, B, cin, h, h), generator=g, dtype=torch.uint8).to(DEV)
    pmask = torch.randint(0, 2, (C, B, cin, h, h), generator=g, dtype=torch.uint8).to(DEV)

    def run():
        dx = torch.zeros(C, B, cin, h, h, device=DEV)
        part = torch.zeros(C, cin, ops.bnstats_tiles(B, h, h), 2, dtype=torch.float64,
                           device=DEV)
        bb = (bx, sc, sh, mean, part) + ((pidx, pmask, 0.5) if pooled else ())
        ops.conv2d_dgrad(dy, w, dx, C, B, cin, h, h, cout, 3, 1, 1, counts=counts, bn_bwd=bb)
        return dx, part

    on, off = _both(run)
    _eq_valid(on[0], off[0], counts)
    assert torch.allclose(on[1], off[1], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("C,h,pool_hw", [(1, 16, 14), (2, 16, 14)])
def test_fwd_relu_pool_inlaunch(C, h, pool_hw):
    """SimpleCNN conv2 -> ReLU -> pool2 on zero-ringed 16x16 planes (fh_conv2d_fwd_relu_pool):
    the last arriver pools its tile image as an unsplit launch does."""
    B, cin, cout = 32, 32, 64
    x, w, b, dy, counts = _data(C, B, cin, h, cout, 11 + C)
    x[..., pool_hw:, :] = 0.0
    x[..., :, pool_hw:] = 0.0
    ph = pool_hw // 2

    def run():
        y = torch.zeros(C, B, cout, h, h, device=DEV)
        py = torch.zeros(C, B, cout, ph, ph, device=DEV)
        pi = torch.zeros(C, B, cout, ph, ph, dtype=torch.uint8, device=DEV)
        ops.conv2d_fwd_relu_pool(x, w, b, y, py, pi, C, B, cin, h, cout, pool_hw, counts=counts)
        return py, pi

    on, off = _both(run)
    _eq_valid(on[0], off[0], counts)
    _eq_valid(on[1], off[1], counts)


def test_dual_backward_inlaunch():
    """A held WGRAD + its split DGRAD as one dual-role launch (fh_conv_pair): the DGRAD role
    reduces in-launch; dW / dX equal the epilogue-launch path's."""
    C, B, cin, h, cout = 1, 32, 64, 8, 128
    x, w, b, dy, counts = _data(C, B, cin, h, cout, 5)

    def run():
        dw = torch.zeros(C, cout, cin, 3, 3, device=DEV)
        db = torch.zeros(C, cout, device=DEV)
        dx = torch.zeros(C, B, cin, h, h, device=DEV)
        ops.conv_pair(2)
        ops.conv2d_wgrad(x, dy, dw, db, C, B, cin, h, h, cout, 3, 1, 1, counts=counts)
        ops.conv2d_dgrad(dy, w, dx, C, B, cin, h, h, cout, 3, 1, 1, counts=counts)
        ops.conv_pair(0)
        return dw, db, dx

    on, off = _both(run)
    assert torch.equal(on[0], off[0]) and torch.equal(on[1], off[1])
    _eq_valid(on[2], off[2], counts)


def test_training_rounds_inlaunch_vs_epilogue():
    """Whole CIFAR10CNN rounds (one-client and ragged steps: split plans everywhere) with the
    in-launch reductions against the epilogue launches: the trained rows agree to fp32 rounding
    of the BN statistics order (the only arithmetic that differs), and graph replay of the
    in-launch steps reproduces their eager rows bit for bit."""
    from fedhip.engine import PackedTrainer
    from src.shared import models_pytorch as hm
    sizes = [100, 37, 9]
    rows, engs, prev = [], [], ops.SPLIT_TICKETS[0]
    for on, graphs in ((True, False), (True, True), (False, True)):
        ops.SPLIT_TICKETS[0] = on
        try:
            torch.manual_seed(0)
            model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.0).to(DEV)
            eng = PackedTrainer(model, capacity=len(sizes), batch=32, device=DEV)
            eng.use_graphs = graphs
            for k in range(len(sizes)):
                eng.load_module_state(k, model)
            g = torch.Generator().manual_seed(5)
            data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
            labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
            offs = [sum(sizes[:k]) for k in range(len(sizes))]
            plan = eng.make_plan(sizes, 1, generator=torch.Generator().manual_seed(11))
            eng.run_round(data, labels, offs, plan, "sgd", 1e-2, seed=0)
            torch.cuda.synchronize()
            rows.append(eng.params[:len(sizes)].clone())
            engs.append(eng)
        finally:
            ops.SPLIT_TICKETS[0] = prev
    assert torch.equal(rows[0], rows[1])  # eager == replayed, in-launch
    d = (rows[0] - rows[2]).abs().max().item()
    assert d <= 1e-4 * rows[2].abs().max().item(), d
    for eng in engs[:2]:  # the in-launch trainers left every ticket at zero
        assert int(eng.split_tickets.t.abs().sum()) == 0
    assert engs[2].split_tickets is None
