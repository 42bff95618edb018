"""r06: a split direct conv's reduction inside the BatchNorm call after it (fh_conv_bn_defer,
splitbn.h): one launch per (channel, client) instead of splitk_epilogue_kernel + bn_finalize /
maxpool2_bnfin / bn_bwd_apply.  Against the same calls unarmed (the two launches): every
stored tensor bit for bit — the convolution output, the BN affine, saved and running
statistics, the pooled output / argmax / keep-mask, dgamma / dbeta and dx — on split plans
(one or a few clients, ragged counts, with and without dropout); the launches really fused
(fh_conv_bn_defer_status); whole CIFAR10CNN and ResNet rounds bit-identical with the fusion
on and off, eager and replayed.
Reference: BatchNorm2d after Conv2d, src/shared/models_pytorch.py:133-150, 189-194."""
import pytest
import torch

from fedhip import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
B = 32


@pytest.fixture(autouse=True)
def _whole_chip():
    ops.set_fill_fraction(1.0)  # the unit tests' split plans assume the whole-chip planner
    yield


def _counts(nc, seed):
    g = torch.Generator().manual_seed(seed)
    c = [B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,), generator=g)]
    return torch.tensor(c, dtype=torch.int32, device=DEV)


def _both(fn):
    """fn(armed) for armed = True, False: (results_armed, results_plain); the armed run fused."""
    d0, t0 = ops.bn_defer_status()
    on = fn(True)
    torch.cuda.synchronize()
    d1, t1 = ops.bn_defer_status()
    off = fn(False)
    torch.cuda.synchronize()
    d2, t2 = ops.bn_defer_status()
    assert d1 > d0 and t1 - t0 == d1 - d0, (d0, t0, d1, t1)  # deferred and all taken
    assert (d2, t2) == (d1, t1)
    return on, off


def _eq(a, b, cnt=None):
    if cnt is None:
        assert torch.equal(a, b)
        return
    for z in range(a.shape[0]):
        k = int(cnt[z])
        assert torch.equal(a[z, :k], b[z, :k]), z


def _arm(armed):
    if armed:
        prev = ops.SPLIT_BN[0]
        ops.SPLIT_BN[0] = True  # off by default: measured no faster (ops.SPLIT_BN)
        try:
            ops.conv_bn_defer(8192)  # every shape here, whatever the default policy
        finally:
            ops.SPLIT_BN[0] = prev


@pytest.mark.parametrize("nc,ci,co,hw,pool,dm", [
    (1, 64, 64, 16, False, False), (1, 64, 64, 16, True, True), (1, 64, 128, 8, False, False),
    (1, 128, 128, 8, True, True), (2, 64, 128, 8, True, False), (3, 32, 64, 16, False, False)])
def test_fwd_reduction_in_finalize_bitwise(nc, ci, co, hw, pool, dm):
    torch.manual_seed(nc * 7 + ci + hw)
    cnt = _counts(nc, ci + hw)
    x = torch.randn(nc, B, ci, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) / (3.0 * ci ** 0.5)
    b = torch.randn(nc, co, device=DEV) * 0.1
    gamma = torch.rand(nc, co, device=DEV) + 0.5
    beta = torch.randn(nc, co, device=DEV) * 0.2
    in_sc = torch.rand(nc, ci, device=DEV) + 0.5
    in_sh = torch.randn(nc, ci, device=DEV) * 0.1

    def run(armed):
        y = torch.full((nc, B, co, hw, hw), 7.0, device=DEV)
        part = torch.zeros(nc, co, ops.bnstats_tiles(B, hw, hw), 2, dtype=torch.float64,
                           device=DEV)
        rm, rv = torch.zeros(nc, co, device=DEV) + 0.3, torch.ones(nc, co, device=DEV)
        sm, si, sc, sh = (torch.zeros(nc, co, device=DEV) for _ in range(4))
        _arm(armed)
        ops.conv2d_fwd(x, w, b, y, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt,
                       in_affine=(in_sc, in_sh), bn_stats=part)
        out = [y, rm, rv, sm, si, sc, sh]
        if pool:
            h2 = hw // 2
            q = torch.zeros(nc, B, co, h2, h2, device=DEV)
            idx = torch.zeros(nc, B, co, h2, h2, dtype=torch.uint8, device=DEV)
            msk = torch.zeros_like(idx) if dm else None
            ops.maxpool2_fwd_bnfinalize(part, gamma, beta, rm, rv, sm, si, sc, sh, y, q, idx, nc,
                                        B, co, hw, hw, mask=msk, drop_mode=1 if dm else 0,
                                        p_drop=0.3, seed=17, counts=cnt)
            out += [q, idx] + ([msk] if dm else [])
        else:
            ops.bn_finalize_tiles(part, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, co, hw * hw,
                                  counts=cnt)
        return out

    on, off = _both(run)
    _eq(on[0], off[0], cnt)
    for a, c in zip(on[1:7], off[1:7]):
        _eq(a, c)
    for a, c in zip(on[7:], off[7:]):
        _eq(a, c, cnt)


@pytest.mark.parametrize("nc,ci,co,hw,pooled,dm", [
    (1, 64, 64, 16, False, False), (1, 64, 128, 8, False, False), (1, 32, 64, 16, True, True),
    (1, 64, 128, 8, True, True), (2, 32, 64, 16, True, False), (3, 64, 128, 8, False, False)])
def test_dgrad_reduction_in_bn_backward_bitwise(nc, ci, co, hw, pooled, dm):
    """CIFAR10CNN conv k+1's DGRAD -> BN k's backward: unpooled (bn_bwd_tiles) and through the
    2x2 max-pool + dropout (bn_bwd_pool_tiles)."""
    torch.manual_seed(nc * 11 + ci + hw + pooled)
    cnt = _counts(nc, co + hw)
    H = 2 * hw if pooled else hw
    p = 0.3 if dm else 0.0
    bx = torch.randn(nc, B, ci, H, H, device=DEV) * 1.3 + 0.1
    gamma = torch.rand(nc, ci, device=DEV) + 0.5
    gamma[:, ::5] *= -1
    beta = torch.randn(nc, ci, device=DEV) * 0.3
    rm, rv = torch.zeros(nc, ci, device=DEV), torch.ones(nc, ci, device=DEV)
    sm, si = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    sc, sh = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    ops.bn_fwd_stats(bx, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, ci, H * H, counts=cnt)
    idx = msk = None
    if pooled:
        q = torch.zeros(nc, B, ci, hw, hw, device=DEV)
        idx = torch.zeros(nc, B, ci, hw, hw, dtype=torch.uint8, device=DEV)
        msk = torch.zeros_like(idx) if dm else None
        ops.maxpool2_fwd(bx, q, idx, nc, B, ci, H, H, mask=msk, drop_mode=1 if dm else 0,
                         p_drop=p, seed=3, counts=cnt, in_affine=(sc, sh))
    dy = torch.randn(nc, B, co, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) * 0.1

    def run(armed):
        dq = torch.zeros(nc, B, ci, hw, hw, device=DEV)
        part = torch.zeros(nc, ci, ops.bnstats_tiles(B, hw, hw), 2, dtype=torch.float64,
                           device=DEV)
        bb = (bx, sc, sh, sm, part) + ((idx, msk, p) if pooled else ())
        _arm(armed)
        ops.conv2d_dgrad(dy, w, dq, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt, bn_bwd=bb)
        dx = torch.full_like(bx, 5.0)
        dg, db = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
        if pooled:
            ops.bn_bwd_pool_tiles(part, dq, idx, bx, gamma, beta, sm, si, dx, dg, db, nc, B, ci,
                                  H, H, pmask=msk, p_drop=p, counts=cnt)
        else:
            ops.bn_bwd_tiles(part, dq, bx, gamma, sm, si, dx, dg, db, nc, B, ci, H * H,
                             counts=cnt)
        return dx, dg, db

    on, off = _both(run)
    _eq(on[0], off[0], cnt)
    _eq(on[1], off[1])
    _eq(on[2], off[2])


def test_unconsumed_reduction_materialises():
    """An armed split FWD whose output is read by something other than its BN call: the
    skipped epilogue runs first (the reader sees the reduced output)."""
    nc, ci, co, hw = 1, 64, 64, 16
    torch.manual_seed(3)
    x = torch.randn(nc, B, ci, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) / 24.0
    ys, parts = [], []
    for armed in (True, False):
        y = torch.zeros(nc, B, co, hw, hw, device=DEV)
        part = torch.zeros(nc, co, ops.bnstats_tiles(B, hw, hw), 2, dtype=torch.float64,
                           device=DEV)
        d0, _ = ops.bn_defer_status()
        _arm(armed)
        ops.conv2d_fwd(x, w, None, y, nc, B, ci, hw, hw, co, 3, 1, 1, bn_stats=part)
        d1, _ = ops.bn_defer_status()
        assert (d1 > d0) == armed
        y2 = torch.zeros_like(y)  # a conv reading y: the pending reduction launches first
        ops.conv2d_fwd(y, w, None, y2, nc, B, co, hw, hw, co, 3, 1, 1)
        torch.cuda.synchronize()
        ys.append((y, y2))
        parts.append(part)
    assert torch.equal(ys[0][0], ys[1][0]) and torch.equal(ys[0][1], ys[1][1])
    assert torch.equal(parts[0], parts[1])


def _rounds(model_name, sizes, split_bn, graphs, **kw):
    from fedhip.engine import PackedTrainer
    from src.shared import models_pytorch as hm
    prev, prev_max = ops.SPLIT_BN[0], ops.SPLIT_BN_MAX[0]
    ops.SPLIT_BN[0] = split_bn
    ops.SPLIT_BN_MAX[0] = 8192  # the 16x16 and 32x32 maps too
    try:
        torch.manual_seed(0)
        model = hm.ModelFactory.create_model(model_name, **kw).to(DEV)
        eng = PackedTrainer(model, capacity=len(sizes), batch=B, device=DEV)
        eng.use_graphs = graphs
        for k in range(len(sizes)):
            eng.load_module_state(k, model)
        g = torch.Generator().manual_seed(5)
        data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
        labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
        offs = [sum(sizes[:k]) for k in range(len(sizes))]
        gen = torch.Generator().manual_seed(11)
        for r in range(2):
            plan = eng.make_plan(sizes, 1, generator=gen)
            eng.run_round(data, labels, offs, plan, "sgd", 1e-2, seed=r)
        torch.cuda.synchronize()
        return eng.params[:len(sizes)].clone(), eng.bufs[:len(sizes)].clone()
    finally:
        ops.SPLIT_BN[0], ops.SPLIT_BN_MAX[0] = prev, prev_max


@pytest.mark.parametrize("model_name,kw", [("cifar10_cnn", {"dropout_rate": 0.3}),
                                           ("federated_resnet", {"num_blocks": [1, 1, 1]})])
def test_rounds_bit_identical_with_split_bn(model_name, kw):
    """One-client and ragged steps (split plans): the trained rows and BN buffers with the
    fused launches equal the two-launch path's bit for bit, eager and replayed."""
    sizes = [100, 37, 9]
    d0, t0 = ops.bn_defer_status()
    p_on, b_on = _rounds(model_name, sizes, True, False, **kw)
    d1, t1 = ops.bn_defer_status()
    assert d1 > d0 and t1 - t0 == d1 - d0
    p_g, b_g = _rounds(model_name, sizes, True, True, **kw)
    p_off, b_off = _rounds(model_name, sizes, False, True, **kw)
    assert torch.equal(p_on, p_off) and torch.equal(b_on, b_off)
    assert torch.equal(p_g, p_off) and torch.equal(b_g, b_off)
