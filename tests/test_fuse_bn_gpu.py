"""BatchNorm apply + ReLU folded into its consumers (fh_bn_fwd_stats, fh_conv2d_fwd_bnrelu,
fh_conv2d_wgrad_bnrelu, fh_maxpool2_fwd_bnrelu) is bit-identical to the materialised path
(fh_bn_fwd_train's apply pass + plain conv / pool): the consumer evaluates the same fp32
operations on load.  Whole CIFAR10CNN rounds (graph replay, dropout, ragged batches) and
the single ops on ragged client counts."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round(fuse, opt, sizes, rounds=2, bn_epilogue=False, bn_bwd_epilogue=False,
           resnet=False):
    torch.manual_seed(0)
    if resnet:  # ResNet-8 (K3): stride-1 and stride-2 blocks, projection shortcuts
        model = hm.ModelFactory.create_model("federated_resnet", num_blocks=[1, 1, 1]).to(DEV)
    else:
        model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.3).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.net.fuse_bn = fuse
    eng.net.bn_epilogue = bn_epilogue
    eng.net.bn_bwd_epilogue = bn_bwd_epilogue
    for k in range(S):
        eng.load_module_state(k, model)
    eng.init_params = eng.params.clone()
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), 3, 32, 32, generator=g).to(DEV)
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
def test_fused_bn_rounds_bit_identical(opt):
    sizes = [130, 70, 33, 9]
    a, ma = _round(True, opt, sizes)
    b, mb = _round(False, opt, sizes)
    assert a.net._fused and not b.net._fused
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.bufs, b.bufs)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)


@pytest.mark.parametrize("nc,C,hw", [(1, 32, 32), (3, 64, 16), (5, 128, 8)])
def test_fused_ops_match_apply_pass(nc, C, hw):
    B = 32
    torch.manual_seed(nc + C)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, C, hw, hw, device=DEV) * 1.5 + 0.2
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    gamma[:, ::7] *= -1  # negative scales: the ReLU mask is not monotone in x
    beta = torch.randn(nc, C, device=DEV) * 0.3
    rm0, rv0 = torch.zeros(nc, C, device=DEV), torch.ones(nc, C, device=DEV)
    # materialised path
    rm1, rv1 = rm0.clone(), rv0.clone()
    sm1, si1 = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
    r = torch.zeros_like(x)
    ops.bn_fwd_train(x, r, gamma, beta, rm1, rv1, sm1, si1, nc, B, C, hw * hw, relu=True,
                     counts=cnt)
    # statistics + affine
    rm2, rv2 = rm0.clone(), rv0.clone()
    sm2, si2 = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
    sc, sh = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
    ops.bn_fwd_stats(x, gamma, beta, rm2, rv2, sm2, si2, sc, sh, nc, B, C, hw * hw, counts=cnt)
    for u, v in ((rm1, rm2), (rv1, rv2), (sm1, sm2), (si1, si2)):
        assert torch.equal(u, v)
    # conv forward on r vs on x with the affine
    co = 64
    w = torch.randn(nc, co, C, 3, 3, device=DEV) * 0.05
    bias = torch.randn(nc, co, device=DEV) * 0.1
    y1 = torch.zeros(nc, B, co, hw, hw, device=DEV)
    y2 = torch.zeros_like(y1)
    ops.conv2d_fwd(r, w, bias, y1, nc, B, C, hw, hw, co, 3, 1, 1, counts=cnt)
    ops.conv2d_fwd(x, w, bias, y2, nc, B, C, hw, hw, co, 3, 1, 1, counts=cnt, in_affine=(sc, sh))
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(y1[z, :k], y2[z, :k])
    # weight gradient with x as the staged input
    dy = torch.randn(nc, B, co, hw, hw, device=DEV)
    dw1 = torch.zeros(nc, co, C, 3, 3, device=DEV)
    db1 = torch.zeros(nc, co, device=DEV)
    dw2, db2 = torch.zeros_like(dw1), torch.zeros_like(db1)
    ops.conv2d_wgrad(r, dy, dw1, db1, nc, B, C, hw, hw, co, 3, 1, 1, counts=cnt)
    ops.conv2d_wgrad(x, dy, dw2, db2, nc, B, C, hw, hw, co, 3, 1, 1, counts=cnt,
                     in_affine=(sc, sh))
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    # max-pool (+ generated dropout mask) on r vs on x with the affine
    oh = hw // 2
    q1 = torch.zeros(nc, B, C, oh, oh, device=DEV)
    q2 = torch.zeros_like(q1)
    i1 = torch.zeros(nc, B, C, oh, oh, dtype=torch.uint8, device=DEV)
    i2 = torch.zeros_like(i1)
    m1, m2 = torch.zeros_like(i1), torch.zeros_like(i1)
    ops.maxpool2_fwd(r, q1, i1, nc, B, C, hw, hw, mask=m1, drop_mode=1, p_drop=0.3, seed=9,
                     counts=cnt)
    ops.maxpool2_fwd(x, q2, i2, nc, B, C, hw, hw, mask=m2, drop_mode=1, p_drop=0.3, seed=9,
                     counts=cnt, in_affine=(sc, sh))
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(q1[z, :k], q2[z, :k]) and torch.equal(i1[z, :k], i2[z, :k])
        assert torch.equal(m1[z, :k], m2[z, :k])


def _ulps(a, b):
    """Largest distance in units in the last place between two fp32 tensors."""
    ia = a.contiguous().view(torch.int32).to(torch.int64)
    ib = b.contiguous().view(torch.int32).to(torch.int64)
    ia = torch.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = torch.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return int((ia - ib).abs().max())


# client counts that take the unsplit epilogue (many clients) and the split-K epilogue
# kernel (one client: the planner splits the input channels), every map width, with and
# without a BN-on-load input, ragged counts
@pytest.mark.parametrize("nc,ci,co,hw,affine", [(1, 32, 32, 32, True), (1, 3, 32, 32, False),
                                                (1, 64, 128, 8, True), (3, 32, 64, 16, True),
                                                (32, 32, 32, 32, True), (32, 64, 64, 16, False),
                                                (24, 128, 128, 8, True), (9, 64, 128, 8, False)])
def test_epilogue_bn_stats_match_separate_pass(nc, ci, co, hw, affine):
    """fh_conv2d_fwd_bnstats + fh_bn_finalize_tiles vs fh_conv2d_fwd_bnrelu + fh_bn_fwd_stats:
    y bit-identical; the per-tile fp64 partials equal fp64 sums of the stored y; the BN
    outputs (save_mean/invstd, running stats, the consumer's affine) within 1 ulp (the two
    paths add the same fp64 terms in different orders)."""
    B = 32
    torch.manual_seed(nc * 7 + co)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, ci, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) * 0.1
    bias = torch.randn(nc, co, device=DEV) * 0.2 + 0.5
    aff = None
    if affine:
        aff = (torch.rand(nc, ci, device=DEV) + 0.5, torch.randn(nc, ci, device=DEV) * 0.2)
    y1 = torch.zeros(nc, B, co, hw, hw, device=DEV)
    y2 = torch.zeros_like(y1)
    part = torch.full((nc, co, ops.bnstats_tiles(B, hw, hw), 2), float("nan"),
                      dtype=torch.float64, device=DEV)
    ops.conv2d_fwd(x, w, bias, y1, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt, in_affine=aff)
    ops.conv2d_fwd(x, w, bias, y2, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt, in_affine=aff,
                   bn_stats=part)
    torch.cuda.synchronize()
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(y1[z, :k], y2[z, :k])
    # partials: fp64 sums of the stored values of each 256-pixel tile (zeros past the count)
    T = part.shape[2]
    yz = y2.double().permute(0, 2, 1, 3, 4).reshape(nc, co, B * hw * hw)
    for z in range(nc):
        yz[z, :, int(cnt[z]) * hw * hw:] = 0.0
    yt = torch.nn.functional.pad(yz, (0, T * 256 - B * hw * hw)).reshape(nc, co, T, 256)
    assert not torch.isnan(part).any()
    torch.testing.assert_close(part[..., 0], yt.sum(-1), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(part[..., 1], (yt * yt).sum(-1), rtol=1e-12, atol=1e-9)
    # BN outputs
    gamma = torch.rand(nc, co, device=DEV) + 0.5
    beta = torch.randn(nc, co, device=DEV) * 0.3
    outs = []
    for use_part in (False, True):
        rm, rv = torch.zeros(nc, co, device=DEV), torch.ones(nc, co, device=DEV)
        sm, si = torch.zeros(nc, co, device=DEV), torch.zeros(nc, co, device=DEV)
        sc, sh = torch.zeros(nc, co, device=DEV), torch.zeros(nc, co, device=DEV)
        if use_part:
            ops.bn_finalize_tiles(part, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, co, hw * hw,
                                  counts=cnt)
        else:
            ops.bn_fwd_stats(y1, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, co, hw * hw,
                             counts=cnt)
        outs.append((rm, rv, sm, si, sc, sh))
    for u, v in zip(*outs):
        assert _ulps(u, v) <= 1


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_epilogue_bn_stats_rounds_match(opt):
    """Whole CIFAR10CNN rounds with the statistics from the conv epilogues vs the separate
    statistics pass: the same training up to the fp64 summation order of the statistics."""
    sizes = [130, 70, 33, 9]
    a, ma = _round(True, opt, sizes, bn_epilogue=True)
    b, mb = _round(True, opt, sizes, bn_epilogue=False)
    P = a.layout.P
    d = (a.params[:, :P] - b.params[:, :P]).norm(dim=1)
    upd = (b.params[:, :P] - b.init_params[:, :P]).norm(dim=1)
    assert bool((d <= 1e-3 * upd).all()), (d, upd)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert abs(x.loss - y.loss) <= 1e-4 * max(1.0, abs(y.loss))


def test_fused_entry_points_refuse_unsupported_shapes():
    x = torch.zeros(1, 4, 32, 14, 14, device=DEV)  # 14x14: no direct-conv path
    sc, sh = torch.ones(1, 32, device=DEV), torch.zeros(1, 32, device=DEV)
    w = torch.zeros(1, 64, 32, 3, 3, device=DEV)
    y = torch.zeros(1, 4, 64, 14, 14, device=DEV)
    with pytest.raises(ops.FedHipError):
        ops.conv2d_fwd(x, w, None, y, 1, 4, 32, 14, 14, 64, 3, 1, 1, in_affine=(sc, sh))


@pytest.mark.parametrize("nc,C,hw,dm", [(1, 32, 32, 1), (5, 64, 16, 1), (3, 128, 8, 0),
                                        (24, 32, 32, 1)])
def test_pool_finalize_matches_separate_launches(nc, C, hw, dm):
    """fh_maxpool2_fwd_bnfinalize == fh_bn_finalize_tiles + fh_maxpool2_fwd_bnrelu: the BN
    outputs within 1 ulp (tree vs sequential merge of the same fp64 partials); the pooled
    values, window argmax and dropout keep-mask bit-identical to the separate pool launch
    given the affine the fused kernel publishes."""
    B = 32
    torch.manual_seed(nc * 11 + C)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    ci = 16
    x = torch.randn(nc, B, ci, hw, hw, device=DEV)
    w = torch.randn(nc, C, ci, 3, 3, device=DEV) * 0.1
    bias = torch.randn(nc, C, device=DEV) * 0.2
    c = torch.zeros(nc, B, C, hw, hw, device=DEV)
    part = torch.zeros(nc, C, ops.bnstats_tiles(B, hw, hw), 2, dtype=torch.float64, device=DEV)
    ops.conv2d_fwd(x, w, bias, c, nc, B, ci, hw, hw, C, 3, 1, 1, counts=cnt, bn_stats=part)
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    gamma[:, ::5] *= -1
    beta = torch.randn(nc, C, device=DEV) * 0.3
    outs = []
    for fused in (False, True):
        rm, rv = torch.zeros(nc, C, device=DEV), torch.ones(nc, C, device=DEV)
        sm, si = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
        sc, sh = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
        q = torch.zeros(nc, B, C, hw // 2, hw // 2, device=DEV)
        idx = torch.zeros(nc, B, C, hw // 2, hw // 2, dtype=torch.uint8, device=DEV)
        msk = torch.zeros_like(idx)
        if fused:
            ops.maxpool2_fwd_bnfinalize(part, gamma, beta, rm, rv, sm, si, sc, sh, c, q, idx, nc,
                                        B, C, hw, hw, mask=msk, drop_mode=dm, p_drop=0.3, seed=5,
                                        counts=cnt)
        else:
            ops.bn_finalize_tiles(part, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, C, hw * hw,
                                  counts=cnt)
            ops.maxpool2_fwd(c, q, idx, nc, B, C, hw, hw, mask=msk, drop_mode=dm, p_drop=0.3,
                             seed=5, counts=cnt, in_affine=(sc, sh))
        outs.append((rm, rv, sm, si, sc, sh, q, idx, msk))
    for u, v in zip(outs[0][:6], outs[1][:6]):
        assert _ulps(u, v) <= 1
    # the pool given the fused kernel's own affine
    rm, rv, sm, si, sc, sh, q2, i2, m2 = outs[1]
    q3 = torch.zeros_like(q2)
    i3, m3 = torch.zeros_like(i2), torch.zeros_like(m2)
    ops.maxpool2_fwd(c, q3, i3, nc, B, C, hw, hw, mask=m3, drop_mode=dm, p_drop=0.3, seed=5,
                     counts=cnt, in_affine=(sc, sh))
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(q2[z, :k], q3[z, :k]) and torch.equal(i2[z, :k], i3[z, :k])
        if dm:
            assert torch.equal(m2[z, :k], m3[z, :k]) and torch.equal(m2[z, :k], outs[0][8][z, :k])


# unsplit (many clients) and split-K (one client) DGRAD epilogues, every map width, ragged
@pytest.mark.parametrize("nc,ci,co,hw", [(1, 32, 32, 32), (32, 32, 32, 32), (3, 64, 64, 16),
                                         (1, 64, 64, 16), (24, 128, 128, 8), (1, 128, 128, 8),
                                         (5, 32, 64, 16)])
def test_dgrad_bn_bwd_stats_match_separate_pass(nc, ci, co, hw):
    """fh_conv2d_dgrad_bnstats + fh_bn_bwd_tiles vs fh_conv2d_dgrad + fh_bn_bwd (relu, mask
    recomputed from x): the stored g is dX with the ReLU mask applied, bit for bit; the
    per-tile fp64 partials equal fp64 sums of g and of the fp32 (x - mean) * g; dgamma /
    dbeta within 1 ulp and dx within 1e-5 of its scale (the same fp64 terms added in another
    order can move the fp32 mean-of-g / k by an ulp)."""
    B = 32
    torch.manual_seed(nc * 13 + ci + hw)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    bx = torch.randn(nc, B, ci, hw, hw, device=DEV) * 1.3 + 0.1  # the BN input (conv output)
    gamma = torch.rand(nc, ci, device=DEV) + 0.5
    gamma[:, ::6] *= -1
    beta = torch.randn(nc, ci, device=DEV) * 0.3
    rm, rv = torch.zeros(nc, ci, device=DEV), torch.ones(nc, ci, device=DEV)
    sm, si = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    sc, sh = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    ops.bn_fwd_stats(bx, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, ci, hw * hw, counts=cnt)
    dy = torch.randn(nc, B, co, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) * 0.1
    # separate: dgrad, then reduce + apply
    dr = torch.zeros(nc, B, ci, hw, hw, device=DEV)
    ops.conv2d_dgrad(dy, w, dr, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt)
    dx1 = torch.zeros_like(dr)
    dg1, db1 = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    ops.bn_bwd(dr, None, bx, gamma, sm, si, dx1, dg1, db1, nc, B, ci, hw * hw, relu=True,
               counts=cnt, beta=beta)
    # fused: dgrad with the mask + statistics, then the apply pass
    g = torch.zeros_like(dr)
    part = torch.full((nc, ci, ops.bnstats_tiles(B, hw, hw), 2), float("nan"),
                      dtype=torch.float64, device=DEV)
    ops.conv2d_dgrad(dy, w, g, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt,
                     bn_bwd=(bx, sc, sh, sm, part))
    dx2 = torch.zeros_like(dr)
    dg2, db2 = torch.zeros_like(dg1), torch.zeros_like(db1)
    ops.bn_bwd_tiles(part, g, bx, gamma, sm, si, dx2, dg2, db2, nc, B, ci, hw * hw, counts=cnt)
    torch.cuda.synchronize()
    keep = bx * sc[:, None, :, None, None] + sh[:, None, :, None, None] > 0
    gref = torch.where(keep, dr, torch.zeros_like(dr))
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(g[z, :k], gref[z, :k])
    assert not torch.isnan(part).any()
    T = part.shape[2]
    prod = (bx - sm[:, None, :, None, None]) * gref  # fp32, as bn_bwd_reduce_kernel
    terms = []
    for t in (gref, prod):
        tz = t.double().permute(0, 2, 1, 3, 4).reshape(nc, ci, B * hw * hw)
        for z in range(nc):
            tz[z, :, int(cnt[z]) * hw * hw:] = 0.0
        terms.append(torch.nn.functional.pad(tz, (0, T * 256 - B * hw * hw)).reshape(nc, ci, T, 256))
    torch.testing.assert_close(part[..., 0], terms[0].sum(-1), rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(part[..., 1], terms[1].sum(-1), rtol=1e-12, atol=1e-9)
    assert _ulps(dg1, dg2) <= 1 and _ulps(db1, db2) <= 1
    for z in range(nc):
        k = int(cnt[z])
        scale = dx1[z, :k].abs().max().item()
        assert (dx1[z, :k] - dx2[z, :k]).abs().max().item() <= 1e-5 * scale


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_dgrad_bn_bwd_epilogue_rounds_match(opt):
    """Whole CIFAR10CNN rounds with the BN backward statistics from the dgrad epilogues vs
    the reduce pass: the same training up to the fp64 summation order."""
    sizes = [130, 70, 33, 9]
    a, ma = _round(True, opt, sizes, bn_epilogue=True, bn_bwd_epilogue=True)
    b, mb = _round(True, opt, sizes, bn_epilogue=True, bn_bwd_epilogue=False)
    P = a.layout.P
    d = (a.params[:, :P] - b.params[:, :P]).norm(dim=1)
    upd = (b.params[:, :P] - b.init_params[:, :P]).norm(dim=1)
    assert bool((d <= 1e-3 * upd).all()), (d, upd)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert abs(x.loss - y.loss) <= 1e-4 * max(1.0, abs(y.loss))


@pytest.mark.parametrize("nc,ci,co,hw,dm", [(1, 32, 64, 16, True), (32, 32, 64, 16, True),
                                            (3, 64, 128, 8, False), (1, 64, 128, 8, True),
                                            (24, 64, 128, 8, True)])
def test_dgrad_bn_bwd_stats_through_pool(nc, ci, co, hw, dm):
    """fh_conv2d_dgrad_bnstats with pidx (the BN-ReLU output went through a 2x2 max-pool and
    dropout) + fh_bn_bwd_pool_tiles vs fh_conv2d_dgrad + fh_bn_bwd_pool: dX bit-identical,
    partials = fp64 sums of the routed, masked g and (x - mean) g over each pooled tile,
    dgamma / dbeta within 1 ulp, dx within 1e-5 of its scale."""
    B, p = 32, 0.3
    H = 2 * hw
    torch.manual_seed(nc * 17 + ci + hw)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    bx = torch.randn(nc, B, ci, H, H, device=DEV) * 1.3 + 0.1
    gamma = torch.rand(nc, ci, device=DEV) + 0.5
    gamma[:, ::6] *= -1
    beta = torch.randn(nc, ci, device=DEV) * 0.3
    rm, rv = torch.zeros(nc, ci, device=DEV), torch.ones(nc, ci, device=DEV)
    sm, si = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    sc, sh = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    ops.bn_fwd_stats(bx, gamma, beta, rm, rv, sm, si, sc, sh, nc, B, ci, H * H, counts=cnt)
    q = torch.zeros(nc, B, ci, hw, hw, device=DEV)
    idx = torch.zeros(nc, B, ci, hw, hw, dtype=torch.uint8, device=DEV)
    msk = torch.zeros_like(idx) if dm else None
    ops.maxpool2_fwd(bx, q, idx, nc, B, ci, H, H, mask=msk, drop_mode=1 if dm else 0,
                     p_drop=p, seed=3, counts=cnt, in_affine=(sc, sh))
    pd = p if dm else 0.0
    dy = torch.randn(nc, B, co, hw, hw, device=DEV)
    w = torch.randn(nc, co, ci, 3, 3, device=DEV) * 0.1
    dq1 = torch.zeros(nc, B, ci, hw, hw, device=DEV)
    ops.conv2d_dgrad(dy, w, dq1, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt)
    dx1 = torch.zeros_like(bx)
    dg1, db1 = torch.zeros(nc, ci, device=DEV), torch.zeros(nc, ci, device=DEV)
    ops.bn_bwd_pool(dq1, idx, None, bx, gamma, sm, si, dx1, dg1, db1, nc, B, ci, H, H,
                    relu=True, pmask=msk, p_drop=pd, counts=cnt, beta=beta)
    dq2 = torch.zeros_like(dq1)
    part = torch.full((nc, ci, ops.bnstats_tiles(B, hw, hw), 2), float("nan"),
                      dtype=torch.float64, device=DEV)
    ops.conv2d_dgrad(dy, w, dq2, nc, B, ci, hw, hw, co, 3, 1, 1, counts=cnt,
                     bn_bwd=(bx, sc, sh, sm, part, idx, msk, pd))
    dx2 = torch.zeros_like(bx)
    dg2, db2 = torch.zeros_like(dg1), torch.zeros_like(db1)
    ops.bn_bwd_pool_tiles(part, dq2, idx, bx, gamma, beta, sm, si, dx2, dg2, db2, nc, B, ci, H,
                          H, pmask=msk, p_drop=pd, counts=cnt)
    torch.cuda.synchronize()
    for z in range(nc):
        k = int(cnt[z])
        assert torch.equal(dq1[z, :k], dq2[z, :k])
    assert not torch.isnan(part).any()
    # routed g on the pooled grid: the gradient at the argmax element, ReLU-masked there
    gu = dq1 if msk is None else torch.where(msk.bool(), dq1 * (1.0 / (1.0 - pd)),
                                              torch.zeros_like(dq1))
    dyy, dxx = (idx.long() >> 1), (idx.long() & 1)
    yy = 2 * torch.arange(hw, device=DEV).view(hw, 1) + dyy
    xx = 2 * torch.arange(hw, device=DEV).view(1, hw) + dxx
    xa = torch.gather(bx.reshape(nc, B, ci, H * H), 3, (yy * H + xx).reshape(nc, B, ci, -1))
    xa = xa.reshape(nc, B, ci, hw, hw)
    keep = xa * sc[:, None, :, None, None] + sh[:, None, :, None, None] > 0
    g = torch.where(keep, gu, torch.zeros_like(gu))
    prod = (xa - sm[:, None, :, None, None]) * g
    T = part.shape[2]
    for col, t in ((0, g), (1, prod)):
        tz = t.double().permute(0, 2, 1, 3, 4).reshape(nc, ci, B * hw * hw)
        for z in range(nc):
            tz[z, :, int(cnt[z]) * hw * hw:] = 0.0
        ref = torch.nn.functional.pad(tz, (0, T * 256 - B * hw * hw)).reshape(nc, ci, T, 256)
        torch.testing.assert_close(part[..., col], ref.sum(-1), rtol=1e-12, atol=1e-9)
    assert _ulps(dg1, dg2) <= 1 and _ulps(db1, db2) <= 1
    for z in range(nc):
        k = int(cnt[z])
        scale = dx1[z, :k].abs().max().item()
        assert (dx1[z, :k] - dx2[z, :k]).abs().max().item() <= 1e-5 * scale


# ---------------------------------------------------------------- FederatedResNet (r02)
@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_resnet_fused_bn_rounds_bit_identical(opt):
    """ResNet-8 with bn1 applied on load by conv2 (fwd + wgrad) and its statistics from a
    separate statistics pass (fh_bn_fwd_stats): bit-identical to the materialised path."""
    sizes = [70, 33, 9]
    a, ma = _round(True, opt, sizes, resnet=True)
    b, mb = _round(False, opt, sizes, resnet=True)
    assert a.net._fused and not b.net._fused
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.bufs, b.bufs)
    assert torch.equal(a.state1, b.state1)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy) == (y.loss, y.accuracy)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_resnet_epilogue_bn_stats_rounds_match(opt):
    """ResNet-8 rounds with the forward BN statistics from the conv epilogues (stem bn1,
    stride-1 bn1, every bn2 via fh_bn_apply_tiles) and bn1's backward statistics from conv2's
    dgrad epilogue vs the separate passes: the same training up to the fp64 summation order
    of the statistics."""
    sizes = [70, 33, 9]
    a, ma = _round(True, opt, sizes, bn_epilogue=True, bn_bwd_epilogue=True, resnet=True)
    b, mb = _round(True, opt, sizes, resnet=True)
    P = a.layout.P
    d = (a.params[:, :P] - b.params[:, :P]).norm(dim=1)
    upd = (b.params[:, :P] - b.init_params[:, :P]).norm(dim=1)
    assert bool((d <= 1e-3 * upd).all()), (d, upd)
    torch.testing.assert_close(a.bufs, b.bufs, rtol=1e-4, atol=1e-5)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert abs(x.loss - y.loss) <= 1e-4 * max(1.0, abs(y.loss))


@pytest.mark.parametrize("nc,C,hw,res", [(1, 64, 32, False), (3, 64, 32, True),
                                         (5, 128, 16, True), (8, 256, 8, True)])
def test_bn_apply_tiles_matches_fwd_train(nc, C, hw, res):
    """fh_conv2d_fwd_bnstats + fh_bn_apply_tiles vs fh_bn_fwd_train on the same conv output
    (ReLU, with and without the residual, ragged counts): the saved / running statistics
    within 1 ulp (the same fp64 terms added in a different order), y within 1e-5 (a 1-ulp
    scale difference moves x*alpha + beta' by an ulp of x*alpha, not of y); y past a
    client's count untouched."""
    B = 32
    torch.manual_seed(nc * 11 + C)
    cnt = torch.tensor([B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,))],
                       dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, C, hw, hw, device=DEV)
    w = torch.randn(nc, C, C, 3, 3, device=DEV) * 0.05
    c = torch.zeros(nc, B, C, hw, hw, device=DEV)
    part = torch.full((nc, C, ops.bnstats_tiles(B, hw, hw), 2), float("nan"),
                      dtype=torch.float64, device=DEV)
    ops.conv2d_fwd(x, w, None, c, nc, B, C, hw, hw, C, 3, 1, 1, counts=cnt, bn_stats=part)
    r = torch.randn(nc, B, C, hw, hw, device=DEV) if res else None
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    beta = torch.randn(nc, C, device=DEV) * 0.3
    outs = []
    for tiles in (False, True):
        y = torch.full_like(c, 7.0)
        rm, rv = torch.zeros(nc, C, device=DEV), torch.ones(nc, C, device=DEV)
        sm, si = torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
        if tiles:
            ops.bn_apply_tiles(part, c, y, gamma, beta, rm, rv, sm, si, nc, B, C, hw * hw,
                               relu=True, res=r, counts=cnt)
        else:
            ops.bn_fwd_train(c, y, gamma, beta, rm, rv, sm, si, nc, B, C, hw * hw, relu=True,
                             res=r, counts=cnt)
        outs.append((y, rm, rv, sm, si))
    torch.cuda.synchronize()
    for u, v in list(zip(*outs))[1:]:
        assert _ulps(u, v) <= 1
    torch.testing.assert_close(outs[1][0], outs[0][0], rtol=1e-5, atol=1e-5)
    y = outs[1][0]
    for z in range(nc):
        assert bool((y[z, int(cnt[z]):] == 7.0).all())
