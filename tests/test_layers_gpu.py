"""BatchNorm2d (+ReLU, +residual) kernels vs a float64 torch reference of the same op,
per client over its valid images (nn.BatchNorm2d train/eval, models_pytorch.py:108-120,
176-187).  Shapes cover the split-reduction geometry: one client / many clients,
small and large HW, HW % 4 != 0 (scalar path), ragged counts."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fedhip import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")

CASES = [  # (clients, batch, C, H, W)
    (1, 32, 32, 32, 32),
    (3, 32, 64, 16, 16),
    (7, 32, 128, 8, 8),
    (2, 32, 64, 4, 4),
    (4, 16, 8, 7, 7),     # HW = 49: scalar path
    (1, 8, 5, 3, 5),      # HW = 15
]


def _counts(nc, B, seed):
    g = np.random.default_rng(seed)
    c = [B] + [int(v) for v in g.integers(1, B + 1, size=nc - 1)]
    return c


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("relu,residual", [(False, False), (True, False), (True, True)])
def test_bn_train_fwd_bwd(case, relu, residual):
    nc, B, C, H, W = case
    HW = H * W
    torch.manual_seed(sum(case) + relu + 2 * residual)
    cnt = _counts(nc, B, sum(case))
    x = torch.randn(nc, B, C, H, W, device=DEV) * 2 + 0.5
    res = torch.randn_like(x) if residual else None
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    beta = torch.randn(nc, C, device=DEV) * 0.1
    rmean = torch.randn(nc, C, device=DEV) * 0.1
    rvar = torch.rand(nc, C, device=DEV) + 0.5
    rm0, rv0 = rmean.clone(), rvar.clone()
    y = torch.zeros_like(x)
    sm = torch.zeros(nc, C, device=DEV)
    si = torch.zeros(nc, C, device=DEV)
    counts = torch.tensor(cnt, dtype=torch.int32, device=DEV)
    ops.bn_fwd_train(x, y, gamma, beta, rmean, rvar, sm, si, nc, B, C, HW, relu=relu, res=res,
                     counts=counts)
    dy = torch.randn_like(x)
    dx = torch.zeros_like(x)
    dres = torch.zeros_like(x) if residual else None
    dg = torch.zeros(nc, C, device=DEV)
    db = torch.zeros(nc, C, device=DEV)
    ops.bn_bwd(dy, y, x, gamma, sm, si, dx, dg, db, nc, B, C, HW, relu=relu, dres=dres,
               counts=counts)
    torch.cuda.synchronize()
    for z in range(nc):
        n = cnt[z]
        xr = x[z, :n].double().cpu().requires_grad_(True)
        g = gamma[z].double().cpu().requires_grad_(True)
        b = beta[z].double().cpu().requires_grad_(True)
        rm, rv = rm0[z].double().cpu(), rv0[z].double().cpu()
        out = F.batch_norm(xr, rm, rv, g, b, training=True, momentum=0.1, eps=1e-5)
        if residual:
            out = out + res[z, :n].double().cpu()
        if relu:
            out = F.relu(out)
        out.backward(dy[z, :n].double().cpu())
        yz = y[z, :n].double().cpu()
        assert (yz - out.detach()).abs().max().item() <= 2e-5 * (1 + out.abs().max().item())
        assert torch.allclose(rmean[z].double().cpu(), rm, rtol=1e-5, atol=1e-6)
        assert torch.allclose(rvar[z].double().cpu(), rv, rtol=1e-5, atol=1e-6)
        # float32 arithmetic against fp64: tolerances relative to the gradient scale
        gs = xr.grad.abs().max().item()
        assert (dx[z, :n].double().cpu() - xr.grad).abs().max().item() <= 1e-4 * gs + 1e-6
        assert torch.allclose(dg[z].double().cpu(), g.grad, rtol=1e-4, atol=1e-4)
        assert torch.allclose(db[z].double().cpu(), b.grad, rtol=1e-4, atol=1e-4)
        if residual:
            gm = dy[z, :n] * (y[z, :n] > 0) if relu else dy[z, :n]
            assert torch.equal(dres[z, :n], gm)


@pytest.mark.parametrize("case", CASES[:3] + CASES[4:5])
def test_bn_eval(case):
    nc, B, C, H, W = case
    HW = H * W
    torch.manual_seed(7)
    x = torch.randn(nc, B, C, H, W, device=DEV)
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    beta = torch.randn(nc, C, device=DEV) * 0.1
    rmean = torch.randn(nc, C, device=DEV) * 0.1
    rvar = torch.rand(nc, C, device=DEV) + 0.5
    y = torch.zeros_like(x)
    ops.bn_fwd_eval(x, y, gamma, beta, rmean, rvar, nc, B, C, HW, relu=True)
    for z in range(nc):
        ref = F.relu(F.batch_norm(x[z].double(), rmean[z].double(), rvar[z].double(),
                                  gamma[z].double(), beta[z].double(), training=False, eps=1e-5))
        assert (y[z].double() - ref).abs().max().item() <= 1e-5 * (1 + ref.abs().max().item())


def test_bn_deterministic():
    nc, B, C, H, W = 2, 32, 32, 32, 32
    torch.manual_seed(3)
    x = torch.randn(nc, B, C, H, W, device=DEV)
    gamma = torch.ones(nc, C, device=DEV)
    beta = torch.zeros(nc, C, device=DEV)
    outs = []
    for _ in range(2):
        y = torch.empty_like(x)
        sm = torch.empty(nc, C, device=DEV)
        si = torch.empty(nc, C, device=DEV)
        ops.bn_fwd_train(x, y, gamma, beta, None, None, sm, si, nc, B, C, H * W)
        outs.append((y, sm, si))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("case", [(2, 32, 32, 32), (3, 17, 64, 16), (1, 32, 128, 8), (2, 5, 8, 6)])
@pytest.mark.parametrize("p_drop", [0.0, 0.5])
def test_bn_bwd_pool_matches_unfused(case, p_drop):
    """fh_bn_bwd_pool == fh_maxpool2_bwd followed by fh_bn_bwd, bit for bit."""
    nc, B, C, H = case
    W = H
    torch.manual_seed(H + C)
    cnt = _counts(nc, B, H)
    counts = torch.tensor(cnt, dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, C, H, W, device=DEV)
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    beta = torch.randn(nc, C, device=DEV) * 0.1
    y = torch.zeros_like(x)
    sm = torch.zeros(nc, C, device=DEV)
    si = torch.zeros(nc, C, device=DEV)
    ops.bn_fwd_train(x, y, gamma, beta, None, None, sm, si, nc, B, C, H * W, relu=True,
                     counts=counts)
    q = torch.zeros(nc, B, C, H // 2, W // 2, device=DEV)
    idx = torch.zeros(nc, B, C, H // 2, W // 2, dtype=torch.uint8, device=DEV)
    mask = torch.zeros_like(idx) if p_drop > 0 else None
    ops.maxpool2_fwd(y, q, idx, nc, B, C, H, W, mask=mask, drop_mode=1 if p_drop > 0 else 0,
                     p_drop=p_drop, seed=3, counts=counts)
    dq = torch.randn_like(q)
    # unfused reference path
    dr = torch.zeros_like(x)
    ops.maxpool2_bwd(dq, idx, dr, nc, B, C, H, W, mask=mask, p_drop=p_drop, counts=counts)
    dx1, dg1, db1 = torch.zeros_like(x), torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
    ops.bn_bwd(dr, y, x, gamma, sm, si, dx1, dg1, db1, nc, B, C, H * W, relu=True, counts=counts)
    dx2, dg2, db2 = torch.zeros_like(x), torch.zeros(nc, C, device=DEV), torch.zeros(nc, C, device=DEV)
    ops.bn_bwd_pool(dq, idx, y, x, gamma, sm, si, dx2, dg2, db2, nc, B, C, H, W, relu=True,
                    pmask=mask, p_drop=p_drop, counts=counts)
    torch.cuda.synchronize()
    if W % 4 == 0:  # same float4 element order in both paths
        for z in range(nc):
            n = cnt[z]
            assert torch.equal(dx1[z, :n], dx2[z, :n])
        assert torch.equal(dg1, dg2) and torch.equal(db1, db2)
    else:           # fused path runs scalar (fp64 partial sums in another order)
        for z in range(nc):
            n = cnt[z]
            torch.testing.assert_close(dx1[z, :n], dx2[z, :n], rtol=1e-5, atol=1e-6)
        torch.testing.assert_close(dg1, dg2, rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(db1, db2, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("case", [(2, 32, 32, 16, 16), (3, 9, 64, 8, 8), (2, 7, 8, 7, 7)])
def test_bn_bwd_recomputed_relu_mask_is_exact(case):
    """yout=None: the ReLU mask recomputed from x equals the stored forward output's."""
    nc, B, C, H, W = case
    torch.manual_seed(C)
    cnt = _counts(nc, B, C)
    counts = torch.tensor(cnt, dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, C, H, W, device=DEV)
    gamma = torch.rand(nc, C, device=DEV) + 0.5
    beta = torch.randn(nc, C, device=DEV) * 0.3
    y = torch.zeros_like(x)
    sm = torch.zeros(nc, C, device=DEV)
    si = torch.zeros(nc, C, device=DEV)
    ops.bn_fwd_train(x, y, gamma, beta, None, None, sm, si, nc, B, C, H * W, relu=True,
                     counts=counts)
    dy = torch.randn_like(x)
    outs = []
    for yout, bt in ((y, None), (None, beta)):
        dx = torch.zeros_like(x)
        dg = torch.zeros(nc, C, device=DEV)
        db = torch.zeros(nc, C, device=DEV)
        ops.bn_bwd(dy, yout, x, gamma, sm, si, dx, dg, db, nc, B, C, H * W, relu=True,
                   counts=counts, beta=bt)
        outs.append((dx, dg, db))
    torch.cuda.synchronize()
    for z in range(nc):
        assert torch.equal(outs[0][0][z, :cnt[z]], outs[1][0][z, :cnt[z]])
    assert torch.equal(outs[0][1], outs[1][1]) and torch.equal(outs[0][2], outs[1][2])


@pytest.mark.parametrize("mom,wd,first", [(0.9, 0.0, False), (0.9, 0.0, True), (0.0, 0.0, False),
                                          (0.9, 0.01, False)])
def test_sgd_vector_and_scalar_paths_agree(mom, wd, first):
    """fh_sgd_step takes the float4 kernel for 16-B-aligned, n % 4 == 0 slabs (every packed
    parameter slab) and the scalar kernel otherwise; both must give the same bits, and the
    torch.optim.SGD update (training.py:244-255 builds it with momentum 0.9)."""
    n = 3 * 65536 + 64
    gen = torch.Generator(device="cpu").manual_seed(7)
    p0, g0, b0 = (torch.randn(n, generator=gen) for _ in range(3))
    outs = []
    for off in (0, 1):  # offset 1 float: misaligned -> scalar kernel
        p, g, b = (torch.zeros(n + 4, device="cuda") for _ in range(3))
        p[off:off + n], g[off:off + n], b[off:off + n] = p0.cuda(), g0.cuda(), b0.cuda()
        ops.sgd_step(p[off:off + n], g[off:off + n], b[off:off + n], 0.01, mom, wd, first)
        torch.cuda.synchronize()
        outs.append((p[off:off + n].cpu(), b[off:off + n].cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    # ATen's rounding, exactly: the add-with-alpha steps (g + wd*p, p - lr*b) are single-
    # rounding fmadds (emulated in fp64: the fp32 product is exact there), the momentum
    # update b*mom + g is two fp32 roundings (optim.hip builds with -ffp-contract=off)
    def fmadd(a, b, alpha):  # fl32(a + alpha*b) with one rounding
        return (a.double() + b.double() * torch.tensor(alpha, dtype=torch.float32).double()
                ).float()
    gv = fmadd(g0, p0, wd) if wd != 0.0 else g0
    bref = gv if (first or mom == 0.0) else b0 * mom + gv
    assert torch.equal(outs[0][0], fmadd(p0, bref, -0.01))
    if mom != 0.0:
        assert torch.equal(outs[0][1], bref)
    else:
        assert torch.equal(outs[0][1], b0)  # no momentum: the buffer is never touched


@pytest.mark.parametrize("wd,decoupled", [(0.0, False), (0.01, True), (0.01, False)])
def test_adam_vector_and_scalar_paths_agree(wd, decoupled):
    """fh_adam_step: float4 kernel on aligned slabs, scalar kernel otherwise — same bits
    (Adam / AdamW of training.py:244-255; torch parity is test_train_gpu's)."""
    n = 3 * 65536 + 64
    gen = torch.Generator(device="cpu").manual_seed(11)
    p0, g0, m0 = (torch.randn(n, generator=gen) for _ in range(3))
    v0 = torch.rand(n, generator=gen)
    outs = []
    for off in (0, 1):
        t = [torch.zeros(n + 4, device="cuda") for _ in range(4)]
        for buf, x in zip(t, (p0, g0, m0, v0)):
            buf[off:off + n] = x.cuda()
        ops.adam_step(*(buf[off:off + n] for buf in t), step=3, lr=1e-3, weight_decay=wd,
                      decoupled=decoupled)
        torch.cuda.synchronize()
        outs.append([t[i][off:off + n].cpu() for i in (0, 2, 3)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("p_drop", [0.0, 0.25])
def test_pitched_maxpool_matches_dense(p_drop):
    """Max-pool fwd / bwd on 14x14 maps embedded in 16x16 planes (SimpleCNN's direct-conv
    layout) == the dense kernels, bit for bit, and nothing outside the maps is written."""
    nc, B, C, H = 3, 32, 32, 14
    torch.manual_seed(2)
    counts = torch.tensor([32, 17, 5], dtype=torch.int32, device=DEV)
    x = torch.randn(nc, B, C, H, H, device=DEV)
    xp = torch.full((nc, B, C, 16, 16), 7.0, device=DEV)
    xp[..., :H, :H] = x
    q = torch.zeros(nc, B, C, 7, 7, device=DEV)
    qp = torch.full((nc, B, C, 16, 16), -3.0, device=DEV)  # pooled map into a 16x16 plane
    i1, i2 = (torch.zeros(nc, B, C, 7, 7, dtype=torch.uint8, device=DEV) for _ in range(2))
    m1, m2 = (torch.zeros_like(i1) if p_drop else None for _ in range(2))
    dm = 1 if p_drop else 0
    ops.maxpool2_fwd(x, q, i1, nc, B, C, H, H, mask=m1, drop_mode=dm, p_drop=p_drop, seed=4,
                     counts=counts)
    ops.maxpool2_fwd(xp, qp, i2, nc, B, C, H, H, mask=m2, drop_mode=dm, p_drop=p_drop, seed=4,
                     counts=counts)
    dq = torch.randn(nc, B, C, 7, 7, device=DEV)
    dqp = torch.full((nc, B, C, 16, 16), 5.0, device=DEV)
    dqp[..., :7, :7] = dq
    dx = torch.zeros(nc, B, C, H, H, device=DEV)
    dxp = torch.zeros(nc, B, C, 16, 16, device=DEV)
    ops.maxpool2_bwd(dq, i1, dx, nc, B, C, H, H, mask=m1, p_drop=p_drop, xin=x, counts=counts)
    ops.maxpool2_bwd(dqp, i2, dxp, nc, B, C, H, H, mask=m2, p_drop=p_drop, xin=xp, counts=counts)
    torch.cuda.synchronize()
    for z in range(nc):
        k = int(counts[z])
        assert torch.equal(q[z, :k], qp[z, :k, :, :7, :7])
        assert torch.equal(i1[z, :k], i2[z, :k])
        if p_drop:
            assert torch.equal(m1[z, :k], m2[z, :k])
        assert torch.equal(dx[z, :k], dxp[z, :k, :, :H, :H])
    assert bool((qp[..., 7:] == -3.0).all()) and bool((qp[..., 7:, :] == -3.0).all())
    assert bool((dxp[..., H:] == 0).all()) and bool((dxp[..., H:, :] == 0).all())
