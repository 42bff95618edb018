"""HIP implicit-GEMM conv / linear vs a torch fp32 CPU reference (F.conv2d +
autograd), client-batched, including partial last batches (counts < batch).

Tolerance: fp32 MFMA accumulation order differs from mkldnn's, so outputs are
compared with  |gpu - ref| <= 2e-5 * sqrt(K) * max|ref| + 1e-6  where K is the
reduction length of the product (stated per test).
"""
import math

import pytest
import torch
import torch.nn.functional as F

from fedhip import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(gpu, ref, K, what):
    gpu = gpu.detach().cpu().double()
    ref = ref.detach().cpu().double()
    tol = 2e-5 * math.sqrt(K) * ref.abs().max().item() + 1e-6
    err = (gpu - ref).abs().max().item()
    assert err <= tol, f"{what}: max err {err:.3e} > tol {tol:.3e}"


CASES = [
    # nclients, batch, cin, h, w, cout, k, stride, pad
    (3, 8, 3, 32, 32, 32, 3, 1, 1),
    (2, 5, 32, 16, 16, 64, 3, 1, 1),
    (2, 4, 64, 8, 8, 128, 3, 1, 1),
    (2, 4, 1, 28, 28, 32, 3, 1, 1),
    (2, 3, 32, 14, 14, 64, 3, 1, 1),
    (2, 4, 64, 16, 16, 128, 3, 2, 1),
    (2, 4, 64, 16, 16, 128, 1, 2, 0),
    (2, 4, 128, 8, 8, 256, 3, 2, 1),
    (1, 2, 96, 7, 9, 40, 3, 1, 1),
    # direct-conv path (3x3/s1/p1, square 32/16/8): full tiles, split-K, multi-image tiles
    (4, 32, 32, 32, 32, 32, 3, 1, 1),
    (1, 32, 32, 32, 32, 32, 3, 1, 1),
    (2, 32, 64, 16, 16, 64, 3, 1, 1),
    (3, 30, 128, 8, 8, 128, 3, 1, 1),
    (1, 32, 128, 8, 8, 128, 3, 1, 1),
    (2, 7, 64, 8, 8, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", CASES)
def test_conv_fwd_bwd(case):
    C, B, cin, h, w, cout, k, s, p = case
    g = torch.Generator().manual_seed(1234)
    x = torch.randn(C, B, cin, h, w, generator=g)
    wt = torch.randn(C, cout, cin, k, k, generator=g) * (1.0 / math.sqrt(cin * k * k))
    bias = torch.randn(C, cout, generator=g)
    counts = torch.tensor([B - (i % 2) for i in range(C)], dtype=torch.int32)
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    dy = torch.randn(C, B, cout, oh, ow, generator=g)

    xd, wd, bd, dyd = x.to(DEV), wt.to(DEV), bias.to(DEV), dy.to(DEV)
    y = torch.zeros(C, B, cout, oh, ow, device=DEV)
    ops.conv2d_fwd(xd, wd, bd, y, C, B, cin, h, w, cout, k, s, p, counts=counts.to(DEV))
    dx = torch.zeros(C, B, cin, h, w, device=DEV)
    ops.conv2d_dgrad(dyd, wd, dx, C, B, cin, h, w, cout, k, s, p, counts=counts.to(DEV))
    dw = torch.zeros(C, cout, cin, k, k, device=DEV)
    db = torch.zeros(C, cout, device=DEV)
    ops.conv2d_wgrad(xd, dyd, dw, db, C, B, cin, h, w, cout, k, s, p, counts=counts.to(DEV))
    torch.cuda.synchronize()

    for z in range(C):
        n = int(counts[z])
        xr = x[z, :n].clone().requires_grad_(True)
        wr = wt[z].clone().requires_grad_(True)
        br = bias[z].clone().requires_grad_(True)
        yr = F.conv2d(xr, wr, br, stride=s, padding=p)
        yr.backward(dy[z, :n])
        _close(y[z, :n], yr, cin * k * k, f"fwd z={z}")
        _close(dx[z, :n], xr.grad, cout * k * k, f"dgrad z={z}")
        _close(dw[z], wr.grad, n * oh * ow, f"wgrad z={z}")
        _close(db[z], br.grad, n * oh * ow, f"bgrad z={z}")


@pytest.mark.parametrize("case", [(2, 9, 32, 32, 32, 64), (3, 16, 64, 16, 16, 32),
                                  (1, 32, 128, 8, 8, 128)])
def test_conv_relu_and_accumulate(case):
    """Fused ReLU epilogue (fwd) and dx += (dgrad into a residual gradient)."""
    C, B, cin, h, w, cout = case
    g = torch.Generator().manual_seed(99)
    x = torch.randn(C, B, cin, h, w, generator=g).to(DEV)
    wt = (torch.randn(C, cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)).to(DEV)
    bias = torch.randn(C, cout, generator=g).to(DEV)
    dy = torch.randn(C, B, cout, h, w, generator=g).to(DEV)
    y = torch.zeros(C, B, cout, h, w, device=DEV)
    y2 = torch.zeros_like(y)
    ops.conv2d_fwd(x, wt, bias, y, C, B, cin, h, w, cout, 3, 1, 1)
    ops.conv2d_fwd(x, wt, bias, y2, C, B, cin, h, w, cout, 3, 1, 1, relu=True)
    assert torch.equal(y2, torch.relu(y))
    base = torch.randn(C, B, cin, h, w, generator=g).to(DEV)
    dx = torch.zeros_like(base)
    ops.conv2d_dgrad(dy, wt, dx, C, B, cin, h, w, cout, 3, 1, 1)
    acc = base.clone()
    ops.conv2d_dgrad(dy, wt, acc, C, B, cin, h, w, cout, 3, 1, 1, accumulate=True)
    assert torch.equal(acc, base + dx)


@pytest.mark.parametrize("C,B,cin,h,cout,k,pad", [(8, 32, 64, 32, 128, 3, 1),
                                                   (1, 32, 128, 16, 256, 3, 1),
                                                   (2, 11, 64, 16, 128, 1, 0)])
def test_dgrad_s2_accumulate(C, B, cin, h, cout, k, pad):
    """Stride-2 DGRAD (parity phases) into a residual gradient: dx += result equals
    base + (the written result), and untouched images (past counts) keep their values
    (ResNet adds the conv1 dgrad onto the shortcut's, models_pytorch.py:182-194)."""
    g = torch.Generator().manual_seed(5)
    oh = h // 2
    wt = (torch.randn(C, cout, cin, k, k, generator=g) / math.sqrt(cin * k * k)).to(DEV)
    dy = torch.randn(C, B, cout, oh, oh, generator=g).to(DEV)
    base = torch.randn(C, B, cin, h, h, generator=g).to(DEV)
    counts = torch.tensor([B - (i % 3) for i in range(C)], dtype=torch.int32, device=DEV)
    dx = torch.zeros_like(base)
    ops.conv2d_dgrad(dy, wt, dx, C, B, cin, h, h, cout, k, 2, pad, counts=counts)
    acc = base.clone()
    ops.conv2d_dgrad(dy, wt, acc, C, B, cin, h, h, cout, k, 2, pad, counts=counts, accumulate=True)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(counts[z])
        assert torch.equal(acc[z, :n], base[z, :n] + dx[z, :n])
        assert torch.equal(acc[z, n:], base[z, n:])


@pytest.mark.parametrize("C,B,inf,outf", [(3, 32, 3136, 128), (2, 17, 128, 10), (2, 32, 2048, 512)])
def test_linear_fwd_bwd(C, B, inf, outf):
    g = torch.Generator().manual_seed(7)
    x = torch.randn(C, B, inf, generator=g)
    wt = torch.randn(C, outf, inf, generator=g) / math.sqrt(inf)
    bias = torch.randn(C, outf, generator=g)
    dy = torch.randn(C, B, outf, generator=g)
    counts = torch.tensor([B - i for i in range(C)], dtype=torch.int32)
    cd = counts.to(DEV)
    y = torch.zeros(C, B, outf, device=DEV)
    ops.linear_fwd(x.to(DEV), wt.to(DEV), bias.to(DEV), y, C, B, inf, outf, relu=True, counts=cd)
    dx = torch.zeros(C, B, inf, device=DEV)
    ops.linear_dgrad(dy.to(DEV), wt.to(DEV), dx, C, B, inf, outf, counts=cd)
    dw = torch.zeros(C, outf, inf, device=DEV)
    db = torch.zeros(C, outf, device=DEV)
    ops.linear_wgrad(x.to(DEV), dy.to(DEV), dw, db, C, B, inf, outf, counts=cd)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(counts[z])
        xr = x[z, :n].clone().requires_grad_(True)
        wr = wt[z].clone().requires_grad_(True)
        br = bias[z].clone().requires_grad_(True)
        yr = F.linear(xr, wr, br)
        yr.backward(dy[z, :n])
        _close(y[z, :n], torch.relu(yr), inf, "linear fwd")
        _close(dx[z, :n], xr.grad, outf, "linear dgrad")
        _close(dw[z], wr.grad, n, "linear wgrad")
        _close(db[z], br.grad, n, "linear bgrad")


EXACT = [  # nclients, batch, cin, h, cout, k, stride, pad (square maps)
    (1, 32, 32, 32, 32, 3, 1, 1),
    (2, 32, 32, 32, 64, 3, 1, 1),
    (8, 32, 32, 32, 32, 3, 1, 1),
    (3, 30, 64, 16, 64, 3, 1, 1),
    (1, 32, 64, 16, 128, 3, 1, 1),
    (5, 32, 128, 8, 128, 3, 1, 1),
    (2, 13, 64, 8, 64, 3, 1, 1),
    # r03 quadrant-wave WGRAD: one split per tile (>= 512 tiles: dW / db written directly,
    # no reduction launch), ragged counts
    (32, 8, 128, 8, 128, 3, 1, 1),
    (2, 9, 3, 32, 32, 3, 1, 1),
    (2, 8, 64, 16, 128, 3, 2, 1),
    (2, 8, 64, 16, 128, 1, 2, 0),
    (3, 6, 32, 28, 64, 3, 1, 1),
    # stride-2 DGRAD by parity phases (ResNet down-sampling: 3x3/p1 and the 1x1 shortcut),
    # full-width (no split-K) and one-client (split-K + phase epilogue) grids
    (8, 32, 64, 32, 128, 3, 2, 1),
    (8, 32, 64, 32, 128, 1, 2, 0),
    (1, 32, 128, 16, 256, 3, 2, 1),
    (1, 32, 128, 16, 256, 1, 2, 0),
    (3, 19, 32, 8, 48, 3, 2, 1),
    # stride-2 FWD on the direct kernel (S=2: 32->16, 16->8): split-K at one client,
    # ragged counts, Cout off the tile (48), scalar weight staging (Cin % 4 != 0)
    (3, 32, 64, 32, 96, 3, 2, 1),
    (2, 17, 32, 16, 48, 3, 2, 1),
    (2, 8, 6, 16, 40, 3, 2, 1),
    (1, 5, 6, 32, 32, 3, 2, 1),
    # single input channel (SimpleCNN conv1 on 28x28 MNIST maps): direct c1 FWD / WGRAD,
    # ragged counts, several pixel chunks, 64 output channels
    (3, 17, 1, 28, 32, 3, 1, 1),
    (1, 32, 1, 28, 32, 3, 1, 1),
    (2, 9, 1, 16, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", EXACT)
def test_conv_exact_integer(case):
    """Small-integer operands: every product and partial sum is exact in fp32, so
    any summation order gives the exact answer — the HIP results must equal the
    fp64 reference bit for bit (catches a dropped or doubled term that a
    relative tolerance at large K would hide)."""
    C, B, cin, h, cout, k, s, p = case
    w_ = h
    g = torch.Generator().manual_seed(sum(case))
    x = torch.randint(-2, 3, (C, B, cin, h, w_), generator=g).float()
    wt = torch.randint(-2, 3, (C, cout, cin, k, k), generator=g).float()
    bias = torch.randint(-2, 3, (C, cout), generator=g).float()
    oh = (h + 2 * p - k) // s + 1
    dy = torch.randint(-2, 3, (C, B, cout, oh, oh), generator=g).float()
    counts = torch.tensor([B - (i * 3) % min(B, 7) for i in range(C)], dtype=torch.int32)
    cd = counts.to(DEV)
    y = torch.zeros(C, B, cout, oh, oh, device=DEV)
    dx = torch.zeros(C, B, cin, h, w_, device=DEV)
    dw = torch.zeros(C, cout, cin, k, k, device=DEV)
    db = torch.zeros(C, cout, device=DEV)
    xd, wd, dyd = x.to(DEV), wt.to(DEV), dy.to(DEV)
    ops.conv2d_fwd(xd, wd, bias.to(DEV), y, C, B, cin, h, w_, cout, k, s, p, counts=cd)
    ops.conv2d_dgrad(dyd, wd, dx, C, B, cin, h, w_, cout, k, s, p, counts=cd)
    ops.conv2d_wgrad(xd, dyd, dw, db, C, B, cin, h, w_, cout, k, s, p, counts=cd)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(counts[z])
        xr = x[z, :n].double().requires_grad_(True)
        wr = wt[z].double().requires_grad_(True)
        br = bias[z].double().requires_grad_(True)
        yr = F.conv2d(xr, wr, br, stride=s, padding=p)
        yr.backward(dy[z, :n].double())
        assert torch.equal(y[z, :n].cpu().double(), yr.detach()), f"fwd z={z}"
        assert torch.equal(dx[z, :n].cpu().double(), xr.grad), f"dgrad z={z}"
        assert torch.equal(dw[z].cpu().double(), wr.grad), f"wgrad z={z}"
        assert torch.equal(db[z].cpu().double(), br.grad), f"bgrad z={z}"


@pytest.mark.parametrize("h", [32, 16])
def test_conv_s2_relu_epilogue(h):
    """Stride-2 forward (direct kernel) with the fused ReLU epilogue == relu(plain)."""
    C, B, cin, cout = 2, 12, 64, 128
    g = torch.Generator().manual_seed(h)
    x = torch.randn(C, B, cin, h, h, generator=g).to(DEV)
    wt = (torch.randn(C, cout, cin, 3, 3, generator=g) / math.sqrt(cin * 9)).to(DEV)
    bias = torch.randn(C, cout, generator=g).to(DEV)
    y = torch.zeros(C, B, cout, h // 2, h // 2, device=DEV)
    y2 = torch.zeros_like(y)
    ops.conv2d_fwd(x, wt, bias, y, C, B, cin, h, h, cout, 3, 2, 1)
    ops.conv2d_fwd(x, wt, bias, y2, C, B, cin, h, h, cout, 3, 2, 1, relu=True)
    assert torch.equal(y2, torch.relu(y))


@pytest.mark.parametrize("C,B,cin,h,cout,acc", [(8, 32, 64, 32, 128, False),
                                                (1, 32, 128, 16, 256, False),
                                                (3, 19, 32, 16, 48, True),
                                                (2, 32, 64, 32, 128, True)])
def test_dgrad_s2_shortcut_exact_integer(C, B, cin, h, cout, acc):
    """fh_conv2d_dgrad_s2_shortcut (conv1 3x3/s2 and the 1x1/s2 projection shortcut of a
    ResNet down-sampling block in one launch): small-integer operands, so the result must
    equal the fp64 sum of both input gradients bit for bit — unsplit grids, the split-K
    grid (one client), ragged counts, accumulate onto a residual gradient; images past a
    client's count untouched."""
    g = torch.Generator().manual_seed(C * 100 + cin)
    oh = h // 2
    wt = torch.randint(-2, 3, (C, cout, cin, 3, 3), generator=g).float()
    wsc = torch.randint(-2, 3, (C, cout, cin, 1, 1), generator=g).float()
    dy = torch.randint(-2, 3, (C, B, cout, oh, oh), generator=g).float()
    dsc = torch.randint(-2, 3, (C, B, cout, oh, oh), generator=g).float()
    base = torch.randint(-3, 4, (C, B, cin, h, h), generator=g).float()
    counts = torch.tensor([B - (i * 3) % min(B, 7) for i in range(C)], dtype=torch.int32)
    dx = base.to(DEV) if acc else torch.full((C, B, cin, h, h), 9.0, device=DEV)
    assert ops.conv2d_dgrad_s2_shortcut(dy.to(DEV), wt.to(DEV), dsc.to(DEV), wsc.to(DEV), dx, C, B,
                                        cin, h, h, cout, counts=counts.to(DEV), accumulate=acc)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(counts[z])
        xr = torch.zeros(n, cin, h, h, dtype=torch.float64, requires_grad=True)
        y = F.conv2d(xr, wt[z].double(), stride=2, padding=1)
        ysc = F.conv2d(xr, wsc[z].double(), stride=2)
        (y * dy[z, :n].double()).sum().add((ysc * dsc[z, :n].double()).sum()).backward()
        ref = xr.grad + (base[z, :n].double() if acc else 0.0)
        assert torch.equal(dx[z, :n].cpu().double(), ref), f"z={z}"
        tail = base[z, n:] if acc else torch.full_like(base[z, n:], 9.0)
        assert torch.equal(dx[z, n:].cpu(), tail)


def test_dgrad_s2_shortcut_declines_unsupported():
    """Outside the direct stride-2 kernel (8x8 map, cin % 32 != 0) the fused entry point
    issues nothing and returns False (the caller runs the two dgrads)."""
    z = torch.zeros
    assert not ops.conv2d_dgrad_s2_shortcut(z(1, 2, 16, 4, 4, device=DEV), z(1, 16, 8, 3, 3, device=DEV),
                                            z(1, 2, 16, 4, 4, device=DEV), z(1, 16, 8, 1, 1, device=DEV),
                                            z(1, 2, 8, 8, 8, device=DEV), 1, 2, 8, 8, 8, 16)


@pytest.mark.parametrize("C,B,cin,h,cout", [(1, 32, 32, 32, 32), (1, 32, 64, 16, 64),
                                            (1, 27, 32, 32, 32), (2, 32, 128, 8, 128),
                                            (1, 9, 64, 8, 64)])
def test_conv_lane_fill_exact(C, B, cin, h, cout):
    """Narrow grids at a one-client lane's fill fraction (0.25: no split-K below 128
    workgroups, fedhip/lanes.py): small-integer operands, so FWD, DGRAD and the two
    statistics epilogues (BN forward sums of y; BN backward sums of the ReLU-masked gradient
    and of (bn_x - mean) * g) must equal the fp64 reference exactly."""
    g = torch.Generator().manual_seed(C * 1000 + B + cin + h)
    x = torch.randint(-2, 3, (C, B, cin, h, h), generator=g).float()
    wt = torch.randint(-2, 3, (C, cout, cin, 3, 3), generator=g).float()
    bias = torch.randint(-2, 3, (C, cout), generator=g).float()
    dy = torch.randint(-2, 3, (C, B, cout, h, h), generator=g).float()
    bx = torch.randint(-3, 4, (C, B, cin, h, h), generator=g).float()    # BN input below
    sc = torch.randint(1, 3, (C, cin), generator=g).float()
    sh = torch.randint(-1, 2, (C, cin), generator=g).float()
    mean = torch.randint(-1, 2, (C, cin), generator=g).float()
    counts = torch.tensor([B - (i * 5) % 4 for i in range(C)], dtype=torch.int32)
    cd = counts.to(DEV)
    tiles = ops.bnstats_tiles(B, h, h)
    y = torch.zeros(C, B, cout, h, h, device=DEV)
    y1 = torch.zeros_like(y)
    dx = torch.zeros(C, B, cin, h, h, device=DEV)
    gx = torch.zeros_like(dx)
    part = torch.zeros(C, cout, tiles, 2, dtype=torch.float64, device=DEV)
    bpart = torch.zeros(C, cin, tiles, 2, dtype=torch.float64, device=DEV)
    xd, wd, bd, dyd = x.to(DEV), wt.to(DEV), bias.to(DEV), dy.to(DEV)
    ops.set_fill_fraction(0.25)
    try:
        ops.conv2d_fwd(xd, wd, bd, y, C, B, cin, h, h, cout, 3, 1, 1, counts=cd)
        ops.conv2d_fwd(xd, wd, bd, y1, C, B, cin, h, h, cout, 3, 1, 1, counts=cd, bn_stats=part)
        ops.conv2d_dgrad(dyd, wd, dx, C, B, cin, h, h, cout, 3, 1, 1, counts=cd)
        ops.conv2d_dgrad(dyd, wd, gx, C, B, cin, h, h, cout, 3, 1, 1, counts=cd,
                         bn_bwd=(bx.to(DEV), sc.to(DEV), sh.to(DEV), mean.to(DEV), bpart))
    finally:
        ops.set_fill_fraction(1.0)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(counts[z])
        xr = x[z, :n].double().requires_grad_(True)
        yr = F.conv2d(xr, wt[z].double(), bias[z].double(), padding=1)
        yr.backward(dy[z, :n].double())
        assert torch.equal(y[z, :n].cpu().double(), yr.detach()), f"fwd z={z}"
        assert torch.equal(y1[z, :n].cpu().double(), yr.detach()), f"fwd+stats z={z}"
        assert torch.equal(dx[z, :n].cpu().double(), xr.grad), f"dgrad z={z}"
        ps = part[z].sum(dim=1).cpu()  # tiles summed: per channel (sum y, sum y^2)
        assert torch.equal(ps[:, 0], yr.detach().sum(dim=(0, 2, 3))), f"bn sum z={z}"
        assert torch.equal(ps[:, 1], (yr.detach() ** 2).sum(dim=(0, 2, 3))), f"bn sq z={z}"
        on = (bx[z, :n].double() * sc[z].double().view(-1, 1, 1) +
              sh[z].double().view(-1, 1, 1)) > 0
        gr = torch.where(on, xr.grad, torch.zeros_like(xr.grad))
        assert torch.equal(gx[z, :n].cpu().double(), gr), f"dgrad+bnstats z={z}"
        bs = bpart[z].sum(dim=1).cpu()
        assert torch.equal(bs[:, 0], gr.sum(dim=(0, 2, 3))), f"bn bwd sum z={z}"
        dot = ((bx[z, :n].double() - mean[z].double().view(-1, 1, 1)) * gr).sum(dim=(0, 2, 3))
        assert torch.equal(bs[:, 1], dot), f"bn bwd dot z={z}"
