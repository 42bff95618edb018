"""Fused classifier kernels vs the separate launches they replace (and an fp64 truth).

* fh_linear_head_ce: last linear forward + cross-entropy + that layer's wgrad / dgrad + the
  dropout/ReLU backward of its input (reference: CIFAR10CNN fc3 models_pytorch.py:159-165,
  SimpleCNN fc2 :96-97, FederatedResNet fc :241-246; criterion training.py:193-203).
* fh_linear_bwd_fused: a linear layer's wgrad + dgrad + the dropout/ReLU backward of its
  input in one launch (the same MFMA bodies: bit-identical to the separate kernels).
* fh_linear_fwd on the skinny FORWARD kernel (in_f % 32 == 0, <= 32 images): exact on
  integer-valued operands for split and unsplit plans, ragged batches, partial output tiles."""
import pytest
import torch

from fedhip import ops

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _counts(nc, B, seed):
    g = torch.Generator().manual_seed(seed)
    c = [B] + [int(v) for v in torch.randint(1, B + 1, (nc - 1,), generator=g)]
    return torch.tensor(c, dtype=torch.int32, device=DEV)


def _dropped_relu(nc, B, F, p, seed):
    """h = relu(N(0,1)), keep-mask, e = h * mask / (1 - p) (what feeds the next layer)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    h = torch.relu(torch.randn(nc, B, F, generator=g, device=DEV))
    mask = (torch.rand(nc, B, F, generator=g, device=DEV) >= p).to(torch.uint8)
    e = torch.where(mask.bool(), h * (1.0 / (1.0 - p)), torch.zeros_like(h))
    return h, mask, e


@pytest.mark.parametrize("nc,F,K,p", [(5, 256, 10, 0.3), (3, 128, 10, 0.25), (4, 256, 100, 0.0),
                                      (1, 256, 10, 0.3)])
def test_head_matches_separate_ops(nc, F, K, p):
    B = 32
    cnt = _counts(nc, B, F + K)
    g = torch.Generator(device=DEV).manual_seed(K)
    h, mask, x = _dropped_relu(nc, B, F, p, 7 + F)
    w = torch.randn(nc, K, F, generator=g, device=DEV) * 0.1
    b = torch.randn(nc, K, generator=g, device=DEV) * 0.1
    y = torch.randint(0, K, (nc, B), generator=g, device=DEV)
    relu = p > 0.0  # the ResNet-like case: no ReLU / dropout in front of the layer
    mk = mask if p > 0.0 else None
    # separate launches (the round-1 path)
    lg1, dl1 = torch.zeros(nc, B, K, device=DEV), torch.zeros(nc, B, K, device=DEV)
    loss1 = torch.zeros(nc, device=DEV)
    acc1 = (torch.zeros(nc, dtype=torch.float64, device=DEV),
            torch.zeros(nc, dtype=torch.int64, device=DEV), torch.zeros(nc, dtype=torch.int64, device=DEV))
    ops.linear_fwd(x, w, b, lg1, nc, B, F, K, counts=cnt)
    ops.ce_fwd_bwd(lg1, y, dl1, nc, B, K, loss_out=loss1, acc_loss=acc1[0], acc_correct=acc1[1],
                   acc_seen=acc1[2], counts=cnt)
    dw1, db1 = torch.zeros(nc, K, F, device=DEV), torch.zeros(nc, K, device=DEV)
    ops.linear_wgrad(x, dl1, dw1, db1, nc, B, F, K, counts=cnt)
    dd = torch.zeros(nc, B, F, device=DEV)
    ops.linear_dgrad(dl1, w, dd, nc, B, F, K, counts=cnt)
    dx1 = torch.zeros(nc, B, F, device=DEV)
    ops.dropout_bwd(dd, dx1, nc, B, F, mask=mk, p_drop=p, relu_out=h if relu else None, counts=cnt)
    # fused
    lg2, dl2 = torch.zeros_like(lg1), torch.zeros_like(dl1)
    loss2 = torch.zeros(nc, device=DEV)
    acc2 = tuple(t.clone().zero_() for t in acc1)
    dw2, db2, dx2 = torch.zeros_like(dw1), torch.zeros_like(db1), torch.zeros_like(dx1)
    ops.linear_head_ce(x, w, b, y, lg2, dl2, dw2, db2, dx2, nc, B, F, K, loss_out=loss2,
                       acc_loss=acc2[0], acc_correct=acc2[1], acc_seen=acc2[2], mask=mk,
                       p_drop=p, relu_in=relu, counts=cnt)
    torch.cuda.synchronize()
    # fp64 truth of the same step
    for z in range(nc):
        n = int(cnt[z])
        xd, wd, bd = x[z, :n].double(), w[z].double(), b[z].double()
        lt = xd @ wd.T + bd
        lsm = torch.log_softmax(lt, dim=1)
        tgt = y[z, :n]
        loss_t = -lsm[torch.arange(n), tgt].mean()
        dlt = (lsm.exp() - torch.nn.functional.one_hot(tgt, K).double()) / n
        dwt, dbt = dlt.T @ xd, dlt.sum(0)
        dxt = dlt @ wd
        if relu:
            dxt = torch.where(mask[z, :n].bool() & (h[z, :n] > 0), dxt / (1.0 - p),
                              torch.zeros_like(dxt))
        for got, sep, ref in ((lg2[z, :n], lg1[z, :n], lt), (dl2[z, :n], dl1[z, :n], dlt),
                              (dw2[z], dw1[z], dwt), (db2[z], db1[z], dbt),
                              (dx2[z, :n], dx1[z, :n], dxt)):
            scale = ref.abs().max().item() + 1e-12
            e_new = (got.double() - ref).abs().max().item() / scale
            e_old = (sep.double() - ref).abs().max().item() / scale
            assert e_new <= max(4 * e_old, 2e-6), (e_new, e_old)
        assert abs(loss2[z].item() - loss_t.item()) <= 2e-6 * max(1.0, abs(loss_t.item()))
        assert abs(loss2[z].item() - loss1[z].item()) <= 2e-6 * max(1.0, abs(loss1[z].item()))
    # accumulators: same increments (loss sums as float64 of the fp32 batch losses)
    torch.testing.assert_close(acc2[0], loss2.double())
    assert torch.equal(acc2[2], cnt.to(torch.int64))
    pred_ok = 0
    for z in range(nc):
        n = int(cnt[z])
        pred_ok += int((lg2[z, :n].argmax(1) == y[z, :n]).sum())
    assert int(acc2[1].sum()) == pred_ok


@pytest.mark.parametrize("nc,in_f,out_f,p,relu", [(3, 512, 256, 0.3, True),
                                                  (32, 2048, 512, 0.0, False),
                                                  (1, 2048, 512, 0.0, False),
                                                  (7, 512, 256, 0.5, True),
                                                  # SimpleCNN fc1 (3136 = 24.5 x 128): the
                                                  # last WGRAD block's spare waves, one-tile
                                                  # DGRAD; fused grid and the wide two-launch
                                                  (3, 3136, 128, 0.0, False),
                                                  (32, 3136, 128, 0.0, False)])
def test_linear_bwd_fused_bit_identical(nc, in_f, out_f, p, relu):
    """One launch == linear_wgrad + linear_dgrad + dropout_bwd, bit for bit (same MFMA
    bodies; the ReLU decided on the dropped input e equals the one on h where kept)."""
    B = 32
    cnt = _counts(nc, B, in_f + nc)
    g = torch.Generator(device=DEV).manual_seed(in_f + nc)
    h, mask, x = _dropped_relu(nc, B, in_f, p, 3 + nc)
    if not relu:
        x = torch.randn(nc, B, in_f, generator=g, device=DEV)
    dy = torch.randn(nc, B, out_f, generator=g, device=DEV)
    w = torch.randn(nc, out_f, in_f, generator=g, device=DEV) * 0.05
    dw1, db1 = torch.zeros(nc, out_f, in_f, device=DEV), torch.zeros(nc, out_f, device=DEV)
    dd, dx1 = torch.zeros(nc, B, in_f, device=DEV), torch.zeros(nc, B, in_f, device=DEV)
    ops.linear_wgrad(x, dy, dw1, db1, nc, B, in_f, out_f, counts=cnt)
    ops.linear_dgrad(dy, w, dd, nc, B, in_f, out_f, counts=cnt)
    if relu:
        ops.dropout_bwd(dd, dx1, nc, B, in_f, mask=mask, p_drop=p, relu_out=h, counts=cnt)
    else:
        dx1 = dd
    dw2, db2, dx2 = torch.zeros_like(dw1), torch.zeros_like(db1), torch.zeros_like(dx1)
    assert ops.linear_bwd_fused(x, dy, w, dw2, db2, dx2, nc, B, in_f, out_f,
                                mask=mask if relu else None, p_drop=p,
                                relu_ref=x if relu else None, counts=cnt)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(dx1[z, :n], dx2[z, :n])


def test_linear_bwd_fused_declines_unsupported_shapes():
    x = torch.zeros(1, 32, 100, device=DEV)  # in_f % 32 != 0
    dy = torch.zeros(1, 32, 128, device=DEV)
    w = torch.zeros(1, 128, 100, device=DEV)
    assert not ops.linear_bwd_fused(x, dy, w, torch.zeros(1, 128, 100, device=DEV), None,
                                    torch.zeros_like(x), 1, 32, 100, 128)


@pytest.mark.parametrize("nc,in_f,out_f", [(1, 2048, 512), (32, 2048, 512), (5, 512, 256),
                                           (3, 3136, 128), (9, 128, 64)])
@pytest.mark.parametrize("mode", [1, 2])
def test_linear_fwd_dropout_equals_two_launches(nc, in_f, out_f, mode):
    """fh_linear_fwd_dropout == fh_dropout_fwd(fh_linear_fwd(x)), bit for bit, unsplit and
    split-K plans (1 client splits K), generated and injected keep-masks."""
    B, p = 32, 0.3
    cnt = _counts(nc, B, in_f + out_f)
    g = torch.Generator(device=DEV).manual_seed(nc + in_f)
    x = torch.randn(nc, B, in_f, generator=g, device=DEV)
    w = torch.randn(nc, out_f, in_f, generator=g, device=DEV) * 0.05
    b = torch.randn(nc, out_f, generator=g, device=DEV) * 0.1
    h = torch.zeros(nc, B, out_f, device=DEV)
    e1, e2 = torch.zeros_like(h), torch.zeros_like(h)
    m1 = torch.zeros(nc, B, out_f, dtype=torch.uint8, device=DEV)
    if mode == 2:
        m1 = (torch.rand(nc, B, out_f, generator=g, device=DEV) > p).to(torch.uint8)
    m2 = m1.clone()
    ops.linear_fwd(x, w, b, h, nc, B, in_f, out_f, relu=True, counts=cnt)
    ops.dropout_fwd(h, e1, m1, nc, B, out_f, p, mode, seed=77, counts=cnt)
    ops.linear_fwd_dropout(x, w, b, e2, m2, nc, B, in_f, out_f, p, drop_mode=mode, seed=77,
                           counts=cnt)
    torch.cuda.synchronize()
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(e1[z, :n], e2[z, :n]) and torch.equal(m1[z, :n], m2[z, :n])


@pytest.mark.parametrize("nc,plane", [(3, 16), (1, 14), (33, 16)])
def test_linear_bwd_fused_pool_equals_two_launches(nc, plane):
    """fh_linear_bwd_fused_pool (SimpleCNN fc1 after pool2, models_pytorch.py:91-95) writes
    the pool INPUT's gradient directly: bit-identical to fh_linear_bwd_fused (the pooled
    gradient) + fh_maxpool2_bwd_ymask (routed to the argmax, ReLU mask = pooled output > 0),
    the same dW / db, and the planes' elements outside the 14x14 map untouched."""
    B, C, OH, OW, out_f = 32, 64, 7, 7, 128
    in_f = C * OH * OW
    cnt = _counts(nc, B, 11)
    g = torch.Generator(device=DEV).manual_seed(nc)
    # pooled ReLU output: non-negative with exact zeros (the mask matters)
    x = torch.relu(torch.randn(nc, B, C, OH, OW, generator=g, device=DEV))
    idx = torch.randint(0, 4, (nc, B, C, OH, OW), generator=g, device=DEV).to(torch.uint8)
    dy = torch.randn(nc, B, out_f, generator=g, device=DEV)
    w = torch.randn(nc, out_f, in_f, generator=g, device=DEV) * 0.02
    dw1, db1 = torch.zeros(nc, out_f, in_f, device=DEV), torch.zeros(nc, out_f, device=DEV)
    dw2, db2 = torch.zeros_like(dw1), torch.zeros_like(db1)
    dp = torch.zeros(nc, B, in_f, device=DEV)
    assert ops.linear_bwd_fused(x.view(nc, B, in_f), dy, w, dw1, db1, dp, nc, B, in_f, out_f,
                                counts=cnt)
    sentinel = 7.0  # outside the map: must stay untouched
    da1 = torch.full((nc, B, C, plane, plane), sentinel, device=DEV)
    da1[..., :14, :14] = 0.0
    ops.maxpool2_bwd_ymask(dp.view(nc, B, C, OH, OW), idx, x, da1, nc, B, C, 14, 14, counts=cnt)
    da2 = torch.full_like(da1, sentinel)
    da2[..., :14, :14] = 0.0
    assert ops.linear_bwd_fused_pool(x.view(nc, B, in_f), dy, w, dw2, db2, da2, idx, nc, B, C, OH,
                                     OW, out_f, counts=cnt)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(da1[z, :n], da2[z, :n])
        if plane > 14:
            assert bool((da2[z, :, :, 14:, :] == sentinel).all())


@pytest.mark.parametrize("nc,B,in_f,out_f", [(1, 32, 2048, 512), (32, 32, 3136, 128),
                                             (7, 17, 256, 100), (64, 20, 128, 96),
                                             (3, 32, 512, 256), (2, 1, 96, 33)])
def test_linear_fwd_skinny_exact(nc, B, in_f, out_f):
    """Integer-valued x, w, bias (every partial sum exact in fp32): y equals the fp64 product
    exactly, whatever the split plan (1 client: 32-k chunks; 128-in layers: one split),
    ReLU applied, rows past each client's count untouched."""
    g = torch.Generator().manual_seed(in_f + out_f)
    x = torch.randint(-3, 4, (nc, B, in_f), generator=g).float()
    w = torch.randint(-3, 4, (nc, out_f, in_f), generator=g).float()
    b = torch.randint(-5, 6, (nc, out_f), generator=g).float()
    cnt = _counts(nc, B, nc + in_f)
    y = torch.full((nc, B, out_f), 7.0, device=DEV)
    ops.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), y, nc, B, in_f, out_f, relu=True, counts=cnt)
    torch.cuda.synchronize()
    ref = torch.relu(torch.einsum("zbk,zok->zbo", x.double(), w.double()) + b.double()[:, None])
    yc = y.cpu()
    for z in range(nc):
        n = int(cnt[z])
        assert torch.equal(yc[z, :n].double(), ref[z, :n]), z
        assert torch.all(yc[z, n:] == 7.0)

