"""Per-sample-clipped DP-SGD (north_star extension; parity unpinned by the reference,
which has no DP-SGD) against the CPU oracle oracle/dpsgd_ref.py.

* sigma = 0: one packed step (3 clients, one with a partial batch) == the fp64
  per-sample-loop oracle replaying the GPU's max-pool / ReLU decisions, within the
  fp32-vs-fp64 tolerance used by the training parity tests;
* C huge: clipping inactive -> identical to the ordinary (non-private) gradient step;
* sigma > 0: the added noise has std sigma*C/B per coordinate (first SGD step moves
  parameters by lr * noise), zero mean;
* BatchNorm models are refused (no per-sample gradient)."""
import math

import numpy as np
import pytest
import torch

from fedhip import ops
from fedhip._lib import FedHipError
from fedhip.engine import DPSGDConfig, PackedTrainer
from oracle import dpsgd_ref, train_ref
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _engine(sizes, dpsgd, seed=0, lr=0.05):
    torch.manual_seed(seed)
    model = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.0)
    eng = PackedTrainer(model.to(DEV), capacity=len(sizes), batch=32, device=DEV, dpsgd=dpsgd)
    for k in range(len(sizes)):
        eng.load_module_state(k, model)
    eng.begin_round("sgd", lr)
    g = torch.Generator().manual_seed(seed + 1)
    xs = [torch.randn(n, 1, 28, 28, generator=g) for n in sizes]
    ys = [torch.randint(0, 10, (n,), generator=g) for n in sizes]
    for k in range(len(sizes)):
        eng.net.x[k, :sizes[k]].copy_(xs[k])
        eng.net.y[k, :sizes[k]].copy_(ys[k])
    return eng, xs, ys


def _decisions(eng, slots):
    relus = [b[:slots].cpu() > 0 for b in eng.net.relu_output_buffers()]
    per = []
    for slot in range(slots):
        pools = []
        for buf, H, W in eng.net.pool_index_buffers():
            a = buf[slot].long().cpu()
            OH, OW = a.shape[-2:]
            oh = torch.arange(OH).view(1, 1, OH, 1)
            ow = torch.arange(OW).view(1, 1, 1, OW)
            pools.append((2 * oh + a // 2) * W + (2 * ow + a % 2))
        per.append((pools, [r[slot] for r in relus]))
    return per


@pytest.mark.parametrize("max_norm", [0.05, 1.0])
def test_dpsgd_step_matches_oracle(max_norm):
    sizes = [32, 32, 7]
    eng, xs, ys = _engine(sizes, DPSGDConfig(max_grad_norm=max_norm, noise_multiplier=0.0))
    snap = {}
    eng.on_step = lambda e, n: snap.setdefault("d", _decisions(e, n))
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    eng.step(3, counts)
    torch.cuda.synchronize()
    for k, n in enumerate(sizes):
        ref32 = train_ref.make_model("simple_cnn", 0, dropout_rate=0.0)
        ref64 = train_ref.make_model("simple_cnn", None, dropout_rate=0.0).double()
        ref64.load_state_dict({a: b.double() for a, b in ref32.state_dict().items()})
        p0 = train_ref.param_vector(ref64).clone()
        pools, relus = snap["d"][k]
        pools = [p[:n] for p in pools]
        relus = [r[:n] for r in relus]
        opt32 = train_ref.make_optimizer(ref32, "sgd", 0.05)
        opt64 = train_ref.make_optimizer(ref64, "sgd", 0.05)
        c32, _ = dpsgd_ref.dpsgd_step(ref32, opt32, xs[k], ys[k], max_norm, pools=pools,
                                      relus=relus)
        c64, _ = dpsgd_ref.dpsgd_step(ref64, opt64, xs[k].double(), ys[k], max_norm,
                                      pools=pools, relus=relus)
        got = eng._coef[k, :n].double().cpu()
        assert torch.allclose(got, torch.tensor(c64, dtype=torch.float64), rtol=1e-4, atol=1e-6)
        if max_norm < 0.1:
            assert max(c64) < 1.0  # clipping active
        p32 = train_ref.param_vector(ref32).double()
        p64 = train_ref.param_vector(ref64)
        pg = eng.params[k, :eng.layout.P].double().cpu()
        e_hip = (pg - p64).norm().item()
        e_cpu = (p32 - p64).norm().item()
        assert e_hip <= 4 * e_cpu + 1e-4 * (p64 - p0).norm().item() + 1e-7 * p64.norm().item(), \
            (k, e_hip, e_cpu)


def test_dpsgd_without_clipping_equals_plain_step():
    sizes = [32, 20]
    a, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=1e9, noise_multiplier=0.0))
    b, _, _ = _engine(sizes, None)
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    a.step(2, counts)
    b.step(2, counts)
    torch.cuda.synchronize()
    assert torch.all(a._coef[0, :32] == 1.0) and torch.all(a._coef[1, :20] == 1.0)
    d = (a.params - b.params).abs().max().item()
    assert d <= 1e-6 * b.params.abs().max().item(), d


def test_dpsgd_noise_scale():
    sizes = [32, 16]
    lr, C, sig = 0.05, 1.0, 2.0
    a, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=C, noise_multiplier=sig), lr=lr)
    b, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=C, noise_multiplier=0.0), lr=lr)
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    a.step(2, counts)
    b.step(2, counts)
    torch.cuda.synchronize()
    P = a.layout.P
    for k, n in enumerate(sizes):
        d = ((b.params[k, :P] - a.params[k, :P]) / lr).double()  # = sigma*C/B * xi
        exp = sig * C / n
        assert abs(d.std().item() / exp - 1) < 0.01
        assert abs(d.mean().item()) < 5 * exp / math.sqrt(P)
    assert torch.equal(a.params[:, P:], b.params[:, P:])  # row padding untouched


def test_dpsgd_refuses_batchnorm_models():
    model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.0).to(DEV)
    eng = PackedTrainer(model, capacity=1, batch=32, device=DEV, dpsgd=DPSGDConfig())
    eng.load_module_state(0, model)
    eng.begin_round("sgd", 0.01)
    with pytest.raises(FedHipError, match="BatchNorm"):
        eng.step(1, torch.tensor([32], dtype=torch.int32, device=DEV))


def test_dpsgd_noise_key_is_secret():
    """Two trainers with the same public seeds (round seed, step, slot) draw different noise
    unless the caller fixes DPSGDConfig.seed (a public key would let anyone
    regenerate the noise and subtract it)."""
    sizes = [32, 16]
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    cfg = dict(max_grad_norm=1.0, noise_multiplier=1.0)
    a, _, _ = _engine(sizes, DPSGDConfig(**cfg))
    b, _, _ = _engine(sizes, DPSGDConfig(**cfg))
    c, _, _ = _engine(sizes, DPSGDConfig(seed=5, **cfg))
    d, _, _ = _engine(sizes, DPSGDConfig(seed=5, **cfg))
    for e in (a, b, c, d):
        e.step(2, counts)
    torch.cuda.synchronize()
    P = a.layout.P
    assert not torch.equal(a.params[:, :P], b.params[:, :P])
    assert torch.equal(c.params[:, :P], d.params[:, :P])


def test_persample_conv_slabs_exact():
    """fh_conv2d_wgrad_persample (one WGRAD pixel split per image, r04): each image's slab row
    is that image's own weight / bias gradient, slab_sqnorm its squared norm and slab_wsum the
    coefficient-weighted sum in image order — exact on small-integer operands and dyadic
    coefficients (ragged counts: rows past a client's count are never read)."""
    from fedhip import ops
    import torch.nn.functional as F
    C, B, cin, h, cout = 2, 7, 32, 16, 64
    g = torch.Generator().manual_seed(3)
    x = torch.randint(-2, 3, (C, B, cin, h, h), generator=g).float()
    dy = torch.randint(-2, 3, (C, B, cout, h, h), generator=g).float()
    counts = torch.tensor([7, 5], dtype=torch.int32)
    coef = torch.tensor([[1.0, 0.5, 0.25, 1.0, 0.125, 0.5, 1.0]] * C)
    slab = ops.PersampleSlab(DEV)
    cd = counts.to(DEV)
    ops.conv2d_wgrad_persample(x.to(DEV), dy.to(DEV), slab, C, B, cin, h, h, cout, counts=cd)
    sq = torch.zeros(C, B, dtype=torch.float64, device=DEV)
    ops.slab_sqnorm(slab, sq, counts=cd)
    dw = torch.zeros(C, cout, cin, 3, 3, device=DEV)
    db = torch.zeros(C, cout, device=DEV)
    ops.slab_wsum(slab, coef.to(DEV), dw, db, counts=cd)
    torch.cuda.synchronize()
    nw = cout * cin * 9
    boff = (C * B * nw * 4 + 255) // 256 * 256
    wrows = slab.buf[:C * B * nw * 4].view(torch.float32).view(C, B, nw).cpu()
    brows = slab.buf[boff:boff + C * B * cout * 4].view(torch.float32).view(C, B, cout).cpu()
    for z in range(C):
        accw = torch.zeros(cout, cin, 3, 3, dtype=torch.float64)
        accb = torch.zeros(cout, dtype=torch.float64)
        for i in range(int(counts[z])):
            wr = torch.zeros(cout, cin, 3, 3, dtype=torch.float64, requires_grad=True)
            br = torch.zeros(cout, dtype=torch.float64, requires_grad=True)
            F.conv2d(x[z, i:i + 1].double(), wr, br, padding=1).backward(dy[z, i:i + 1].double())
            assert torch.equal(wrows[z, i].double(), wr.grad.reshape(-1)), (z, i)
            assert torch.equal(brows[z, i].double(), br.grad), (z, i)
            assert sq[z, i].item() == float((wr.grad ** 2).sum() + (br.grad ** 2).sum())
            accw += coef[z, i].double() * wr.grad
            accb += coef[z, i].double() * br.grad
        assert torch.equal(dw[z].cpu().double(), accw), z
        assert torch.equal(db[z].cpu().double(), accb), z


def test_persample_c1_pool_slabs_sum_to_wgrad():
    """conv1's per-image slabs from pool1's gradient sum (coefficients 1) to the ordinary
    fused-pool conv1 weight gradient (fh_conv2d_c1_pool_wgrad) exactly, on integer data."""
    from fedhip import ops
    C, B, h = 2, 6, 28
    g = torch.Generator().manual_seed(4)
    x = torch.randint(-2, 3, (C, B, 1, h, h), generator=g).float().to(DEV)
    dpool = torch.zeros(C, B, 32, 16, 16)
    dpool[..., :14, :14] = torch.randint(-2, 3, (C, B, 32, 14, 14), generator=g).float()
    yp = torch.zeros(C, B, 32, 16, 16)
    yp[..., :14, :14] = torch.randint(-1, 2, (C, B, 32, 14, 14), generator=g).float()
    idx = torch.randint(0, 4, (C, B, 32, 14, 14), generator=g).to(torch.uint8).to(DEV)
    dpool, yp = dpool.to(DEV), yp.to(DEV)
    cd = torch.tensor([6, 4], dtype=torch.int32, device=DEV)
    slab = ops.PersampleSlab(DEV)
    ops.conv2d_c1_pool_wgrad_persample(x, dpool, idx, yp, slab, C, B, h, h, 32, counts=cd)
    dw = torch.zeros(C, 32, 1, 3, 3, device=DEV)
    db = torch.zeros(C, 32, device=DEV)
    ops.slab_wsum(slab, torch.ones(C, B, device=DEV), dw, db, counts=cd)
    dw2, db2 = torch.zeros_like(dw), torch.zeros_like(db)
    ops.conv2d_c1_pool_wgrad(x, dpool, idx, yp, dw2, db2, C, B, h, h, 32, counts=cd)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2) and torch.equal(db, db2)
    assert dw.abs().sum() > 0


@pytest.mark.parametrize("opt", ["sgd", "adamw"])
def test_dpsgd_fused_step_bit_identical(opt):
    """fh_dpsgd_step_slabs (r04) == slab_wsum of each per-image slab + dpsgd_noise over the
    row + the plain optimizer step, bit for bit (params, grads, optimizer state), with ragged
    counts and rows longer than the noised prefix."""
    from fedhip import ops
    C, B, cin, h, cout = 3, 9, 32, 16, 64
    g = torch.Generator().manual_seed(11)
    x = torch.randn(C, B, cin, h, h, generator=g).to(DEV)
    dy = torch.randn(C, B, cout, h, h, generator=g).to(DEV)
    cd = torch.tensor([9, 6, 1], dtype=torch.int32, device=DEV)
    coef = torch.rand(C, B, generator=g).to(DEV)
    slab = ops.PersampleSlab(DEV)
    ops.conv2d_wgrad_persample(x, dy, slab, C, B, cin, h, h, cout, counts=cd)
    nw = cout * cin * 9
    off_w, off_b, P = 40, 40 + nw, 40 + nw + cout + 52
    Ppad = (P + 60 + 63) // 64 * 64
    out = []
    for fused in (True, False):
        gen = torch.Generator().manual_seed(5)
        params = torch.randn(C, Ppad, generator=gen).to(DEV)
        grads = torch.randn(C, Ppad, generator=gen).to(DEV)
        s1 = torch.randn(C, Ppad, generator=gen).abs().to(DEV)
        s2 = torch.randn(C, Ppad, generator=gen).abs().to(DEV)
        dw, db = grads[:, off_w:off_w + nw], grads[:, off_b:off_b + cout]
        if fused:
            ops.dpsgd_step_slabs(params, grads, s1, s2, C, slab.ranges(grads, dw, db), coef, cd, B,
                                 P, 2.5, seed=77, opt=opt, lr=0.01, step=3)
        else:
            ops.slab_wsum(slab, coef, dw, db, counts=cd)
            ops.dpsgd_noise(grads, P, C, B, 2.5, seed=77, counts=cd)
            if opt == "sgd":
                ops.sgd_step(params, grads, s1, 0.01, 0.9, first_step=False)
            else:
                ops.adam_step(params, grads, s1, s2, 3, 0.01, weight_decay=0.01, decoupled=True)
        torch.cuda.synchronize()
        out.append((params, grads, s1, s2))
    for a, b in zip(*out):
        assert torch.equal(a, b)


@pytest.mark.parametrize("in_f,out_f", [(3136, 128), (128, 10)])
def test_linear_wgrad_rowscale_bit_identical(in_f, out_f):
    """fh_linear_wgrad_rowscale == scale_rows + linear_wgrad, bit for bit (ragged counts)."""
    from fedhip import ops
    C, B = 3, 32
    g = torch.Generator().manual_seed(in_f)
    x = torch.randn(C, B, in_f, generator=g).to(DEV)
    dy = torch.randn(C, B, out_f, generator=g).to(DEV)
    coef = torch.rand(C, B, generator=g).to(DEV)
    cd = torch.tensor([32, 17, 1], dtype=torch.int32, device=DEV)
    dw1, db1 = torch.zeros(C, out_f, in_f, device=DEV), torch.zeros(C, out_f, device=DEV)
    dw2, db2 = torch.zeros_like(dw1), torch.zeros_like(db1)
    ops.linear_wgrad_rowscale(x, dy, coef, dw1, db1, C, B, in_f, out_f, counts=cd)
    s = ops.scale_rows(dy, coef, torch.empty_like(dy), C, B, out_f, counts=cd)
    ops.linear_wgrad(x, s, dw2, db2, C, B, in_f, out_f, counts=cd)
    torch.cuda.synchronize()
    assert torch.equal(dw1, dw2) and torch.equal(db1, db2)


def test_dpsgd_norm_clip_matches_per_layer_path():
    """fh_dpsgd_norm_clip (r04: every image's norm over linear + slab sources and its clip
    coefficient in one launch) == the per-layer norm launches + fh_dpsgd_clip_coef (fp64 sums
    in another order: equal to 1e-12 relative; coefficients to fp32 rounding)."""
    from fedhip import ops
    C, B = 3, 12
    g = torch.Generator().manual_seed(8)
    cd = torch.tensor([12, 7, 1], dtype=torch.int32, device=DEV)
    x1, d1 = torch.randn(C, B, 128, generator=g).to(DEV), torch.randn(C, B, 10, generator=g).to(DEV)
    x2, d2 = torch.randn(C, B, 3136, generator=g).to(DEV), torch.randn(C, B, 128, generator=g).to(DEV)
    s2 = ops.PersampleSlab(DEV)
    ops.conv2d_wgrad_persample(torch.randn(C, B, 32, 16, 16, generator=g).to(DEV),
                               torch.randn(C, B, 64, 16, 16, generator=g).to(DEV) * 1e-3, s2, C, B,
                               32, 16, 16, 64, counts=cd)
    sq_b = torch.zeros(C, B, dtype=torch.float64, device=DEV)
    coef_b = torch.zeros(C, B, device=DEV)
    ops.linear_persample_sqnorm(x1, d1, sq_b, C, B, 128, 10, counts=cd)
    ops.linear_persample_sqnorm(x2, d2, sq_b, C, B, 3136, 128, counts=cd)
    ops.slab_sqnorm(s2, sq_b, counts=cd)
    norms = torch.cat([cd[z].item() * sq_b[z, :int(cd[z])].sqrt() for z in range(C)])
    max_norm = float(norms.median())  # some images clipped, some not
    ops.dpsgd_clip_coef(sq_b, coef_b, C, B, max_norm, counts=cd)
    sq_a = torch.zeros(C, B, dtype=torch.float64, device=DEV)
    coef_a = torch.zeros(C, B, device=DEV)
    ops.dpsgd_norm_clip([(x1, d1, 128, 10), (x2, d2, 3136, 128)], [s2], coef_a, C, B, max_norm,
                        sqnorm=sq_a, counts=cd)
    torch.cuda.synchronize()
    for z in range(C):
        n = int(cd[z])
        torch.testing.assert_close(sq_a[z, :n], sq_b[z, :n], rtol=1e-12, atol=0)
        torch.testing.assert_close(coef_a[z, :n], coef_b[z, :n], rtol=2e-7, atol=0)
        assert torch.all(coef_a[z, n:] == 0)
    assert (coef_a < 1).any() and (coef_a == 1).any()  # both branches of the clip exercised


@pytest.mark.parametrize("seed_cfg", [None, 9])
def test_dpsgd_dual_pooled_bit_identical(seed_cfg):
    """conv2's per-image WGRAD slabs held for its DGRAD (one dual-role launch) with pool2's
    backward routed inside (r05) == the two-launch path with the separate maxpool2_bwd launch,
    bit for bit (params, optimizer state), ragged clients, noise on (fixed noise key)."""
    sizes = [32, 32, 17, 5]
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    cfg = dict(max_grad_norm=0.5, noise_multiplier=0.7, seed=seed_cfg if seed_cfg else 3)
    out = []
    for dual, pooled in ((2, True), (0, False), (0, True)):
        eng, _, _ = _engine(sizes, DPSGDConfig(**cfg))
        eng.net.dual_bwd, eng.net.pooled_dy_bwd = dual, pooled
        for _ in range(3):
            eng.step(3, counts)
        torch.cuda.synchronize()
        out.append(eng)
    for e in out[1:]:
        assert torch.equal(out[0].params, e.params)
        assert torch.equal(out[0].state1, e.state1)


def test_linear_wgrad_rowscale_multi_bit_identical():
    """fh_linear_wgrad_rowscale_multi (r05) == one fh_linear_wgrad_rowscale per layer, bit for
    bit (ragged counts, with and without bias), and DP-SGD steps with it == without it."""
    from fedhip import ops
    g = torch.Generator().manual_seed(21)
    C, B = 3, 32
    cd = torch.tensor([32, 17, 1], dtype=torch.int32, device=DEV)
    coef = torch.rand(C, B, generator=g).to(DEV)
    shapes = [(3136, 128, True), (128, 10, True), (256, 64, False)]
    ins = [(torch.randn(C, B, fi, generator=g).to(DEV), torch.randn(C, B, fo, generator=g).to(DEV))
           for fi, fo, _ in shapes]
    outs = []
    for multi in (True, False):
        dws = [torch.zeros(C, fo, fi, device=DEV) for fi, fo, _ in shapes]
        dbs = [torch.zeros(C, fo, device=DEV) if bias else None for fi, fo, bias in shapes]
        if multi:
            ops.linear_wgrad_rowscale_multi(
                [(x, dy, dw, db, fi, fo) for (x, dy), dw, db, (fi, fo, _) in
                 zip(ins, dws, dbs, shapes)], coef, C, B, counts=cd)
        else:
            for (x, dy), dw, db, (fi, fo, _) in zip(ins, dws, dbs, shapes):
                ops.linear_wgrad_rowscale(x, dy, coef, dw, db, C, B, fi, fo, counts=cd)
        torch.cuda.synchronize()
        outs.append((dws, dbs))
    for a, b in zip(outs[0][0] + outs[0][1], outs[1][0] + outs[1][1]):
        assert (a is None and b is None) or torch.equal(a, b)
    sizes = [32, 32, 17, 5]
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    engs = []
    for multi in (True, False):
        eng, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=0.5, noise_multiplier=0.7, seed=4))
        eng.net.lin_wgrad_multi = multi
        for _ in range(2):
            eng.step(2, counts)
        torch.cuda.synchronize()
        engs.append(eng)
    assert torch.equal(engs[0].params, engs[1].params)


@pytest.mark.parametrize("sizes", [[32, 32, 17, 5], [9]])
def test_c1_slabs_with_norm_clip_bit_identical(sizes):
    """fh_conv2d_c1_pool_wgrad_persample_clip (r05: the norm / clip launch folded into the
    per-image conv1 slab launch) == the two launches: the same coefficients, squared norms and
    DP-SGD steps, bit for bit (ragged counts, narrow and wide grids)."""
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    engs = []
    for fused in (True, False):
        eng, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=0.3, noise_multiplier=0.6, seed=8))
        eng.net.c1_norm_fused = fused
        for _ in range(2):
            eng.step(len(sizes), counts)
        torch.cuda.synchronize()
        engs.append(eng)
    assert torch.equal(engs[0].params, engs[1].params)
    assert torch.equal(engs[0].state1, engs[1].state1)


@pytest.mark.parametrize("sizes", [[32, 17, 5], [23]])
def test_dpsgd_deferred_dgrad_reduction_bit_identical(sizes):
    """r05 fh_conv_defer_dgrad in DP-SGD: conv1's per-image slab launch (with the norm / clip
    tail) sums conv2's split DGRAD partials while staging — the same steps, bit for bit."""
    counts = torch.tensor(sizes, dtype=torch.int32, device=DEV)
    engs = []
    taken = []
    for defer in (True, False):
        eng, _, _ = _engine(sizes, DPSGDConfig(max_grad_norm=0.4, noise_multiplier=0.5, seed=2))
        eng.net.defer_dgrad = defer
        d0 = ops.defer_status()
        for _ in range(2):
            eng.step(len(sizes), counts)
        torch.cuda.synchronize()
        d1 = ops.defer_status()
        taken.append((d1[0] - d0[0], d1[1] - d0[1]))
        engs.append(eng)
    # defer=True: both steps left conv2's DGRAD partials to conv1's slab launch
    assert taken[0][0] >= 2 and taken[0][1] >= 2 and taken[1] == (0, 0), taken
    assert torch.equal(engs[0].params, engs[1].params)
    assert torch.equal(engs[0].state1, engs[1].state1)
