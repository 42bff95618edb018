"""FedAvg (bit-exact), update-level DP (exact with injected noise, statistical
with Philox noise) and optimizer kernels vs the CPU oracle / torch.optim."""
import math

import numpy as np
import pytest
import torch

from fedhip import ops
from oracle import fedavg_ref, privacy_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("C,P", [(4, 421642), (32, 421642), (7, 1001), (1, 13), (64, 4096)])
def test_fedavg_bit_exact(C, P):
    rng = np.random.default_rng(C * 1000 + P)
    rows = rng.standard_normal((C, P)).astype(np.float32) * 0.1
    n = [int(v) for v in rng.integers(10, 5000, size=C)]
    w = fedavg_ref.calculate_sample_weights(n)
    ref = fedavg_ref.weighted_average(list(rows), w)
    rd = torch.from_numpy(rows).to(DEV)
    wd = torch.tensor(w, dtype=torch.float32, device=DEV)
    out = torch.empty(P, dtype=torch.float32, device=DEV)
    ops.fedavg_weighted_sum(rd, wd, out)
    got = out.cpu().numpy()
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_fedavg_row_index_and_accumulate():
    rng = np.random.default_rng(3)
    C, P = 9, 3000
    rows = rng.standard_normal((C, P)).astype(np.float32)
    order = [4, 0, 8, 2, 6, 1, 3, 7, 5]
    w = [0.05 * (i + 1) for i in range(C)]
    half = 4
    ref = fedavg_ref.weighted_average([rows[i] for i in order], w)
    rd = torch.from_numpy(rows).to(DEV)
    idx = torch.tensor(order, dtype=torch.int32, device=DEV)
    wd = torch.tensor(w, dtype=torch.float32, device=DEV)
    out = torch.empty(P, device=DEV)
    # two chunks, accumulate = sequential semantics preserved
    ops.fedavg_weighted_sum(rd, wd[:half], out, row_index=idx[:half])
    ops.fedavg_weighted_sum(rd, wd[half:], out, row_index=idx[half:], accumulate=True)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_dp_clip_and_injected_noise_exact():
    rng = np.random.default_rng(11)
    C, P = 5, 20000
    segs = [0, 288, 320, 18752, 18816, 20000]
    glob = rng.standard_normal(P).astype(np.float32) * 0.1
    local = np.stack([glob + rng.standard_normal(P).astype(np.float32) * s
                      for s in (0.001, 0.01, 0.05, 0.0001, 0.2)])
    noise = rng.standard_normal((C, P)).astype(np.float32)
    eps, delta, maxn = 1.0, 1e-5, 1.0
    seg_off = torch.tensor(segs, dtype=torch.int64, device=DEV)
    ld = torch.from_numpy(local).to(DEV)
    gd = torch.from_numpy(np.tile(glob, (C, 1))).to(DEV)
    sq = ops.dp_delta_sqnorm(ld, gd, seg_off, C)
    total, coef, clipped, sigma = ops.dp_clip_coef(sq, maxn, eps, delta)
    out = torch.empty_like(ld)
    ops.dp_apply(ld, gd, out, coef, clipped, sigma, noise=torch.from_numpy(noise).to(DEV))
    out = out.cpu().numpy()
    for z in range(C):
        tens = [local[z, a:b] for a, b in zip(segs[:-1], segs[1:])]
        gten = [glob[a:b] for a, b in zip(segs[:-1], segs[1:])]
        nz = [noise[z, a:b] for a, b in zip(segs[:-1], segs[1:])]
        ref, sens, tot, was = privacy_ref.apply_update_dp(tens, gten, maxn, eps, delta, nz)
        ref = np.concatenate(ref)
        assert bool(clipped[z].item()) == was
        assert abs(total[z].item() - tot) <= 1e-6 * tot
        assert math.isclose(sigma[z].item(), privacy_ref.sigma(sens, eps, delta), rel_tol=1e-6)
        # clip coefficient can differ in the last ulp (norm summation order): <= 2 ulp
        d = np.abs(out[z].astype(np.float64) - ref)
        assert d.max() <= 4 * np.finfo(np.float32).eps * max(1.0, np.abs(ref).max())


def test_dp_philox_noise_statistics():
    C, P = 3, 1 << 20
    ld = torch.zeros(C, P, device=DEV)
    seg_off = torch.tensor([0, P], dtype=torch.int64, device=DEV)
    sq = ops.dp_delta_sqnorm(ld, None, seg_off, C)
    total, coef, clipped, sigma = ops.dp_clip_coef(sq, 1.0, 1.0, 1e-5)
    sigma.fill_(2.0)
    out = torch.empty_like(ld)
    ops.dp_apply(ld, None, out, coef, clipped, sigma, seed=1234)
    o = out.double()
    # reference statistical KAT (privacy_validator.py:103-108): mean|n|/sigma in [0.5, 2];
    # tightened to E|N(0,s)|/s = sqrt(2/pi) +- 1 %, std within 1 %, rows independent.
    r = (o.abs().mean(dim=1) / 2.0).cpu().numpy()
    assert np.all(np.abs(r - math.sqrt(2 / math.pi)) < 0.01 * math.sqrt(2 / math.pi))
    assert torch.all((o.std(dim=1) / 2.0 - 1).abs() < 0.01)
    assert abs(o.mean().item()) < 0.01
    assert not torch.equal(out[0], out[1])


def test_dp_noise_keyed_by_client_id():
    """row_ids: the noise of a client depends on its global id, not on the row it occupies
    (two ranks both have a row 0; their clients must not draw the same noise)."""
    P = 4099
    seg_off = torch.tensor([0, P], dtype=torch.int64, device=DEV)
    ld = torch.zeros(4, P, device=DEV)
    sq = ops.dp_delta_sqnorm(ld, None, seg_off, 4)
    _, coef, clipped, sigma = ops.dp_clip_coef(sq, 1.0, 1.0, 1e-5)
    sigma.fill_(1.0)
    ids = torch.tensor([7, 3, 12, 0], dtype=torch.int64, device=DEV)
    full = torch.empty_like(ld)
    ops.dp_apply(ld, None, full, coef, clipped, sigma, seed=99, row_ids=ids)
    # "rank 1" holds clients 12 and 3 in its rows 0 and 1: same noise as above
    part = torch.empty(2, P, device=DEV)
    ops.dp_apply(ld[:2], None, part, coef[:2], clipped[:2], sigma[:2], seed=99,
                 row_ids=ids[[2, 1]].contiguous())
    assert torch.equal(part[0], full[2]) and torch.equal(part[1], full[1])
    # without ids the key is the row: row 0 of both launches would collide
    plain = torch.empty(2, P, device=DEV)
    ops.dp_apply(ld[:2], None, plain, coef[:2], clipped[:2], sigma[:2], seed=99)
    assert not torch.equal(plain[0], full[0]) or int(ids[0]) == 0
    for i in range(4):
        for j in range(i + 1, 4):
            assert not torch.equal(full[i], full[j])
    with pytest.raises(Exception):
        ops.dp_apply(ld[:2], None, plain, coef[:2], clipped[:2], sigma[:2], seed=99,
                     row_ids=ids[:3])


def _torch_opt_steps(kind, p0, grads, lr):
    p = torch.nn.Parameter(p0.clone())
    if kind == "sgd":
        opt = torch.optim.SGD([p], lr=lr, momentum=0.9)
    elif kind == "adam":
        opt = torch.optim.Adam([p], lr=lr)
    else:
        opt = torch.optim.AdamW([p], lr=lr)
    for g in grads:
        p.grad = g.clone()
        opt.step()
    return p.detach()


@pytest.mark.parametrize("kind", ["sgd", "adam", "adamw"])
def test_optimizer_vs_torch_optim(kind):
    g = torch.Generator().manual_seed(5)
    n = 100003
    p0 = torch.randn(n, generator=g) * 0.1
    grads = [torch.randn(n, generator=g) * 0.01 for _ in range(4)]
    lr = 0.01 if kind == "sgd" else 1e-3
    ref = _torch_opt_steps(kind, p0, grads, lr)
    p = p0.to(DEV)
    s1 = torch.zeros(n, device=DEV)
    s2 = torch.zeros(n, device=DEV)
    for t, gr in enumerate(grads, 1):
        gd = gr.to(DEV)
        if kind == "sgd":
            ops.sgd_step(p, gd, s1, lr, 0.9, first_step=(t == 1))
        else:
            ops.adam_step(p, gd, s1, s2, t, lr, weight_decay=(0.01 if kind == "adamw" else 0.0),
                          decoupled=(kind == "adamw"))
    d = (p.cpu() - ref).abs().max().item()
    assert d <= 2e-7 * max(1.0, ref.abs().max().item()), d
