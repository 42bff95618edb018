"""CPU checks of the DP-SGD oracle (oracle/dpsgd_ref.py) — parity unpinned by the
reference (no DP-SGD there); pinned instead against torch.func and the plain step."""
import torch
import torch.nn.functional as F
from torch.func import functional_call, grad, vmap

from oracle import dpsgd_ref, train_ref


def _model():
    return train_ref.make_model("simple_cnn", 3, dropout_rate=0.0)


def test_per_sample_loop_equals_vmap_grad():
    m = _model()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(4, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (4,), generator=g)
    loop = dpsgd_ref.per_sample_grads(m, x, y)
    params = {k: v.detach() for k, v in m.named_parameters()}

    def loss(p, xi, yi):
        return F.cross_entropy(functional_call(m, p, (xi.unsqueeze(0),)), yi.unsqueeze(0))

    vg = vmap(grad(loss), in_dims=(None, 0, 0))(params, x, y)
    names = [k for k, _ in m.named_parameters()]
    for i in range(4):
        for j, k in enumerate(names):
            torch.testing.assert_close(loop[i][j], vg[k][i], rtol=1e-5, atol=1e-7)


def test_unclipped_noiseless_step_is_plain_sgd():
    a, b = _model(), _model()
    g = torch.Generator().manual_seed(1)
    x = torch.randn(6, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (6,), generator=g)
    oa = train_ref.make_optimizer(a, "sgd", 0.1)
    ob = train_ref.make_optimizer(b, "sgd", 0.1)
    coefs, _ = dpsgd_ref.dpsgd_step(a, oa, x, y, max_norm=1e9)
    assert coefs == [1.0] * 6
    train_ref.train_step(b, ob, x, y)
    torch.testing.assert_close(train_ref.param_vector(a), train_ref.param_vector(b),
                               rtol=1e-5, atol=1e-7)


def test_clipped_norms_bounded():
    m = _model()
    g = torch.Generator().manual_seed(2)
    x = torch.randn(5, 1, 28, 28, generator=g)
    y = torch.randint(0, 10, (5,), generator=g)
    grads = dpsgd_ref.per_sample_grads(m, x, y)
    opt = train_ref.make_optimizer(m, "sgd", 0.0)
    coefs, norms = dpsgd_ref.dpsgd_step(m, opt, x, y, max_norm=0.01)
    for gi, c, nrm in zip(grads, coefs, norms):
        clipped = sum(float(((t * c) ** 2).sum()) for t in gi) ** 0.5
        assert clipped <= 0.01 * (1 + 1e-5)
        assert abs(nrm - sum(float((t.double() ** 2).sum()) for t in gi) ** 0.5) < 1e-6 * nrm
    assert abs(dpsgd_ref.sigma(1.0, 1e-5) - 4.844805262605097) < 1e-9
