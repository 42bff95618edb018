"""The drop-in evaluation surface on the GPU.

  LocalTrainer.evaluate_model    src/shared/training.py:307-360 — against golden G7, the
                                 reference's own metrics + exact logits for three models
  model(x)  (fedhip/infer.py)     the eval-mode forward every caller of the nn.Module uses
  train_local_model(validation_loader=..., early_stopping_patience=...)
                                 training.py:110-138 + _validate_epoch :214-242 — per-epoch
                                 validation loss / accuracy against the oracle and the
                                 early-stopping decision it implies

Tolerances: logits within 2e-4 of their magnitude (fp32 convolutions, other summation
order); predictions and every count exact wherever the reference's top-2 margin is
clear of that tolerance (all G7 cases are)."""
import json
import os

import pytest
import torch

from fedhip import infer
from oracle import train_ref
from src.shared import models_pytorch as hm
from src.shared.training import LocalTrainer
from test_oracle_golden import g7_case

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "golden.json")))


def _gpu_model(ref, name, kw):
    m = hm.ModelFactory.create_model(name, **kw)
    m.load_state_dict(ref.state_dict())
    return m.to(DEV)


@pytest.mark.parametrize("key", [k for k in GOLD if k.startswith("G7/")])
def test_evaluate_model_matches_reference_g7(key):
    g = GOLD[key]
    ref, xt, yt = g7_case(g)  # the reference's trained model, rebuilt by the oracle
    exp, logits = train_ref.evaluate_model(ref, xt, yt, batch=32)
    model = _gpu_model(ref, g["model"], g["kwargs"])
    loader = torch.utils.data.DataLoader(torch.utils.data.TensorDataset(xt, yt), batch_size=32,
                                         shuffle=False)
    got = LocalTrainer(model, device=DEV).evaluate_model(loader)
    tol = 2e-4 * float(logits.abs().max()) + 1e-5
    top2 = logits.topk(2, dim=1).values
    assert bool(((top2[:, 0] - top2[:, 1]) > 4 * tol).all()), "G7 margins are clear"
    assert got == g["metrics"]  # the reference's own evaluate_model output, exactly
    assert got == exp
    # model(x): the same eval-mode forward, batch by batch and in one ragged call
    model.eval()
    with torch.no_grad():
        lg = torch.cat([model(xt[i:i + 32].to(DEV)).cpu() for i in range(0, len(xt), 32)])
        one = model(xt.to(DEV)).cpu()
    assert (lg - logits).abs().max().item() <= tol
    assert (one - logits).abs().max().item() <= tol


def test_forward_sees_weight_changes_between_calls():
    """Outside an evaluation loop every call reloads the module's weights (including
    p.data writes, which torch's version counter does not see)."""
    torch.manual_seed(2)
    model = hm.ModelFactory.create_model("simple_cnn").to(DEV).eval()
    x = torch.randn(5, 1, 28, 28, device=DEV)
    with torch.no_grad():
        a = model(x).clone()
        model.fc2.bias.data.add_(1.0)  # no version bump
        b = model(x)
    assert torch.allclose(b - a, torch.ones_like(a), atol=1e-5)
    # inside frozen() the weights are taken once: a change made meanwhile is not seen
    with torch.no_grad(), infer.frozen(model):
        c = model(x).clone()
        model.fc2.bias.data.add_(1.0)
        d = model(x)
    assert torch.equal(c, d)
    with torch.no_grad():
        e = model(x)
    assert torch.allclose(e - d, torch.ones_like(d), atol=1e-5)


def _oracle_validate(model, batches):
    """_validate_epoch (training.py:214-242): eval mode, mean of batch losses, accuracy."""
    model.eval()
    run, correct, seen = 0.0, 0, 0
    with torch.no_grad():
        for x, y in batches:
            out = model(x)
            run += torch.nn.functional.cross_entropy(out, y).item()
            correct += int((out.argmax(1) == y).sum())
            seen += y.numel()
    return run / len(batches), correct / seen


@pytest.mark.parametrize("name,kw,shape,patience", [
    ("simple_cnn", {"dropout_rate": 0.0}, (1, 28, 28), 1),
    ("cifar10_cnn", {"dropout_rate": 0.0}, (3, 32, 32), 2),
])
def test_validation_and_early_stopping(name, kw, shape, patience):
    """Per-epoch validation against the oracle, and early stopping at the epoch the
    validation losses dictate (training.py:124-131: stop after `patience` epochs without a
    new best)."""
    g = torch.Generator().manual_seed(31)
    n, nv, epochs, lr = 96, 40, 6, 0.08  # a high lr on noise labels: val loss turns up
    x, y = torch.randn(n, *shape, generator=g), torch.randint(0, 10, (n,), generator=g)
    xv, yv = torch.randn(nv, *shape, generator=g), torch.randint(0, 10, (nv,), generator=g)
    tb = [(x[i:i + 32], y[i:i + 32]) for i in range(0, n, 32)]
    vb = [(xv[i:i + 32], yv[i:i + 32]) for i in range(0, nv, 32)]
    ref = train_ref.make_model(name, 5, **kw)
    model = _gpu_model(ref, name, kw)
    opt = train_ref.make_optimizer(ref, "sgd", lr)
    ref_val = []
    for _ in range(epochs):
        for xb, yb in tb:
            train_ref.train_step(ref, opt, xb, yb)
        ref_val.append(_oracle_validate(ref, vb))

    tr = LocalTrainer(model, device=DEV)
    got_val = []
    inner = tr._validate_epoch
    tr._validate_epoch = lambda eng, loader: got_val.append(inner(eng, loader)) or got_val[-1]
    mk = lambda xs, ys: torch.utils.data.DataLoader(  # noqa: E731
        torch.utils.data.TensorDataset(xs, ys), batch_size=32, shuffle=False)
    m = tr.train_local_model(mk(x, y), epochs=epochs, learning_rate=lr, optimizer_type="sgd",
                             validation_loader=mk(xv, yv), save_checkpoints=False,
                             early_stopping_patience=patience)
    # the epochs both ran: losses within training drift, accuracies within a few samples
    for e, ((lv, av), (rl, ra)) in enumerate(zip(got_val, ref_val)):
        assert abs(lv - rl) <= 2e-2 * abs(rl) + 1e-3 * (e + 1), (e, lv, rl)
        assert abs(av - ra) <= 3.0 / nv + 1e-12, (e, av, ra)
    # the stop epoch implied by the GPU's own validation losses, and by the oracle's
    def stop_epoch(vals):
        best, wait = float("inf"), 0
        for e, (lv, _) in enumerate(vals):
            if lv < best:
                best, wait = lv, 0
            else:
                wait += 1
                if wait >= patience:
                    return e + 1
        return len(vals)
    assert m.epochs_completed == len(got_val) == stop_epoch(got_val)
    margins = [abs(a[0] - b[0]) for a, b in zip(ref_val[1:], ref_val[:-1])]
    if min(margins[:m.epochs_completed]) > 0.05:
        assert m.epochs_completed == stop_epoch(ref_val[:m.epochs_completed]) or \
            m.epochs_completed == stop_epoch(ref_val)
    assert m.samples_processed == n * m.epochs_completed
