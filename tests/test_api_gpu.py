"""Drop-in API behaviour on the GPU: FedAvgAggregator, DifferentialPrivacyEngine,
validator, RankRound (1 rank) — each checked against the CPU oracle."""
from datetime import datetime

import numpy as np
import pytest
import torch

from fedhip.round import DPConfig, RankRound
from oracle import fedavg_ref, privacy_ref
from src.aggregation.fedavg import AdaptiveFedAvg, FedAvgAggregator, FedAvgError
from src.shared import models_pytorch as hm
from src.shared.models import ModelUpdate
from src.shared.privacy import PrivacyError, create_privacy_engine

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
SHAPES = [("fc2.weight", (10, 128)), ("fc2.bias", (10,)), ("w3", (7, 3, 3, 3))]


def rows_for(C, seed, scale=0.05):
    rng = np.random.default_rng(seed)
    return [{n: rng.standard_normal(s).astype(np.float32) * scale for n, s in SHAPES}
            for _ in range(C)]


def upd(cid, w, n, budget=0.5, loss=0.5, on_gpu=False):
    d = {k: torch.from_numpy(v.copy()) for k, v in w.items()}
    if on_gpu:
        d = {k: v.to(DEV) for k, v in d.items()}
    return ModelUpdate(client_id=cid, round_number=2, model_weights=d, num_samples=n,
                       training_loss=loss, privacy_budget_used=budget, compression_ratio=0.8,
                       timestamp=datetime.now())


@pytest.mark.parametrize("validate", [False, True])
def test_aggregate_updates_bit_exact(validate):
    rows = rows_for(9, 1)
    ns = [100 * (i + 1) for i in range(9)]
    ups = [upd(f"c{i}", rows[i], ns[i], on_gpu=(i % 2 == 0)) for i in range(9)]
    gm = FedAvgAggregator(min_clients=2, validate_updates=validate).aggregate_updates(ups)
    w = fedavg_ref.calculate_sample_weights(ns)
    for n, _ in SHAPES:
        ref = fedavg_ref.weighted_average([r[n].reshape(-1) for r in rows], w)
        got = gm.model_weights[n].reshape(-1).cpu().numpy()
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), n
    assert gm.participating_clients == [f"c{i}" for i in range(9)]


def test_filter_truncate_and_reject():
    rows = rows_for(6, 2)
    rows[1]["fc2.weight"][0, 0] = 11.0          # |w| > 10
    rows[3]["fc2.bias"][2] = np.nan              # NaN
    ns = [10, 20, 30, 40, 50, 60]
    budgets = [0.5, 0.5, 4.0, 0.5, 0.5, 1.0]     # eps 4.0 -> rejected (validation.py:95)
    ups = [upd(f"v{i}", rows[i], ns[i], budgets[i]) for i in range(6)]
    gm = FedAvgAggregator(min_clients=2, max_clients=2).aggregate_updates(ups)
    # survivors v0, v4, v5 -> max_clients=2 keeps the two largest (stable): v5, v4
    assert gm.participating_clients == ["v5", "v4"]
    with pytest.raises(FedAvgError, match="Insufficient valid updates"):
        FedAvgAggregator(min_clients=2).aggregate_updates(
            [upd(f"e{i}", rows_for(1, 9 + i)[0], 5, 2.0) for i in range(3)])


def test_adaptive_reference_behaviour():
    rows = rows_for(3, 3)
    ups = [upd(f"a{i}", rows[i], 10 + i) for i in range(3)]
    # reference :443-447 compares a float against a list when performance_weight != 0
    with pytest.raises(FedAvgError):
        AdaptiveFedAvg().aggregate_updates(ups)
    gm = AdaptiveFedAvg(performance_weight=0.0).aggregate_updates(ups)
    assert len(gm.participating_clients) == 3


def test_convergence_metric_matches_torch():
    a, b = rows_for(2, 4)
    from src.shared.models import GlobalModel
    old = GlobalModel(1, {k: torch.from_numpy(v) for k, v in a.items()}, {}, [], 0.0)
    new = GlobalModel(2, {k: torch.from_numpy(v) for k, v in b.items()}, {}, [], 0.0)
    got = FedAvgAggregator().calculate_convergence_metrics(old, new)
    diff = sum(torch.norm(new.model_weights[k] - old.model_weights[k]).item() for k in a)
    norm = sum(torch.norm(new.model_weights[k]).item() for k in a)
    assert abs(got - min(1.0, diff / norm)) < 1e-6


@pytest.mark.parametrize("scale", [0.01, 1e-5])
def test_privacy_engine_injected_noise_exact(scale):
    d = rows_for(1, 5, scale)[0]
    grads = {k: torch.from_numpy(v).to(DEV) for k, v in d.items()}
    noise = {k: torch.randn(v.shape, generator=torch.Generator().manual_seed(1)) for k, v in d.items()}
    eng = create_privacy_engine(epsilon=1.0, delta=1e-5, max_grad_norm=1.0)
    out = eng.add_noise(grads, 1.0, 1e-5, noise={k: v.to(DEV) for k, v in noise.items()})
    names = [n for n, _ in SHAPES]
    clipped, sens, total, was = privacy_ref.clip([d[n] for n in names], 1.0)
    ref = privacy_ref.add_noise(clipped, [noise[n].numpy() for n in names])
    for n, r in zip(names, ref):
        got = out[n].cpu().numpy()
        assert np.abs(got.astype(np.float64) - r).max() <= 4 * np.finfo(np.float32).eps * max(1, np.abs(r).max())
    with pytest.raises(PrivacyError, match="budget exhausted"):  # reference: 2nd call raises
        eng.add_noise(grads, 1.0, 1e-5)


def test_privacy_engine_noise_statistics():
    g = {"w": torch.zeros(1 << 20, device=DEV)}
    eng = create_privacy_engine(epsilon=2.0, delta=1e-5, max_grad_norm=1.0)
    gen = eng.noise_generator
    n = gen.generate_noise(torch.Size([1 << 20]), 1.0, 2.0, 1e-5).double()
    sigma = privacy_ref.sigma(1.0, 2.0, 1e-5)
    assert abs(n.std().item() / sigma - 1) < 0.01
    out = eng.add_noise(g, 2.0, 1e-5)  # total norm 0 -> sensitivity 0 -> no noise
    assert torch.count_nonzero(out["w"]).item() == 0


def test_clip_gradients_api():
    d = rows_for(1, 6, 0.01)[0]
    grads = {k: torch.from_numpy(v).to(DEV) for k, v in d.items()}
    eng = create_privacy_engine()
    out = eng.clip_gradients(grads, 1.0)
    clipped, _, _, _ = privacy_ref.clip([d[n] for n, _ in SHAPES], 1.0)
    for (n, _), c in zip(SHAPES, clipped):
        assert np.abs(out[n].cpu().numpy() - c).max() <= 2 * np.finfo(np.float32).eps * np.abs(c).max()


def test_rank_round_dp_and_fedavg():
    """RankRound on one GPU: per-client DP with injected-free Philox noise has the right
    sigma; FedAvg of the resulting rows is bit-exact with the oracle."""
    torch.manual_seed(0)
    m = hm.ModelFactory.create_model("simple_cnn", dropout_rate=0.0).to(DEV)
    sizes = [40, 33, 64, 9]
    rr = RankRound(m, sizes, list(range(4)), epochs=1, device=DEV,
                   dp=DPConfig(epsilon=4.0, delta=1e-5, max_grad_norm=1.0))
    total = sum(sizes)
    data = torch.randn(total, 1, 28, 28, device=DEV)
    lab = torch.randint(0, 10, (total,), device=DEV)
    offs = np.cumsum([0] + [sizes[k] for k in rr.slots][:-1]).tolist()
    g0 = rr.global_flat.clone()
    captured = {}
    orig = rr._apply_dp

    def spy(S, seed):
        orig(S, seed)
        captured["rows"] = rr.trainer.params[:S, :rr.P].clone()
    rr._apply_dp = spy
    rr.run(data, lab, offs, "sgd", 0.01, seed=3)
    rows = captured["rows"].cpu().numpy()
    w = fedavg_ref.calculate_sample_weights(sizes)
    ref = fedavg_ref.weighted_average([rows[rr.slot_of[k]] for k in range(4)], w)
    assert np.array_equal(rr.global_flat.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    total_norm, clipped, sigma = rr.last_dp
    for z in range(4):
        exp = privacy_ref.sigma(min(total_norm[z].item(), 1.0), 4.0, 1e-5)
        assert abs(sigma[z].item() - exp) <= 1e-6 * exp
        if clipped[z].item():  # delta noise std should be sigma
            delta = torch.from_numpy(rows[z]) - g0.cpu()
            assert abs(delta.std().item() / exp - 1) < 0.02
