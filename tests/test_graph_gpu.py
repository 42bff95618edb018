"""Graph-replayed rounds are bit-identical to eager rounds.

PackedTrainer.run_round replays every step after the first from a captured HIP
graph whose per-step inputs (batch indices, counts, epoch resets, dropout key,
Adam bias corrections) come from device memory.  Same plan, same seeds: the
parameters, BN buffers and metrics must match the eager path bit for bit,
including dropout masks and Adam's per-step scalars."""
import pytest
import torch

from fedhip.engine import PackedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _round(model_name, kw, shape, sizes, opt, use_graphs, rounds=2):
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(model_name, **kw).to(DEV)
    S = len(sizes)
    eng = PackedTrainer(model, capacity=S, batch=32, device=DEV)
    eng.use_graphs = use_graphs
    for k in range(S):
        eng.load_module_state(k, model)
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), *shape, generator=g).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(S)]
    gen = torch.Generator().manual_seed(11)
    metrics = []
    for r in range(rounds):
        plan = eng.make_plan(sizes, 1, generator=gen)
        metrics.append(eng.run_round(data, labels, offs, plan, optimizer_type=opt, lr=1e-3,
                                     seed=r))
    torch.cuda.synchronize()
    return eng, metrics


@pytest.mark.parametrize("model_name,kw,shape,opt", [
    ("cifar10_cnn", {"dropout_rate": 0.5}, (3, 32, 32), "sgd"),
    ("cifar10_cnn", {"dropout_rate": 0.5}, (3, 32, 32), "adam"),
    ("simple_cnn", {"dropout_rate": 0.5}, (1, 28, 28), "adamw"),
])
def test_graph_rounds_match_eager(model_name, kw, shape, opt):
    sizes = [100, 70, 40, 9]
    a, ma = _round(model_name, kw, shape, sizes, opt, use_graphs=True)
    b, mb = _round(model_name, kw, shape, sizes, opt, use_graphs=False)
    assert len(a._graphs) > 0 and len(b._graphs) == 0
    assert torch.equal(a.params, b.params)
    assert torch.equal(a.bufs, b.bufs)
    assert torch.equal(a.state1, b.state1) and torch.equal(a.state2, b.state2)
    for ra, rb in zip(ma, mb):
        for x, y in zip(ra, rb):
            assert (x.loss, x.accuracy, x.samples_processed) == (y.loss, y.accuracy,
                                                                y.samples_processed)
    assert a.num_batches_tracked == b.num_batches_tracked
