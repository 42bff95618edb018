"""Concurrent lanes (fedhip/lanes.py) are bit-identical to training each lane alone.

A LanedTrainer cuts the slots into contiguous lanes that run concurrently on
their own HIP streams (own activation buffers, split-K scratch and graphs) over
one shared state matrix.  Each lane must produce exactly what a standalone
PackedTrainer of the same capacity produces for those clients with the same
plan and dropout keys: any cross-lane race (shared scratch, stream ordering of
the per-step rows, graph pools) shows up as a bit difference."""
import pytest
import torch

from fedhip import ops
from fedhip.engine import PackedTrainer
from fedhip.lanes import LanedTrainer
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


def _data(sizes, shape):
    g = torch.Generator().manual_seed(5)
    data = torch.randn(sum(sizes), *shape, generator=g).to(DEV)
    labels = torch.randint(0, 10, (sum(sizes),), generator=g).to(DEV)
    offs = [sum(sizes[:k]) for k in range(len(sizes))]
    return data, labels, offs


@pytest.mark.parametrize("model_name,kw,shape,opt", [
    ("cifar10_cnn", {"dropout_rate": 0.3}, (3, 32, 32), "sgd"),
    ("simple_cnn", {"dropout_rate": 0.25}, (1, 28, 28), "adam"),
])
def test_lanes_match_standalone(model_name, kw, shape, opt):
    sizes = [300, 120, 100, 64, 33, 9]
    cut = [0, 1, 4, 6]
    steps = [-(-n // 32) for n in sizes]
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model(model_name, **kw).to(DEV)
    data, labels, offs = _data(sizes, shape)

    lt = LanedTrainer(model, steps, batch=32, device=DEV, cut=cut)
    for k in range(len(sizes)):
        lt.load_module_state(k, model)
    gen = torch.Generator().manual_seed(11)
    for r in range(2):
        plans = lt.make_plan(sizes, 1, generator=gen)
        lt.run_round(data, labels, offs, plans, optimizer_type=opt, lr=1e-3, seed=r)
    torch.cuda.synchronize()

    gen = torch.Generator().manual_seed(11)
    alone = [PackedTrainer(model, cut[i + 1] - cut[i], batch=32, device=DEV)
             for i in range(len(cut) - 1)]
    for i, tr in enumerate(alone):
        tr.net.salt = lt.lanes[i].net.salt
        for k in range(cut[i], cut[i + 1]):
            tr.load_module_state(k - cut[i], model)
    for r in range(2):
        for i, tr in enumerate(alone):
            a, b = cut[i], cut[i + 1]
            plan = tr.make_plan(sizes[a:b], 1, generator=gen)
            ops.set_fill_fraction(lt.fill[i])  # the lane's split-K plan (1-client lane: 0.25)
            try:
                tr.run_round(data, labels, offs[a:b], plan, optimizer_type=opt, lr=1e-3, seed=r)
            finally:
                ops.set_fill_fraction(1.0)
    torch.cuda.synchronize()
    for i, tr in enumerate(alone):
        a, b = cut[i], cut[i + 1]
        assert torch.equal(lt.params[a:b], tr.params), f"lane {i} params"
        assert torch.equal(lt.bufs[a:b], tr.bufs), f"lane {i} BN buffers"
        assert torch.equal(lt.acc_loss[a:b], tr.acc_loss)
        assert torch.equal(lt.acc_correct[a:b], tr.acc_correct)
    assert len(lt.lanes) == 3 and all(len(ln._graphs) > 0 for ln in lt.lanes[:2])
    assert lt.fill == [0.25, 0.75, 0.5]  # isolated client, widest lane, the rest
    # the lanes replayed libfedhip-recorded step programs (csrc/program.hip), each one
    # verified complete against its captured graph — not the graph fallback
    for ln in lt.lanes:
        assert ln.launch_mode == "program"
        for graph, prog in ln._graphs.values():
            assert prog is not None and prog.kernels >= 10 and prog.complete_for(graph)
    for ln in lt.lanes:
        ln.release_graphs()
    assert all(not ln._graphs for ln in lt.lanes)


def test_program_replays_graph_bit_for_bit():
    """One trainer, every step after the first replayed as a recorded program vs as the
    captured graph: same kernels, same arguments -> identical parameters / buffers."""
    sizes = [96, 70, 40]
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("cifar10_cnn", dropout_rate=0.3).to(DEV)
    data, labels, offs = _data(sizes, (3, 32, 32))
    out = []
    for mode in ("graph", "program"):
        tr = PackedTrainer(model, len(sizes), batch=32, device=DEV)
        tr.launch_mode = mode
        for k in range(len(sizes)):
            tr.load_module_state(k, model)
        gen = torch.Generator().manual_seed(3)
        plan = tr.make_plan(sizes, 1, generator=gen)
        tr.run_round(data, labels, offs, plan, optimizer_type="adam", lr=1e-3, seed=4)
        torch.cuda.synchronize()
        progs = [p for _, p in tr._graphs.values()]
        assert progs and all((p is not None) == (mode == "program") for p in progs)
        out.append((tr.params.clone(), tr.bufs.clone(), tr.acc_loss.clone()))
        tr.release_graphs()
    for a, b in zip(*out):
        assert torch.equal(a, b)

