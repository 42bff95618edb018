"""§8f-4 on the GPU: convergence weight-change norms computed on the chip vs the
reference's values (golden G9), and the packed <-> weight-dict edge round trip."""
import json
import os

import pytest
import torch

from fedhip import wire
from fedhip.net import ParamLayout
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                   "golden.json")))


def _flat(name, seed):
    torch.manual_seed(seed)
    m = hm.ModelFactory.create_model(name)
    return ParamLayout.from_module(m), torch.cat([p.detach().reshape(-1) for p in m.parameters()])


@pytest.mark.parametrize("name", ["simple_cnn", "cifar10_cnn"])
def test_weight_change_metrics_vs_reference(name):
    g = GOLD[f"G9/weight_change_{name}"]
    L, a = _flat(name, g["seeds"][0])
    _, b = _flat(name, g["seeds"][1])
    seg = torch.tensor(L.seg_offsets(), dtype=torch.int64, device=DEV)
    res = wire.weight_change_metrics(a.to(DEV), b.to(DEV), seg)
    # the chip accumulates in fp64; torch's CPU fp32 norm accumulates in fp32 (cascade sum
    # over up to 1M elements): measured 1.6e-6 relative on SimpleCNN.  Tolerance 1e-5.
    assert abs(res["norm"] - g["norm"]) <= 1e-5 * g["norm"]
    assert abs(res["relative"] - g["relative"]) <= 1e-5 * g["relative"]


def test_packed_edge_round_trip():
    L, a = _flat("cifar10_cnn", 0)
    _, b = _flat("cifar10_cnn", 1)
    Ppad = (L.P + 63) // 64 * 64
    rows = torch.zeros(2, Ppad, device=DEV)
    rows[0, :L.P], rows[1, :L.P] = a.to(DEV), b.to(DEV)
    dicts = wire.packed_to_weight_dicts(rows, L, 2)
    assert list(dicts[0]) == L.names
    back = wire.weight_dicts_to_packed(dicts, L, DEV)
    assert torch.equal(back, rows)
