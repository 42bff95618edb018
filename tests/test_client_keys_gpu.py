"""Philox row keys by GLOBAL client id (csrc/fh_common.h philox_row, engine key block): a
client's dropout keep-masks and crop / flip draws depend on (round seed, step, client id)
only — the same whichever clients share its rank, lane or slot (the reference trains each
client in its own process with its own RNG, federated_simulation.py:309-318).
The trained weights are not compared across layouts: split-K plans follow the number of
packed clients, so their fp32 summation order does."""
import numpy as np
import pytest
import torch

from fedhip import ops
from fedhip.round import RankRound
from src.shared import models_pytorch as hm

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")
SIZES = [40, 70, 33, 64, 45]  # steps 2, 3, 2, 2, 2 at batch 32


def _draws(my_clients, lanes):
    """Per step: {client: (keep-masks of every dropout site, crop/flip draws)}."""
    torch.manual_seed(0)
    model = hm.ModelFactory.create_model("cifar10_cnn").to(DEV)
    assert model.dropout_rate > 0
    rr = RankRound(model, SIZES, my_clients, device=DEV, lanes=lanes, shuffle_seed=5,
                   transform=ops.DataTransform.cifar10(train=True))
    g = torch.Generator().manual_seed(3)
    imgs = {k: torch.randint(0, 256, (n, 32, 32, 3), generator=g, dtype=torch.uint8)
            for k, n in enumerate(SIZES)}
    labs = {k: torch.randint(0, 10, (n,), generator=g) for k, n in enumerate(SIZES)}
    data = torch.cat([imgs[k] for k in rr.slots]).to(DEV)
    labels = torch.cat([labs[k] for k in rr.slots]).to(DEV)
    offs = np.cumsum([0] + [SIZES[k] for k in rr.slots][:-1]).tolist()
    out = []
    for i, ln in enumerate(rr.trainer.lanes):
        ln.aug_record = torch.zeros(ln.capacity, 32, 4, dtype=torch.uint8, device=DEV)
        ids = rr.slots[rr.trainer.cut[i]:rr.trainer.cut[i + 1]]

        def on_step(e, n, ids=ids, step=[0]):
            rec = {ids[r]: ([b[r].cpu().clone() for b in e.net.mask_buffers()],
                            e.aug_record[r].cpu().clone()) for r in range(n)}
            out.append((step[0], rec))
            step[0] += 1
        ln.on_step = on_step
    rr.run(data, labels, offs, "sgd", 0.01, seed=11)
    torch.cuda.synchronize()
    per = {}
    for g_, rec in out:
        for k, v in rec.items():
            per[(g_, k)] = v
    return per


def test_dropout_and_augmentation_follow_the_client_not_its_slot():
    a = _draws([0, 1, 2, 3, 4], lanes=1)       # five clients packed in one lane
    b = _draws([3, 2], lanes=1)                # two of them, other slots
    c = _draws([4, 1, 2, 3, 0], lanes=3)       # the five over concurrent lanes
    shared = [key for key in b if key in a]
    assert len(shared) >= 4
    for key in shared:
        (ma, ua), (mb, ub) = a[key], b[key]
        assert all(torch.equal(x, y) for x, y in zip(ma, mb)), key
        assert torch.equal(ua, ub), key
    for key in a:
        (ma, ua), (mc, uc) = a[key], c[key]
        assert all(torch.equal(x, y) for x, y in zip(ma, mc)), key
        assert torch.equal(ua, uc), key
    # and two clients at the same step never share a stream
    m0, m1 = a[(0, 0)][0], a[(0, 1)][0]
    assert not all(torch.equal(x, y) for x, y in zip(m0, m1))
