"""§8f-2: the on-device input pipeline (fh_gather_u8) against the oracle's restatement
of the reference loaders' torchvision transforms (oracle/data_ref.py).

Bit-exact given the same crop/flip draws (recorded by the kernel); the draws
themselves are checked statistically (uniform offsets, fair flips)."""
import numpy as np
import pytest
import torch

from fedhip import ops
from oracle import data_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda")


@pytest.mark.parametrize("tf,shape", [
    (ops.DataTransform.cifar10(train=True), (32, 32, 3)),
    (ops.DataTransform.cifar10(train=False), (32, 32, 3)),
    (ops.DataTransform.mnist(), (28, 28)),
])
def test_gather_u8_matches_oracle(tf, shape):
    g = torch.Generator().manual_seed(0)
    N, S, B = 500, 3, 32
    data = torch.randint(0, 256, (N, *shape), generator=g, dtype=torch.uint8)
    labels = torch.randint(0, 10, (N,), generator=g)
    idx = torch.randint(0, N, (S, B), generator=g)
    counts = torch.tensor([32, 17, 0], dtype=torch.int32)
    C = 1 if len(shape) == 2 else shape[2]
    x = torch.full((S, B, C, shape[0], shape[1]), -7.0, device=DEV)
    y = torch.full((S, B), -1, dtype=torch.int64, device=DEV)
    aug = torch.zeros(S, B, 4, dtype=torch.uint8, device=DEV)
    ops.gather_u8(data.to(DEV), labels.to(DEV), idx.to(DEV), x, y, tf, S, B,
                  counts=counts.to(DEV), seed=1234, aug_out=aug)
    xs, ys, au = x.cpu().numpy(), y.cpu().numpy(), aug.cpu().numpy()
    for z in range(S):
        for b in range(B):
            if b >= counts[z]:
                assert (xs[z, b] == -7.0).all() and ys[z, b] == -1  # padding untouched
                continue
            i, j, fl = (int(au[z, b, 0]), int(au[z, b, 1]), bool(au[z, b, 2])) if tf.pad or tf.flip \
                else (0, 0, False)
            exp = data_ref.transform(data[idx[z, b]].numpy(), tf.mean, tf.std, tf.pad, i, j, fl)
            assert np.array_equal(xs[z, b].view(np.uint32), exp.view(np.uint32)), (z, b)
            assert ys[z, b] == labels[idx[z, b]]


def test_gather_u8_draws_are_uniform():
    tf = ops.DataTransform.cifar10(train=True)
    S, B = 64, 32
    data = torch.zeros(10, 32, 32, 3, dtype=torch.uint8, device=DEV)
    labels = torch.zeros(10, dtype=torch.int64, device=DEV)
    idx = torch.zeros(S, B, dtype=torch.int64, device=DEV)
    x = torch.empty(S, B, 3, 32, 32, device=DEV)
    aug = torch.zeros(S, B, 4, dtype=torch.uint8, device=DEV)
    ops.gather_u8(data, labels, idx, x, None, tf, S, B, seed=99, aug_out=aug)
    a = aug.cpu().numpy().reshape(-1, 4).astype(np.int64)
    n = a.shape[0]
    for col in (0, 1):
        hist = np.bincount(a[:, col], minlength=9)
        assert hist.shape[0] == 9  # offsets in [0, 8]
        assert np.all(np.abs(hist - n / 9) < 5 * np.sqrt(n / 9))
    assert abs(a[:, 2].mean() - 0.5) < 5 * 0.5 / np.sqrt(n)
    assert not np.array_equal(a[:, 0], a[:, 1])  # independent draws
