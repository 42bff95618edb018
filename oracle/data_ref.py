"""CPU restatement of the reference's per-sample input transforms — TEST ORACLE.

Reference: src/shared/data_loader.py
  :298-306  MNIST train/test: ToTensor + Normalize((0.1307,), (0.3081,))
  :454-463  CIFAR-10 train: RandomCrop(32, padding=4) + RandomHorizontalFlip + ToTensor +
            Normalize((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)); test: the last two

The transforms are torchvision's (requirements: torchvision, unpinned), which is
NOT installed in this image: this restates torchvision's published algorithm —
to_tensor: HWC uint8 -> CHW float32 .div(255); normalize: tensor.sub_(mean).div_(std)
with float32 mean/std; RandomCrop(size, padding): constant-0 pad of the uint8 image,
then crop at (i, j) with i, j uniform in [0, 2*padding]; RandomHorizontalFlip: mirror
with probability 0.5 (applied after the crop).  The random draws themselves (torch's
global RNG in loader workers) are not reproducible across implementations: the
oracle takes the (i, j, flip) draws as inputs.  Parity unpinned vs torchvision itself
(no fixture can be generated here); test infrastructure only.
"""
from __future__ import annotations

import numpy as np


def to_tensor(img_hwc: np.ndarray) -> np.ndarray:
    """uint8 HWC (or HW) -> float32 CHW in [0, 1]."""
    a = img_hwc if img_hwc.ndim == 3 else img_hwc[:, :, None]
    return (a.transpose(2, 0, 1).astype(np.float32) / np.float32(255))


def normalize(t_chw: np.ndarray, mean, std) -> np.ndarray:
    m = np.asarray(mean, np.float32)[:, None, None]
    s = np.asarray(std, np.float32)[:, None, None]
    return (t_chw - m) / s


def crop_flip(img_hwc: np.ndarray, pad: int, i: int, j: int, flip: bool) -> np.ndarray:
    a = img_hwc if img_hwc.ndim == 3 else img_hwc[:, :, None]
    H, W = a.shape[:2]
    if pad:
        p = np.zeros((H + 2 * pad, W + 2 * pad, a.shape[2]), a.dtype)
        p[pad:pad + H, pad:pad + W] = a
        a = p[i:i + H, j:j + W]
    if flip:
        a = a[:, ::-1]
    return a


def transform(img_hwc, mean, std, pad=0, i=0, j=0, flip=False):
    """Normalize(ToTensor(RandomHorizontalFlip(RandomCrop(img)))) with given draws."""
    return normalize(to_tensor(crop_flip(img_hwc, pad, i, j, flip)), mean, std)
