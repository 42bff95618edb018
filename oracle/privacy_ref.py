"""Update-level DP restated in numpy/Python doubles.

Reference: src/shared/privacy.py
  GradientClipper.clip_gradients          :107-144
  GaussianNoiseGenerator.generate_noise   :183-219  (sigma formula :209)
  add_noise_to_gradients                  :221-254
  DifferentialPrivacyEngine.add_noise     :284-311
and the caller src/client/federated_trainer.py:434-462 (delta, reconstitution).
"""
from __future__ import annotations

import math

import numpy as np


def tensor_norm_fp32(t):
    """grad.norm().item(): torch's CPU fp32 norm (the reference's own arithmetic), as double."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(t, dtype=np.float32)).norm().item()


def clip(tensors, max_norm):
    """privacy.py:117-140. Returns (clipped list, min(total, max_norm), total, clipped?)."""
    total = 0.0
    for t in tensors:
        total += tensor_norm_fp32(t) ** 2
    total = math.sqrt(total)
    if total > max_norm:
        coef = np.float32(max_norm / total)
        out = [(np.asarray(t, np.float32) * coef).astype(np.float32) for t in tensors]
        was = True
    else:
        out = [np.array(t, dtype=np.float32, copy=True) for t in tensors]
        was = False
    return out, min(total, max_norm), total, was


def sigma(sensitivity, epsilon, delta):
    """privacy.py:209."""
    return sensitivity * math.sqrt(2 * math.log(1.25 / delta)) / epsilon


def add_noise(tensors, noises):
    """privacy.py:244-245 with the noise supplied (the reference draws torch.normal)."""
    return [(np.asarray(t, np.float32) + np.asarray(n, np.float32)).astype(np.float32)
            for t, n in zip(tensors, noises)]


def apply_update_dp(local, global_, max_norm, epsilon, delta, noises):
    """federated_trainer.py:438-459: delta -> clip -> +noise -> global + noisy."""
    deltas = [(np.asarray(l, np.float32) - np.asarray(g, np.float32)).astype(np.float32)
              for l, g in zip(local, global_)]
    clipped, sens, total, was = clip(deltas, max_norm)
    noisy = add_noise(clipped, noises)
    out = [(np.asarray(g, np.float32) + n).astype(np.float32) for g, n in zip(global_, noisy)]
    return out, sens, total, was
