"""FedAvg restated in numpy (bit-exact with the reference's torch CPU loop).

Reference: src/aggregation/fedavg.py
  _calculate_sample_weights  :247-256   w_k = n_k / sum(n)   (Python double)
  _normalize_weights         :258-265
  _weighted_average          :267-289   acc = 0; acc += fl32(w_k) * x_k  (mul-round, add-round)
  aggregate_updates          :56-124    filter -> max_clients truncation -> weights -> average
"""
from __future__ import annotations

import numpy as np


def calculate_sample_weights(num_samples):
    """fedavg.py:247-256."""
    total = sum(num_samples)
    if total == 0:
        return [1.0 / len(num_samples)] * len(num_samples)
    return [n / total for n in num_samples]


def normalize_weights(weights):
    """fedavg.py:258-265."""
    total = sum(weights)
    if total == 0:
        return [1.0 / len(weights)] * len(weights)
    return [w / total for w in weights]


def weighted_average(rows, weights):
    """fedavg.py:267-289 on flat fp32 rows: sequential fl32(w)*x then fl32 add."""
    rows = [np.asarray(r, dtype=np.float32) for r in rows]
    acc = np.zeros_like(rows[0])
    for r, w in zip(rows, weights):
        acc = (acc + (np.float32(w) * r).astype(np.float32)).astype(np.float32)
    return acc


def select_max_clients(num_samples, max_clients):
    """fedavg.py:82-86: stable sort by num_samples descending, keep the first max_clients.
    Returns the kept positions in their new order."""
    order = sorted(range(len(num_samples)), key=lambda i: num_samples[i], reverse=True)
    return order[:max_clients]
