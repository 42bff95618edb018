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


def validate_update(client_id, round_number, num_samples, training_loss, budget, compression,
                    layers, max_weight_magnitude=10.0, min_samples=1):
    """ModelUpdateValidator.validate_model_update (validation.py:28-111), timestamps excluded.
    layers: list of fp32 arrays. Returns True/False (the aggregator swallows the exception)."""
    if not client_id or not isinstance(client_id, str) or round_number < 0:
        return False
    if num_samples < min_samples or training_loss < 0:
        return False
    if not layers:
        return False
    for a in layers:
        a = np.asarray(a, np.float32)
        if np.isnan(a).any() or np.isinf(a).any():
            return False
        if np.abs(a).max() > max_weight_magnitude:
            return False
    if not (0 <= budget <= 1) or not (0 <= compression <= 1):
        return False
    return True


def filter_updates(updates, validate=True):
    """fedavg.py:209-245 on dicts with keys client_id, num_samples, training_loss, budget,
    compression, round, layers (list). Shape-compatibility pass keeps every update whose
    layer shapes match the first survivor's (the reference's pop-while-iterating bug,
    fedavg.py:236-243, is NOT reproduced; see DESIGN.md divergence D6)."""
    out = []
    for u in updates:
        if u["num_samples"] <= 0 or u["training_loss"] < 0:
            continue
        if validate and not validate_update(u["client_id"], u.get("round", 0), u["num_samples"],
                                            u["training_loss"], u["budget"], u["compression"],
                                            u["layers"]):
            continue
        out.append(u)
    if len(out) > 1:
        ref = [np.shape(a) for a in out[0]["layers"]]
        out = [out[0]] + [u for u in out[1:] if [np.shape(a) for a in u["layers"]] == ref]
    return out
