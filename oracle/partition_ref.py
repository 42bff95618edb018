"""Client data partitioning restated (host-side index bookkeeping) — ORACLE.

Reference: src/shared/data_loader.py DataPartitioner
  _create_iid_partitions            :118-137
  _create_non_iid_partitions        :139-177  (Dirichlet per class)
  _create_pathological_partitions   :179-237
Consumes Python `random` and `numpy.random` global state in exactly the
reference's order, so with the same seeds the index lists are identical
(pinned by golden G6).
"""
from __future__ import annotations

import random
from collections import defaultdict

import numpy as np


def iid(n, num_clients):
    indices = list(range(n))
    random.shuffle(indices)
    per = n // num_clients
    out = {}
    for c in range(num_clients):
        s = c * per
        e = n if c == num_clients - 1 else s + per
        out[c] = indices[s:e]
    return out


def non_iid(labels, num_clients, alpha, min_samples=10):
    class_indices = defaultdict(list)
    for i, l in enumerate(labels):
        class_indices[l].append(i)
    out = defaultdict(list)
    for _, idx in class_indices.items():
        prop = np.random.dirichlet([alpha] * num_clients)
        prop = np.maximum(prop, min_samples / len(idx))
        prop = prop / prop.sum()
        np.random.shuffle(idx)
        s = 0
        for c in range(num_clients):
            k = int(prop[c] * len(idx))
            e = len(idx) if c == num_clients - 1 else s + k
            out[c].extend(idx[s:e])
            s = e
    for c in out:
        random.shuffle(out[c])
    return dict(out)


def pathological(labels, num_clients, min_samples=10):
    n = len(labels)
    num_classes = len(set(labels))
    class_indices = defaultdict(list)
    for i, l in enumerate(labels):
        class_indices[l].append(i)
    out = defaultdict(list)
    cpc = max(1, num_classes // num_clients)
    class_list = list(class_indices.keys())
    random.shuffle(class_list)
    assign = {}
    for c in range(num_clients):
        start = (c * cpc) % num_classes
        assign[c] = [class_list[(start + i) % num_classes] for i in range(cpc)]
    for c, classes in assign.items():
        for cl in classes:
            idx = class_indices[cl].copy()
            random.shuffle(idx)
            share = len(idx) // sum(1 for _, cs in assign.items() if cl in cs)
            out[c].extend(idx[:share])
    for c in range(num_clients):
        if len(out[c]) < min_samples:
            used = set()
            for v in out.values():
                used.update(v)
            avail = list(set(range(n)) - used)
            need = min_samples - len(out[c])
            if avail:
                out[c].extend(random.sample(avail, min(need, len(avail))))
    return dict(out)


def partition(labels, num_clients, strategy="iid", alpha=0.5, min_samples=10):
    labels = [int(l) for l in labels]
    if strategy == "iid":
        return iid(len(labels), num_clients)
    if strategy == "non_iid":
        return non_iid(labels, num_clients, alpha, min_samples)
    if strategy == "pathological":
        return pathological(labels, num_clients, min_samples)
    raise ValueError(f"Unknown partition strategy: {strategy}")
