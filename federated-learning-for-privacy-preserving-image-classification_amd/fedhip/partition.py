"""Client shard bookkeeping: DataPartitioner semantics, bit-exact.

Reference: src/shared/data_loader.py:65-237 (DataPartitioner: iid, Dirichlet
non-iid, pathological) and :343-351 (per-client 90/10 train/validation
random_split).  Index lists depend on Python ``random`` and ``numpy.random``
global state; this module draws from them in the reference's exact order, so
with the same seeds every client receives the same sample indices (pinned by
tests against golden G6).  Host-side integer work only.
"""
from __future__ import annotations

import random
from collections import defaultdict
from typing import Dict, List, Sequence

import numpy as np
import torch


def _by_class(labels: Sequence[int]):
    groups = defaultdict(list)
    for i, lab in enumerate(labels):
        groups[lab].append(i)
    return groups


def partition(labels: Sequence[int], num_clients: int, strategy: str = "iid", alpha: float = 0.5,
              min_samples_per_client: int = 10) -> Dict[int, List[int]]:
    labels = [int(v) for v in labels]
    n = len(labels)
    if strategy == "iid":
        order = list(range(n))
        random.shuffle(order)
        share = n // num_clients
        cuts = [c * share for c in range(num_clients)] + [n]
        return {c: order[cuts[c]:(cuts[c + 1] if c < num_clients - 1 else n)]
                for c in range(num_clients)}
    if strategy == "non_iid":
        shards = defaultdict(list)
        for _, members in _by_class(labels).items():
            p = np.random.dirichlet([alpha] * num_clients)
            p = np.maximum(p, min_samples_per_client / len(members))
            p = p / p.sum()
            np.random.shuffle(members)
            start = 0
            for c in range(num_clients):
                stop = len(members) if c == num_clients - 1 else start + int(p[c] * len(members))
                shards[c].extend(members[start:stop])
                start = stop
        for c in shards:
            random.shuffle(shards[c])
        return dict(shards)
    if strategy == "pathological":
        groups = _by_class(labels)
        ncls = len(set(labels))
        per = max(1, ncls // num_clients)
        classes = list(groups.keys())
        random.shuffle(classes)
        owned = {c: [classes[((c * per) % ncls + i) % ncls] for i in range(per)]
                 for c in range(num_clients)}
        shards = defaultdict(list)
        for c, cs in owned.items():
            for cl in cs:
                pool = groups[cl].copy()
                random.shuffle(pool)
                k = len(pool) // sum(1 for _, o in owned.items() if cl in o)
                shards[c].extend(pool[:k])
        for c in range(num_clients):
            if len(shards[c]) < min_samples_per_client:
                used = set()
                for v in shards.values():
                    used.update(v)
                spare = list(set(range(n)) - used)
                if spare:
                    shards[c].extend(random.sample(spare, min(min_samples_per_client - len(shards[c]),
                                                              len(spare))))
        return dict(shards)
    raise ValueError(f"Unknown partition strategy: {strategy}")


def train_split_sizes(shard_sizes: Sequence[int], validation_split: float = 0.1) -> List[int]:
    """data_loader.py:345-351: train = n - int(n * validation_split)."""
    return [n - int(n * validation_split) for n in shard_sizes]


def train_split(indices: Sequence[int], validation_split: float = 0.1, generator=None):
    """torch.utils.data.random_split(client_dataset, [train, val]) index semantics."""
    n = len(indices)
    val = int(n * validation_split)
    perm = torch.randperm(n, generator=generator).tolist()
    idx = list(indices)
    return [idx[i] for i in perm[:n - val]], [idx[i] for i in perm[n - val:]]


def lpt_assign(sizes: Sequence[int], bins: int) -> List[List[int]]:
    """Longest-processing-time assignment of clients to GPUs (by sample count)."""
    order = sorted(range(len(sizes)), key=lambda i: (-sizes[i], i))
    load = [0] * bins
    out: List[List[int]] = [[] for _ in range(bins)]
    for i in order:
        b = min(range(bins), key=lambda j: (load[j], j))
        out[b].append(i)
        load[b] += sizes[i]
    return out


def _steps(n: int, epochs: int, batch: int) -> int:
    return epochs * -(-n // batch)


def rank_time_model(steps: Sequence[int], ratio: float) -> float:
    """Modelled round time of one rank (in units of one client-step of packed work): its
    clients' local epochs are dependent SGD chains, so the rank cannot finish before its
    longest chain (ratio x that chain's steps: a chain step is latency-bound) nor before its
    total client-steps are through (the packed / concurrent-lane throughput term)."""
    return ratio * max(steps, default=0) + sum(steps)


def chain_assign(sizes: Sequence[int], bins: int, epochs: int = 1, batch: int = 32,
                 ratio: float = 0.0) -> List[List[int]]:
    """Client -> rank assignment for a FIXED client set (strong scaling, r06).  Plain LPT
    balances images, but a Dirichlet shard's local steps are a dependent chain: the rank holding
    the longest client pays that chain's latency whatever else it holds (KT at 8 GPUs: the
    131-step client plus two more, 61.4 ms, against 39-48 ms for the other ranks).  With
    ratio > 0 clients go, in descending steps, to the rank whose modelled time
    (rank_time_model) after adding them is least — the long chain's rank then takes little
    else; the result is kept only if its modelled makespan beats LPT's.  ratio = per-step
    chain latency / per-client-step packed cost, fitted per model on MI355X (bench.CONFIGS
    `chain_ratio`, profiles/r06_strong/)."""
    base = lpt_assign(sizes, bins)
    if ratio <= 0 or bins <= 1:
        return base
    st = [_steps(n, epochs, batch) for n in sizes]
    order = sorted(range(len(sizes)), key=lambda i: (-st[i], -sizes[i], i))
    out: List[List[int]] = [[] for _ in range(bins)]
    longest = [0] * bins
    total = [0] * bins
    for i in order:
        b = min(range(bins), key=lambda j: (ratio * max(longest[j], st[i]) + total[j] + st[i],
                                            total[j], j))
        out[b].append(i)
        longest[b] = max(longest[b], st[i])
        total[b] += st[i]
    span = lambda a: max(rank_time_model([st[k] for k in r], ratio) for r in a)
    return out if span(out) < span(base) else base
