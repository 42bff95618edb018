"""One federated round on one GPU rank: local training -> update-level DP -> FedAvg.

Reference control flow replaced (per round):
  FederatedTrainer._perform_local_training  src/client/federated_trainer.py:390-426
  FederatedTrainer._apply_differential_privacy  :428-469
  FederatedLearningServicer._perform_aggregation  src/coordinator/grpc_server.py:465-506
    -> FedAvgAggregator.aggregate_updates  src/aggregation/fedavg.py:56-124

Multi-GPU (one process per GPU, torch.distributed over RCCL): clients are
LPT-assigned to ranks by sample count; each rank trains its clients as one
packed job, forms its partial FedAvg sum  S_r = sum_{k in r} fl32(w_k) x_k
(w_k = n_k / sum_all n, host double, client-list order inside the rank), and
one all_reduce(SUM) of the P-float vector over xGMI yields the new global
model on every rank (no broadcast needed).  With one rank the sum is the
reference's sequential loop, bit for bit.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from . import ops
from .lanes import LanedTrainer


@dataclass
class DPConfig:
    epsilon: float
    delta: float = 1e-5
    max_grad_norm: float = 1.0


class RankRound:
    def __init__(self, template_model, all_train_sizes: Sequence[int], my_clients: Sequence[int],
                 epochs: int = 1, batch: int = 32, device="cuda", dp: Optional[DPConfig] = None,
                 group=None, lanes=None):
        self.device = torch.device(device)
        self.B, self.epochs, self.dp, self.group = batch, epochs, dp, group
        self.all_sizes = list(all_train_sizes)
        # slots: this rank's clients ordered by descending step count (stable)
        self.clients = sorted(my_clients)
        self.slots = sorted(self.clients, key=lambda k: (-math.ceil(self.all_sizes[k] / batch), k))
        self.slot_of = {k: i for i, k in enumerate(self.slots)}
        steps = [epochs * math.ceil(self.all_sizes[k] / batch) for k in self.slots]
        self.trainer = LanedTrainer(template_model, steps or [0], batch=batch, device=self.device,
                                    lanes=lanes)
        L = self.trainer.layout
        self.P = L.P
        self.global_flat = torch.zeros(self.P, device=self.device)
        with torch.no_grad():
            for n, p in template_model.named_parameters():
                L.view(self.global_flat.view(1, -1), n)[0].copy_(p.detach().reshape(-1))
        # FedAvg weights: samples_processed = epochs * train size (federated_trainer.py:481),
        # w_k = n_k / sum(n) in Python double (fedavg.py:255), rounded to fp32 at the multiply.
        processed = [epochs * n for n in self.all_sizes]
        total = sum(processed)
        self.weights = [n / total for n in processed]
        self.w32 = torch.tensor([self.weights[k] for k in self.clients], dtype=torch.float32,
                                device=self.device)
        self.rows = torch.tensor([self.slot_of[k] for k in self.clients], dtype=torch.int32,
                                 device=self.device)
        self.partial = torch.zeros(self.P, device=self.device)
        self.round_index = 0

    def set_global(self, flat: torch.Tensor):
        self.global_flat.copy_(flat)

    def run(self, data, labels, slot_offsets: Sequence[int], optimizer_type="sgd", lr=0.01,
            seed=0, generator=None):
        """One round. data/labels: this rank's train shards, slot k's at slot_offsets[k]."""
        tr = self.trainer
        S = len(self.slots)
        tr.params[:S, :self.P].copy_(self.global_flat.expand(S, -1))  # all start from global
        sizes = [self.all_sizes[k] for k in self.slots]
        plan = tr.make_plan(sizes, self.epochs, generator=generator)
        metrics = tr.run_round(data, labels, slot_offsets, plan, optimizer_type=optimizer_type,
                               lr=lr, seed=seed)
        if self.dp is not None:
            self._apply_dp(S, seed)
        # FedAvg: this rank's partial sum in client-list order, then RCCL all-reduce.
        ops.fedavg_weighted_sum(tr.params, self.w32, self.partial, row_index=self.rows, P=self.P)
        if self.group is not None or (dist.is_available() and dist.is_initialized()):
            dist.all_reduce(self.partial, op=dist.ReduceOp.SUM, group=self.group)
        self.global_flat.copy_(self.partial)
        self.round_index += 1
        return metrics

    def _apply_dp(self, S, seed):
        """federated_trainer.py:434-462 for every client at once (budget bookkeeping is the
        caller's: privacy.py's tracker is host state)."""
        tr, dp = self.trainer, self.dp
        sq = ops.dp_delta_sqnorm(tr.params, self.global_flat.view(1, -1).expand(S, -1),
                                 tr.seg_offsets, S)
        total, coef, clipped, sigma = ops.dp_clip_coef(sq, dp.max_grad_norm, dp.epsilon, dp.delta)
        g = self.global_flat.view(1, -1).expand(S, -1)
        ops.dp_apply(tr.params, g, tr.params, coef, clipped, sigma, P=self.P,
                     seed=(seed * 6364136223846793005 + 1442695040888963407) & ((1 << 64) - 1))
        self.last_dp = (total, clipped, sigma)
