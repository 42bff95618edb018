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
reference's sequential loop, bit for bit.  With more ranks the association of
the all-reduce differs from that loop by a few ulp; ``exact=True`` instead
all-gathers every client's row and runs the sequential FedAvg kernel over all
clients in global client order on every rank (fedavg.py:278-285 bit for bit, at
C x P floats of gather traffic per rank instead of one P-float all-reduce).
"""
from __future__ import annotations

import math
import os
import secrets
import sys
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist

from . import ops
from .lanes import HOST_TIMING as _HOST_TIMING  # diagnostics: per-round host split
from .lanes import LanedTrainer


@dataclass
class DPConfig:
    epsilon: float
    delta: float = 1e-5
    max_grad_norm: float = 1.0


class RankRound:
    def __init__(self, template_model, all_train_sizes: Sequence[int], my_clients: Sequence[int],
                 epochs: int = 1, batch: int = 32, device="cuda", dp: Optional[DPConfig] = None,
                 group=None, lanes=None, compression=None, transform=None, dp_seed=None,
                 shuffle_seed=None, exact=False):
        self.device = torch.device(device)
        self._template = template_model
        self.B, self.epochs, self.dp, self.group = batch, epochs, dp, group
        self.all_sizes = list(all_train_sizes)
        # slots: this rank's clients ordered by descending step count (stable)
        self.clients = sorted(my_clients)
        self.slots = sorted(self.clients, key=lambda k: (-math.ceil(self.all_sizes[k] / batch), k))
        self.slot_of = {k: i for i, k in enumerate(self.slots)}
        steps = [epochs * math.ceil(self.all_sizes[k] / batch) for k in self.slots]
        self.distributed = group is not None or (dist.is_available() and dist.is_initialized())
        self.rank = dist.get_rank(group) if self.distributed else 0
        self.trainer = LanedTrainer(template_model, steps or [0], batch=batch, device=self.device,
                                    lanes=lanes, salt=self.rank)
        if self.slots:  # dropout / augmentation keyed by global client id (not rank / lane)
            self.trainer.set_client_ids(self.slots)
        self.transform = transform  # ops.DataTransform when the shards are raw uint8 images
        self.trainer.transform = transform
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
        # update-level DP noise: Philox keyed by (round key, global client id, element), so
        # no two clients — on any rank or lane — ever draw the same noise; the round key
        # comes from a secret base seed (os.urandom) unless the caller fixes one (tests /
        # reproducible benchmarks: a public seed makes the noise recomputable, i.e. no
        # privacy)
        self.slot_ids = torch.tensor(list(self.slots), dtype=torch.int64, device=self.device)
        self.dp_seed = secrets.randbits(63) if dp_seed is None else int(dp_seed)
        # data shuffling when run() gets no generator: every client draws its epochs'
        # permutations from its own generator keyed by (shuffle seed, round seed, client
        # id) — independent of the rank / lane / slot it lands on
        self.shuffle_seed = secrets.randbits(62) if shuffle_seed is None else int(shuffle_seed)
        self.partial = torch.zeros(self.P, device=self.device)
        # global BN running statistics for evaluation (f-1; divergence D13): FedAvg of the
        # clients' buffers with the same weights.  Clients keep their own buffers (D4).
        self.Q = L.Q
        self.global_bufs = torch.zeros(max(self.Q, 1), device=self.device)
        with torch.no_grad():
            for n, b in template_model.named_buffers():
                if n in L.buf_names:
                    L.bview(self.global_bufs.view(1, -1), n)[0].copy_(b.detach().reshape(-1))
        self.round_index = 0
        self._evaluator = None
        # test / diagnostic hooks: on_trained(params, S) sees the trained rows before DP /
        # compression / FedAvg; dp_noise [S, P] replaces the Philox draw (exact replay)
        self.on_trained = None
        self.dp_noise = None
        self.last_plan = None
        # update compression before FedAvg (f-3; insertion point D14): delta vs the global
        self.compression = compression
        self._cplan = None
        if compression is not None:
            from .compress import SegmentPlan
            self._cplan = SegmentPlan(L.seg_offsets(), self.device)
        self.exact = bool(exact) and self.distributed
        if self.exact:
            self._init_exact()

    def _init_exact(self):
        """Exact-mode FedAvg layout: every rank's client list (host, once), rows padded to
        the largest rank's count, and the gather position of each global client."""
        world = dist.get_world_size(self.group)
        lists = [None] * world
        dist.all_gather_object(lists, list(self.clients), group=self.group)
        maxS = max(1, max(len(c) for c in lists))
        pos = {}
        for r, cl in enumerate(lists):
            for i, k in enumerate(cl):
                if k in pos:  # the all-reduce path would count it twice, this one once
                    raise ops.FedHipError(f"exact FedAvg: client {k} is listed by more than "
                                          f"one rank")
                pos[k] = r * maxS + i
        order = sorted(pos)  # global client order: the reference's sequential loop
        if order != list(range(len(self.all_sizes))):
            raise ops.FedHipError(f"exact FedAvg: the ranks' client lists cover {len(order)} "
                                  f"of {len(self.all_sizes)} clients")
        self._x_world, self._x_maxS = world, maxS
        self._x_w32 = torch.tensor([self.weights[k] for k in order], dtype=torch.float32,
                                   device=self.device)
        self._x_idx = torch.tensor([pos[k] for k in order], dtype=torch.int32, device=self.device)
        self._x_mine = torch.tensor([self.slot_of[k] for k in self.clients], dtype=torch.int64,
                                    device=self.device)
        self._x_buf = {}

    def _exact_fedavg(self, rows, n, out):
        """out = sum over ALL clients, in global client order, of fl32(w_k) * row_k: this
        rank's rows (client-list order, zero padded) all-gathered, then fh_fedavg_weighted_sum."""
        world, maxS = self._x_world, self._x_maxS
        buf = self._x_buf.get(n)
        if buf is None:
            buf = self._x_buf[n] = (torch.zeros(maxS, n, device=self.device),
                                    torch.empty(world, maxS, n, device=self.device))
        send, recv = buf
        S = len(self.clients)
        if S:
            torch.index_select(rows[:, :n], 0, self._x_mine, out=send[:S])
        dist.all_gather(list(recv.unbind(0)), send, group=self.group)
        ops.fedavg_weighted_sum(recv.view(world * maxS, n), self._x_w32, out,
                                row_index=self._x_idx, P=n)

    def client_shuffle_seed(self, seed: int, client: int) -> int:
        """Seed of the torch.Generator client `client` draws its round-`seed` batch
        permutations from (one torch.randperm per local epoch, fedhip/engine.plan_round)."""
        return (self.shuffle_seed * 0x9E3779B97F4A7C15 + seed * 0xBF58476D1CE4E5B9
                + client * 0x94D049BB133111EB) & 0x7FFFFFFFFFFFFFFF

    def set_global(self, flat: torch.Tensor):
        self.global_flat.copy_(flat)

    def run(self, data, labels, slot_offsets: Sequence[int], optimizer_type="sgd", lr=0.01,
            seed=0, generator=None, serialize_lanes=False):
        """One round. data/labels: this rank's train shards, slot k's at slot_offsets[k]."""
        tr = self.trainer
        S = len(self.slots)
        _t = [time.perf_counter()] if _HOST_TIMING else None
        tr.params[:S, :self.P].copy_(self.global_flat.expand(S, -1))  # all start from global
        sizes = [self.all_sizes[k] for k in self.slots]
        cseeds = None
        if generator is None:
            cseeds = [self.client_shuffle_seed(seed, k) for k in self.slots]
        plan = tr.make_plan(sizes, self.epochs, generator=generator, client_seeds=cseeds)
        self.last_plan = plan
        if _t:
            _t.append(time.perf_counter())
        metrics = tr.run_round(data, labels, slot_offsets, plan, optimizer_type=optimizer_type,
                               lr=lr, seed=seed, serialize=serialize_lanes)
        if _t:
            _t.append(time.perf_counter())
        if self.on_trained is not None:
            self.on_trained(tr.params, S)
        if self.dp is not None:
            self._apply_dp(S, seed)
        if self.compression is not None:
            from .compress import compress_rows
            compress_rows(self._cplan, self.compression, tr.params, S,
                          base=self.global_flat.view(1, -1).expand(S, -1))
        distributed = self.distributed
        if self.exact:  # bit-exact multi-rank FedAvg: all-gather + one sequential sum
            self._exact_fedavg(tr.params, self.P, self.global_flat)
            if self.Q:
                self._exact_fedavg(tr.bufs, self.Q, self.global_bufs)
            self.round_index += 1
            self._host_timing(_t)
            return metrics
        # FedAvg: this rank's partial sum in client-list order, then RCCL all-reduce.
        ops.fedavg_weighted_sum(tr.params, self.w32, self.partial, row_index=self.rows, P=self.P)
        if distributed:
            dist.all_reduce(self.partial, op=dist.ReduceOp.SUM, group=self.group)
        self.global_flat.copy_(self.partial)
        if self.Q:
            ops.fedavg_weighted_sum(tr.bufs, self.w32, self.global_bufs, row_index=self.rows,
                                    P=self.Q)
            if distributed:
                dist.all_reduce(self.global_bufs, op=dist.ReduceOp.SUM, group=self.group)
        self.round_index += 1
        self._host_timing(_t)
        return metrics

    def _host_timing(self, _t):
        if _t:
            torch.cuda.synchronize(self.device)
            _t.append(time.perf_counter())
            print("round host ms: plan %.1f, run_round %.1f, dp/fedavg+sync %.1f" % tuple(
                1e3 * (b - a) for a, b in zip(_t, _t[1:])), file=sys.stderr)

    def evaluate(self, data, labels, template_model=None):
        """Eval-mode metrics of the current global model on a device-resident test set
        (fedhip/evaluate.py; LocalTrainer.evaluate_model's keys + 'loss')."""
        if self._evaluator is None:
            from .evaluate import GlobalEvaluator
            self._evaluator = GlobalEvaluator(template_model or self._template, self.device)
        return self._evaluator.evaluate(self.global_flat, self.global_bufs, data, labels,
                                        transform=self.transform)

    def _apply_dp(self, S, seed):
        """federated_trainer.py:434-462 for every client at once (budget bookkeeping is the
        caller's: privacy.py's tracker is host state)."""
        tr, dp = self.trainer, self.dp
        sq = ops.dp_delta_sqnorm(tr.params, self.global_flat.view(1, -1).expand(S, -1),
                                 tr.seg_offsets, S)
        total, coef, clipped, sigma = ops.dp_clip_coef(sq, dp.max_grad_norm, dp.epsilon, dp.delta)
        g = self.global_flat.view(1, -1).expand(S, -1)
        key = (self.dp_seed * 6364136223846793005 + seed * 1442695040888963407
               + self.round_index) & ((1 << 64) - 1)
        ops.dp_apply(tr.params, g, tr.params, coef, clipped, sigma, P=self.P, seed=key,
                     row_ids=self.slot_ids[:S], noise=self.dp_noise)
        self.last_dp = (total, clipped, sigma)
