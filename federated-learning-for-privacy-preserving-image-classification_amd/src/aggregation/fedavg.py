"""FedAvg aggregation with the reference's API; the weighted sum runs on HIP.

Reference: src/aggregation/fedavg.py — FedAvgAggregator (:25-357),
AdaptiveFedAvg (:360-467), create_fedavg_aggregator (:470-484).

The arithmetic of _weighted_average (:267-289) — zeros, then for each client
in list order ``acc += fl32(w_k) * x_k`` with a rounded multiply and a
rounded add — is done by fh_fedavg_weighted_sum over all layers at once, bit
for bit.  Filtering, truncation and weights are host bookkeeping with the
reference's semantics, with one deliberate fix: incompatible
updates are all removed (the reference pops by index while iterating a
snapshot and can drop the wrong client).

``aggregate_packed`` is the additive batched entry point used by the
client-packed engine: parameters already resident as [clients, P] rows.
"""
from __future__ import annotations

import logging
from datetime import datetime
from typing import Any, Dict, List, Optional, Sequence

import numpy as np
import torch

from fedhip import ops

from ..shared.interfaces import AggregationServiceInterface
from ..shared.models import GlobalModel, ModelUpdate, ModelWeights
from ..shared.validation import ModelUpdateValidator, validate_model_compatibility

logger = logging.getLogger(__name__)


class FedAvgError(Exception):
    """Any aggregation failure (reference :20-22)."""


class FedAvgAggregator(AggregationServiceInterface):
    def __init__(self, min_clients: int = 2, max_clients: Optional[int] = None,
                 validate_updates: bool = True, device: Optional[torch.device] = None):
        self.min_clients, self.max_clients = min_clients, max_clients
        self.validate_updates = validate_updates
        self.validator = ModelUpdateValidator() if validate_updates else None
        self.aggregation_history: List[Dict[str, Any]] = []
        self.device = torch.device(device) if device is not None else torch.device("cuda")

    # ------------------------------------------------------------------ main API
    def aggregate_updates(self, updates: List[ModelUpdate],
                          weights: Optional[List[float]] = None) -> GlobalModel:
        try:
            t0 = datetime.now()
            self._validate_aggregation_inputs(updates, weights)
            valid = self._filter_and_validate_updates(updates)
            if len(valid) < self.min_clients:
                raise FedAvgError(f"Insufficient valid updates: {len(valid)} < {self.min_clients}")
            if self.max_clients and len(valid) > self.max_clients:
                valid = sorted(valid, key=lambda u: u.num_samples, reverse=True)[:self.max_clients]
            agg_w = self._calculate_sample_weights(valid) if weights is None \
                else self._normalize_weights(weights[:len(valid)])
            out = self._weighted_average(valid, agg_w)
            total = sum(u.num_samples for u in valid)
            avg_loss = sum(u.training_loss * w for u, w in zip(valid, agg_w))
            gm = GlobalModel(round_number=valid[0].round_number, model_weights=out,
                             accuracy_metrics={},
                             participating_clients=[u.client_id for u in valid],
                             convergence_score=0.0, created_at=datetime.now())
            self._record_aggregation_stats(valid, agg_w, total, avg_loss,
                                           (datetime.now() - t0).total_seconds())
            return gm
        except Exception as e:
            logger.error(f"FedAvg aggregation failed: {e}")
            raise FedAvgError(f"FedAvg aggregation failed: {e}") from e

    def aggregate_packed(self, packed: torch.Tensor, num_samples: Sequence[int],
                         row_index: Optional[Sequence[int]] = None,
                         out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Weighted FedAvg of client rows already on the device ([clients, P] fp32).
        Rows are summed in the order of `row_index` (default: row order)."""
        C = len(num_samples)
        if C == 0:
            raise FedAvgError("No updates to aggregate")
        w = self._calculate_sample_weights_n(list(num_samples))
        dev = packed.device
        w32 = torch.tensor(w, dtype=torch.float32, device=dev)
        idx = None if row_index is None else torch.tensor(list(row_index), dtype=torch.int32,
                                                          device=dev)
        if out is None:
            out = torch.empty(packed.shape[1], dtype=torch.float32, device=dev)
        ops.fedavg_weighted_sum(packed, w32, out, row_index=idx)
        return out

    def validate_update(self, update: ModelUpdate) -> bool:
        try:
            if not self.validate_updates or not self.validator:
                return True
            return self.validator.validate_model_update(update)
        except Exception as e:
            logger.error(f"Update validation failed for client {update.client_id}: {e}")
            return False

    def compress_global_model(self, model: GlobalModel) -> bytes:
        import io
        buf = io.BytesIO()
        torch.save({k: v.cpu() for k, v in model.model_weights.items()}, buf)
        return buf.getvalue()

    def calculate_convergence_metrics(self, old_model: GlobalModel,
                                      new_model: GlobalModel) -> float:
        """sum_l ||new_l - old_l|| / sum_l ||new_l||, clamped to [0,1] (reference :144-190);
        both norm vectors come from one fused device pass each."""
        try:
            if not old_model or not new_model:
                return 1.0
            names = [n for n in new_model.model_weights if n in old_model.model_weights]
            if not names:
                return 0.0
            new_row, seg = self._pack([new_model.model_weights[n] for n in names])
            old_row, _ = self._pack([old_model.model_weights[n] for n in names])
            d2 = ops.dp_delta_sqnorm(new_row, old_row, seg, 1)[0]
            n2 = ops.dp_delta_sqnorm(new_row, None, seg, 1)[0]
            diff = float(torch.sqrt(d2.float().double()).sum())
            norm = float(torch.sqrt(n2.float().double()).sum())
            score = diff / norm if norm > 0 else 0.0
            return min(1.0, max(0.0, score))
        except Exception as e:
            logger.error(f"Convergence calculation failed: {e}")
            return 0.0

    # ------------------------------------------------------------------ internals
    def _pack(self, tensors):
        dev = self.device
        flats = [t.detach().to(device=dev, dtype=torch.float32).reshape(-1) for t in tensors]
        offs = [0]
        for f in flats:
            offs.append(offs[-1] + f.numel())
        return torch.cat(flats).view(1, -1), torch.tensor(offs, dtype=torch.int64, device=dev)

    def _validate_aggregation_inputs(self, updates, weights):
        if not updates:
            raise FedAvgError("No model updates provided")
        if weights is not None:
            if len(weights) != len(updates):
                raise FedAvgError("Number of weights must match number of updates")
            if any(w < 0 for w in weights):
                raise FedAvgError("All weights must be non-negative")
            if sum(weights) == 0:
                raise FedAvgError("Sum of weights cannot be zero")

    def _filter_and_validate_updates(self, updates: List[ModelUpdate]) -> List[ModelUpdate]:
        valid = []
        for u in updates:
            try:
                if u.num_samples <= 0:
                    logger.warning(f"Skipping update from {u.client_id}: invalid sample count")
                    continue
                if u.training_loss < 0:
                    logger.warning(f"Skipping update from {u.client_id}: invalid training loss")
                    continue
                if self.validate_updates and not self.validate_update(u):
                    logger.warning(f"Skipping update from {u.client_id}: validation failed")
                    continue
                valid.append(u)
            except Exception as e:
                logger.error(f"Error validating update from {u.client_id}: {e}")
        if len(valid) > 1:
            ref = valid[0].model_weights
            keep = [valid[0]]
            for u in valid[1:]:
                try:
                    validate_model_compatibility(ref, u.model_weights)
                    keep.append(u)
                except Exception as e:
                    logger.warning(f"Removing incompatible update from {u.client_id}: {e}")
            valid = keep
        return valid

    @staticmethod
    def _calculate_sample_weights_n(ns: List[int]) -> List[float]:
        total = sum(ns)
        if total == 0:
            return [1.0 / len(ns)] * len(ns)
        return [n / total for n in ns]

    def _calculate_sample_weights(self, updates: List[ModelUpdate]) -> List[float]:
        return self._calculate_sample_weights_n([u.num_samples for u in updates])

    def _normalize_weights(self, weights: List[float]) -> List[float]:
        total = sum(weights)
        if total == 0:
            return [1.0 / len(weights)] * len(weights)
        return [w / total for w in weights]

    def _weighted_average(self, updates: List[ModelUpdate], weights: List[float]) -> ModelWeights:
        """Device-packed: client rows [C, P] -> one fused FedAvg launch -> layer views.
        Layers missing from update 0 are ignored; layers missing from a later update
        contribute nothing for that client (reference :278-287)."""
        if not updates:
            raise FedAvgError("No updates to aggregate")
        ref = updates[0].model_weights
        names = list(ref)
        sizes = [ref[n].numel() for n in names]
        offs = np.cumsum([0] + sizes).tolist()
        P = offs[-1]
        dev = self.device
        rows = torch.zeros(len(updates), P, dtype=torch.float32, device=dev)
        for k, u in enumerate(updates):
            for n, o, s in zip(names, offs, sizes):
                t = u.model_weights.get(n)
                if t is not None:
                    rows[k, o:o + s].copy_(t.detach().reshape(-1))
            for n in u.model_weights:
                if n not in ref:
                    logger.warning(f"Layer {n} not found in reference model")
        w32 = torch.tensor(weights, dtype=torch.float32, device=dev)
        out = torch.empty(P, dtype=torch.float32, device=dev)
        ops.fedavg_weighted_sum(rows, w32, out)
        return {n: out[o:o + s].view(ref[n].shape).to(ref[n].device)
                for n, o, s in zip(names, offs, sizes)}

    def _record_aggregation_stats(self, updates, weights, total_samples, avg_training_loss,
                                  aggregation_time):
        self.aggregation_history.append({
            "timestamp": datetime.now().isoformat(), "num_clients": len(updates),
            "total_samples": total_samples, "avg_training_loss": avg_training_loss,
            "aggregation_time": aggregation_time,
            "client_weights": {u.client_id: w for u, w in zip(updates, weights)},
            "client_samples": {u.client_id: u.num_samples for u in updates}})
        self.aggregation_history = self.aggregation_history[-100:]

    def get_aggregation_stats(self) -> Dict[str, Any]:
        if not self.aggregation_history:
            return {"message": "No aggregation history available"}
        recent = self.aggregation_history[-10:]
        return {"total_aggregations": len(self.aggregation_history),
                "recent_aggregations": len(recent),
                "avg_clients_per_round": float(np.mean([s["num_clients"] for s in recent])),
                "avg_samples_per_round": float(np.mean([s["total_samples"] for s in recent])),
                "avg_aggregation_time": float(np.mean([s["aggregation_time"] for s in recent])),
                "avg_training_loss": float(np.mean([s["avg_training_loss"] for s in recent])),
                "client_participation": self._calculate_client_participation()}

    def _calculate_client_participation(self) -> Dict[str, Any]:
        counts: Dict[str, int] = {}
        for s in self.aggregation_history:
            for cid in s["client_weights"]:
                counts[cid] = counts.get(cid, 0) + 1
        rounds = len(self.aggregation_history)
        return {"unique_clients": len(counts),
                "avg_participation_rate": float(np.mean(list(counts.values()))) / rounds,
                "most_active_clients": sorted(counts.items(), key=lambda x: x[1],
                                              reverse=True)[:5]}


class AdaptiveFedAvg(FedAvgAggregator):
    """Sample weights blended with a loss-history performance term (reference :360-467)."""

    def __init__(self, min_clients: int = 2, max_clients: Optional[int] = None,
                 validate_updates: bool = True, performance_weight: float = 0.1,
                 device: Optional[torch.device] = None):
        super().__init__(min_clients, max_clients, validate_updates, device)
        self.performance_weight = performance_weight
        self.client_performance_history: Dict[str, Dict[str, Any]] = {}

    def aggregate_updates(self, updates, weights=None):
        try:
            for u in updates:
                h = self.client_performance_history.setdefault(
                    u.client_id, {"losses": [], "sample_counts": [], "participation_count": 0})
                h["losses"] = (h["losses"] + [u.training_loss])[-10:]
                h["sample_counts"] = (h["sample_counts"] + [u.num_samples])[-10:]
                h["participation_count"] += 1
            if weights is None:
                weights = self._calculate_adaptive_weights(updates)
            return super().aggregate_updates(updates, weights)
        except Exception as e:
            raise FedAvgError(f"Adaptive FedAvg aggregation failed: {e}") from e

    def _calculate_adaptive_weights(self, updates):
        base = self._calculate_sample_weights(updates)
        if self.performance_weight == 0:
            return base
        hist = self.client_performance_history
        max_loss = max(h["losses"] for h in hist.values() if h["losses"])
        adj = []
        for u in updates:
            h = hist.get(u.client_id)
            if h is None:
                adj.append(1.0)
                continue
            avg = float(np.mean(h["losses"]))
            adj.append(1.0 - avg / max_loss if max_loss > 0 else 1.0)
        pw = self.performance_weight
        return self._normalize_weights([(1 - pw) * b + pw * a for b, a in zip(base, adj)])


def create_fedavg_aggregator(aggregator_type: str = "standard", **kwargs) -> FedAvgAggregator:
    return AdaptiveFedAvg(**kwargs) if aggregator_type == "adaptive" else FedAvgAggregator(**kwargs)
