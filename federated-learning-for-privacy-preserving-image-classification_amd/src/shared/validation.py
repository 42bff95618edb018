"""Model-update validation (reference src/shared/validation.py:21-111, 256-282).

The per-tensor value checks (NaN, Inf, max |w| <= 10) run as one fused HIP
reduction over all layers of an update (fh_update_stats); field, budget,
compression and timestamp checks are host-side, as in the reference.
"""
from __future__ import annotations

import logging
from datetime import datetime, timedelta
from typing import Dict

import torch

from fedhip import ops

from .models import ModelUpdate

logger = logging.getLogger(__name__)


class ValidationError(Exception):
    """An update failed validation."""


def _layer_stats(weights: Dict[str, torch.Tensor]):
    """(names, max|w| per layer, nonfinite flag per layer) computed on the device."""
    names = list(weights)
    dev = next((t.device for t in weights.values() if t.is_cuda), torch.device("cuda"))
    flats = [weights[n].detach().to(device=dev, dtype=torch.float32).reshape(-1) for n in names]
    offs = [0]
    for f in flats:
        offs.append(offs[-1] + f.numel())
    row = torch.cat(flats).view(1, -1)
    seg = torch.tensor(offs, dtype=torch.int64, device=dev)
    absmax, bad = ops.update_stats(row, seg, 1)
    return names, absmax[0].cpu().tolist(), bad[0].cpu().tolist()


class ModelUpdateValidator:
    def __init__(self, max_weight_magnitude: float = 10.0, min_samples: int = 1):
        self.max_weight_magnitude = max_weight_magnitude
        self.min_samples = min_samples

    def validate_model_update(self, update: ModelUpdate) -> bool:
        """True, or raises ValidationError naming the first failed check."""
        try:
            self._validate_basic_fields(update)
            self._validate_model_weights(update.model_weights)
            self._validate_privacy_and_compression(update)
            self._validate_timestamp(update.timestamp)
            return True
        except Exception as e:
            logger.error(f"Model update validation failed for client {update.client_id}: {e}")
            raise ValidationError(f"Model update validation failed: {e}") from e

    def _validate_basic_fields(self, u: ModelUpdate) -> None:
        if not u.client_id or not isinstance(u.client_id, str):
            raise ValidationError("Client ID must be a non-empty string")
        if u.round_number < 0:
            raise ValidationError("Round number must be non-negative")
        if u.num_samples < self.min_samples:
            raise ValidationError(f"Number of samples must be at least {self.min_samples}")
        if u.training_loss < 0:
            raise ValidationError("Training loss must be non-negative")

    def _validate_model_weights(self, weights: Dict[str, torch.Tensor]) -> None:
        if not weights:
            raise ValidationError("Model weights cannot be empty")
        for n, t in weights.items():
            if not isinstance(t, torch.Tensor):
                raise ValidationError(f"Weight for layer {n} must be a torch.Tensor")
        names, absmax, bad = _layer_stats(weights)
        for n, m, b in zip(names, absmax, bad):
            if b:
                t = weights[n]
                kind = "NaN" if bool(torch.isnan(t).any()) else "Infinite"
                raise ValidationError(f"{kind} values found in layer {n}")
            if m > self.max_weight_magnitude:
                raise ValidationError(f"Weight magnitude {m} exceeds maximum "
                                      f"{self.max_weight_magnitude} in layer {n}")

    def _validate_privacy_and_compression(self, u: ModelUpdate) -> None:
        if not 0 <= u.privacy_budget_used <= 1:
            raise ValidationError("Privacy budget used must be between 0 and 1")
        if not 0 <= u.compression_ratio <= 1:
            raise ValidationError("Compression ratio must be between 0 and 1")

    def _validate_timestamp(self, ts: datetime) -> None:
        now = datetime.now()
        if ts < now - timedelta(hours=24):
            raise ValidationError("Model update timestamp is too old")
        if ts > now + timedelta(minutes=5):
            raise ValidationError("Model update timestamp is in the future")


def validate_model_compatibility(weights1: Dict[str, torch.Tensor],
                                 weights2: Dict[str, torch.Tensor]) -> bool:
    if set(weights1) != set(weights2):
        raise ValidationError("Model compatibility validation failed: "
                              "Model weights have different layer names")
    for n in weights1:
        if weights1[n].shape != weights2[n].shape:
            raise ValidationError(f"Model compatibility validation failed: "
                                  f"Layer {n} has incompatible shapes")
    return True
