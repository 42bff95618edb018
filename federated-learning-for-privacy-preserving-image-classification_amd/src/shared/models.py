"""Boundary records of the local-training / aggregation path.

Field names and meanings are the reference's (src/shared/models.py:20-97), so
objects built by the existing coordinator / client code are accepted as-is.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from datetime import datetime
from typing import Dict, List, Optional

import torch

ModelWeights = Dict[str, torch.Tensor]


@dataclass
class PrivacyConfig:
    epsilon: float
    delta: float
    max_grad_norm: float
    noise_multiplier: float

    def __post_init__(self):
        checks = [(self.epsilon > 0, "Epsilon must be positive"),
                  (0 <= self.delta < 1, "Delta must be in [0, 1)"),
                  (self.max_grad_norm > 0, "Max gradient norm must be positive"),
                  (self.noise_multiplier >= 0, "Noise multiplier must be non-negative")]
        for ok, msg in checks:
            if not ok:
                raise ValueError(msg)


@dataclass
class ModelUpdate:
    client_id: str
    round_number: int
    model_weights: Dict[str, torch.Tensor]
    num_samples: int
    training_loss: float
    privacy_budget_used: float
    compression_ratio: float
    timestamp: datetime

    def validate(self) -> bool:
        return bool(self.client_id) and self.round_number >= 0 and self.num_samples > 0 \
            and self.training_loss >= 0 and 0 <= self.privacy_budget_used <= 1 \
            and 0 <= self.compression_ratio <= 1


@dataclass
class GlobalModel:
    round_number: int
    model_weights: Dict[str, torch.Tensor]
    accuracy_metrics: Dict[str, float]
    participating_clients: List[str]
    convergence_score: float
    created_at: datetime = field(default_factory=datetime.now)

    def get_accuracy(self, dataset: str = "test") -> Optional[float]:
        return self.accuracy_metrics.get(f"{dataset}_accuracy")


@dataclass
class TrainingMetrics:
    loss: float
    accuracy: float
    epochs_completed: int
    training_time: float
    samples_processed: int
