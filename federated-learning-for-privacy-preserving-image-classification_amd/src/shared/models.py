"""Boundary records shared by the hot path and the code around it.

Every record the reference declares in src/shared/models.py:13-169 is exported here with
the same field names, field order, defaults and checks, so objects built by the existing
coordinator / client / gRPC code are accepted as-is and the callers' imports resolve
(tests/golden/boundary_names.json lists them; tests/test_boundary_cpu.py checks them):

* the records the HIP path produces / consumes — PrivacyConfig (:21), ModelUpdate (:50),
  GlobalModel (:75), TrainingMetrics (:90);
* the records of the control plane it sits under — ComputePowerLevel (:13),
  ClientCapabilities (:41), RegistrationResponse (:101), ModelResponse (:110),
  AckResponse (:119), RoundConfig (:127), TrainingStatus (:139), CompressedUpdate (:150);
* the aliases ModelWeights / ClientID / RoundNumber (:167-169).
"""
from __future__ import annotations

import enum
from dataclasses import dataclass, field
from datetime import datetime
from typing import Any, Dict, List, Optional

import torch

ModelWeights = Dict[str, torch.Tensor]
ClientID = str
RoundNumber = int


class ComputePowerLevel(enum.Enum):
    """Coarse client compute class (the capability adapter picks model / batch from it)."""
    LOW = "low"
    MEDIUM = "medium"
    HIGH = "high"


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
class ClientCapabilities:
    compute_power: ComputePowerLevel
    network_bandwidth: int          # Mbps
    available_samples: int
    supported_models: List[str]
    privacy_requirements: PrivacyConfig


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


# ---- control-plane messages (the gRPC servicer / client build and read these) ----------

@dataclass
class RegistrationResponse:
    success: bool
    client_id: str
    message: str
    global_model_version: int


@dataclass
class ModelResponse:
    success: bool
    model_weights: Optional[Dict[str, torch.Tensor]]
    round_number: int
    message: str


@dataclass
class AckResponse:
    success: bool
    message: str
    next_round_eta: Optional[datetime]


@dataclass
class RoundConfig:
    round_number: int
    min_clients: int
    max_clients: int
    local_epochs: int
    batch_size: int
    learning_rate: float
    timeout_seconds: int


@dataclass
class TrainingStatus:
    current_round: int
    active_clients: int
    round_progress: float           # fraction of the round done, 0..1
    global_accuracy: float
    convergence_score: float
    estimated_completion: Optional[datetime]


@dataclass
class CompressedUpdate:
    client_id: str
    round_number: int
    compressed_weights: bytes
    compression_metadata: Dict[str, Any]
    original_size: int
    compressed_size: int

    @property
    def compression_ratio(self) -> float:
        """compressed / original bytes (0 for an empty original, as the reference)."""
        return 0.0 if self.original_size == 0 else self.compressed_size / self.original_size
