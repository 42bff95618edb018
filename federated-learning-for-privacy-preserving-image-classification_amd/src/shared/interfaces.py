"""Service contracts (reference src/shared/interfaces.py:17-182), all seven.

The HIP path implements three of them — AggregationServiceInterface (FedAvgAggregator),
ModelInterface (FederatedCNNBase), PrivacyEngineInterface (DifferentialPrivacyEngine).  The
other four are the contracts of the control plane this package drops in under
(coordinator, client service, data loader, compressor); they are restated so that the
reference's own implementations of them (src/shared/data_loader.py:18,
src/shared/compression.py:16, ...) import and subclass them unchanged when this package
shadows src.shared.interfaces (tests/test_boundary_cpu.py).
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List

import torch

from .models import (AckResponse, ClientCapabilities, ClientID, CompressedUpdate, GlobalModel,
                     ModelResponse, ModelUpdate, ModelWeights, RegistrationResponse, RoundConfig,
                     RoundNumber, TrainingMetrics, TrainingStatus)


class CoordinatorServiceInterface(ABC):
    """Round orchestration seen by clients (reference :17)."""

    @abstractmethod
    def register_client(self, client_id: ClientID,
                        capabilities: ClientCapabilities) -> RegistrationResponse: ...

    @abstractmethod
    def get_global_model(self, client_id: ClientID, round_number: RoundNumber) -> ModelResponse: ...

    @abstractmethod
    def submit_model_update(self, client_id: ClientID, model_update: ModelUpdate) -> AckResponse: ...

    @abstractmethod
    def start_training_round(self, round_config: RoundConfig) -> bool: ...

    @abstractmethod
    def get_training_status(self) -> TrainingStatus: ...


class ClientServiceInterface(ABC):
    """One client's side of a round (reference :46)."""

    @abstractmethod
    def initialize_local_model(self, global_model: torch.nn.Module) -> None: ...

    @abstractmethod
    def train_local_model(self, epochs: int, batch_size: int) -> TrainingMetrics: ...

    @abstractmethod
    def apply_differential_privacy(self, model_update: ModelUpdate,
                                   epsilon: float) -> ModelUpdate: ...

    @abstractmethod
    def compress_model_update(self, model_update: ModelUpdate) -> CompressedUpdate: ...

    @abstractmethod
    def sync_with_coordinator(self) -> bool: ...


class AggregationServiceInterface(ABC):
    """FedAvg and friends (reference :75)."""

    @abstractmethod
    def aggregate_updates(self, updates: List[ModelUpdate], weights: List[float]) -> GlobalModel: ...

    @abstractmethod
    def validate_update(self, update: ModelUpdate) -> bool: ...

    @abstractmethod
    def compress_global_model(self, model: GlobalModel) -> CompressedUpdate: ...

    @abstractmethod
    def calculate_convergence_metrics(self, old_model: GlobalModel,
                                      new_model: GlobalModel) -> float: ...


class ModelInterface(ABC):
    """What the federation needs from a network (reference :99)."""

    @abstractmethod
    def get_model_weights(self) -> ModelWeights: ...

    @abstractmethod
    def set_model_weights(self, weights: ModelWeights) -> None: ...

    @abstractmethod
    def get_parameter_count(self) -> int: ...

    @abstractmethod
    def estimate_memory_usage(self) -> int: ...


class DataLoaderInterface(ABC):
    """Per-client data access (reference :123)."""

    @abstractmethod
    def load_training_data(self, client_id: ClientID) -> torch.utils.data.DataLoader: ...

    @abstractmethod
    def load_validation_data(self) -> torch.utils.data.DataLoader: ...

    @abstractmethod
    def get_data_statistics(self, client_id: ClientID) -> Dict[str, Any]: ...


class PrivacyEngineInterface(ABC):
    """Update-level differential privacy (reference :142)."""

    @abstractmethod
    def add_noise(self, gradients: ModelWeights, epsilon: float, delta: float) -> ModelWeights: ...

    @abstractmethod
    def clip_gradients(self, gradients: ModelWeights, max_norm: float) -> ModelWeights: ...

    @abstractmethod
    def calculate_privacy_budget(self, epsilon: float, delta: float, steps: int) -> float: ...

    @abstractmethod
    def validate_privacy_parameters(self, epsilon: float, delta: float) -> bool: ...


class CompressionInterface(ABC):
    """Weight-dict codecs (reference :166)."""

    @abstractmethod
    def compress_weights(self, weights: ModelWeights) -> bytes: ...

    @abstractmethod
    def decompress_weights(self, compressed_data: bytes) -> ModelWeights: ...

    @abstractmethod
    def get_compression_ratio(self, original_size: int, compressed_size: int) -> float: ...
