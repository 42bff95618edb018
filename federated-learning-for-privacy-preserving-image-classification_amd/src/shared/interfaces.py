"""Plugin contracts of the hot path (reference src/shared/interfaces.py:75-163).

Only the three interfaces the HIP path implements are restated; the
coordinator / client-service / data-loader contracts are outside the path.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import List

from .models import GlobalModel, ModelUpdate, ModelWeights


class AggregationServiceInterface(ABC):
    @abstractmethod
    def aggregate_updates(self, updates: List[ModelUpdate], weights: List[float]) -> GlobalModel:
        ...

    @abstractmethod
    def validate_update(self, update: ModelUpdate) -> bool:
        ...

    @abstractmethod
    def calculate_convergence_metrics(self, old_model: GlobalModel,
                                      new_model: GlobalModel) -> float:
        ...


class ModelInterface(ABC):
    @abstractmethod
    def get_model_weights(self) -> ModelWeights:
        ...

    @abstractmethod
    def set_model_weights(self, weights: ModelWeights) -> None:
        ...


class PrivacyEngineInterface(ABC):
    @abstractmethod
    def add_noise(self, gradients: ModelWeights, epsilon: float, delta: float) -> ModelWeights:
        ...

    @abstractmethod
    def clip_gradients(self, gradients: ModelWeights, max_norm: float) -> ModelWeights:
        ...

