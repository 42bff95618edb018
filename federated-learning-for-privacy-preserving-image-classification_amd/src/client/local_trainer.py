"""north_star path `src/client/local_trainer`: the HIP-backed LocalTrainer.

The reference defines LocalTrainer in src/shared/training.py:28 and the client
consumes it from src/client/federated_trainer.py:127; both import paths work.
"""
from ..shared.training import (FederatedTrainingConfig, LocalTrainer, TrainingError,  # noqa: F401
                               create_adaptive_config)
from ..shared.models import TrainingMetrics  # noqa: F401
