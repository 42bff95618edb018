"""fedhip — MI355X-native hot path for federated CNN training.

Layers:
  _lib     ctypes binding of libfedhip.so (include/fedhip.h)
  ops      tensor-level wrappers (client-packed device tensors)
  net      client-packed forward/backward programs per model family
  engine   PackedTrainer: many clients' local training as one GPU job
  round    federated round driver (local training -> DP -> FedAvg, multi-GPU)
"""
from ._lib import FedHipError, load  # noqa: F401

__version__ = "0.1.0"
