"""CPU restatement of the gRPC-edge arithmetic — TEST ORACLE.

Reference:
  src/aggregation/convergence.py:189-217  ConvergenceDetector._calculate_weight_change_metrics
  src/shared/serialization.py:28-48       ModelWeightSerializer.serialize_weights (torch.save)
Pinned against the reference by tests/golden (G9).  Test infrastructure only.
"""
from __future__ import annotations

import math

from .privacy_ref import tensor_norm_fp32


def weight_change_metrics(current: dict, previous: dict) -> dict:
    """Per layer fp32 torch norms (.item()) of (current - previous) and current, squared
    and summed in Python doubles; relative = norm / ||current|| (0 when ||current|| = 0)."""
    total, total_cur = 0.0, 0.0
    for name, cur in current.items():
        if name in previous:
            total += tensor_norm_fp32(cur - previous[name]) ** 2
            total_cur += tensor_norm_fp32(cur) ** 2
    norm = math.sqrt(total)
    cur_norm = math.sqrt(total_cur)
    return {"norm": norm, "relative": norm / cur_norm if cur_norm > 0 else 0.0}
