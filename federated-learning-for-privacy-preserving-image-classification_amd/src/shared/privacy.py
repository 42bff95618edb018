"""Update-level differential privacy with the reference's API, on HIP.

Reference: src/shared/privacy.py — PrivacyBudgetTracker (:25-92),
GradientClipper (:95-168), GaussianNoiseGenerator (:171-254),
DifferentialPrivacyEngine (:257-417), PrivacyAccountant (:419-484),
create_privacy_engine (:487-512), estimate_privacy_parameters (:515-556).

Arithmetic (all on the device, libfedhip dp kernels):
  total  = sqrt(sum_t norm(g_t)^2)  (per-tensor fp32 norms, summed in double)
  clip   : g_t * fl32(C/total) if total > C else g_t
  sigma  = min(total, C) * sqrt(2 ln(1.25/delta)) / epsilon
  noisy  = clipped + N(0, sigma^2)  — Philox4x32-10 on the device (the
           reference draws torch.normal on its device; the distribution and
           the formula are the same, the stream is not — noise can be injected
           with `noise=` for exact replay).
Budget bookkeeping is host state exactly as in the reference, including its
behaviour that the second add_noise() on one engine exhausts the budget.
"""
from __future__ import annotations

import logging
import math
import secrets
from datetime import datetime
from typing import Any, Dict, List, Optional, Tuple

import torch

from fedhip import ops

from .interfaces import PrivacyEngineInterface
from .models import ModelWeights, PrivacyConfig

logger = logging.getLogger(__name__)


class PrivacyError(Exception):
    """Raised by every privacy operation that fails (reference :20-22)."""


# ---------------------------------------------------------------- device helpers
def _pack(tensors: List[torch.Tensor], device) -> Tuple[torch.Tensor, torch.Tensor, List]:
    """Flatten a list of tensors into one [1, P] device row + segment offsets."""
    flats = [t.detach().to(device=device, dtype=torch.float32).reshape(-1) for t in tensors]
    row = torch.cat(flats).view(1, -1) if flats else torch.zeros(1, 0, device=device)
    offs = [0]
    for f in flats:
        offs.append(offs[-1] + f.numel())
    return row, torch.tensor(offs, dtype=torch.int64, device=device), offs


def _unpack(row: torch.Tensor, like: List[torch.Tensor], offs: List[int]) -> List[torch.Tensor]:
    return [row[0, offs[i]:offs[i + 1]].reshape(t.shape).to(t.device) for i, t in enumerate(like)]


def _device_for(tensors, default):
    for t in tensors:
        if t.is_cuda:
            return t.device
    return default if default is not None and torch.device(default).type == "cuda" \
        else torch.device("cuda")


class PrivacyBudgetTracker:
    """epsilon/delta spend ledger (host bookkeeping)."""

    def __init__(self, initial_epsilon: float, initial_delta: float):
        self.initial_epsilon, self.initial_delta = initial_epsilon, initial_delta
        self.consumed_epsilon = self.consumed_delta = 0.0
        self.consumption_history: List[Dict[str, Any]] = []
        self.start_time = datetime.now()

    def consume_budget(self, epsilon: float, delta: float, operation: str = "training"):
        self.consumed_epsilon += epsilon
        self.consumed_delta += delta
        self.consumption_history.append({
            "timestamp": datetime.now().isoformat(), "epsilon": epsilon, "delta": delta,
            "operation": operation, "total_epsilon": self.consumed_epsilon,
            "total_delta": self.consumed_delta})

    def get_remaining_budget(self) -> Tuple[float, float]:
        return (max(0, self.initial_epsilon - self.consumed_epsilon),
                max(0, self.initial_delta - self.consumed_delta))

    def is_budget_exhausted(self, required_epsilon: float = 0, required_delta: float = 0) -> bool:
        re, rd = self.get_remaining_budget()
        return re < required_epsilon or rd < required_delta

    def get_budget_status(self) -> Dict[str, Any]:
        re, rd = self.get_remaining_budget()
        return {"initial_epsilon": self.initial_epsilon, "initial_delta": self.initial_delta,
                "consumed_epsilon": self.consumed_epsilon, "consumed_delta": self.consumed_delta,
                "remaining_epsilon": re, "remaining_delta": rd,
                "epsilon_utilization": self.consumed_epsilon / self.initial_epsilon,
                "delta_utilization": self.consumed_delta / self.initial_delta,
                "operations_count": len(self.consumption_history),
                "tracking_duration": (datetime.now() - self.start_time).total_seconds()}


class GradientClipper:
    """Global-L2 clipping of a tensor dict (device kernels: fp64 norm, fp32 rescale)."""

    def __init__(self, max_grad_norm: float, device=None):
        self.max_grad_norm = max_grad_norm
        self.device = device

    def _clip_row(self, row, segs):
        sq = ops.dp_delta_sqnorm(row, None, segs, 1)
        return ops.dp_clip_coef(sq, self.max_grad_norm, 1.0, 0.5)

    def clip_gradients(self, gradients: ModelWeights) -> Tuple[ModelWeights, float]:
        try:
            names = [n for n, g in gradients.items() if g is not None]
            tens = [gradients[n] for n in names]
            dev = _device_for(tens, self.device)
            row, segs, offs = _pack(tens, dev)
            total, coef, clipped, _ = self._clip_row(row, segs)
            zero_sigma = torch.zeros(1, device=dev)
            out = torch.empty_like(row)
            ops.dp_apply(row, None, out, coef, clipped, zero_sigma,
                         noise=torch.zeros_like(row))
            res = dict(zip(names, _unpack(out, tens, offs)))
            result = {n: (res[n] if g is not None else None) for n, g in gradients.items()}
            return result, min(float(total.item()), self.max_grad_norm)
        except Exception as e:
            raise PrivacyError(f"Gradient clipping failed: {e}") from e

    def estimate_sensitivity(self, gradients_batch: List[ModelWeights]) -> float:
        best = 0.0
        for grads in gradients_batch:
            tens = [g for g in grads.values() if g is not None]
            if not tens:
                continue
            row, segs, _ = _pack(tens, _device_for(tens, self.device))
            total, _, _, _ = self._clip_row(row, segs)
            best = max(best, float(total.item()))
        return best


class GaussianNoiseGenerator:
    """Gaussian mechanism noise, generated on the device.

    seed None (default) draws a secret 64-bit Philox key from os.urandom, as the
    reference's torch.normal draws from an RNG state nobody else holds (privacy.py:212).
    A fixed seed is for tests and replay only: anyone who knows it can regenerate the
    noise and subtract it, which removes the privacy guarantee."""

    def __init__(self, device: Optional[torch.device] = None, seed: Optional[int] = None):
        self.device = device
        self._seed = secrets.randbits(64) if seed is None else int(seed)
        self._calls = 0

    @staticmethod
    def noise_scale(sensitivity: float, epsilon: float, delta: float) -> float:
        if epsilon <= 0:
            raise ValueError("Epsilon must be positive")
        if delta <= 0 or delta >= 1:
            raise ValueError("Delta must be in (0, 1)")
        return sensitivity * math.sqrt(2 * math.log(1.25 / delta)) / epsilon

    def _next_seed(self):
        self._calls += 1
        return (self._seed * 0x9E3779B97F4A7C15 + self._calls) & ((1 << 64) - 1)

    def generate_noise(self, shape: torch.Size, sensitivity: float, epsilon: float,
                       delta: float) -> torch.Tensor:
        try:
            sigma = self.noise_scale(sensitivity, epsilon, delta)
            dev = self.device if self.device is not None and torch.device(self.device).type == "cuda" \
                else torch.device("cuda")
            n = int(torch.Size(shape).numel())
            zero = torch.zeros(1, n, device=dev)
            out = torch.empty_like(zero)
            one = torch.ones(1, device=dev)
            ops.dp_apply(zero, None, out, one, torch.zeros(1, dtype=torch.int32, device=dev),
                         torch.full((1,), sigma, dtype=torch.float32, device=dev),
                         seed=self._next_seed())
            return out.view(shape)
        except Exception as e:
            raise PrivacyError(f"Noise generation failed: {e}") from e

    def add_noise_to_gradients(self, gradients: ModelWeights, sensitivity: float, epsilon: float,
                               delta: float, noise: Optional[ModelWeights] = None) -> ModelWeights:
        try:
            sigma = self.noise_scale(sensitivity, epsilon, delta)
            names = [n for n, g in gradients.items() if g is not None]
            tens = [gradients[n] for n in names]
            dev = _device_for(tens, self.device)
            row, segs, offs = _pack(tens, dev)
            out = torch.empty_like(row)
            nz = None if noise is None else _pack([noise[n] for n in names], dev)[0]
            ops.dp_apply(row, None, out, torch.ones(1, device=dev),
                         torch.zeros(1, dtype=torch.int32, device=dev),
                         torch.full((1,), sigma, dtype=torch.float32, device=dev), noise=nz,
                         seed=self._next_seed())
            res = dict(zip(names, _unpack(out, tens, offs)))
            return {n: (res[n] if g is not None else None) for n, g in gradients.items()}
        except Exception as e:
            raise PrivacyError(f"Adding noise to gradients failed: {e}") from e


class DifferentialPrivacyEngine(PrivacyEngineInterface):
    """PrivacyEngineInterface implementation (reference :257-417)."""

    def __init__(self, privacy_config: PrivacyConfig, device: Optional[torch.device] = None,
                 seed: Optional[int] = None):
        """seed: see GaussianNoiseGenerator (None = secret key from os.urandom)."""
        self.config = privacy_config
        self.device = device
        self.clipper = GradientClipper(privacy_config.max_grad_norm, device)
        self.noise_generator = GaussianNoiseGenerator(device, seed)
        self.budget_tracker = PrivacyBudgetTracker(privacy_config.epsilon, privacy_config.delta)

    def add_noise(self, gradients: ModelWeights, epsilon: float, delta: float,
                  noise: Optional[ModelWeights] = None) -> ModelWeights:
        """Clip to max_grad_norm, add N(0, sigma^2) with sensitivity = clipped norm, spend budget.
        Fused on the device: one norm pass, one clip+noise pass."""
        try:
            if not self.validate_privacy_parameters(epsilon, delta):
                raise PrivacyError("Invalid privacy parameters")
            if self.budget_tracker.is_budget_exhausted(epsilon, delta):
                raise PrivacyError("Privacy budget exhausted")
            names = [n for n, g in gradients.items() if g is not None]
            tens = [gradients[n] for n in names]
            dev = _device_for(tens, self.device)
            row, segs, offs = _pack(tens, dev)
            sq = ops.dp_delta_sqnorm(row, None, segs, 1)
            total, coef, clipped, sigma = ops.dp_clip_coef(sq, self.config.max_grad_norm,
                                                           epsilon, delta)
            out = torch.empty_like(row)
            nz = None if noise is None else _pack([noise[n] for n in names], dev)[0]
            ops.dp_apply(row, None, out, coef, clipped, sigma, noise=nz,
                         seed=self.noise_generator._next_seed())
            self.budget_tracker.consume_budget(epsilon, delta, "gradient_noise")
            res = dict(zip(names, _unpack(out, tens, offs)))
            return {n: (res[n] if g is not None else None) for n, g in gradients.items()}
        except Exception as e:
            logger.error(f"Adding DP noise failed: {e}")
            raise PrivacyError(f"Adding DP noise failed: {e}") from e

    def clip_gradients(self, gradients: ModelWeights, max_norm: float) -> ModelWeights:
        return GradientClipper(max_norm, self.device).clip_gradients(gradients)[0]

    def calculate_privacy_budget(self, epsilon: float, delta: float, steps: int) -> float:
        """Simplified advanced composition (reference :319-333)."""
        if steps <= 1:
            return epsilon
        return epsilon * math.sqrt(2 * steps * math.log(1 / delta)) + \
            steps * epsilon * (math.exp(epsilon) - 1)

    def validate_privacy_parameters(self, epsilon: float, delta: float) -> bool:
        if epsilon <= 0 or delta <= 0 or delta >= 1:
            return False
        if epsilon > 10.0:
            logger.warning(f"Epsilon {epsilon} is very high, privacy may be weak")
        if delta > 1e-3:
            logger.warning(f"Delta {delta} is high, privacy may be weak")
        return True

    def get_privacy_analysis(self) -> Dict[str, Any]:
        c = self.config
        eps_s = "strong" if c.epsilon < 1.0 else "moderate" if c.epsilon < 5.0 else "weak"
        del_s = "strong" if c.delta < 1e-5 else "moderate" if c.delta < 1e-3 else "weak"
        rank = ["strong", "moderate", "weak"]
        return {"privacy_config": {"epsilon": c.epsilon, "delta": c.delta,
                                   "max_grad_norm": c.max_grad_norm,
                                   "noise_multiplier": c.noise_multiplier},
                "budget_status": self.budget_tracker.get_budget_status(),
                "privacy_strength": {"epsilon_strength": eps_s, "delta_strength": del_s,
                                     "overall_strength": min(eps_s, del_s, key=rank.index)},
                "recommendations": self._get_privacy_recommendations()}

    def _get_privacy_recommendations(self) -> List[str]:
        c, recs = self.config, []
        if c.epsilon > 5.0:
            recs.append("Consider reducing epsilon for stronger privacy")
        if c.delta > 1e-3:
            recs.append("Consider reducing delta for better privacy guarantees")
        if c.max_grad_norm > 10.0:
            recs.append("Consider reducing gradient clipping norm to improve privacy")
        if self.budget_tracker.get_remaining_budget()[0] < c.epsilon * 0.1:
            recs.append("Privacy budget nearly exhausted, consider resetting or reducing usage")
        return recs or ["Privacy configuration looks good"]

    def reset_budget(self, new_epsilon: Optional[float] = None, new_delta: Optional[float] = None):
        self.budget_tracker = PrivacyBudgetTracker(new_epsilon or self.config.epsilon,
                                                   new_delta or self.config.delta)
        if new_epsilon:
            self.config.epsilon = new_epsilon
        if new_delta:
            self.config.delta = new_delta


class PrivacyAccountant:
    """Basic-composition ledger (reference :419-484)."""

    def __init__(self):
        self.privacy_ledger: List[Dict[str, Any]] = []
        self.total_epsilon = self.total_delta = 0.0

    def add_mechanism(self, mechanism_type: str, epsilon: float, delta: float,
                      sensitivity: float, noise_scale: float,
                      metadata: Optional[Dict[str, Any]] = None):
        self.privacy_ledger.append({"timestamp": datetime.now().isoformat(),
                                    "mechanism_type": mechanism_type, "epsilon": epsilon,
                                    "delta": delta, "sensitivity": sensitivity,
                                    "noise_scale": noise_scale, "metadata": metadata or {}})
        self.total_epsilon += epsilon
        self.total_delta += delta

    def get_total_privacy_cost(self) -> Tuple[float, float]:
        return self.total_epsilon, self.total_delta

    def get_privacy_ledger(self) -> List[Dict[str, Any]]:
        return list(self.privacy_ledger)

    def export_ledger(self, filepath: str):
        import json
        with open(filepath, "w") as f:
            json.dump({"total_epsilon": self.total_epsilon, "total_delta": self.total_delta,
                       "ledger": self.privacy_ledger}, f, indent=2)


def create_privacy_engine(epsilon: float = 1.0, delta: float = 1e-5, max_grad_norm: float = 1.0,
                          noise_multiplier: float = 1.0,
                          device: Optional[torch.device] = None) -> DifferentialPrivacyEngine:
    return DifferentialPrivacyEngine(PrivacyConfig(epsilon=epsilon, delta=delta,
                                                   max_grad_norm=max_grad_norm,
                                                   noise_multiplier=noise_multiplier), device)


def estimate_privacy_parameters(target_accuracy: float = 0.9, dataset_size: int = 10000,
                                num_rounds: int = 100) -> Dict[str, float]:
    """Heuristic parameter suggestion (reference :515-556)."""
    base = 1.0 if dataset_size > 5000 else 2.0
    eps = base * 2 if target_accuracy > 0.95 else base * 0.5 if target_accuracy < 0.85 else base
    return {"epsilon": eps / math.sqrt(num_rounds), "delta": 1.0 / dataset_size,
            "max_grad_norm": 1.0 if target_accuracy > 0.9 else 2.0, "noise_multiplier": 1.0}
