"""LocalTrainer with the reference's API, computing on MI355X through libfedhip.

Reference: src/shared/training.py:28-403 (LocalTrainer), :406-501 (config
helpers).  The caller (src/client/federated_trainer.py:400-407) is unchanged:
``train_local_model(train_loader, epochs, learning_rate, optimizer_type, ...)``
returns the same TrainingMetrics.

What differs, by design (divergence log):
  D12  no per-batch host synchronisation: loss / correct counts accumulate on
       the device and are read once per epoch (values identical);
  --   only CrossEntropyLoss is supported as loss_function (the reference's
       default and the only loss any caller passes).
"""
from __future__ import annotations

import json
import logging
import os
import time
from datetime import datetime
from typing import Any, Dict, List, Optional

import torch
import torch.nn as nn

from fedhip import infer
from fedhip._lib import FedHipError
from fedhip.engine import PackedTrainer

from .models import TrainingMetrics
from .models_pytorch import FederatedCNNBase

logger = logging.getLogger(__name__)


class TrainingError(Exception):
    """Raised for any failure inside local training (reference :23-25)."""


def _check_loss(loss_function):
    if loss_function is None:
        return
    ok = isinstance(loss_function, nn.CrossEntropyLoss) and loss_function.weight is None \
        and loss_function.reduction == "mean" and loss_function.label_smoothing == 0.0 \
        and loss_function.ignore_index == -100
    if not ok:
        raise FedHipError("only nn.CrossEntropyLoss() (mean reduction, no weights/smoothing) "
                          "is implemented on the HIP path")


class LocalTrainer:
    """One client's local training loop on the HIP engine (one packed slot)."""

    def __init__(self, model: FederatedCNNBase, device: Optional[torch.device] = None,
                 checkpoint_dir: Optional[str] = None):
        self.model = model
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        if self.device.type != "cuda":
            raise TrainingError(f"LocalTrainer computes on a HIP device; got {self.device} "
                                "(there is no CPU path)")
        self.checkpoint_dir = checkpoint_dir
        self.model.to(self.device)
        self.current_epoch = 0
        self.training_history: List[Dict[str, Any]] = []
        self._engines: Dict[int, PackedTrainer] = {}
        self._flags: Dict[tuple, torch.Tensor] = {}
        if checkpoint_dir:
            os.makedirs(checkpoint_dir, exist_ok=True)
        logger.info(f"LocalTrainer initialized on device: {self.device}")

    # ------------------------------------------------------------------ plumbing
    def _engine(self, batch: int) -> PackedTrainer:
        b = max(32, ((batch + 31) // 32) * 32)
        if b not in self._engines:
            self._engines[b] = PackedTrainer(self.model, capacity=1, batch=b, device=self.device)
        return self._engines[b]

    def _i32(self, value: int) -> torch.Tensor:
        key = ("i32", value)
        if key not in self._flags:
            self._flags[key] = torch.tensor([value], dtype=torch.int32, device=self.device)
        return self._flags[key]

    def _stage(self, eng, data, targets):
        n = data.shape[0]
        eng.net.x[0, :n].copy_(data.reshape(n, *eng.net.in_shape), non_blocking=True)
        eng.net.y[0, :n].copy_(targets, non_blocking=True)
        return n

    def _max_batch(self, loader) -> int:
        bs = getattr(loader, "batch_size", None)
        if bs:
            return int(bs)
        return max(int(d.shape[0]) for d, _ in loader)

    # ------------------------------------------------------------------ training
    def train_local_model(self, train_loader, epochs: int, learning_rate: float = 0.001,
                          optimizer_type: str = "adam", loss_function: Optional[nn.Module] = None,
                          validation_loader=None, save_checkpoints: bool = True,
                          early_stopping_patience: Optional[int] = None) -> TrainingMetrics:
        try:
            t0 = time.time()
            _check_loss(loss_function)
            eng = self._engine(self._max_batch(train_loader))
            eng.load_module_state(0, self.model)
            eng.begin_round(optimizer_type, learning_rate)  # fresh optimizer (reference :89)
            best_val, patience, total = float("inf"), 0, 0
            losses, accs = [], []
            for epoch in range(epochs):
                self.current_epoch = epoch
                loss, acc, seen = self._train_epoch(eng, train_loader)
                total += seen
                val_loss = val_acc = None
                if validation_loader:
                    val_loss, val_acc = self._validate_epoch(eng, validation_loader)
                losses.append(loss)
                accs.append(acc)
                msg = f"Epoch {epoch + 1}/{epochs} - Loss: {loss:.4f}, Acc: {acc:.4f}"
                if val_loss is not None:
                    msg += f", Val Loss: {val_loss:.4f}, Val Acc: {val_acc:.4f}"
                logger.info(msg)
                if save_checkpoints and self.checkpoint_dir:
                    eng.store_module_state(0, self.model)
                    self._save_checkpoint(epoch, loss, val_loss)
                if early_stopping_patience and validation_loader:
                    if val_loss < best_val:
                        best_val, patience = val_loss, 0
                    else:
                        patience += 1
                        if patience >= early_stopping_patience:
                            logger.info(f"Early stopping at epoch {epoch + 1}")
                            break
            eng.store_module_state(0, self.model)
            self._expose_last_gradients(eng)
            elapsed = time.time() - t0
            final_loss = losses[-1] if losses else 0.0
            final_acc = accs[-1] if accs else 0.0
            metrics = TrainingMetrics(loss=final_loss, accuracy=final_acc,
                                      epochs_completed=len(losses), training_time=elapsed,
                                      samples_processed=total)
            self.training_history.append({
                "timestamp": datetime.now().isoformat(), "epochs": len(losses),
                "final_loss": final_loss, "final_accuracy": final_acc,
                "training_time": elapsed, "samples_processed": total})
            return metrics
        except Exception as e:  # reference :169-171: everything becomes TrainingError
            logger.error(f"Local training failed: {e}")
            raise TrainingError(f"Local training failed: {e}") from e

    def _train_epoch(self, eng, loader):
        """One pass over the loader; metrics accumulate on the device (one sync per epoch)."""
        nb = 0
        for data, targets in loader:
            n = self._stage(eng, data, targets)
            eng.step(1, self._i32(n), reset=self._i32(1 if nb == 0 else 0))
            nb += 1
        if nb == 0:
            raise ZeroDivisionError("division by zero")  # reference: running_loss / len(loader)
        loss = float(eng.acc_loss[0].item()) / nb
        correct, seen = int(eng.acc_correct[0].item()), int(eng.acc_seen[0].item())
        return loss, correct / seen, seen

    def _validate_epoch(self, eng, loader):
        nb = 0
        for data, targets in loader:
            n = self._stage(eng, data, targets)
            eng.eval_batch(1, self._i32(n), reset=self._i32(1 if nb == 0 else 0))
            nb += 1
        loss = float(eng.acc_loss[0].item()) / nb
        return loss, int(eng.acc_correct[0].item()) / int(eng.acc_seen[0].item())

    def _expose_last_gradients(self, eng):
        """param.grad = last step's gradient (what the reference leaves after backward)."""
        with torch.no_grad():
            for name, p in self.model.named_parameters():
                p.grad = eng.layout.view(eng.grads, name)[0].reshape(p.shape).clone()

    # ------------------------------------------------------------------ evaluation
    def evaluate_model(self, test_loader) -> Dict[str, float]:
        """Eval-mode accuracy overall and per class (reference :307-360)."""
        try:
            self.model.eval()
            correct = total = 0
            cls_ok: Dict[int, int] = {}
            cls_n: Dict[int, int] = {}
            with infer.frozen(self.model):  # weights loaded into the engine once
                for data, targets in test_loader:
                    out = self.model(data.to(self.device))
                    pred = out.argmax(dim=1).cpu()
                    t = targets.cpu()
                    total += t.numel()
                    hit = pred == t
                    correct += int(hit.sum())
                    for lab, h in zip(t.tolist(), hit.tolist()):
                        cls_ok[lab] = cls_ok.get(lab, 0) + int(h)
                        cls_n[lab] = cls_n.get(lab, 0) + 1
            res = {"overall_accuracy": correct / total, "total_samples": total,
                   "correct_predictions": correct}
            for c in cls_n:
                res[f"class_{c}_accuracy"] = cls_ok[c] / cls_n[c]
            return res
        except Exception as e:
            raise TrainingError(f"Model evaluation failed: {e}") from e

    # ------------------------------------------------------------------ checkpoints
    def _save_checkpoint(self, epoch: int, train_loss: float, val_loss: Optional[float] = None):
        if not self.checkpoint_dir:
            return
        ckpt = {"epoch": epoch, "model_state_dict": self.model.state_dict(),
                "train_loss": train_loss, "val_loss": val_loss,
                "timestamp": datetime.now().isoformat(), "model_info": self.model.get_model_info()}
        torch.save(ckpt, os.path.join(self.checkpoint_dir, f"checkpoint_epoch_{epoch}.pt"))
        torch.save(ckpt, os.path.join(self.checkpoint_dir, "latest_checkpoint.pt"))

    def load_checkpoint(self, checkpoint_path: str) -> Dict[str, Any]:
        try:
            ckpt = torch.load(checkpoint_path, map_location=self.device, weights_only=True)
            self.model.load_state_dict(ckpt["model_state_dict"])
            self.current_epoch = ckpt["epoch"]
            return {"epoch": ckpt["epoch"], "train_loss": ckpt["train_loss"],
                    "val_loss": ckpt.get("val_loss"), "timestamp": ckpt.get("timestamp")}
        except Exception as e:
            raise TrainingError(f"Failed to load checkpoint: {e}") from e

    # ------------------------------------------------------------------ misc API
    def get_model_gradients(self) -> Dict[str, torch.Tensor]:
        return {n: p.grad.clone() for n, p in self.model.named_parameters() if p.grad is not None}

    def set_model_gradients(self, gradients: Dict[str, torch.Tensor]):
        for n, p in self.model.named_parameters():
            if n in gradients:
                p.grad = gradients[n].clone()

    def get_training_history(self) -> List[Dict[str, Any]]:
        return list(self.training_history)

    def save_training_history(self, filepath: str):
        with open(filepath, "w") as f:
            json.dump(self.training_history, f, indent=2)

    def reset_training_state(self):
        self.current_epoch = 0
        self.training_history = []


class FederatedTrainingConfig:
    """Per-round local hyper-parameters (reference :406-452)."""

    FIELDS = ("local_epochs", "batch_size", "learning_rate", "optimizer_type",
              "early_stopping_patience", "save_checkpoints", "validation_split")

    def __init__(self, local_epochs: int = 5, batch_size: int = 32, learning_rate: float = 0.001,
                 optimizer_type: str = "adam", early_stopping_patience: Optional[int] = None,
                 save_checkpoints: bool = True, validation_split: float = 0.1):
        self.local_epochs, self.batch_size, self.learning_rate = local_epochs, batch_size, learning_rate
        self.optimizer_type, self.early_stopping_patience = optimizer_type, early_stopping_patience
        self.save_checkpoints, self.validation_split = save_checkpoints, validation_split

    def to_dict(self) -> Dict[str, Any]:
        return {k: getattr(self, k) for k in self.FIELDS}

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "FederatedTrainingConfig":
        return cls(**d)


def create_adaptive_config(client_capabilities: Dict[str, Any]) -> FederatedTrainingConfig:
    """Capability-driven epochs / batch / lr (reference :455-501)."""
    tiers = {"high": (10, 64, 0.001), "medium": (5, 32, 0.001)}
    epochs, bs, lr = tiers.get(client_capabilities.get("compute_power", "medium"), (3, 16, 0.0005))
    samples = client_capabilities.get("available_samples", 1000)
    if samples < 500:
        bs = min(bs, 16)
    elif samples > 5000:
        bs = min(bs * 2, 128)
    if client_capabilities.get("network_bandwidth", 10) < 5:
        epochs = max(epochs + 2, 7)
    return FederatedTrainingConfig(local_epochs=epochs, batch_size=bs, learning_rate=lr,
                                   optimizer_type="adam", early_stopping_patience=None,
                                   save_checkpoints=True, validation_split=0.1)


def validate_training_data(train_loader) -> Dict[str, Any]:
    """Pre-flight check of a (data, targets) loader (reference :504-560).

    Host-side only: it looks at the loader's length and its first batch (NCHW float data,
    integer targets) and never raises — problems come back as {'valid': False, 'error': …},
    the same keys and messages as the reference."""
    try:
        n = len(train_loader)
        if n == 0:
            raise ValueError("Training data loader is empty")
        batch = next(iter(train_loader))
        if len(batch) != 2:
            raise ValueError("Expected (data, targets) tuple from data loader")
        data, targets = batch
        if not isinstance(data, torch.Tensor):
            raise ValueError("Data must be a torch.Tensor")
        if not isinstance(targets, torch.Tensor):
            raise ValueError("Targets must be a torch.Tensor")
        if data.dim() != 4:
            raise ValueError(f"Expected 4D data tensor, got shape {data.shape}")
        b, c, h, w = data.shape
        out = {"valid": True, "num_batches": n, "batch_size": b, "data_shape": (c, h, w),
               "num_classes": int(torch.unique(targets).numel()),
               "data_type": str(data.dtype), "targets_type": str(targets.dtype)}
        logger.info("Training data validation passed: %s", out)
        return out
    except Exception as e:  # the reference reports, it does not raise
        logger.error("Training data validation failed: %s", e)
        return {"valid": False, "error": str(e)}
