"""Global-model evaluation on HIP: eval-mode forward of ONE model over a test set.

SURVEY.md §8(f-1).  The reference's coordinator never evaluates the global
model; the nearest code is ``LocalTrainer.evaluate_model``
(src/shared/training.py:307-360: eval mode, ``torch.max`` argmax, overall and
per-class accuracy) — this computes the same metrics for the aggregated model,
batched for the chip, and is what bench.py's rounds-to-target measurement
calls after every FedAvg.

Layout: the test set stays resident in HBM as one [N, *in_shape] tensor; a
launch covers ``slots x batch`` consecutive images as ``slots`` packed
"clients" that all read the same parameter row (client stride 0 — the kernels
take strides, so no copy of the weights is made).  Full chunks are read in
place; only a ragged final chunk is copied into the padded input buffer.
Metrics accumulate on the device (fh_eval_metrics) and are read once.

BatchNorm: the global model's running statistics are the FedAvg of the
clients' (RankRound.global_bufs) — a recorded divergence: the
reference federates parameters only, so its global model would evaluate with
freshly initialised buffers (mean 0, var 1).
"""
from __future__ import annotations

import math
from typing import Dict

import torch

from . import ops
from ._lib import FedHipError, load
from .net import PackedNet


class GlobalEvaluator:
    def __init__(self, model, device="cuda", slots: int = 64, batch: int = 32):
        load()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise FedHipError("GlobalEvaluator needs a HIP device; there is no CPU path")
        self.slots, self.batch = slots, batch
        self.net = PackedNet(model, slots, batch, self.device)
        self.layout = self.net.layout
        self.K = self.net.num_classes
        z = lambda *s, **k: torch.zeros(*s, device=self.device, **k)
        self.loss_sum = z(slots, dtype=torch.float64)
        self.correct = z(slots, dtype=torch.int64)
        self.class_correct = z(self.K, dtype=torch.int64)
        self.class_total = z(self.K, dtype=torch.int64)
        self.full_counts = torch.full((slots,), batch, dtype=torch.int32, device=self.device)
        self._x_pad, self._y_pad = self.net.x, self.net.y
        self._tail_counts = {}

    def _counts_for(self, m):
        if m not in self._tail_counts:
            c = [max(0, min(self.batch, m - z * self.batch)) for z in range(self.slots)]
            self._tail_counts[m] = torch.tensor(c, dtype=torch.int32, device=self.device)
        return self._tail_counts[m]

    def evaluate(self, params_flat: torch.Tensor, bufs_flat: torch.Tensor, data: torch.Tensor,
                 labels: torch.Tensor, transform=None) -> Dict[str, float]:
        """params_flat [>=P] (named_parameters order), bufs_flat [>=Q] (BN running stats),
        data [N, *in_shape] fp32 — or raw uint8 images [N, H, W(, C)] with `transform`
        (ops.DataTransform; its eval form, ToTensor + Normalize, is applied on the chip) —
        labels [N] int64, all on the device."""
        net, S, B = self.net, self.slots, self.batch
        N = int(data.shape[0])
        if data.dtype == torch.uint8:
            return self._evaluate_u8(params_flat, bufs_flat, data, labels, transform)
        if tuple(data.shape[1:]) != tuple(net.in_shape) or labels.shape[0] != N:
            raise FedHipError(f"evaluate: data {tuple(data.shape)} / labels "
                              f"{tuple(labels.shape)} do not match input {net.in_shape}")
        if labels.dtype != torch.int64 or not (data.is_contiguous() and labels.is_contiguous()):
            raise FedHipError("evaluate: data/labels must be contiguous, labels int64")
        rows = params_flat.reshape(1, -1).expand(S, -1)
        brows = bufs_flat.reshape(1, -1).expand(S, -1)
        for t in (self.loss_sum, self.correct, self.class_correct, self.class_total):
            t.zero_()
        chunk = S * B
        try:
            for start in range(0, N, chunk):
                m = min(chunk, N - start)
                if m == chunk:
                    net.x = data[start:start + chunk].view(S, B, *net.in_shape)
                    net.y = labels[start:start + chunk].view(S, B)
                    counts, n = self.full_counts, S
                else:
                    net.x, net.y = self._x_pad, self._y_pad
                    net.x.view(chunk, -1)[:m].copy_(data[start:start + m].view(m, -1))
                    net.y.view(chunk)[:m].copy_(labels[start:start + m])
                    counts, n = self._counts_for(m), math.ceil(m / B)
                net.forward(rows, brows, n, counts, train=False)
                ops.eval_metrics(net.logits, net.y, n, B, self.K, counts=counts,
                                 loss_sum=self.loss_sum, correct=self.correct,
                                 class_correct=self.class_correct, class_total=self.class_total)
        finally:
            net.x, net.y = self._x_pad, self._y_pad
        return self._metrics(N)

    def _evaluate_u8(self, params_flat, bufs_flat, data, labels, transform):
        if transform is None:
            raise FedHipError("evaluate: uint8 images need a DataTransform")
        tf = transform.eval()
        net, S, B = self.net, self.slots, self.batch
        N = int(data.shape[0])
        chunk = S * B
        nchunks = -(-N // chunk)
        if getattr(self, "_idx_n", None) != N:
            self._idx = torch.arange(nchunks * chunk, device=self.device).clamp_(max=max(N - 1, 0))
            self._idx_n = N
        rows = params_flat.reshape(1, -1).expand(S, -1)
        brows = bufs_flat.reshape(1, -1).expand(S, -1)
        for t in (self.loss_sum, self.correct, self.class_correct, self.class_total):
            t.zero_()
        for start in range(0, N, chunk):
            m = min(chunk, N - start)
            counts, n = ((self.full_counts, S) if m == chunk else
                         (self._counts_for(m), math.ceil(m / B)))
            idx = self._idx[start:start + chunk].view(S, B)
            ops.gather_u8(data, labels, idx, net.x, net.y, tf, n, B, counts=counts)
            net.forward(rows, brows, n, counts, train=False)
            ops.eval_metrics(net.logits, net.y, n, B, self.K, counts=counts,
                             loss_sum=self.loss_sum, correct=self.correct,
                             class_correct=self.class_correct, class_total=self.class_total)
        return self._metrics(N)

    def _metrics(self, N):
        correct = int(self.correct.sum().item())
        cc, ct = self.class_correct.tolist(), self.class_total.tolist()
        out = {"overall_accuracy": correct / N if N else 0.0, "total_samples": N,
               "correct_predictions": correct,
               "loss": float(self.loss_sum.sum().item()) / N if N else 0.0}
        for k in range(self.K):
            if ct[k]:
                out[f"class_{k}_accuracy"] = cc[k] / ct[k]
        return out
