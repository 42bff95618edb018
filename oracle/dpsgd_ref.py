"""CPU restatement of per-sample-clipped DP-SGD — TEST ORACLE (parity unpinned by the
reference, which has no DP-SGD: its DP clips whole update deltas, src/shared/privacy.py:107-144).

One step (Abadi et al. form, with the reference's own Gaussian-mechanism sigma,
privacy.py:209, as the default noise multiplier):
    g_i  = grad of CE(model(x_i), y_i)            (per sample, loss of that sample alone)
    c_i  = min(1, C / ||g_i||_2)                   (norm over ALL parameters, in float64)
    g    = (sum_i c_i g_i + noise) / B ;  optimizer.step() with g
Per-sample gradients by an explicit per-sample loop (the same values torch.func's
vmap(grad) yields); `pools` / `relus` replay another implementation's max-pool argmax
and ReLU masks (the fp64 "same decisions" check of the GPU tests)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from .train_ref import _Dropout


def sigma(epsilon, delta):
    """privacy.py:209 noise multiplier (sensitivity 1)."""
    return math.sqrt(2.0 * math.log(1.25 / delta)) / epsilon


def per_sample_grads(model, data, targets, pools=None, relus=None):
    params = list(model.parameters())
    out = []
    for i in range(data.shape[0]):
        drop = _Dropout(0.0,
                        pools=[p[i:i + 1] for p in pools] if pools is not None else None,
                        relus=[r[i:i + 1] for r in relus] if relus is not None else None)
        model.zero_grad()
        logits = model(data[i:i + 1], drop)
        F.cross_entropy(logits, targets[i:i + 1]).backward()
        out.append([p.grad.detach().clone() for p in params])
    return out


def dpsgd_step(model, opt, data, targets, max_norm, noise=None, pools=None, relus=None):
    """Returns (coefs, norms).  noise: list of tensors shaped like the parameters (already
    multiplied by sigma*C) or None."""
    model.train()
    grads = per_sample_grads(model, data, targets, pools, relus)
    B = data.shape[0]
    params = list(model.parameters())
    acc = [torch.zeros_like(p) for p in params]
    coefs, norms = [], []
    for g in grads:
        norm = math.sqrt(sum(float((t.double() ** 2).sum()) for t in g))
        c = min(1.0, max_norm / norm) if norm > 0 else 1.0
        coefs.append(c)
        norms.append(norm)
        for a, t in zip(acc, g):
            a.add_(t * c)
    for k, (p, a) in enumerate(zip(params, acc)):
        if noise is not None:
            a = a + noise[k]
        p.grad = a / B
    opt.step()
    return coefs, norms
