"""Single-model forward on HIP (nn.Module.forward of the drop-in models).

Used by LocalTrainer._validate_epoch / evaluate_model and by anyone calling
``model(x)``.  A small cache of one-slot PackedTrainers (keyed by model id and
padded batch) holds the buffers; parameters and BN statistics are copied in
from the module for each call and, in train mode, the updated running
statistics are copied back (BatchNorm's train-mode side effect).
"""
from __future__ import annotations

import weakref

import torch

from ._lib import FedHipError

_CACHE: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def _round_batch(n):
    return max(32, ((n + 31) // 32) * 32)


def engine_for(model, batch, device):
    from .engine import PackedTrainer
    per = _CACHE.setdefault(model, {})
    key = (_round_batch(batch), str(device))
    if key not in per:
        per[key] = PackedTrainer(model, capacity=1, batch=key[0], device=device)
    return per[key]


def module_forward(model, x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        raise FedHipError("HIP models compute on a HIP device only; move the model and input "
                          "to 'cuda' (there is no CPU path)")
    n = x.shape[0]
    eng = engine_for(model, n, x.device)
    eng.load_module_state(0, model)
    net = eng.net
    net.x[0, :n].copy_(x.reshape(n, *net.in_shape))
    counts = torch.tensor([n], dtype=torch.int32, device=x.device)
    net.forward(eng.params, eng.bufs, 1, counts, train=model.training)
    if model.training:
        eng.num_batches_tracked[0] += 1
        eng.store_module_state(0, model)
    return net.logits[0, :n].clone()
