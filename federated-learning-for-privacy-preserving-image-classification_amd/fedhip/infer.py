"""Single-model forward on HIP (nn.Module.forward of the drop-in models).

Used by LocalTrainer.evaluate_model and by anyone calling ``model(x)``.  A small
cache of one-slot PackedTrainers (keyed by model id and padded batch) holds the
buffers.  A plain call copies the module's parameters and BN statistics in (the
module may have been changed in any way since the last call, ``p.data`` writes
included) and, in train mode, copies the updated running statistics back
(BatchNorm's train-mode side effect).  Inside ``frozen(model)`` — a loop that
only evaluates, as LocalTrainer.evaluate_model's — the weights are loaded once per
engine and every further batch reuses them.
"""
from __future__ import annotations

import contextlib
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


_FROZEN: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


@contextlib.contextmanager
def frozen(model):
    """Evaluation loop over `model` whose weights do not change meanwhile: load them into
    the HIP engine once instead of once per batch."""
    prev = _FROZEN.get(model)
    _FROZEN[model] = set()  # engines already loaded inside this block
    try:
        yield
    finally:
        if prev is None:
            _FROZEN.pop(model, None)
        else:
            _FROZEN[model] = prev


def module_forward(model, x: torch.Tensor) -> torch.Tensor:
    if not x.is_cuda:
        raise FedHipError("HIP models compute on a HIP device only; move the model and input "
                          "to 'cuda' (there is no CPU path)")
    n = x.shape[0]
    eng = engine_for(model, n, x.device)
    loaded = _FROZEN.get(model) if not model.training else None
    if loaded is None or id(eng) not in loaded:
        eng.load_module_state(0, model)
        if loaded is not None:
            loaded.add(id(eng))
    net = eng.net
    net.x[0, :n].copy_(x.reshape(n, *net.in_shape))
    counts = torch.tensor([n], dtype=torch.int32, device=x.device)
    net.forward(eng.params, eng.bufs, 1, counts, train=model.training)
    if model.training:
        eng.num_batches_tracked[0] += 1
        eng.store_module_state(0, model)
    return net.logits[0, :n].clone()
