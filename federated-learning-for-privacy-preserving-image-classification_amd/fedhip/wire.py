"""The gRPC edge of the packed path: wire format and convergence norms.

Wire format.  The reference ships a client's weights as
``torch.save(get_model_weights())`` bytes, hex-encoded into the message
(src/shared/serialization.py:28-48, :105; grpc_utils.py:127).  A packed round
holds every client as a row of one device matrix, so the edge is one
device->host copy of the [clients, P] block, then per client the same dict of
fresh tensors (named_parameters order, clones — never views, or torch.save would
write the whole packed storage) serialised exactly as the reference does:
byte-identical output (golden G9).  The inverse stacks received updates into
packed rows with one host->device copy.

Convergence.  ConvergenceDetector._calculate_weight_change_metrics
(src/aggregation/convergence.py:189-217): per layer ||current - previous|| and
||current|| (torch fp32 norms, .item()), squared and summed in double.  Here the
two per-layer reductions over P run on the chip (fh_dp_delta_sqnorm, fp64
accumulation), each layer's norm is rounded to fp32 like torch's result, and the
nseg-long sums are finished on the host in double.  The reference's torch CPU
norm accumulates in fp32, so the two agree to ~1e-6 relative (tested at 1e-5).
"""
from __future__ import annotations

import io
import math
from typing import Dict, List, Sequence

import torch

from . import ops


def client_weights(rows_cpu: torch.Tensor, layout, slot: int) -> Dict[str, torch.Tensor]:
    """get_model_weights() of packed client `slot` (models_pytorch.py:25-28): fresh tensors
    in named_parameters order."""
    return {n: rows_cpu[slot, o:o + _numel(s)].reshape(s).clone()
            for n, s, o in zip(layout.names, layout.shapes, layout.offsets)}


def _numel(shape):
    n = 1
    for s in shape:
        n *= s
    return n


def serialize_weights(weights: Dict[str, torch.Tensor]) -> bytes:
    """ModelWeightSerializer.serialize_weights (serialization.py:28-48): torch.save bytes."""
    buf = io.BytesIO()
    torch.save(weights, buf)
    return buf.getvalue()


def packed_to_weight_dicts(rows: torch.Tensor, layout, nclients: int) -> List[Dict[str, torch.Tensor]]:
    """All clients' weight dicts from device rows [>=nclients, >=P] with ONE D2H copy."""
    host = rows[:nclients, :layout.P].to("cpu")
    return [client_weights(host, layout, z) for z in range(nclients)]


def weight_dicts_to_packed(dicts: Sequence[Dict[str, torch.Tensor]], layout, device,
                           row_stride: int = None) -> torch.Tensor:
    """Received weight dicts -> packed device rows [C, row_stride] (one H2D copy); rows are
    zero-padded to `row_stride` (default: P rounded up to 64 floats, as PackedTrainer)."""
    P = layout.P
    stride = row_stride or ((P + 63) // 64) * 64
    host = torch.zeros(len(dicts), stride, dtype=torch.float32, pin_memory=False)
    for z, d in enumerate(dicts):
        for n, s, o in zip(layout.names, layout.shapes, layout.offsets):
            t = d[n]
            if tuple(t.shape) != tuple(s):
                raise ValueError(f"client {z}: {n} has shape {tuple(t.shape)}, expected {s}")
            host[z, o:o + t.numel()] = t.reshape(-1).to(torch.float32)
    return host.to(device)


def weight_change_metrics(current: torch.Tensor, previous: torch.Tensor,
                          seg_offsets: torch.Tensor) -> Dict[str, float]:
    """{'norm': ||current - previous||, 'relative': norm / ||current||} over the layers
    (convergence.py:189-217).  current / previous: flat device rows [>=P]; seg_offsets:
    device int64 [nseg+1] layer boundaries."""
    nseg = seg_offsets.numel() - 1
    cur = current.reshape(1, -1)
    diff_sq = ops.dp_delta_sqnorm(cur, previous.reshape(1, -1), seg_offsets, 1)
    cur_sq = ops.dp_delta_sqnorm(cur, None, seg_offsets, 1)
    d = diff_sq.reshape(-1).tolist()
    c = cur_sq.reshape(-1).tolist()
    total, total_cur = 0.0, 0.0
    for t in range(nseg):
        dn = float(torch.tensor(math.sqrt(d[t]), dtype=torch.float32))  # torch fp32 .item()
        cn = float(torch.tensor(math.sqrt(c[t]), dtype=torch.float32))
        total += dn ** 2
        total_cur += cn ** 2
    norm = math.sqrt(total)
    cur_norm = math.sqrt(total_cur)
    return {"norm": norm, "relative": norm / cur_norm if cur_norm > 0 else 0.0}
