"""Update compression of packed client rows on HIP (csrc/compress.hip).

Reference: src/shared/compression.py — QuantizationCompressor (:123-247) and
TopKSparsificationCompressor (:250-368), applied per parameter tensor.  The
reference never wires compression into its live path; the
insertion point chosen here is the client update delta right
before FedAvg:

    w_k <- w_global + decompress(compress(w_k - w_global))     per tensor

which is what a server would reconstruct from a compressed upload of the delta.
``RankRound(compression=...)`` applies it to every client row of a round in
one pass per kernel (no host sync).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import torch

from ._lib import FedHipError, call, load, ptr, stream_handle
from .ops import _ws


@dataclass
class CompressionConfig:
    """algorithm: "quantization" (bits, symmetric) or "topk" (sparsity_ratio)."""
    algorithm: str = "topk"
    sparsity_ratio: float = 0.9
    bits: int = 8
    symmetric: bool = True

    def __post_init__(self):
        if self.algorithm not in ("quantization", "topk"):
            raise FedHipError(f"unknown compression algorithm {self.algorithm!r}")


def topk_k(numel: int, sparsity_ratio: float) -> int:
    """k = int(n * (1 - ratio)), at least 1 (compression.py:255, 333-338)."""
    r = max(0.0, min(1.0, sparsity_ratio))
    k = int(numel * (1 - r))
    return 1 if k == 0 else k


class SegmentPlan:
    """Device-side segment table of one parameter layout: seg_offsets [nseg+1] (int64),
    chunk_offsets [nseg+1] (int32, cumulative chunk counts) and per-ratio k tables."""

    def __init__(self, seg_offsets: Sequence[int], device):
        lib = load()
        self.device = torch.device(device)
        self.chunk = int(lib.fh_compress_chunk_elems())
        offs = [int(o) for o in seg_offsets]
        self.lengths = [b - a for a, b in zip(offs[:-1], offs[1:])]
        if not self.lengths or min(self.lengths) <= 0:
            raise FedHipError("compression needs non-empty segments")
        co = [0]
        for n in self.lengths:
            co.append(co[-1] + -(-n // self.chunk))
        self.nseg, self.nchunks = len(self.lengths), co[-1]
        self.seg_offsets = torch.tensor(offs, dtype=torch.int64, device=self.device)
        self.chunk_offsets = torch.tensor(co, dtype=torch.int32, device=self.device)
        self._k = {}

    def seg_k(self, ratio: float) -> torch.Tensor:
        if ratio not in self._k:
            self._k[ratio] = torch.tensor([topk_k(n, ratio) for n in self.lengths],
                                          dtype=torch.int64, device=self.device)
        return self._k[ratio]


def _cs(t):
    return 0 if t is None else t.stride(0)


def quantize_rows(plan: SegmentPlan, x, nclients, bits=8, symmetric=True, base=None, out=None,
                  codes=None, scale_out=None, zp_out=None):
    """out = base + dequantize(quantize(x - base)) per (client row, segment)."""
    lib = load()
    need = int(lib.fh_quantize_workspace(nclients, plan.nchunks))
    ws = _ws(x.device).get(max(need, 1))
    call("fh_quantize_rows", ptr(x), x.stride(0), ptr(base), _cs(base), ptr(out), _cs(out),
         ptr(codes), _cs(codes), nclients, ptr(plan.seg_offsets), ptr(plan.chunk_offsets),
         plan.nseg, plan.nchunks, int(bits), int(bool(symmetric)), ptr(scale_out), ptr(zp_out),
         ptr(ws), ws.numel(), stream_handle())
    return out


def topk_rows(plan: SegmentPlan, x, nclients, sparsity_ratio=0.9, base=None, out=None,
              keep=None):
    """out = base + topk_dense(x - base) per (client row, segment)."""
    lib = load()
    need = int(lib.fh_topk_workspace(nclients, plan.nseg, plan.nchunks))
    ws = _ws(x.device).get(max(need, 1))
    call("fh_topk_rows", ptr(x), x.stride(0), ptr(base), _cs(base), ptr(out), _cs(out),
         ptr(keep), _cs(keep), nclients, ptr(plan.seg_offsets), ptr(plan.chunk_offsets),
         ptr(plan.seg_k(float(sparsity_ratio))), plan.nseg, plan.nchunks, ptr(ws), ws.numel(),
         stream_handle())
    return out


def compress_rows(plan: SegmentPlan, cfg: CompressionConfig, rows, nclients,
                  base: Optional[torch.Tensor] = None):
    """In place: rows[:nclients] <- base + decompress(compress(rows - base))."""
    if cfg.algorithm == "topk":
        return topk_rows(plan, rows, nclients, cfg.sparsity_ratio, base=base, out=rows)
    return quantize_rows(plan, rows, nclients, cfg.bits, cfg.symmetric, base=base, out=rows)
