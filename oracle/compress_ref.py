"""CPU restatement of the reference's update compressors — TEST ORACLE.

Reference: src/shared/compression.py
  :123-247  QuantizationCompressor (_quantize_tensor :203-228, _dequantize_tensor :230-244)
  :250-368  TopKSparsificationCompressor (_sparsify_tensor :327-344, _desparsify_tensor :346-365)

numpy, fp32 arithmetic in the reference's order.  Pinned against the reference
itself by tests/golden (G8).  Test infrastructure only: the product path is
csrc/compress.hip.

Tie rule (top-k): torch.topk's order among equal magnitudes is unspecified; this
restatement (and the HIP kernel) keeps, among the elements whose |x| equals the
k-th largest magnitude, the ones with the LOWEST flat indices.
"""
from __future__ import annotations

import numpy as np


def quant_params(x: np.ndarray, bits: int = 8, symmetric: bool = True):
    """(scale: Python float, zero_point: int) of compression.py:205-213."""
    bits = max(1, min(32, bits))
    levels = 2 ** bits
    if symmetric:
        max_val = float(np.abs(x).max())
        scale = (2 * max_val) / (levels - 1)
        zero_point = (levels - 1) // 2
    else:
        min_val, max_val = float(x.min()), float(x.max())
        scale = (max_val - min_val) / (levels - 1)
        zero_point = -round(min_val / scale)
    return scale, zero_point


def quantize(x: np.ndarray, bits: int = 8, symmetric: bool = True):
    """codes (uint8/int16/int32 by bits), scale, zero_point: round(x / fl32(scale) + zp),
    clamped to [0, levels-1] (compression.py:215-226; round = half to even)."""
    bits = max(1, min(32, bits))
    levels = 2 ** bits
    scale, zp = quant_params(x, bits, symmetric)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.rint(x.astype(np.float32) / np.float32(scale) + np.float32(zp))
    q = np.clip(q, 0, levels - 1)
    q = np.nan_to_num(q, nan=0.0)  # scale 0: x86 converts the NaN codes to 0
    dt = np.uint8 if bits <= 8 else (np.int16 if bits <= 16 else np.int32)
    return q.astype(dt), scale, zp


def dequantize(codes: np.ndarray, scale: float, zero_point: int) -> np.ndarray:
    """(q.float() - zp) * fl32(scale) in fp32 (compression.py:234)."""
    return (codes.astype(np.float32) - np.float32(zero_point)) * np.float32(scale)


def topk_k(numel: int, sparsity_ratio: float) -> int:
    """k = int(n * (1 - ratio)), at least 1 (compression.py:255, 333-338)."""
    r = max(0.0, min(1.0, sparsity_ratio))
    k = int(numel * (1 - r))
    return 1 if k == 0 else k


def topk_indices(x: np.ndarray, k: int) -> np.ndarray:
    """Flat indices of the k largest |x| (ascending index order), lowest-index tie rule."""
    a = np.abs(x.reshape(-1))
    order = np.lexsort((np.arange(a.size), -a.astype(np.float64)))
    return np.sort(order[:k])


def topk_dense(x: np.ndarray, sparsity_ratio: float) -> np.ndarray:
    """decompress(compress(x)): zeros except the top-k entries (compression.py:346-365)."""
    flat = x.reshape(-1)
    idx = topk_indices(flat, topk_k(flat.size, sparsity_ratio))
    out = np.zeros_like(flat)
    out[idx] = flat[idx]
    return out.reshape(x.shape)
