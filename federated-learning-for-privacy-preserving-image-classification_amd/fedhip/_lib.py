"""ctypes binding of libfedhip.so (the C ABI declared in include/fedhip.h).

This module is the ONLY way Python reaches the HIP kernels.  There is no
fallback: if the library is missing, or no HIP device is present, calls raise
``FedHipError`` — the product path never silently drops to a CPU/PyTorch
implementation.

``torch`` is imported first so that the HIP runtime torch ships
(libamdhip64.so.7) is the one libfedhip binds to: both share the soname, so
the dynamic loader reuses torch's copy and device pointers / streams are
interchangeable.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_float, c_int32, c_int64, c_size_t, c_uint64, c_void_p

import torch  # noqa: F401  (must precede CDLL: shared HIP runtime)

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_ROOT, "lib", "libfedhip.so")


class FedHipError(RuntimeError):
    """A libfedhip entry point returned a non-zero status."""


P = c_void_p  # every tensor argument is a raw device pointer
I32, I64, F32, F64, U64, SZ = c_int32, c_int64, c_float, c_double, c_uint64, c_size_t

# name -> (restype, [argtypes]); mirrors include/fedhip.h one for one.
SIGNATURES = {
    "fh_last_error": (ctypes.c_char_p, []),
    "fh_version": (I32, []),
    "fh_fedavg_weighted_sum": (I32, [P, I64, P, P, I32, I64, P, I32, P]),
    "fh_update_stats": (I32, [P, I64, I32, P, I32, P, P, P]),
    "fh_dp_delta_sqnorm": (I32, [P, I64, P, I64, I32, P, I32, P, P]),
    "fh_dp_clip_coef": (I32, [P, I32, I32, F64, F64, F64, P, P, P, P, P]),
    "fh_dp_apply": (I32, [P, I64, P, I64, P, I64, I32, I64, P, P, P, P, I64, U64, P, P]),
    "fh_sgd_step": (I32, [P, P, P, I64, F32, F32, F32, I32, P]),
    "fh_adam_step": (I32, [P, P, P, P, I64, F64, F64, F64, F64, F64, I32, F64, F64, P, P]),
    "fh_sgd_step_slabs": (I32, [P, P, P, I64, I64, I32, P, I32, F32, F32, F32, I32, P]),
    "fh_adam_step_slabs": (I32, [P, P, P, P, I64, I64, I32, P, I32, F64, F64, F64, F64, F64, I32,
                                 F64, F64, P, P]),
    "fh_conv2d_fwd_workspace": (SZ, [I32, I32, I32, I32, I32, I32, I32, I32, I32, I32]),
    "fh_conv2d_dgrad_workspace": (SZ, [I32, I32, I32, I32, I32, I32, I32, I32, I32, I32]),
    "fh_conv2d_fwd": (I32, [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32,
                            I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_dgrad": (I32, [P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32, I32,
                              I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_dgrad_bnstats": (I32, [P, I64, P, I64, P, I64, P, I64, P, P, I64, P, P, P, I64,
                                      P, I64, F32, P, I32, I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_wgrad_workspace": (SZ, [I32, I32, I32, I32, I32, I32, I32, I32, I32, I32]),
    "fh_conv2d_wgrad": (I32, [P, I64, P, I64, P, I64, P, I64, P, SZ, P, I32, I32, I32, I32,
                              I32, I32, I32, I32, I32, I32, P]),
    "fh_linear_fwd_workspace": (SZ, [I32, I32, I32, I32]),
    "fh_linear_dgrad_workspace": (SZ, [I32, I32, I32, I32]),
    "fh_linear_fwd": (I32, [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_linear_fwd_dropout": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32,
                                    I32, I32, I32, F32, U64, P, P, SZ, P]),
    "fh_linear_dgrad": (I32, [P, I64, P, I64, P, I64, P, I32, I32, I32, I32, P, SZ, P]),
    "fh_linear_wgrad_workspace": (SZ, [I32, I32, I32, I32]),
    "fh_linear_wgrad": (I32, [P, I64, P, I64, P, I64, P, I64, P, SZ, P, I32, I32, I32, I32, P]),
    "fh_linear_bwd_fused": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, F32,
                                  P, I64, P, I32, I32, I32, I32, P]),
    "fh_linear_bwd_fused_pool": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P, I64,
                                       P, I32, I32, I32, I32, I32, I32, I32, I32, P]),
    "fh_linear_head_ce": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P, P, P, P, P,
                                P, I64, P, I64, P, I64, P, I64, F32, I32, P, I32, I32, I32, I32,
                                P]),
    "fh_bn_workspace": (SZ, [I32, I32, I32, I32]),
    "fh_bn_fwd_train": (I32, [P, I64, P, I64, P, I64, P, P, I64, P, P, I64, P, P, P, I32, I32,
                              I32, I32, F32, F32, I32, P, SZ, P]),
    "fh_bn_fwd_stats": (I32, [P, I64, P, P, I64, P, P, I64, P, P, P, P, I64, P, I32, I32, I32,
                              I32, F32, F32, P, SZ, P]),
    "fh_conv_bnstats_bytes": (SZ, [I32, I32, I32, I32, I32]),
    "fh_conv2d_fwd_bnstats": (I32, [P, I64, P, P, I64, P, I64, P, I64, P, I64, P, P, I32, I32,
                                    I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_fwd_relu_pool": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P, I32,
                                      I32, I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_maxpool2_fwd_bnfinalize": (I32, [P, P, P, I64, P, P, I64, P, P, P, P, I64, P, I64, P,
                                         I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, F32,
                                         F32, I32, F32, U64, P, P]),
    "fh_bn_finalize_tiles": (I32, [P, P, P, I64, P, P, I64, P, P, P, P, I64, P, I32, I32, I32,
                                   I32, F32, F32, P]),
    "fh_conv2d_dgrad_s2_shortcut": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I32, I32,
                                          I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_maxpool2_bwd_ymask": (I32, [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32,
                                    I32, I32, I32, I32, P]),
    "fh_conv2d_c1_pool_fwd_u8": (I32, [P, P, P, I64, F32, F32, P, I64, P, I64, P, I64, P, I64,
                                       P, I64, P, I64, P, I32, I32, I32, I32, I32, I32, I32, P]),
    "fh_conv2d_c1_pool_fwd": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32,
                                    I32, I32, I32, I32, P]),
    "fh_conv2d_c1_pool_wgrad": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P, SZ, P,
                                      I32, I32, I32, I32, I32, I32, I32, P]),
    "fh_conv2d_c1_pool_wgrad_deferred": (I32, [P, I64, P, I64, P, I64, P, I64, P, I64, P, I64, P,
                                               SZ, P, I32, I32, I32, I32, I32, I32, I32, P, P,
                                               P]),
    "fh_bn_apply_tiles": (I32, [P, P, I64, P, I64, P, I64, P, P, I64, P, P, I64, P, P, P, I32,
                                I32, I32, I32, F32, F32, I32, P]),
    "fh_conv2d_fwd_bnrelu": (I32, [P, I64, P, P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32,
                                   I32, I32, I32, I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_wgrad_deferred": (I32, [P, I64, P, P, I64, P, I64, P, I64, P, I64, P, SZ, P, I32,
                                       I32, I32, I32, I32, I32, I32, I32, I32, I32, P, P, P]),
    "fh_conv2d_wgrad_bnrelu": (I32, [P, I64, P, P, I64, P, I64, P, I64, P, I64, P, SZ, P, I32,
                                     I32, I32, I32, I32, I32, I32, I32, I32, I32, P]),
    "fh_maxpool2_fwd_pitched": (I32, [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32,
                                      I32, F32, U64, P, I32, I32, I32, I32, P]),
    "fh_maxpool2_bwd_pitched": (I32, [P, I64, P, I64, P, I64, F32, P, I64, P, I64, P, I32, I32,
                                      I32, I32, I32, I32, I32, I32, I32, P]),
    "fh_maxpool2_fwd_bnrelu": (I32, [P, I64, P, P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32,
                                     I32, I32, I32, F32, U64, P, P]),
    "fh_bn_fwd_eval": (I32, [P, I64, P, I64, P, I64, P, P, I64, P, P, I64, P, I32, I32, I32,
                             I32, F32, I32, P]),
    "fh_bn_bwd": (I32, [P, I64, P, I64, P, I64, P, P, I64, P, P, P, I64, P, I64, P, P, I64, P,
                        I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_bn_bwd_tiles": (I32, [P, P, I64, P, I64, P, I64, P, P, P, I64, P, P, I64, P, I32, I32,
                              I32, I32, P]),
    "fh_bn_bwd_pool_tiles": (I32, [P, P, I64, P, I64, P, I64, F32, P, I64, P, P, I64, P, P, P,
                                   I64, P, P, I64, P, I32, I32, I32, I32, I32, P]),
    "fh_bn_bwd_pool": (I32, [P, I64, P, I64, P, I64, F32, P, I64, P, I64, P, P, I64, P, P, P, I64,
                             P, P, I64, P, I32, I32, I32, I32, I32, I32, P, SZ, P]),
    "fh_conv2d_persample_sqnorm_workspace": (SZ, [I32] * 10),
    "fh_conv2d_persample_sqnorm": (I32, [P, I64, P, I64, I32, P, P, SZ, P, I32, I32, I32, I32,
                                         I32, I32, I32, I32, I32, I32, P]),
    "fh_linear_persample_sqnorm": (I32, [P, I64, P, I64, I32, P, P, I32, I32, I32, I32, P]),
    "fh_conv2d_wgrad_persample_workspace": (SZ, [I32] * 4),
    "fh_conv2d_wgrad_persample": (I32, [P, I64, P, I64, P, SZ, P, I32, I32, I32, I32, I32, I32,
                                        P]),
    "fh_conv2d_c1_pool_wgrad_persample": (I32, [P, I64, P, I64, P, I64, P, I64, P, SZ, P, I32,
                                                I32, I32, I32, I32, I32, I32, P]),
    "fh_persample_slab_sqnorm": (I32, [P, I32, I32, P, I32, I32, P, P]),
    "fh_linear_wgrad_rowscale_multi": (I32, [P, I32, P, P, I32, I32, P]),
    "fh_linear_wgrad_rowscale": (I32, [P, I64, P, I64, P, P, I64, P, I64, P, I32, I32, I32, I32,
                                       P]),
    "fh_dpsgd_norm_clip": (I32, [P, I32, P, I32, P, I32, I32, F64, P, P, P]),
    "fh_conv2d_c1_pool_wgrad_persample_clip": (I32, [P, I64, P, I64, P, I64, P, I64, P, SZ, P,
                                                     I32, I32, I32, I32, I32, I32, I32, P, I32,
                                                     P, I32, F64, P, P, P]),
    "fh_dpsgd_step_slabs": (I32, [P, P, P, P, I64, I64, I32, P, I32, P, P, I32, I64, F32, U64, P,
                                  I32, F64, F64, F64, F64, F64, F64, I32, I32, F64, F64, P, P]),
    "fh_persample_slab_wsum": (I32, [P, I32, I32, P, P, I32, I32, P, I64, P, I64, P]),
    "fh_dpsgd_clip_coef": (I32, [P, P, I32, I32, F64, P, P]),
    "fh_scale_rows": (I32, [P, I64, P, P, I32, I32, I64, P, I64, P]),
    "fh_dpsgd_noise": (I32, [P, I64, I64, P, I32, I32, F32, U64, P, P]),
    "fh_maxpool2_fwd": (I32, [P, I64, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, I32,
                              F32, U64, P, P]),
    "fh_maxpool2_bwd": (I32, [P, I64, P, I64, P, I64, F32, P, I64, P, I64, P, I32, I32, I32,
                              I32, I32, P]),
    "fh_dropout_fwd": (I32, [P, I64, P, I64, P, I64, P, I32, I32, I64, I32, F32, U64, P, P]),
    "fh_dropout_bwd": (I32, [P, I64, P, I64, F32, P, I64, P, I64, P, I32, I32, I64, P]),
    "fh_ce_fwd_bwd": (I32, [P, I64, P, I64, P, I64, P, P, P, P, P, P, I32, I32, I32, P]),
    "fh_set_fill_fraction": (I32, [F32]),
    "fh_get_fill_fraction": (F32, []),
    "fh_conv_pair": (I32, [I32]),
    "fh_conv_pair_status": (I32, [P, P]),
    "fh_conv_defer_dgrad": (I32, [I32]),
    "fh_conv_defer_status": (I32, [P, P]),
    "fh_conv_bn_defer": (I32, [I32]),
    "fh_conv_bn_defer_status": (I32, [P, P]),
    "fh_set_split_tickets": (I32, [P, I64]),
    "fh_split_tickets_status": (I32, [P]),
    "fh_conv_pooled_dy": (I32, [P, I64, P, I64, P, I64, I32]),
    "fh_launch_ts_set": (I32, [P, P, ctypes.c_uint32, I32, I32, I32]),
    "fh_wall_clock_khz": (I32, [P]),
    "fh_stream_create": (I32, [I32, P, I32, P]),
    "fh_stream_destroy": (I32, [P]),
    "fh_record_begin": (I32, [P]),
    "fh_record_end": (I32, [P, P]),
    "fh_graph_node_counts": (I32, [P, P, P]),
    "fh_program_matches_graph": (I32, [P, P, P]),
    "fh_program_launch": (I32, [P, P]),
    "fh_program_relocate": (I32, [P, P, I32, U64, I64, P]),
    "fh_program_launch_at": (I32, [P, P, U64]),
    "fh_program_destroy": (I32, [P]),
    "fh_copy_bytes": (I32, [P, P, I64, P]),
    "fh_gather_u8": (I32, [P, P, P, I64, P, I64, P, I64, P, I32, I32, I32, I32, I32, P, P, I32,
                           I32, P, P, I64, U64, P, P]),
    "fh_compress_chunk_elems": (I64, []),
    "fh_quantize_workspace": (I64, [I32, I32]),
    "fh_quantize_rows": (I32, [P, I64, P, I64, P, I64, P, I64, I32, P, P, I32, I32, I32, I32, P, P,
                               P, SZ, P]),
    "fh_topk_workspace": (I64, [I32, I32, I32]),
    "fh_topk_rows": (I32, [P, I64, P, I64, P, I64, P, I64, I32, P, P, P, I32, I32, P, SZ, P]),
    "fh_eval_metrics": (I32, [P, I64, P, I64, P, I32, I32, I32, P, P, P, P, P]),
    "fh_avgpool_fwd": (I32, [P, I64, P, I64, P, I32, I32, I32, I32, P]),
    "fh_avgpool_bwd": (I32, [P, I64, P, I64, P, I32, I32, I32, I32, P]),
    "fh_gather_batch": (I32, [P, P, P, I64, P, I64, P, I64, I64, P, I32, I32, P]),
}

_lib = None


def check_build_record(path: str = LIB_PATH, record_path: str | None = None):
    """The in-tree library must match its build record (build_native.py): same source digest
    as the sources beside it, same library bytes.  Raises FedHipError otherwise."""
    import hashlib
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "_fh_build_native", os.path.join(_PKG_ROOT, "build_native.py"))
    bn = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bn)
    rec = bn.read_record(record_path)
    if rec is None:
        raise FedHipError(f"{path} has no build record ({record_path or bn.RECORD}); rebuild "
                          "it with "
                          "`python build_native.py`")
    if rec.get("sources_sha256") != bn.source_digest():
        raise FedHipError(f"{path} was built from other sources than the tree's (stale "
                          "library); rebuild it with `python build_native.py`")
    with open(path, "rb") as fh:
        if hashlib.sha256(fh.read()).hexdigest() != rec.get("lib_sha256"):
            raise FedHipError(f"{path} is not the library its build record describes; "
                              "rebuild it with `python build_native.py`")
    return rec


def load(path: str = LIB_PATH):
    """Load libfedhip.so and bind every declared symbol (raises if absent)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise FedHipError(
            f"libfedhip.so not found at {path}; build it with "
            "`python build_native.py` (HIP/gfx950) — there is no CPU fallback")
    if os.path.abspath(path) == os.path.abspath(LIB_PATH):
        check_build_record(path)
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def ptr(t) -> int | None:
    """Device pointer of a tensor (None passes NULL)."""
    if t is None:
        return None
    return t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def call(name: str, *args):
    """Invoke a status-returning entry point; raise FedHipError on failure."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.fh_last_error().decode(errors="replace")
        raise FedHipError(f"{name} failed (rc={rc}): {msg}")
    return rc


def require_device(t: torch.Tensor, what: str = "tensor"):
    if not t.is_cuda:
        raise FedHipError(f"{what} must live on a HIP device (got {t.device}); "
                          "libfedhip has no CPU path")
