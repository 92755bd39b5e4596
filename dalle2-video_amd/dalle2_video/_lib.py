"""ctypes binding of libdv_hip.so (the C-ABI declared in include/dv_hip.h).

This is the reference-side stub a maintainer would add to bind the HIP path:
plain pointers, ints and the current HIP stream.  There is NO fallback: if
the library is missing or no GPU is present, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DV_HIP_LIB", os.path.join(_HERE, "libdv_hip.so"))

DV_F32, DV_BF16 = 0, 1
ACT_NONE, ACT_SILU = 0, 1

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_longlong
_F = ctypes.c_float

# name -> argtypes (restype is always int except dv_last_error)
_SIGS = {
    "dv_abi_version": [],
    "dv_zero_f32": [_P, _L, _P],
    "dv_conv_fwd_gn_in": [_P, _P, _I, _P, _P, _P, _I, _I, _I, _I, _I, _I, _P, _L, _I, _P],
    "dv_conv_fwd": [_I, _P, _I, _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I,
                    _I, _P, _L, _I, _P],
    "dv_conv_fwd8": [_I, _P, _I, _I, _P, _I, _P, _P, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I,
                     _I, _P, _L, _I, _P],
    "dv_mx8_quant": [_P, _I, _I, _L, _P, _P, _P],
    "dv_mx8_image_bytes": [_I, _I, _P],
    "dv_mx8_pack_conv_weight": [_P, _I, _I, _P, _P],
    "dv_conv_fwd_mx8": [_P, _P, _I, _P, _P, _I, _P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P],
    "dv_xattn_fold_batched": [_I, _P, _I, _F, _P],
    "dv_xattn_fold_bwd_batched": [_P, _I, _F, _P],
    "dv_conv_wgrad_ws": [_I, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_conv_wgrad": [_I, _P, _I, _P, _I, _I, _P, _I, _P, _I, _P, _I, _P, _L, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_conv_wgrad_deferred": [_I, _P, _I, _P, _I, _I, _P, _I, _P, _I, _P, _I, _P, _L, _I, _I, _I, _I, _I, _I,
                               _I, _I, _P, _P],
    "dv_wgrad_reduce_plan": [_P, _I, _P],
    "dv_wgrad_reduce_batched": [_P, _I, _L, _P],
    "dv_wgrad_reduce_one": [_P, _P],
    "dv_cross_embed_image_elems": [_P, _P],
    "dv_cross_embed_pack": [_P, _P, _P],
    "dv_cross_embed_fwd": [_P, _P, _P, _I, _P, _I, _I, _I, _I, _P],
    "dv_cross_embed_wgrad_ws": [_P, _I, _I, _I, _P],
    "dv_cross_embed_wgrad": [_P, _P, _I, _P, _I, _P, _L, _I, _I, _I, _P],
    "dv_conv_small_image_elems": [_I, _I, _I, _P],
    "dv_conv_small_pack": [_P, _P, _I, _I, _I, _P, _P],
    "dv_conv_small_pack_plan": [_P, _I, _P, _P, _P],
    "dv_conv_small_pack_batched": [_P, _I, _L, _P],
    "dv_conv_small_fwd": [_P, _I, _I, _P, _I, _P, _P, _I, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_bias_grad": [_I, _P, _I, _P, _L, _I, _P],
    "dv_pack_conv_weight": [_I, _P, _P, _I, _I, _I, _I, _I, _P],
    "dv_pack_conv_weights_batched": [_P, _I, _L, _P],
    "dv_pack_conv_weight_pairs": [_P, _P, _L, _P],
    "dv_gn_fwd": [_I, _P, _I, _P, _I, _P, _I, _I, _L, _I, _I, _F, _P, _P, _P, _I, _P, _P, _P, _P, _L,
                  _I, _P],
    "dv_gn_fwd_mx8": [_P, _I, _P, _I, _P, _I, _I, _L, _I, _I, _F, _P, _P, _P, _I, _P, _P, _P, _P, _L, _I, _P, _P, _P],
    "dv_gn_bwd": [_I, _P, _I, _P, _I, _P, _I, _I, _L, _I, _I, _P, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _L, _I, _P],
    "dv_gn_path": [_I],
    "dv_ln_fwd": [_I, _P, _I, _P, _I, _P, _I, _L, _I, _P, _P, _F, _P, _P, _P],
    "dv_ln_bwd_ws": [_L, _I, _P],
    "dv_ln_bwd": [_I, _P, _I, _P, _I, _P, _I, _L, _I, _P, _F, _P, _P, _P, _L, _P],
    "dv_ncthw_to_cl": [_I, _P, _P, _I, _I, _I, _I, _I, _I, _P],
    "dv_cl_to_ncthw": [_I, _P, _I, _P, _I, _I, _I, _I, _I, _P],
    "dv_shuffle": [_I, _I, _P, _I, _P, _I, _P, _I, _P, _I, _P, _I, _I, _I, _I, _I, _I, _P],
    "dv_q_sample": [_I, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_mse_loss": [_I, _P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P],
    "dv_mse_loss_bwd": [_I, _P, _I, _P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P],
    "dv_sinusoidal": [_P, _P, _P, _I, _I, _P],
    "dv_linear_group_fwd": [_P, _I, _I, _I, _P, _I, _P],
    "dv_linear_group_bwd": [_P, _I, _I, _I, _P, _I, _P, _I, _P, _P],
    "dv_linear_small_fwd": [_P, _I, _P, _P, _P, _I, _P, _I, _I, _I, _I, _I, _P],
    "dv_linear_small_bwd": [_P, _I, _P, _I, _P, _P, _P, _I, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_adamw": [_P, _P, _P, _P, _L, _L, _F, _F, _F, _F, _F, _F, _F, _P, _P],
    "dv_grad_clip_coef": [_P, _L, _F, _F, _P, _P],
    "dv_p_sample": [_I, _P, _P, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _I, _I, _P],
    "dv_xattn_fold": [_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _P],
    "dv_xattn_fwd": [_I, _P, _I, _P, _I, _L, _L, _I, _P, _P, _P, _P, _F, _P, _P, _P],
    "dv_xattn_bwd_tokens": [_I, _P, _I, _P, _I, _P, _I, _L, _L, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P],
    "dv_xattn_fold_bwd": [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _F, _I, _I, _P],
    "dv_gemm_tn_batched": [_I, _P, _I, _P, _I, _P, _L, _I, _I, _I, _P],
    "dv_gemm_tn_batched_multi": [_I, _I, _P, _P, _P, _P, _P, _L, _I, _I, _I, _P],
    "dv_resize_nearest": [_P, _P, _L, _I, _I, _I, _I, _I, _F, _F, _P],
    "dv_gaussian_blur": [_P, _P, _L, _I, _I, _I, _P, _P],
    "dv_mqa_prep": [_I, _P, _I, _P, _P, _P, _I, _I, _I, _F, _P, _P],
    "dv_mqa_fwd": [_I, _P, _I, _P, _P, _P, _I, _P, _I, _I, _I, _I, _F, _P, _P],
    "dv_mqa_fwd_fp8_ws": [_I, _I, _P],
    "dv_mqa_fwd_fp8": [_P, _I, _P, _P, _P, _L, _P, _I, _P, _I, _I, _I, _I, _P],
    "dv_mqa_bwd_ws": [_I, _I, _I, _I, _I, _I, _I, _P],
    "dv_mqa_bwd": [_I, _P, _I, _P, _I, _P, _I, _P, _P, _P, _P, _I, _P, _P, _L, _P, _I, _P, _I, _I, _I, _I, _F, _I, _P],
    "dv_comm_unique_id": [_P],
    "dv_comm_init": [_P, _I, _I, _I, _P],
    "dv_comm_allreduce": [_P, _P, _L, _I, _I, _P],
    "dv_comm_async_error": [_P],
    "dv_comm_destroy": [_P],
    "dv_comm_abort": [_P],
}


class DvWgradReduceEntry(ctypes.Structure):
    """Mirror of DvWgradReduceEntry (include/dv_hip.h)."""
    _fields_ = [("part", _P), ("dbpart", _P), ("dw", _P), ("db", _P), ("n4", _L), ("blk0", _L),
                ("S", _I), ("G", _I), ("cout", _I), ("acc_w", _I), ("acc_b", _I), ("part_bf16", _I)]


class DvSmallPackEntry(ctypes.Structure):
    """Mirror of DvSmallPackEntry (include/dv_hip.h)."""
    _fields_ = [("w", _P), ("bias", _P), ("image", _P), ("cin", _I), ("cout", _I), ("ksize", _I),
                ("mode", _I), ("wcin", _I)]


class DVError(RuntimeError):
    pass


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DVError(f"libdv_hip.so not found at {LIB_PATH}; build it with "
                          f"`make -C dalle2-video_amd/csrc` (HIP path has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        L.dv_last_error.restype = ctypes.c_char_p
        L.dv_last_error.argtypes = []
        for name, args in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ctypes.c_int
        _lib = L
    return _lib


def exported_symbols():
    return ["dv_last_error", *_SIGS.keys()]


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().dv_last_error().decode(errors="replace")
        raise DVError(f"{name} failed ({rc}): {msg}")


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return DV_F32
    if t.dtype == torch.bfloat16:
        return DV_BF16
    raise DVError(f"unsupported dtype {t.dtype}")


def ctypes_vp(addr):
    return ctypes.c_void_p(addr)


def dtype_name(t):
    return "bf16" if t.dtype == torch.bfloat16 else "float"


def ptr(t):
    """Device address of a tensor for the C-ABI.  Every pointer the library
    takes is a device pointer: a host tensor here would be dereferenced by a
    kernel (a GPU memory fault), so it is rejected before any launch."""
    if t is None:
        return None
    if not t.is_cuda:
        raise DVError("the HIP path runs on the GPU only (got a CPU tensor)")
    return ctypes.c_void_p(t.data_ptr())


def require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise DVError("the HIP path runs on the GPU only (got a CPU tensor)")
