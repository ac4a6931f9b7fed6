"""Loader for the in-tree gfx950 HIP kernel library (``libtoa_hip.so``).

The kernels are plain ``extern "C"`` launchers compiled by ``hipcc
--offload-arch=gfx950`` (see :mod:`tf_operator_amd._build`); they are bound
with :mod:`ctypes` and launched on PyTorch's *current* HIP stream, so they
compose with hipBLASLt GEMMs, RCCL collectives and HIP-graph capture exactly
like native torch ops.

Policy: on a GPU tensor the HIP path is the only path.  If the library is
missing or fails to load, every op raises -- there is no silent eager
fallback on the GPU (CPU tensors use the PyTorch reference implementations
that the numerics tests compare against).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# TOA_HIP_LIB: load another build of the library (in-process A/B of kernel variants)
LIB_PATH = os.environ.get("TOA_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "libtoa_hip.so")

_lock = threading.Lock()
_lib = None
_err = None

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_f = ctypes.c_float
c_p = ctypes.c_void_p

# name -> argtypes (restype is always int = hipError_t)
_SIGS = {
    "toa_sumsq": [c_p, c_i64, c_int, c_p, c_p, c_int, c_p],
    "toa_adamw_flat": [c_p, c_p, c_p, c_int, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_int, c_f, c_p, c_f, c_p],
    "toa_adamw_flat_dstep": [c_p, c_p, c_p, c_int, c_p, c_p, c_i64, c_f, c_f, c_f, c_f, c_f, c_p, c_f, c_p, c_f,
                             c_p],
    "toa_norm_set_fwd_cap": [c_int],
    "toa_lastline_arm": [ctypes.c_char_p, c_i64, c_i64, c_int],
    "toa_lastline_disarm": [],
    "toa_gemm_asm_set_swiglu_persist": [c_int],
    "toa_xent_set_unroll": [c_int],
    "toa_transpose_set_variant": [c_int],
    "toa_wgrad_asm_set_sumsq": [c_p],
    "toa_sum_f32": [c_p, c_i64, c_p, c_p, c_int, c_p],
    "toa_sumsq_ranges": [c_p, c_p, c_p, c_int, c_p, c_p, c_int, c_p],
    "toa_gemm_asm_rope": [c_p, c_i64, c_p, c_i64, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_delta": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_resadd": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_int, c_int, c_int, c_p],
    "toa_adamw_wt": [c_p, c_p, c_p, c_int, c_p, c_p, c_p, c_i64, c_int, c_int, c_f, c_f, c_f, c_f, c_f, c_int, c_f,
                     c_p, c_f, c_p],
    "toa_stream_create_cu_mask": [c_int, c_int, ctypes.POINTER(ctypes.c_void_p)],
    "toa_stream_destroy": [c_p],
    "toa_step_inc": [c_p, c_p],
    "toa_set_stream_variant": [c_int],
    "toa_sgd_flat": [c_p, c_p, c_p, c_i64, c_f, c_f, c_f, c_p],
    "toa_cast_f32_to_bf16": [c_p, c_p, c_i64, c_p],
    "toa_rmsnorm_fwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_f, c_p],
    "toa_rmsnorm_bwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_p],
    "toa_layernorm_fwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_f, c_p],
    "toa_layernorm_bwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_p, c_int, c_int, c_int, c_int,
                          c_p],
    "toa_norm_bwd_blocks": [c_int, c_int],
    "toa_rope_fwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_rope_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_embed_bwd": [c_p, c_p, c_p, c_p, c_int, c_i64, c_int, c_p],
    "toa_swiglu_fwd": [c_p, c_p, c_i64, c_int, c_p],
    "toa_swiglu_bwd": [c_p, c_p, c_p, c_i64, c_int, c_p],
    "toa_xent_fwd": [c_int, c_p, c_p, c_p, c_p, c_i64, c_int, c_i64, c_int, c_p],
    "toa_xent_bwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_i64, c_int, c_p],
    "toa_gemm_bias_act": [c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_gemm_bias_act_dropout": [c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_f,
                                  ctypes.c_uint64, c_p],
    "toa_bias_act_bwd": [c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_p],
    "toa_bias_act_dropout_bwd": [c_int, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_f, ctypes.c_uint64, c_p],
    "toa_dropout_fwd": [c_int, c_p, c_p, c_p, c_i64, c_f, ctypes.c_uint64, ctypes.c_uint64, c_p],
    "toa_accuracy": [c_int, c_p, c_p, c_p, c_int, c_int, c_p],
    "toa_attn_fwd": [c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_p],
    "toa_attn_fwd_asm": [c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_p],
    "toa_attn_fwd_asm_variant": [c_int, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_f, c_p],
    "toa_attn_fwd_asm_timing": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int, c_f,
                                c_p],
    "toa_attn_bwd": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_int,
                     c_f, c_p],
    "toa_wgrad": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_wgrad_split": [c_int, c_int, c_int],
    "toa_wgrad_asm": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_wgrad_asm_variant": [c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_int, c_int, c_int, c_int, c_int,
                              c_p],
    "toa_wgrad_reduce": [c_p, c_p, c_i64, c_int, c_int, c_int, c_int, c_int, c_int, c_p],
    "toa_transpose_bf16": [c_p, c_i64, c_p, c_i64, c_int, c_int, c_p],
    "toa_gemm": [c_int, c_int, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_f, c_int, c_p],
    "toa_gemm_set_algo": [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_int],
    "toa_gemm_current_algo": [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int],
    "toa_bn_fwd_train": [c_int, c_int, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_f, c_f, c_int, c_p, c_p,
                         c_p],
    "toa_bn_fwd_eval": [c_int, c_int, c_p, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_f, c_int, c_p, c_p],
    "toa_bn_bwd": [c_int, c_int, c_p, c_p, c_p, c_int, c_p, c_p, c_i64, c_int, c_p, c_p, c_p, c_p, c_int, c_int, c_p,
                   c_p],
    "toa_gemm_set_no_streamk": [c_int],
    "toa_gemm_prewarm": [],
    "toa_gemm_asm": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_swiglu": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_swiglu_bwd": [c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_swiglu_bwd_variant": [c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_available": [],
    "toa_gemm_asm_trace": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_host_free": [c_p],
    "toa_gemm_asm_stage": [c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_variant": [c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_map": [c_int, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_set_epi_variant": [c_int],
    "toa_gemm_asm_set_phase": [c_int, ctypes.c_uint],
    "toa_wgrad_asm_set_map": [c_int],
    "toa_gemm_asm_set_map": [c_int],
    "toa_gemm_asm_set_persist": [c_int],
    "toa_attn_dkdv_asm_set_arm": [c_int],
    "toa_gemm_asm_timing": [c_int, c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_gemm_asm_probe": [c_p, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_int, c_int, c_int, c_p],
    "toa_attn_set_bwd_variant": [c_int],
    "toa_attn_set_bwd_timing": [c_p],
    "toa_norm_set_row": [c_int],
    "toa_attn_set_fwd_variant": [c_int],
    "toa_attn_set_dkdv_variant": [c_int],
    "toa_attn_dkdv_asm": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int, c_f, c_int,
                          c_p, c_p, c_int, c_p],
    "toa_attn_dkdv_asm_variant": [c_int, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int,
                                  c_f, c_int, c_p, c_p, c_int, c_p],
    "toa_attn_dkdv_asm_timing": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int,
                                 c_f, c_int, c_p, c_p, c_int, c_p],
    "toa_attn_bwd_rope": [c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_p, c_int, c_int, c_int, c_int, c_int,
                          c_int, c_f, c_p],
    "toa_emulate_xfer": [c_p, c_p, c_i64, c_int, ctypes.c_double, c_p],
    "toa_emulate_copy_nocu": [c_p, c_p, c_i64, c_p],
    "toa_flag_publish": [c_p, ctypes.c_uint, c_p],
    "toa_flags_wait": [c_p, c_int, c_int, c_int, ctypes.c_uint, c_p, c_int, c_p],
    "toa_copy_nocu": [c_p, c_p, c_i64, c_p],
    "toa_sum_slices_bf16": [c_p, c_p, c_int, c_i64, c_i64, c_p],
    "toa_gemm_tune": [c_int, c_int, c_i64, c_i64, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_i64, c_f, c_int, c_p, c_p, c_p,
                      c_p, c_p, c_int],
    "toa_gemm_kernel_name": [c_int, c_int, c_i64, c_i64, c_i64, c_i64, c_i64, c_i64, c_int, c_int, c_p, c_int],
}


def _load():
    global _lib, _err
    with _lock:
        if _lib is not None or _err is not None:
            return
        if not os.path.exists(LIB_PATH):
            _err = f"HIP kernel library not built: {LIB_PATH} (run `python -m tf_operator_amd._build`)"
            return
        try:
            lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the box
            _err = f"failed to load {LIB_PATH}: {e}"
            return
        for name, argt in _SIGS.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.argtypes = argt
            fn.restype = c_int
        ws = getattr(lib, "toa_bn_ws_floats", None)
        if ws is not None:
            ws.argtypes, ws.restype = [c_i64, c_int], c_i64
        aw = getattr(lib, "toa_attn_bwd_ws_bytes", None)
        if aw is not None:
            aw.argtypes, aw.restype = [c_int, c_int, c_int, c_int], c_i64
        ha = getattr(lib, "toa_host_coherent_alloc", None)
        if ha is not None:
            ha.argtypes, ha.restype = [ctypes.c_size_t], ctypes.c_void_p
        ww = getattr(lib, "toa_wgrad_workspace", None)
        if ww is not None:
            ww.argtypes, ww.restype = [c_int, c_int, c_int, c_int], c_i64
        _lib = lib


def available() -> bool:
    _load()
    return _lib is not None


def load_error():
    _load()
    return _err


def lib():
    _load()
    if _lib is None:
        raise RuntimeError(_err)
    return _lib


def has(name: str) -> bool:
    return available() and hasattr(_lib, name)


# launchers whose argument / result types _load sets outside _SIGS
_TYPED_ELSEWHERE = {"toa_bn_ws_floats", "toa_attn_bwd_ws_bytes", "toa_host_coherent_alloc", "toa_wgrad_workspace"}


def _fn(name: str):
    """The launcher, refusing one without declared argument types: ctypes
    would pass Python ints as 32-bit C ints, and a 64-bit parameter (a row
    stride) would arrive with garbage in its upper half."""
    if name not in _SIGS and name not in _TYPED_ELSEWHERE:
        raise KeyError(f"{name}: no ctypes signature in ops/_lib.py _SIGS")
    return getattr(lib(), name)


def call(name: str, *args):
    """Invoke launcher `name`; raise on a non-zero hipError_t."""
    rc = _fn(name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    return rc


def call_ret(name: str, *args) -> int:
    """Invoke `name` and return its int result (no error check)."""
    return _fn(name)(*args)


def stream(t: torch.Tensor | None = None):
    dev = t.device if t is not None else None
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def ptr(t: torch.Tensor | None):
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def use_hip(*tensors) -> bool:
    """True when the op must run on the HIP path (any tensor on the GPU)."""
    on_gpu = any(t is not None and t.is_cuda for t in tensors)
    if on_gpu and not available():
        raise RuntimeError(f"tf_operator_amd: GPU tensor but HIP kernels unavailable: {load_error()}")
    return on_gpu


def dtype_code(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return 0
    if t.dtype == torch.float32:
        return 1
    raise TypeError(f"unsupported dtype {t.dtype} (bf16/fp32 only)")
