"""ctypes binding of libautovc_hip.so (the C-ABI declared in include/autovc_hip.h).

This is the only place the product path touches native code.  There is no CPU or
PyTorch fallback: if the library is missing or fails to load, every op raises.
Tensors cross the boundary as raw device pointers (``tensor.data_ptr()``) plus
int64 sizes, and every call is enqueued on torch's current HIP stream.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AUTOVC_HIP_LIB", os.path.join(_HERE, "libautovc_hip.so"))

_lib = None
_lock = threading.Lock()

c_int = ctypes.c_int
c_i64 = ctypes.c_int64
c_f32 = ctypes.c_float
c_ptr = ctypes.c_void_p

# name -> argtypes (restype is always int status unless listed in _RESTYPES)
_SIGS: dict[str, list] = {}
_RESTYPES = {"autovc_last_error": ctypes.c_char_p,
             "autovc_gemm_workspace_floats": c_i64, "autovc_bn_workspace_bytes": c_i64,
             "autovc_lstm_bwd_workspace_floats": c_i64, "autovc_lstm2_bwd_workspace_floats": c_i64, "autovc_loss_workspace_bytes": c_i64,
             "autovc_colsum_workspace_floats": c_i64, "autovc_wavenet_packed_floats": c_i64, "autovc_wavenet_ring_frames": c_i64,
             "autovc_wavenet_workspace_bytes": c_i64, "autovc_lstm2_persist_workspace_bytes": c_i64,
             "autovc_lstm_persist_workspace_bytes": c_i64, "autovc_wino5_rows": c_i64, "autovc_bnconv_workspace_floats": c_i64, "autovc_lstm_xcd_workspace_bytes": c_i64}


def sig(name: str, *argtypes):
    _SIGS[name] = list(argtypes)


sig("autovc_last_error")
sig("autovc_abi_version")
sig("autovc_device_sync")
sig("autovc_stft_mel_f32", c_ptr, c_ptr, c_ptr, c_int, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
    c_int, c_int, c_ptr, c_ptr)
sig("autovc_preprocess_f64", c_ptr, c_int, c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_int,
    c_ptr, c_ptr)
sig("autovc_gemm_workspace_floats", c_int, c_int, c_int)
sig("autovc_gemm_set_lds_reserve", c_int)
sig("autovc_gemm_set_fp32_x6", c_int)
sig("autovc_gemm_fp32_x6")
sig("autovc_gemm_f32_splits", c_int, c_int, c_int, c_int)
sig("autovc_stream_create_cu_mask", c_int, c_ptr, c_ptr)
sig("autovc_stream_destroy", c_ptr)
sig("autovc_event_create", c_ptr)
sig("autovc_event_destroy", c_ptr)
sig("autovc_event_record_any", c_ptr, c_ptr)
sig("autovc_stream_wait_event", c_ptr, c_ptr)
sig("autovc_stamp", c_ptr, c_ptr)
sig("autovc_gemm_bf16_splits", c_int, c_int, c_int, c_int)
sig("autovc_gemm_batched_f32", c_int, c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_int, c_ptr, c_i64, c_i64, c_int,
    c_ptr, c_i64, c_i64, c_int, c_ptr)
sig("autovc_wino5_weights_f32", c_int, c_int, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_conv_weights_batched_f32", c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_bnconv_stats_rows", c_i64)
sig("autovc_bnconv_workspace_floats", c_int, c_int, c_int, c_int)
sig("autovc_bnconv_fwd_bf16_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_int,
    c_ptr, c_ptr)
sig("autovc_bnconv_dx_bf16_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_int,
    c_ptr, c_ptr)
sig("autovc_bnconv_dw_bf16_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_bn_dy_f32", c_i64, c_int, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_bn_apply_bf16", c_i64, c_int, c_ptr, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_wino5_input_f32", c_int, c_int, c_int, c_ptr, c_i64, c_ptr, c_ptr)
sig("autovc_wino5_output_f32", c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_i64, c_ptr)
sig("autovc_wino5_dy_f32", c_int, c_int, c_int, c_ptr, c_i64, c_ptr, c_ptr)
sig("autovc_wino5_wgrad_f32", c_int, c_int, c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_wino5_rows", c_int, c_int)
sig("autovc_wino5_input_bn_f32", c_int, c_int, c_int, c_ptr, c_i64, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_wino5_output_stats_f32", c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_i64, c_ptr, c_ptr)
sig("autovc_wino5_output_bnbwd_f32", c_int, c_int, c_int, c_ptr, c_ptr, c_i64, c_ptr, c_int, c_ptr, c_i64, c_ptr,
    c_ptr)
sig("autovc_wino5_bnbwd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr)
sig("autovc_bn_finalize_f32", c_int, c_i64, c_int, c_ptr, c_ptr, c_ptr, c_f32, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_f32, c_ptr, c_ptr)
sig("autovc_bn_coef_f32", c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_f32, c_ptr, c_ptr)
sig("autovc_bn_partial_rows", c_i64)
sig("autovc_bn_bwd_partial_f32", c_i64, c_int, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_bn_bwd_finalize_f32", c_int, c_int, c_ptr, c_ptr, c_f32, c_ptr, c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_colsum_f64_finalize_f32", c_int, c_int, c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_bn_bwd_finalize_bias_f32", c_int, c_int, c_ptr, c_ptr, c_f32, c_ptr, c_ptr, c_ptr, c_int, c_int, c_int,
    c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_gemm_f32", c_int, c_int, c_int,
    c_ptr, c_i64, c_int, c_int, c_int, c_int,
    c_ptr, c_i64, c_int, c_int, c_int, c_int,
    c_ptr, c_i64, c_ptr, c_ptr, c_int, c_int, c_ptr, c_ptr)
sig("autovc_gemm_bf16_f32", c_int, c_int, c_int,
    c_ptr, c_i64, c_int, c_int, c_int, c_int,
    c_ptr, c_i64, c_int, c_int, c_int, c_int,
    c_ptr, c_i64, c_ptr, c_ptr, c_int, c_int, c_ptr, c_ptr)
sig("autovc_gemm_bf16src_f32", c_int, c_int, c_int, c_ptr, c_i64, c_int,
    c_ptr, c_i64, c_int, c_int, c_int, c_int,
    c_ptr, c_i64, c_ptr, c_ptr, c_int, c_int, c_ptr, c_int, c_ptr)
sig("autovc_bn_workspace_bytes", c_int)
sig("autovc_bn_stats_f32", c_i64, c_int, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_f32, c_ptr,
    c_ptr, c_ptr)
sig("autovc_bn_act_fwd_f32", c_i64, c_int, c_ptr, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_f32, c_int,
    c_ptr, c_i64, c_ptr, c_i64, c_ptr)
sig("autovc_bn_act_bwd_f32", c_i64, c_int, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_i64, c_ptr, c_ptr,
    c_ptr, c_f32, c_int, c_ptr, c_i64, c_ptr, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_lstm_fwd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64,
    c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_lstm2_fwd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_lstm2_fwd_timed_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, ctypes.POINTER(c_f32))
sig("autovc_lstm_fwd_timed_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64,
    c_ptr, c_ptr, c_ptr, ctypes.POINTER(c_f32))
sig("autovc_lstm_bwd_workspace_floats", c_int, c_int, c_int)
sig("autovc_lstm_bwd_set_fused", c_int)
sig("autovc_lstm_bwd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr,
    c_int, c_int, c_ptr, c_ptr)
sig("autovc_lstm2_bwd_workspace_floats", c_int, c_int, c_int)
sig("autovc_lstm2_bwd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_lstm2_persist_workspace_bytes", c_int, c_int, c_int)
sig("autovc_lstm2_persist_supported", c_int, c_int)
sig("autovc_lstm2_fwd_persist_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_lstm2_persist_status", c_ptr, c_ptr)
sig("autovc_fault_status", c_ptr, c_int, c_ptr)
sig("autovc_lstm_persist_set_timeout_ticks", c_int)
sig("autovc_lstm_xcd_supported", c_int, c_int)
sig("autovc_lstm_xcd_workspace_bytes")
sig("autovc_lstm_fwd_xcd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_ptr,
    c_ptr, c_ptr)
sig("autovc_lstm_fwd_xcd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr,
    c_ptr)
sig("autovc_lstm_bwd_xcd_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_lstm_bwd_xcd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr)
sig("autovc_lstm2_fwd_persist_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_lstm_persist_workspace_bytes", c_int, c_int, c_int)
sig("autovc_lstm_persist_supported", c_int, c_int)
sig("autovc_lstm_fwd_persist_f32", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_i64, c_i64, c_ptr, c_ptr,
    c_ptr, c_ptr)
sig("autovc_lstm_fwd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_int, c_ptr)
sig("autovc_lstm2_fwd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_lstm2_bwd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_lstm_bwd_bf16", c_int, c_int, c_int, c_ptr, c_i64, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_int, c_int, c_ptr, c_ptr)
sig("autovc_blstm_fwd_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr)
sig("autovc_blstm_bwd_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr,
    c_ptr)
sig("autovc_frame_concat_f32", c_int, c_int, c_int, c_int, c_int, c_ptr, c_i64, c_ptr, c_ptr, c_ptr)
sig("autovc_frame_concat_bwd_f32", c_int, c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_i64, c_ptr,
    c_int, c_ptr)
sig("autovc_code_gather_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr)
sig("autovc_code_gather_bwd_f32", c_int, c_int, c_int, c_int, c_ptr, c_ptr, c_ptr)
sig("autovc_loss_workspace_bytes")
sig("autovc_loss_f32", c_int, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_loss_bwd_f32", c_int, c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_ptr, c_int, c_int, c_ptr)
sig("autovc_adam_f32", c_i64, c_ptr, c_ptr, c_ptr, c_ptr, c_f32, c_f32, c_f32, c_f32, c_f32, c_f32,
    c_f32, c_ptr)
sig("autovc_conv_pack_f32", c_int, c_int, c_int, c_ptr, c_ptr, c_ptr, c_ptr)
sig("autovc_conv_unpack_grad_f32", c_int, c_int, c_int, c_ptr, c_ptr, c_int, c_ptr)
sig("autovc_transpose_f32", c_int, c_int, c_ptr, c_ptr, c_ptr)
sig("autovc_l2norm_rows_f32", c_int, c_int, c_ptr, c_i64, c_ptr, c_i64, c_ptr)
sig("autovc_colsum_workspace_floats", c_int)
sig("autovc_colsum_f32", c_i64, c_int, c_ptr, c_i64, c_ptr, c_ptr, c_int, c_ptr, c_ptr)
sig("autovc_wavenet_packed_floats", c_int, c_int, c_int, c_int, c_int, c_int)
sig("autovc_wavenet_set_grid", c_int)
sig("autovc_wavenet_get_grid")
sig("autovc_wavenet_grid_explicit")
sig("autovc_wavenet_reset_grid")
sig("autovc_wavenet_last_path")
sig("autovc_wavenet_grid_diag", c_int, c_ptr)
sig("autovc_wavenet_set_timeout_ticks", c_int)
sig("autovc_wavenet_fault", c_int, c_ptr)
sig("autovc_wavenet_ring_frames", c_int, c_int, c_int)
sig("autovc_wavenet_workspace_bytes", c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int)
sig("autovc_wavenet_upsample_f32", c_int, c_int, c_int, c_int, ctypes.POINTER(c_int), c_ptr, c_ptr, c_ptr,
    c_ptr, c_ptr)
sig("autovc_wavenet_generate_f32", c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
    c_int, c_int, c_ptr, c_ptr, c_int, ctypes.c_uint64, c_int, c_f32, c_ptr, c_int, c_ptr, c_ptr, c_ptr,
    c_int, c_ptr)


class HipLibraryError(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise HipLibraryError(
                f"libautovc_hip.so not found at {LIB_PATH}: build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (there is no CPU fallback)")
        # torch first: its libamdhip64.so.7 is then the one the library binds to
        import torch  # noqa: F401
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, argtypes in _SIGS.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = _RESTYPES.get(name, c_int)
        _lib = lib
        return lib


def exported_symbols() -> list[str]:
    return sorted(_SIGS)


def call(name: str, *args):
    """Call an entry point and convert a non-zero status into an exception."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.autovc_last_error().decode(errors="replace")
        if rc == -1:
            raise ValueError(f"{name}: {msg}")
        raise HipLibraryError(f"{name} failed ({rc}): {msg}")
    return rc


def stream_ptr(device=None) -> int:
    import torch
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    return 0 if t is None else t.data_ptr()
