"""ctypes binding of libwsp_hip.so (include/wespeaker_amd.h).

The HIP library is the product path.  There is no CPU fallback: if the shared
library is missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libwsp_hip.so")

WSP_DTYPE_F32 = 0
WSP_DTYPE_S16 = 1
WSP_WINDOW_HAMMING = 0
WSP_WINDOW_POVEY = 1
WSP_WINDOW_HANNING = 2
WSP_WINDOW_RECTANGULAR = 3
WSP_WINDOW_BLACKMAN = 4
# kaldi.fbank window_type names (torchaudio compliance/kaldi.py)
WINDOW_TYPES = {"hamming": WSP_WINDOW_HAMMING, "povey": WSP_WINDOW_POVEY, "hanning": WSP_WINDOW_HANNING,
                "rectangular": WSP_WINDOW_RECTANGULAR, "blackman": WSP_WINDOW_BLACKMAN}


class FbankOpts(ctypes.Structure):
    """wsp_fbank_opts (include/wespeaker_amd.h)."""
    _fields_ = [("num_mel_bins", c_int), ("sample_rate", c_int), ("frame_length_ms", c_double),
                ("frame_shift_ms", c_double), ("window_type", c_int), ("low_freq", c_double),
                ("high_freq", c_double)]

# name -> (restype, argtypes)
SIGNATURES = {
    "wsp_abi_version": (c_int, []),
    "wsp_last_error": (c_char_p, []),
    "wsp_fbank_num_frames": (c_int, [c_int, c_int, c_int]),
    "wsp_fbank": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_int, c_int,
                          c_int, c_int, c_void_p]),
    "wsp_fbank_segments": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_float, c_void_p, c_int,
                                   c_int, c_int, c_int, c_void_p]),
    "wsp_fbank_opts_default": (c_int, [c_void_p]),
    "wsp_fbank_geometry": (c_int, [c_void_p, POINTER(c_int), POINTER(c_int), POINTER(c_int)]),
    "wsp_fbank_mel_banks": (c_int, [c_void_p, c_void_p]),
    "wsp_fbank_ex": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_void_p, c_int, c_void_p]),
    "wsp_fbank_segments_ex": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_float, c_void_p,
                                      c_void_p, c_int, c_void_p]),
    "wsp_model_create": (c_int, [c_char_p, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "wsp_model_destroy": (c_int, [c_void_p]),
    "wsp_model_num_params": (c_int, [c_void_p]),
    "wsp_model_param_info": (c_int, [c_void_p, c_int, POINTER(c_char_p), POINTER(c_int),
                                     POINTER(c_int64)]),
    "wsp_model_set_param": (c_int, [c_void_p, c_int, c_void_p, c_int64]),
    "wsp_model_finalize": (c_int, [c_void_p]),
    "wsp_model_embed_dim": (c_int, [c_void_p]),
    "wsp_model_feat_dim": (c_int, [c_void_p]),
    "wsp_model_workspace_bytes": (c_int, [c_void_p, c_int, c_int, POINTER(c_size_t)]),
    "wsp_model_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_size_t,
                                  c_void_p]),
    "wsp_model_workspace_bytes_segments": (c_int, [c_void_p, c_int, c_int, POINTER(c_size_t)]),
    "wsp_model_forward_segments": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p,
                                           c_size_t, c_void_p]),
    "wsp_model_set_option": (c_int, [c_void_p, c_char_p, c_int]),
    "wsp_model_get_option": (c_int, [c_void_p, c_char_p, POINTER(c_int)]),
    "wsp_frontend_out_frames": (c_int, [c_void_p, c_int, POINTER(c_int)]),
    "wsp_frontend_workspace_bytes": (c_int, [c_void_p, c_int, c_int, POINTER(c_size_t)]),
    "wsp_frontend_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_int, c_void_p, c_size_t,
                                     c_void_p]),
    "wsp_frontend_workspace_bytes_segments": (c_int, [c_void_p, c_int, c_void_p, POINTER(c_size_t)]),
    "wsp_frontend_forward_segments": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int,
                                              c_void_p, c_size_t, c_void_p]),
    "wsp_model_profile": (c_int, [c_void_p, c_int]),
    "wsp_model_profile_query": (c_int, [c_void_p, c_char_p, POINTER(c_int), POINTER(c_double),
                                        POINTER(c_double)]),
    "wsp_cmn": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p]),
    "wsp_cmvn": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "wsp_resampler_create": (c_int, [c_int, c_int, c_int, c_float, c_void_p]),
    "wsp_resampler_destroy": (c_int, [c_void_p]),
    "wsp_resampler_out_len": (c_int, [c_void_p, c_int, c_void_p]),
    "wsp_resample": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "wsp_resampler_kernel": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "wsp_l2_normalize": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "wsp_cosine_pairs": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "wsp_asnorm_stats": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_size_t, c_void_p]),
    "wsp_asnorm_workspace_bytes": (c_int, [c_int, c_int, c_int, POINTER(c_size_t)]),
    "wsp_row_mean_accum": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
}

_lib = None


class WspError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) the HIP library; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise WspError(f"HIP library not built: {LIB_PATH} is missing "
                       "(run `python -c 'import __graft_entry__ as g; g.build()'`)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = load().wsp_last_error().decode("utf-8", "replace")
        raise WspError(f"{what} failed (status {status}): {msg}")


def call(name: str, *args) -> int:
    st = getattr(load(), name)(*args)
    check(st, name)
    return st
