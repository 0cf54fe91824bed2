"""FLAC decoding (host side of the data pipeline): ctypes over
native/libwsp_flac.so, built from native/flac.c by __graft_entry__.build()
(`make -C wespeaker_hubert_amd/native`).  The reference gets FLAC through
torchaudio.load (dataset/processor.py:96-110); see audio.load_audio for the
dtype / normalisation conventions applied on top."""
from __future__ import annotations

import ctypes
import os
from typing import Tuple

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libwsp_flac.so")
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: run __graft_entry__.build() (make -C wespeaker_hubert_amd/native)")
        lib = ctypes.CDLL(LIB_PATH)
        lib.wsp_flac_decode.restype = ctypes.c_int
        lib.wsp_flac_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.POINTER(ctypes.c_int32)),
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int64),
                                        ctypes.c_char_p, ctypes.c_int]
        lib.wsp_flac_free.restype = None
        lib.wsp_flac_free.argtypes = [ctypes.POINTER(ctypes.c_int32)]
        _lib = lib
    return _lib


def decode_flac(data: bytes, name: str = "<flac>") -> Tuple[np.ndarray, int, int]:
    """FLAC stream bytes -> (int32 samples (channels, N), sample_rate, bits per sample)."""
    lib = _load()
    out = ctypes.POINTER(ctypes.c_int32)()
    ch, sr, bits = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    ns = ctypes.c_int64()
    err = ctypes.create_string_buffer(256)
    rc = lib.wsp_flac_decode(bytes(data), len(data), ctypes.byref(out), ctypes.byref(ch), ctypes.byref(sr),
                             ctypes.byref(bits), ctypes.byref(ns), err, len(err))
    if rc != 0:
        raise ValueError(f"{name}: {err.value.decode(errors='replace')}")
    try:
        n = ns.value * ch.value
        x = np.ctypeslib.as_array(out, shape=(n,)).copy() if n else np.zeros(0, np.int32)
    finally:
        lib.wsp_flac_free(out)
    return x.reshape(ch.value, ns.value), sr.value, bits.value
