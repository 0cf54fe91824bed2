"""`torchaudio.transforms.Resample` on the HIP path (wsp_resampler_*).

The reference resamples non-16 kHz audio before fbank with
`torchaudio.transforms.Resample(orig_freq=sr, new_freq=resample_rate)` at
wespeaker/cli/speaker.py:155-157 and wespeaker/dataset/processor.py:242-260.
Same constructor (orig_freq, new_freq, resampling_method="sinc_interp_hann",
lowpass_filter_width=6, rolloff=0.99) and call contract (waveform (..., N) ->
(..., ceil(new*N/orig)); orig == new returns the input); the kernel runs in
libwsp_hip.so.  Algorithm and pinning status: oracle/resample_ref.py.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


class Resample:

    def __init__(self, orig_freq: int = 16000, new_freq: int = 16000, resampling_method: str = "sinc_interp_hann",
                 lowpass_filter_width: int = 6, rolloff: float = 0.99, beta=None):
        if resampling_method != "sinc_interp_hann":
            raise NotImplementedError(f"resampling_method {resampling_method!r}: only sinc_interp_hann "
                                      "(torchaudio's default) is implemented")
        if int(orig_freq) != orig_freq or int(new_freq) != new_freq:
            raise ValueError("frequencies must be integers")
        self.orig_freq, self.new_freq = int(orig_freq), int(new_freq)
        self._h = ctypes.c_void_p()
        _lib.check(_lib.load().wsp_resampler_create(self.orig_freq, self.new_freq, int(lowpass_filter_width),
                                                    float(rolloff), ctypes.byref(self._h)), "wsp_resampler_create")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.load().wsp_resampler_destroy(h)
            except Exception:
                pass
            self._h = None

    def out_len(self, num_samples: int) -> int:
        n = ctypes.c_int()
        _lib.check(_lib.load().wsp_resampler_out_len(self._h, int(num_samples), ctypes.byref(n)),
                   "wsp_resampler_out_len")
        return n.value

    def kernel(self):
        """(reduced_orig, reduced_new, width, f32 kernel [new][taps]) — the host plan."""
        o, n, w, t = (ctypes.c_int() for _ in range(4))
        lib = _lib.load()
        _lib.check(lib.wsp_resampler_kernel(self._h, ctypes.byref(o), ctypes.byref(n), ctypes.byref(w),
                                            ctypes.byref(t), None), "wsp_resampler_kernel")
        k = np.zeros((n.value, t.value), dtype=np.float32)
        if self.orig_freq != self.new_freq:
            _lib.check(lib.wsp_resampler_kernel(self._h, None, None, None, None, k.ctypes.data),
                       "wsp_resampler_kernel")
        return o.value, n.value, w.value, k

    def __call__(self, waveform: torch.Tensor) -> torch.Tensor:
        if self.orig_freq == self.new_freq:
            return waveform
        if not waveform.is_cuda:
            raise RuntimeError("Resample runs on a HIP device tensor (no CPU fallback)")
        shape = waveform.shape
        x = waveform.reshape(-1, shape[-1]).to(torch.float32).contiguous()
        B, N = x.shape
        n_out = self.out_len(N)
        y = torch.empty(B, n_out, dtype=torch.float32, device=x.device)
        with torch.cuda.device(x.device):
            stream = torch.cuda.current_stream(x.device).cuda_stream
            _lib.check(_lib.load().wsp_resample(self._h, x.data_ptr(), B, N, N, y.data_ptr(), n_out, stream),
                       "wsp_resample")
        return y.reshape(shape[:-1] + (n_out,))

    forward = __call__


_CACHE = {}


def resample(waveform: torch.Tensor, orig_freq: int, new_freq: int) -> torch.Tensor:
    """Resample(orig_freq, new_freq)(waveform) with the plan cached per rate pair."""
    if orig_freq == new_freq:
        return waveform
    key = (int(orig_freq), int(new_freq))
    if key not in _CACHE:
        _CACHE[key] = Resample(*key)
    return _CACHE[key](waveform)
