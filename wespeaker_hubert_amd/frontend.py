"""Kaldi fbank front end on the GPU (libwsp_hip.so `wsp_fbank`).

Replaces `torchaudio.compliance.kaldi.fbank(...)` + CMN as called by the
reference at cli/speaker.py:89-104 (int16-valued input, scale 1) and
dataset/processor.py:472-502 (`wav * (1 << 15)`, dither forced to 0 at
extraction, bin/extract.py:66-67).
"""
from __future__ import annotations

import torch

from . import _lib

FRAME_LEN = 400
FRAME_SHIFT = 160
NUM_BINS = 80


def num_frames(num_samples: int) -> int:
    return _lib.load().wsp_fbank_num_frames(int(num_samples), FRAME_LEN, FRAME_SHIFT)


def compute_fbank(wav: torch.Tensor, scale: float = 1.0, cmn: bool = True, num_mel_bins: int = 80,
                  sample_rate: int = 16000, window_type: str = "hamming",
                  out: torch.Tensor = None) -> torch.Tensor:
    """(B, N) float32 / int16 HIP tensor -> (B, T, 80) float32 log-mel (+CMN)."""
    if not wav.is_cuda:
        raise RuntimeError("compute_fbank runs on a HIP device tensor (no CPU fallback)")
    if window_type != "hamming":
        raise NotImplementedError("only window_type='hamming' is implemented")
    if wav.dim() == 1:
        wav = wav.unsqueeze(0)
    if wav.dtype == torch.int16:
        dtype = _lib.WSP_DTYPE_S16
    else:
        wav = wav.float()
        dtype = _lib.WSP_DTYPE_F32
    wav = wav.contiguous()
    B, N = wav.shape
    T = num_frames(N)
    if out is None:
        out = torch.empty(B, T, num_mel_bins, dtype=torch.float32, device=wav.device)
    stream = torch.cuda.current_stream(wav.device).cuda_stream
    _lib.check(_lib.load().wsp_fbank(wav.data_ptr(), dtype, B, N, N, float(scale), out.data_ptr(),
                                     num_mel_bins, sample_rate, _lib.WSP_WINDOW_HAMMING, int(cmn), stream),
               "wsp_fbank")
    return out
