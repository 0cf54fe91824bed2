"""Kaldi fbank front end on the GPU (libwsp_hip.so `wsp_fbank`).

Replaces `torchaudio.compliance.kaldi.fbank(...)` + CMN as called by the
reference at cli/speaker.py:89-104 (int16-valued input, scale 1) and
dataset/processor.py:472-502 (`wav * (1 << 15)`, dither forced to 0 at
extraction, bin/extract.py:66-67).
"""
from __future__ import annotations

import itertools

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


def compute_fbank_segments(wavs, scale: float = 1.0, cmn: bool = True, device=None):
    """Whole utterances of different lengths in one launch (wsp_fbank_segments).

    `wavs`: sequence of 1-D arrays / tensors (int16-valued float or int16), each >= 400
    samples.  Returns (feats [sum T_b][80] float32 on the device, frame_offsets int32
    [B+1] on the device, frame counts list).  Row block b equals
    compute_fbank(wavs[b])[0] exactly."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    lens = [int(len(w)) for w in wavs]
    if any(n < FRAME_LEN for n in lens):
        raise ValueError("every utterance needs >= 400 samples (one 25 ms frame)")
    frames = [num_frames(n) for n in lens]
    cat = torch.cat([torch.as_tensor(w).reshape(-1).to(torch.float32) for w in wavs]).to(device)
    so = torch.tensor([0] + list(itertools.accumulate(lens)), dtype=torch.int32, device=device)
    fo_host = [0] + list(itertools.accumulate(frames))
    fo = torch.tensor(fo_host, dtype=torch.int32, device=device)
    feats = torch.empty(fo_host[-1], NUM_BINS, dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    _lib.check(_lib.load().wsp_fbank_segments(cat.data_ptr(), _lib.WSP_DTYPE_F32, len(lens), so.data_ptr(),
                                              fo.data_ptr(), max(frames), float(scale), feats.data_ptr(),
                                              NUM_BINS, 16000, _lib.WSP_WINDOW_HAMMING, int(cmn), stream),
               "wsp_fbank_segments")
    return feats, fo, frames


def apply_cmn(feats: torch.Tensor) -> torch.Tensor:
    """In-place per-utterance mean subtraction over frames of a (B, T, D) float32
    HIP tensor (wsp_cmn) — apply_cmvn(norm_mean=True, norm_var=False),
    dataset_utils.py:19-26, and the subsegment CMN of extract_embedding_feats."""
    if not feats.is_cuda or feats.dtype != torch.float32 or not feats.is_contiguous() or feats.dim() != 3:
        raise ValueError("apply_cmn expects a contiguous (B, T, D) float32 HIP tensor")
    B, T, D = feats.shape
    stream = torch.cuda.current_stream(feats.device).cuda_stream
    _lib.check(_lib.load().wsp_cmn(feats.data_ptr(), B, T, D, stream), "wsp_cmn")
    return feats
