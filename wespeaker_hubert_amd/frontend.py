"""Kaldi fbank front end on the GPU (libwsp_hip.so `wsp_fbank_ex`).

Replaces `torchaudio.compliance.kaldi.fbank(...)` + CMN as called by the
reference at cli/speaker.py:89-104 (int16-valued input, scale 1, the Speaker's
window_type) and dataset/processor.py:472-502 (`wav * (1 << 15)`, the recipe's
`fbank_args`, dither forced to 0 at extraction, bin/extract.py:66-67), and
`apply_cmvn` (dataset_utils.py:19-26) as bin/extract.py:104-106 applies it.

`FbankArgs` carries the options the reference passes (num_mel_bins,
frame_length, frame_shift, sample_frequency, window_type); the mel filters are
computed by the library's host code from torchaudio's formula when a
configuration is first used.
"""
from __future__ import annotations

import ctypes
import itertools
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from . import _lib

FRAME_LEN = 400     # 25 ms at 16 kHz
FRAME_SHIFT = 160   # 10 ms at 16 kHz
NUM_BINS = 80


@dataclass(frozen=True)
class FbankArgs:
    """kaldi.fbank keyword arguments on the extraction path (processor.compute_fbank
    signature: num_mel_bins, frame_length, frame_shift [ms]; sample_frequency; window_type)."""
    num_mel_bins: int = 80
    frame_length: float = 25.0
    frame_shift: float = 10.0
    sample_rate: int = 16000
    window_type: str = "hamming"

    @classmethod
    def from_config(cls, fbank_args: Optional[dict], sample_rate: int = 16000,
                    window_type: str = "hamming") -> "FbankArgs":
        """dataset_args.fbank_args of a recipe yaml (processor.py:472-476); `dither`
        is forced to 0 at extraction (bin/extract.py:66-67) and so ignored."""
        fa = dict(fbank_args or {})
        fa.pop("dither", None)
        unknown = set(fa) - {"num_mel_bins", "frame_length", "frame_shift"}
        if unknown:
            raise NotImplementedError(f"fbank_args {sorted(unknown)} are not on the extraction path")
        return cls(int(fa.get("num_mel_bins", 80)), float(fa.get("frame_length", 25)),
                   float(fa.get("frame_shift", 10)), int(sample_rate), window_type)

    def opts(self) -> _lib.FbankOpts:
        if self.window_type not in _lib.WINDOW_TYPES:
            raise ValueError(f"Invalid window type {self.window_type}")  # kaldi.py's message
        o = _lib.FbankOpts()
        _lib.check(_lib.load().wsp_fbank_opts_default(ctypes.byref(o)), "wsp_fbank_opts_default")
        o.num_mel_bins = int(self.num_mel_bins)
        o.sample_rate = int(self.sample_rate)
        o.frame_length_ms = float(self.frame_length)
        o.frame_shift_ms = float(self.frame_shift)
        o.window_type = _lib.WINDOW_TYPES[self.window_type]
        return o

    def geometry(self) -> Tuple[int, int, int]:
        """(samples per frame, samples per shift, padded FFT size); raises for
        configurations the kernel does not implement."""
        fl, fs, p = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        o = self.opts()
        _lib.check(_lib.load().wsp_fbank_geometry(ctypes.byref(o), ctypes.byref(fl), ctypes.byref(fs),
                                                  ctypes.byref(p)), "wsp_fbank_geometry")
        return fl.value, fs.value, p.value

    def num_frames(self, num_samples: int) -> int:
        fl, fs, _ = self.geometry()
        return num_frames(num_samples, fl, fs)

    def mel_banks(self) -> np.ndarray:
        """The float32 filters the kernel uses: [num_mel_bins][padded / 2 + 1] (host)."""
        _, _, p = self.geometry()
        w = np.zeros((self.num_mel_bins, p // 2 + 1), dtype=np.float32)
        o = self.opts()
        _lib.check(_lib.load().wsp_fbank_mel_banks(ctypes.byref(o), w.ctypes.data), "wsp_fbank_mel_banks")
        return w


DEFAULT = FbankArgs()


def num_frames(num_samples: int, frame_len: int = FRAME_LEN, frame_shift: int = FRAME_SHIFT) -> int:
    return _lib.load().wsp_fbank_num_frames(int(num_samples), int(frame_len), int(frame_shift))


def compute_fbank(wav: torch.Tensor, scale: float = 1.0, cmn: bool = True, num_mel_bins: int = 80,
                  sample_rate: int = 16000, window_type: str = "hamming",
                  out: torch.Tensor = None, frame_length: float = 25.0, frame_shift: float = 10.0,
                  args: Optional[FbankArgs] = None) -> torch.Tensor:
    """(B, N) float32 / int16 HIP tensor -> (B, T, num_mel_bins) float32 log-mel (+CMN)."""
    if not wav.is_cuda:
        raise RuntimeError("compute_fbank runs on a HIP device tensor (no CPU fallback)")
    if args is None:
        args = FbankArgs(num_mel_bins, frame_length, frame_shift, sample_rate, window_type)
    opts = args.opts()
    if wav.dim() == 1:
        wav = wav.unsqueeze(0)
    if wav.dtype == torch.int16:
        dtype = _lib.WSP_DTYPE_S16
    else:
        wav = wav.float()
        dtype = _lib.WSP_DTYPE_F32
    wav = wav.contiguous()
    B, N = wav.shape
    T = args.num_frames(N)
    if out is None:
        out = torch.empty(B, T, args.num_mel_bins, dtype=torch.float32, device=wav.device)
    stream = torch.cuda.current_stream(wav.device).cuda_stream
    _lib.check(_lib.load().wsp_fbank_ex(wav.data_ptr(), dtype, B, N, N, float(scale), out.data_ptr(),
                                        ctypes.byref(opts), int(cmn), stream), "wsp_fbank_ex")
    return out


def compute_fbank_segments(wavs, scale: float = 1.0, cmn: bool = True, device=None,
                           args: Optional[FbankArgs] = None):
    """Whole utterances of different lengths in one launch (wsp_fbank_segments_ex).

    `wavs`: sequence of 1-D arrays / tensors (int16-valued float or int16), each at
    least one frame long.  Returns (feats [sum T_b][bins] float32 on the device,
    frame_offsets int32 [B+1] on the device, frame counts list).  Row block b equals
    compute_fbank(wavs[b])[0] exactly."""
    args = args or DEFAULT
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    fl, fs, _ = args.geometry()
    lens = [int(len(w)) for w in wavs]
    if any(n < fl for n in lens):
        raise ValueError(f"every utterance needs >= {fl} samples (one {args.frame_length} ms frame)")
    frames = [num_frames(n, fl, fs) for n in lens]
    cat = torch.cat([torch.as_tensor(w).reshape(-1).to(torch.float32) for w in wavs]).to(device)
    so = torch.tensor([0] + list(itertools.accumulate(lens)), dtype=torch.int32, device=device)
    fo_host = [0] + list(itertools.accumulate(frames))
    fo = torch.tensor(fo_host, dtype=torch.int32, device=device)
    feats = torch.empty(fo_host[-1], args.num_mel_bins, dtype=torch.float32, device=device)
    stream = torch.cuda.current_stream(device).cuda_stream
    opts = args.opts()
    _lib.check(_lib.load().wsp_fbank_segments_ex(cat.data_ptr(), _lib.WSP_DTYPE_F32, len(lens), so.data_ptr(),
                                                 fo.data_ptr(), max(frames), float(scale), feats.data_ptr(),
                                                 ctypes.byref(opts), int(cmn), stream),
               "wsp_fbank_segments_ex")
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


def apply_cmvn(feats: torch.Tensor, norm_mean: bool = True, norm_var: bool = False,
               frame_offsets: Optional[torch.Tensor] = None) -> torch.Tensor:
    """apply_cmvn(feats, norm_mean, norm_var) of dataset_utils.py:19-26, in place on the
    device (wsp_cmvn): (B, T, D) per utterance, or a ragged (rows, D) batch with int32
    device `frame_offsets` [B+1]."""
    if not feats.is_cuda or feats.dtype != torch.float32 or not feats.is_contiguous():
        raise ValueError("apply_cmvn expects a contiguous float32 HIP tensor")
    stream = torch.cuda.current_stream(feats.device).cuda_stream
    if frame_offsets is None:
        if feats.dim() != 3:
            raise ValueError("apply_cmvn expects (B, T, D) without frame_offsets")
        B, T, D = feats.shape
        ptr = None
    else:
        if feats.dim() != 2 or not frame_offsets.is_cuda or frame_offsets.dtype != torch.int32:
            raise ValueError("ragged apply_cmvn expects (rows, D) feats and int32 device offsets")
        B, T, D = frame_offsets.numel() - 1, 0, feats.shape[1]
        ptr = frame_offsets.data_ptr()
    _lib.check(_lib.load().wsp_cmvn(feats.data_ptr(), B, T, D, ptr, int(norm_mean), int(norm_var), stream),
               "wsp_cmvn")
    return feats
