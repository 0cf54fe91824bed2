"""ORACLE (test infrastructure only): Kaldi-compatible log-mel fbank in numpy.

Restates `torchaudio.compliance.kaldi.fbank` (third-party dependency of the
reference, `requirements.txt` torchaudio>=0.12, unpinned; NOT installed here)
exactly as the reference calls it:

  * cli/speaker.py:89-104  kaldi.fbank(num_mel_bins=80, frame_length=25,
    frame_shift=10, sample_frequency=sr, window_type=self.window_type) then CMN
    `feat - mean(feat, 0)`; dither / energy at torchaudio defaults (0.0/False).
    Windows: kaldi.py _feature_window_function (hamming, hanning, povey,
    rectangular, blackman).  Recipes' fbank_args: num_mel_bins 40 / 64 / 72 / 80
    at 8 or 16 kHz (examples/sre/v2,v3/conf/resnet.yaml: 40 / 64 bins).
  * dataset/processor.py:472-502  same with `wav * (1 << 15)` and dither
    forced to 0.0 by bin/extract.py:66-67.

Published algorithm (torchaudio compliance/kaldi.py, v0.12-2.x):
  snip_edges framing (n = 1 + (N - 400) // 160) -> per-frame DC removal ->
  pre-emphasis 0.97 with replicate pad (x[0] -= 0.97 x[0]) -> symmetric
  Hamming 0.54 - 0.46 cos(2 pi n / (L-1)) -> zero-pad to 512 -> rFFT ->
  |X|^2 -> 80 triangular mel filters 20 Hz .. Nyquist (mel = 1127 ln(1+f/700),
  filter column for the Nyquist bin = 0) -> log(max(e, FLT_EPSILON)).

The reference's own native restatement of the same algorithm is
runtime/core/frontend/fbank.h:138-198 (+ fft.cc:59-119); it needs glog and is
therefore not compilable here without a stand-in header, so it is read, not
built.  Parity with the reference's own outputs is unpinned (no fixture holds
fbank outputs, torchaudio is absent); the restatement is **proxy-pinned** to an
independent third-party implementation of the same algorithm,
transformers.audio_utils (5.15; the numpy path of its Speech2Text / AST feature
extractors): the frame pipeline agrees within 5e-6 with the same filters and the
filters within 2e-5 (float32 rounding) for 23-128 bins, 8 / 16 kHz and every
window (tests/test_fbank_proxy_cpu.py); `fbank()` is also cross-checked against
`fbank_dft64()` (independent float64 direct-DFT formulation).
"""
from __future__ import annotations

import functools
import math

import numpy as np

FLT_EPS = np.float32(np.finfo(np.float32).eps)


def mel_scale(f):
    return 1127.0 * np.log(1.0 + np.asarray(f) / 700.0)


def mel_banks(num_bins=80, padded=512, sample_freq=16000.0, low_freq=20.0, high_freq=0.0,
              dtype=np.float32) -> np.ndarray:
    return _mel_banks(num_bins, padded, sample_freq, low_freq, high_freq).astype(dtype)


@functools.lru_cache(maxsize=8)
def _mel_banks(num_bins, padded, sample_freq, low_freq, high_freq) -> np.ndarray:
    """torchaudio's get_mel_banks arithmetic: python-double mel_low / delta
    scalars cast to float32, float32 tensor ops in torchaudio's order (checked
    against torch's own evaluation, which promotes exactly like this).  The one
    transcendental, the float32 log of (1 + f / 700), is taken correctly rounded:
    torch's CPU float32 log is host-dependent (SLEEF u10 paths), so torchaudio's
    own filter weights differ between machines by up to 7e-6 (measured: this
    container's Xeon vs the GPU box's host, 41 of 501 weights; numpy's float32 log
    differs again) -- up to 8e-5 in a log-mel value.  This restatement and the
    kernel's generated table (tools/gen_fbank_mel_table.py) use the correctly
    rounded value, i.e. glibc logf."""
    f32 = np.float32
    num_fft_bins = padded // 2
    nyquist = 0.5 * sample_freq
    if high_freq <= 0.0:
        high_freq += nyquist
    fft_bin_width = sample_freq / padded
    mel_low = 1127.0 * math.log(1.0 + low_freq / 700.0)
    mel_high = 1127.0 * math.log(1.0 + high_freq / 700.0)
    delta = f32((mel_high - mel_low) / (num_bins + 1))
    b = np.arange(num_bins, dtype=f32)[:, None]
    left = f32(mel_low) + b * delta
    center = f32(mel_low) + (b + f32(1.0)) * delta
    right = f32(mel_low) + (b + f32(2.0)) * delta
    x = f32(1.0) + (f32(fft_bin_width) * np.arange(num_fft_bins, dtype=f32)) / f32(700.0)
    mel = (f32(1127.0) * np.log(x.astype(np.float64)).astype(f32))[None, :]
    up = (mel - left) / (center - left)
    down = (right - mel) / (right - center)
    w = np.maximum(f32(0), np.minimum(up, down)).astype(f32)
    out = np.concatenate([w, np.zeros((num_bins, 1), dtype=f32)], axis=1)
    out.setflags(write=False)
    return out


def _frames(wave: np.ndarray, frame_len: int, frame_shift: int) -> np.ndarray:
    n = 1 + (len(wave) - frame_len) // frame_shift
    idx = np.arange(frame_len)[None, :] + frame_shift * np.arange(n)[:, None]
    return wave[idx]


def _window(frame_len, dtype, window_type="hamming"):
    """kaldi.py _feature_window_function (symmetric windows; blackman_coeff 0.42)."""
    n = np.arange(frame_len, dtype=np.float64)
    a = 2 * np.pi * n / (frame_len - 1)
    if window_type == "hamming":
        w = 0.54 - 0.46 * np.cos(a)
    elif window_type == "hanning":
        w = 0.5 - 0.5 * np.cos(a)
    elif window_type == "povey":
        w = (0.5 - 0.5 * np.cos(a)) ** 0.85
    elif window_type == "rectangular":
        w = np.ones(frame_len)
    elif window_type == "blackman":
        w = 0.42 - 0.5 * np.cos(a) + 0.08 * np.cos(2 * a)
    else:
        raise ValueError(f"Invalid window type {window_type}")
    return w.astype(dtype)


def _prep(wave, frame_len, frame_shift, dtype, preemph=0.97, window_type="hamming"):
    x = _frames(np.asarray(wave, dtype=dtype), frame_len, frame_shift)
    x = x - x.mean(axis=1, keepdims=True)
    prev = np.concatenate([x[:, :1], x[:, :-1]], axis=1)
    x = x - dtype(preemph) * prev
    return (x * _window(frame_len, dtype, window_type)[None, :]).astype(dtype)


def fbank(wave, num_mel_bins=80, frame_length_ms=25.0, frame_shift_ms=10.0, sample_freq=16000.0,
          dtype=np.float64, cmn=False, window_type="hamming") -> np.ndarray:
    """(T, num_mel_bins) log-mel, computed in `dtype` with numpy's FFT."""
    fl = int(sample_freq * frame_length_ms * 0.001)
    fs = int(sample_freq * frame_shift_ms * 0.001)
    if len(wave) < fl:
        return np.zeros((0, num_mel_bins), dtype=np.float32)
    padded = 1 << int(np.ceil(np.log2(fl)))
    x = _prep(wave, fl, fs, dtype, window_type=window_type)
    spec = np.fft.rfft(x, n=padded, axis=1)
    power = (spec.real ** 2 + spec.imag ** 2).astype(dtype)
    banks = mel_banks(num_mel_bins, padded, sample_freq).astype(dtype)
    mel = power @ banks.T
    out = np.log(np.maximum(mel, FLT_EPS)).astype(np.float32)
    if cmn:
        # speaker.py:102-103 `feat - torch.mean(feat, 0)`: torch's float32 mean
        # uses cascade summation (~exact); numpy's float32 mean over axis 0 of a
        # C-contiguous array accumulates naively (~3e-5 off at T = 498), so the
        # mean is taken in float64 here.
        out = (out - out.astype(np.float64).mean(axis=0, keepdims=True)).astype(np.float32)
    return out


def apply_cmvn(feats, norm_mean=True, norm_var=False):
    """dataset_utils.py:19-26 on (B, T, F) float32, statistics in float64."""
    x = np.asarray(feats, dtype=np.float64)
    if norm_mean:
        x = x - x.mean(axis=1, keepdims=True)
        x = x.astype(np.float32).astype(np.float64)
    if norm_var:
        with np.errstate(invalid="ignore", divide="ignore"):
            x = x / np.sqrt(x.var(axis=1, ddof=1, keepdims=True) + 1e-7)
    return x.astype(np.float32)


def fbank_dft64(wave, num_mel_bins=80, sample_freq=16000.0) -> np.ndarray:
    """Independent float64 formulation (explicit DFT matrix) used to cross-check `fbank`."""
    fl, fs, padded = 400, 160, 512
    x = _prep(wave, fl, fs, np.float64)
    k = np.arange(padded // 2 + 1)[:, None]
    n = np.arange(fl)[None, :]
    ang = 2 * np.pi * k * n / padded
    re = x @ np.cos(ang).T
    im = -(x @ np.sin(ang).T)
    power = re * re + im * im
    mel = power @ mel_banks(num_mel_bins, padded, sample_freq).astype(np.float64).T
    return np.log(np.maximum(mel, FLT_EPS)).astype(np.float32)


def fbank_batch(waves: np.ndarray, cmn=True, dtype=np.float64) -> np.ndarray:
    return np.stack([fbank(w, dtype=dtype, cmn=cmn) for w in waves])
