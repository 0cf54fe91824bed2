"""PCM WAV reading (stdlib `wave`; torchaudio is not a dependency).

Matches `torchaudio.load(path, normalize=False)` for 16-bit PCM files as used at
cli/speaker.py:123-126: int16 sample values, shape (channels, N).  With
`normalize=True` the values are divided by 32768 (torchaudio's float
normalisation).  Resampling is not implemented (SURVEY.md §8(f) "next").
"""
from __future__ import annotations

import wave
from typing import Tuple

import numpy as np


def load_wav(path: str, normalize: bool = False) -> Tuple[np.ndarray, int]:
    with wave.open(path, "rb") as w:
        sr = w.getframerate()
        ch = w.getnchannels()
        width = w.getsampwidth()
        raw = w.readframes(w.getnframes())
    if width != 2:
        raise NotImplementedError(f"{path}: only 16-bit PCM WAV is supported (got {8 * width}-bit)")
    pcm = np.frombuffer(raw, dtype="<i2").reshape(-1, ch).T.copy()
    if normalize:
        return (pcm.astype(np.float32) / 32768.0), sr
    return pcm, sr


def write_wav(path: str, pcm: np.ndarray, sample_rate: int = 16000) -> None:
    pcm = np.asarray(pcm)
    if pcm.ndim == 1:
        pcm = pcm[None, :]
    data = np.clip(np.round(pcm), -32768, 32767).astype("<i2").T.tobytes()
    with wave.open(path, "wb") as w:
        w.setnchannels(pcm.shape[0])
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(data)
