"""CPU restatement of band-limited sinc resampling (TEST INFRASTRUCTURE ONLY —
imported by tests/ and never by the product path).

The reference resamples with `torchaudio.transforms.Resample(orig_freq, new_freq)`
at wespeaker/cli/speaker.py:155-157 (Speaker.extract_embedding_from_pcm) and
wespeaker/dataset/processor.py:242-260 (`resample`, the data pipeline of
bin/extract.py).  torchaudio (third party, unpinned: setup.py:9 'torchaudio>=0.12')
is not installed here, so this file restates its published default algorithm
(`torchaudio.functional.functional._get_sinc_resample_kernel` /
`_apply_sinc_resample_kernel`, method "sinc_interp_hann", lowpass_filter_width 6,
rolloff 0.99):

  g = gcd(orig, new); orig //= g; new //= g
  base = min(orig, new) * rolloff;  width = ceil(lpw * orig / base)
  t[j, k] = clamp(((k - width) / orig - j / new) * base, -lpw, lpw)   k in [0, 2*width + orig)
  kernel[j, k] = sinc(pi t) * cos(pi t / (2 lpw))^2 * base / orig        (f64, stored as f32)
  y[n*new + j] = sum_k kernel[j, k] * x[n*orig + k - width]   (zero outside x)
  len(y) = ceil(new * len(x) / orig);  orig == new returns x unchanged.

Parity with torchaudio itself is UNPINNED (no torchaudio, no reference fixture);
the tests check this restatement against analytic band-limited signals and the
HIP kernel against this restatement.
"""
from __future__ import annotations

import math

import numpy as np


def sinc_hann_kernel(orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99):
    g = math.gcd(int(orig), int(new))
    o, n = int(orig) // g, int(new) // g
    base = min(o, n) * rolloff
    width = math.ceil(lowpass_filter_width * o / base)
    idx = np.arange(-width, width + o, dtype=np.float64)[None, :] / o
    t = (np.arange(0, -n, -1, dtype=np.float64)[:, None] / n + idx) * base
    t = np.clip(t, -lowpass_filter_width, lowpass_filter_width)
    window = np.cos(t * math.pi / lowpass_filter_width / 2) ** 2
    t = t * math.pi
    with np.errstate(invalid="ignore", divide="ignore"):
        k = np.where(t == 0, 1.0, np.sin(t) / t)
    k = k * window * (base / o)
    return k.astype(np.float32), width, o, n


def out_len(orig: int, new: int, num_samples: int) -> int:
    if orig == new:
        return num_samples
    g = math.gcd(int(orig), int(new))
    o, n = int(orig) // g, int(new) // g
    return -(-n * num_samples // o)  # ceil(n * N / o) in integers


def resample(x: np.ndarray, orig: int, new: int, lowpass_filter_width: int = 6, rolloff: float = 0.99) -> np.ndarray:
    """x (..., N) -> (..., ceil(new*N/orig)); float64 accumulation of the f32 kernel."""
    x = np.asarray(x)
    if orig == new:
        return x.copy()
    kern, width, o, n = sinc_hann_kernel(orig, new, lowpass_filter_width, rolloff)
    lead = x.shape[:-1]
    x2 = x.reshape(-1, x.shape[-1]).astype(np.float64)
    N = x2.shape[1]
    L = kern.shape[1]
    xp = np.pad(x2, ((0, 0), (width, width + o)))
    npos = N // o + 1
    # windows[b, p, k] = xp[b, p*o + k]
    idx = np.arange(npos)[:, None] * o + np.arange(L)[None, :]
    win = xp[:, idx]                                   # (R, npos, L)
    y = np.einsum("rpk,jk->rpj", win, kern.astype(np.float64)).reshape(x2.shape[0], -1)
    y = y[:, :out_len(orig, new, N)]
    return y.reshape(lead + (y.shape[-1],)).astype(np.float32)
