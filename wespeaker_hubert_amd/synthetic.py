"""Deterministic synthetic weights and audio for parity tests and the bench.

There are no trained checkpoints offline, so every parity
fixture and every bench run uses seeded random weights.  The generator is keyed
by *parameter name* (not by ordering) so that the reference module
(`wespeaker/models/*.py`, loaded only in the survey container to make golden
fixtures) and this framework's own loader produce bit-identical tensors from
the same `(seed, name, shape)`.

Distributions follow SURVEY.md §8(d): conv/linear weights ~ N(0, 1/fan_in),
BN running_mean ~ N(0, 0.1), running_var ~ U(0.5, 1.5).
"""
from __future__ import annotations

import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

__all__ = ["param_rng", "synth_param", "synth_state_dict", "synth_audio", "synth_feats", "synth_speaker_audio"]


def param_rng(seed: int, name: str) -> np.random.Generator:
    return np.random.default_rng([int(seed) & 0x7FFFFFFF, zlib.crc32(name.encode("utf-8"))])


def synth_param(seed: int, name: str, shape: Tuple[int, ...]) -> np.ndarray:
    """One parameter / buffer of a state_dict, float32 (int64 for counters)."""
    shape = tuple(int(s) for s in shape)
    rng = param_rng(seed, name)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "num_batches_tracked":
        return np.zeros(shape, dtype=np.int64)
    if leaf == "running_mean":
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "running_var":
        return rng.uniform(0.5, 1.5, shape).astype(np.float32)
    if leaf == "weight_g":  # weight-norm magnitude (HuBERT pos_conv): per-tap norms
        return rng.uniform(1.5, 3.0, shape).astype(np.float32)
    if name.endswith("featurizer.weights"):
        return (0.5 * rng.standard_normal(shape)).astype(np.float32)
    is_norm = (".bn" in name or name.startswith("bn") or ".norm" in name
               or "layer_norm" in name or "bns." in name or "seg_bn" in name)
    if leaf == "weight" and len(shape) == 1:
        # BatchNorm / LayerNorm / GroupNorm affine scale
        return rng.uniform(0.8, 1.2, shape).astype(np.float32)
    if leaf == "bias" and (len(shape) == 1 and is_norm):
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "bias":
        return (0.05 * rng.standard_normal(shape)).astype(np.float32)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        gain = 1.0
        # Keep deep residual stacks (ResNet293: 90 blocks) numerically tame:
        # the last BN of every bottleneck / basic block is shrunk, the
        # usual "small residual branch" initialisation.
        return (gain * rng.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
    return (0.05 * rng.standard_normal(shape)).astype(np.float32)


def _residual_tame(name: str, arr: np.ndarray) -> np.ndarray:
    # ResNet blocks: shrink the affine scale of the BN that closes a residual
    # branch (bn2 of BasicBlock, bn3 of Bottleneck) so 90 stacked residual
    # adds stay O(1).
    if name.endswith("bn3.weight") or (".bn2.weight" in name and "layer" in name):
        return (arr * 0.25).astype(arr.dtype)
    return arr


def synth_state_dict(seed: int, shapes: Iterable[Tuple[str, Tuple[int, ...]]],
                     residual_tame: bool = False) -> Dict[str, np.ndarray]:
    out = {}
    for name, shape in shapes:
        arr = synth_param(seed, name, shape)
        if residual_tame:
            arr = _residual_tame(name, arr)
        out[name] = arr
    return out


def synth_audio(seed: int, batch: int, num_samples: int, int16_scale: bool = True) -> np.ndarray:
    """clip(N(0, 0.1), -1, 1) audio; x32768 and rounded to
    integers for the fbank paths (mimics PCM16 read with normalize=False)."""
    rng = np.random.default_rng(int(seed))
    wav = np.clip(0.1 * rng.standard_normal((batch, num_samples)), -1.0, 1.0)
    if int16_scale:
        wav = np.round(wav * 32768.0).clip(-32768, 32767)
    return wav.astype(np.float32)


def synth_feats(seed: int, batch: int, frames: int, dim: int) -> np.ndarray:
    rng = np.random.default_rng(int(seed))
    return rng.standard_normal((batch, frames, dim)).astype(np.float32)


def synth_speaker_audio(seed: int, speakers, utts_per_speaker: int, num_samples: int, sr: int = 16000,
                        snr_db: float = 10.0, jitter: float = 1.0, int16_scale: bool = True) -> np.ndarray:
    """Speaker-structured synthetic speech for EER-level checks (no real corpus
    offline): speaker s (an integer id, seeded by (seed, s)) is a glottal pulse
    train at its own f0 (90-250 Hz) shaped by its own five formant resonances;
    each utterance draws its own f0 contour (+-6 % x jitter), formant jitter (+-4 % x jitter),
    syllable-rate amplitude envelope and white noise at `snr_db`.  Returns
    [len(speakers) * utts_per_speaker][num_samples], speaker-major."""
    out = []
    t = np.arange(num_samples) / sr
    freqs = np.fft.rfftfreq(num_samples, 1.0 / sr)
    for s in speakers:
        srng = np.random.default_rng([int(seed) & 0x7FFFFFFF, int(s), 1])
        f0 = srng.uniform(90.0, 250.0)
        formants = np.sort(srng.uniform([250, 800, 1800, 2600, 3400], [900, 1800, 2800, 3600, 4800]))
        bws = srng.uniform(60.0, 250.0, 5)
        gains = srng.uniform(0.3, 1.0, 5)
        tilt = srng.uniform(0.6, 1.4)
        for u in range(utts_per_speaker):
            urng = np.random.default_rng([int(seed) & 0x7FFFFFFF, int(s), 2, u])
            contour = 1.0 + 0.06 * jitter * np.sin(2 * np.pi * urng.uniform(0.2, 0.8) * t + urng.uniform(0, 2 * np.pi))
            phase = 2 * np.pi * np.cumsum(f0 * contour) / sr
            src = (np.sin(phase) > np.cos(np.pi * 0.85)).astype(np.float64)  # pulse train, ~7.5 % duty
            src -= src.mean()
            fj = formants * (1.0 + 0.04 * jitter * urng.uniform(-1.0, 1.0, 5))
            env = np.zeros_like(freqs)
            for fc, bw, g in zip(fj, bws, gains):
                env += g / (1.0 + ((freqs - fc) / bw) ** 2)
            env *= (1.0 + freqs / 1000.0) ** (-tilt)
            x = np.fft.irfft(np.fft.rfft(src) * env, n=num_samples)
            am = 0.55 + 0.45 * np.sin(2 * np.pi * urng.uniform(3.0, 6.0) * t + urng.uniform(0, 2 * np.pi))
            x *= am
            x /= np.sqrt(np.mean(x ** 2)) + 1e-12
            x += urng.standard_normal(num_samples) * 10 ** (-snr_db / 20.0)
            x *= 0.1 / np.sqrt(np.mean(x ** 2))
            out.append(np.clip(x, -1.0, 1.0))
    wav = np.stack(out)
    if int16_scale:
        wav = np.round(wav * 32768.0).clip(-32768, 32767)
    return wav.astype(np.float32)
