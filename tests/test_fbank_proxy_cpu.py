"""Pins the fbank oracle (oracle/fbank_ref.py, the restatement of
torchaudio.compliance.kaldi.fbank that the GPU kernel is checked against) to an
independent third-party implementation of the same published algorithm:
transformers.audio_utils (5.x; its `spectrogram(..., center=False,
preemphasis=0.97, remove_dc_offset=True, log_mel="log", mel_floor=FLT_EPSILON)` +
`mel_filter_bank(mel_scale="kaldi", triangularize_in_mel_space=True)` is the
numpy path the Speech2Text / AST feature extractors take for
`ta_kaldi.fbank` when torchaudio is absent).  torchaudio itself is not
installed, so this is a proxy pin, like the HuBERT encoder's
(tests/test_hubert_oracle.py):

  * the frame pipeline (snip-edges framing, DC removal, pre-emphasis with the
    replicate pad, the symmetric windows, zero pad to the FFT size, power, log
    with the FLT_EPSILON floor) agrees within 5e-6 (~1 float32 ulp of the log-mel
    values) when both use the same filters, for 23-128 bins at 8 and 16 kHz and
    the hamming / hanning / povey / rectangular / blackman windows;
  * the oracle's filters (torchaudio's float32 arithmetic, as the kernel's host
    code computes them) agree with transformers' float64 Kaldi filters within
    2e-5 — the float32 rounding of torchaudio's own formula.
"""
import numpy as np
import pytest

from oracle import fbank_ref
from wespeaker_hubert_amd.synthetic import synth_audio

ta = pytest.importorskip("transformers.audio_utils")

CASES = [(80, 16000, "hamming"), (80, 16000, "hanning"), (80, 16000, "povey"), (80, 16000, "rectangular"),
         (80, 16000, "blackman"), (40, 16000, "hamming"), (64, 8000, "hamming"), (40, 8000, "povey"),
         (23, 8000, "blackman"), (128, 16000, "hamming")]


def _window(win, n):
    if win == "blackman":  # kaldi.py: 0.42 - 0.5 cos(a n) + 0.08 cos(2 a n) = numpy's blackman
        return np.blackman(n)
    return ta.window_function(n, {"hamming": "hamming", "hanning": "hann", "povey": "povey",
                                  "rectangular": "boxcar"}[win], periodic=False)


@pytest.mark.parametrize("nb,sr,win", CASES)
def test_fbank_oracle_matches_transformers_kaldi_path(nb, sr, win):
    fl, fs = int(sr * 0.025), int(sr * 0.010)
    nfft = 1 << int(np.ceil(np.log2(fl)))
    banks = fbank_ref.mel_banks(nb, nfft, float(sr)).astype(np.float64)  # [nb][nfft / 2 + 1]
    for seed, n in ((3, sr * 2), (4, fl + 7 * fs + 5)):
        w = synth_audio(seed, 1, n)[0].astype(np.float64)
        ref = ta.spectrogram(w, _window(win, fl), frame_length=fl, hop_length=fs, fft_length=nfft, power=2.0,
                             center=False, preemphasis=0.97, mel_filters=banks.T, log_mel="log",
                             mel_floor=1.192092955078125e-07, remove_dc_offset=True).T
        got = fbank_ref.fbank(w, nb, sample_freq=float(sr), window_type=win)
        assert got.shape == ref.shape == (1 + (n - fl) // fs, nb)
        assert np.abs(got - ref).max() <= 5e-6, np.abs(got - ref).max()


@pytest.mark.parametrize("nb,sr", [(80, 16000), (40, 16000), (64, 8000), (40, 8000), (23, 8000)])
def test_mel_banks_match_transformers_kaldi_filters(nb, sr):
    nfft = 512 if sr == 16000 else 256
    ref = ta.mel_filter_bank(num_frequency_bins=nfft // 2 + 1, num_mel_filters=nb, min_frequency=20,
                             max_frequency=sr // 2, sampling_rate=sr, norm=None, mel_scale="kaldi",
                             triangularize_in_mel_space=True).T
    got = fbank_ref.mel_banks(nb, nfft, float(sr)).astype(np.float64)
    assert got.shape == ref.shape
    assert np.abs(got - ref).max() <= 2e-5
    assert np.array_equal(got > 0, ref > 1e-6) or np.abs(got - ref)[(got > 0) != (ref > 1e-6)].max() <= 2e-5
