"""Resampling (torchaudio.transforms.Resample, reference call sites
cli/speaker.py:155-157 and dataset/processor.py:242-260).  The restatement in
oracle/resample_ref.py is checked against analytic band-limited signals (parity
with torchaudio itself is unpinned: torchaudio is absent); the library's host
plan against the restatement on CPU, and the HIP kernel against it on the GPU."""
import numpy as np
import pytest
import torch

from oracle import resample_ref as R

PAIRS = [(8000, 16000), (48000, 16000), (44100, 16000), (22050, 16000), (32000, 16000), (16000, 8000),
         (11025, 16000), (16000, 16000)]


@pytest.mark.parametrize("orig,new", [p for p in PAIRS if p[0] != p[1]])
def test_oracle_reproduces_bandlimited_sine(orig, new):
    N = orig // 2
    nyq = min(orig, new) / 2
    for f in (130.0, 440.0, 2500.0):
        # the 6-zero-crossing Hann sinc's passband: flat to ~0.2 % well below
        # Nyquist, ~1 % at 0.6 x Nyquist
        tol = 2e-3 if f < 0.3 * nyq else 1.2e-2
        x = np.sin(2 * np.pi * f * np.arange(N) / orig)
        y = R.resample(x, orig, new)
        assert len(y) == R.out_len(orig, new, N) == -(-new * N // orig)
        ref = np.sin(2 * np.pi * f * np.arange(len(y)) / new)
        core = slice(64, len(y) - 64)  # away from the zero-padded edges
        assert np.abs(y[core] - ref[core]).max() < tol


def test_oracle_identity_and_lengths():
    x = np.arange(1000, dtype=np.float32)
    np.testing.assert_array_equal(R.resample(x, 16000, 16000), x)
    assert R.out_len(44100, 16000, 44101) == -(-160 * 44101 // 441)
    assert R.out_len(8000, 16000, 0) == 0


@pytest.mark.parametrize("orig,new", PAIRS)
def test_library_plan_matches_oracle_kernel(orig, new):
    from wespeaker_hubert_amd.resample import Resample
    r = Resample(orig, new)
    o, n, w, k = r.kernel()
    for N in (0, 1, 400, 12345, 80000):
        assert r.out_len(N) == R.out_len(orig, new, N)
    if orig == new:
        return
    kr, wr, or_, nr = R.sinc_hann_kernel(orig, new)
    assert (o, n, w) == (or_, nr, wr)
    assert k.shape == kr.shape
    assert np.abs(k - kr).max() <= 1e-7 * max(1.0, float(np.abs(kr).max()))


def test_library_rejects_bad_rates():
    from wespeaker_hubert_amd import _lib
    from wespeaker_hubert_amd.resample import Resample
    with pytest.raises(RuntimeError):
        Resample(0, 16000)
    with pytest.raises(NotImplementedError):
        Resample(8000, 16000, resampling_method="sinc_interp_kaiser")


@pytest.mark.gpu
@pytest.mark.parametrize("orig,new", PAIRS)
def test_gpu_resample_matches_oracle(orig, new):
    from wespeaker_hubert_amd.resample import Resample
    rng = np.random.default_rng(orig + new)
    for N in (1, 777, 12345):
        x = np.round(np.clip(rng.normal(0, 0.1, (3, N)), -1, 1) * 32767).astype(np.float32)
        y = Resample(orig, new)(torch.from_numpy(x).cuda()).cpu().numpy()
        ref = R.resample(x, orig, new)
        assert y.shape == ref.shape
        # fp32 accumulation over <= ~100 taps vs the f64 restatement
        assert np.abs(y - ref).max() <= 2e-6 * 32767
    # leading dims are kept, like torchaudio's (..., time) contract
    x = torch.zeros(2, 2, 1600, device="cuda")
    assert Resample(orig, new)(x).shape == (2, 2, R.out_len(orig, new, 1600))


@pytest.mark.gpu
def test_gpu_speaker_resamples_8k_input(tmp_path):
    """extract_embedding_from_pcm at 8 kHz == oracle resample -> oracle fbank -> oracle model."""
    import yaml
    from oracle import fbank_ref, models_ref
    import wespeaker_hubert_amd as wespeaker
    from wespeaker_hubert_amd import arch as A
    from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict
    arch = "ECAPA_TDNN_c512"
    sd = synth_state_dict(41, A.param_list(A.make_spec(arch, feat_dim=80, embed_dim=192)))
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, tmp_path / "avg_model.pt")
    with open(tmp_path / "config.yaml", "w") as f:
        yaml.safe_dump({"model": arch, "model_args": {"feat_dim": 80, "embed_dim": 192}}, f)
    spk = wespeaker.load_model(str(tmp_path))
    pcm8 = synth_audio(9, 1, 8000 * 3)  # 3 s at 8 kHz, int16-valued
    e = spk.extract_embedding_from_pcm(torch.from_numpy(pcm8), 8000).numpy()
    pcm16 = R.resample(pcm8[0], 8000, 16000)
    feats = fbank_ref.fbank(pcm16, cmn=True)[None]
    with torch.no_grad():
        _, ref = models_ref.forward(arch, torch.from_numpy(feats), {k: torch.from_numpy(v) for k, v in sd.items()})
    ref = ref[0].numpy()
    cos = float(e.astype(np.float64) @ ref / np.linalg.norm(e) / np.linalg.norm(ref))
    assert cos >= 0.9999
