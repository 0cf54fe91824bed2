"""Pins oracle/hubert_ref.py (HuBERT-base restatement)
against the transformers HubertModel proxy fixture (tests/golden/hubert_proxy.npz,
made by tests/golden/make_hubert_proxy.py).  Tolerance: fp32 reorderings only,
|Δ| ≤ 2e-4 per element on LayerNorm-scaled O(1) states."""
import os

import numpy as np
import pytest
import torch

from oracle.hubert_ref import hubert_hidden_states, match_length, pos_conv_weight, s3prl_frontend
from wespeaker_hubert_amd.arch import HUBERT_PREFIX, hubert_num_frames, hubert_params, s3prl_num_frames
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict

GOLD = os.path.join(os.path.dirname(__file__), "golden", "hubert_proxy.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


@pytest.fixture(scope="module")
def sd(gold):
    raw = synth_state_dict(int(gold["weight_seed"]), hubert_params())
    return {k: torch.from_numpy(v) for k, v in raw.items()}


def test_frame_counts():
    assert hubert_num_frames(16000) == 49 and s3prl_num_frames(16000) == 50
    assert hubert_num_frames(8000) == 24 and s3prl_num_frames(8000) == 25
    assert hubert_num_frames(400) == 1


def test_param_layout():
    names = [n for n, _ in hubert_params()]
    assert len(names) == len(set(names))
    assert sum(int(np.prod(s)) for _, s in hubert_params()) == 94371712 - 768 + 13  # HF HubertModel minus masked_spec_embed, + featurizer


@pytest.mark.parametrize("tag", ["short", "s1"])
def test_hidden_states_vs_proxy(gold, sd, tag):
    wav = torch.from_numpy(synth_audio(int(gold[f"{tag}_wav_seed"]), 2, int(gold[f"{tag}_num_samples"]),
                                       int16_scale=False))
    with torch.no_grad():
        hs = hubert_hidden_states(wav, sd)
    assert len(hs) == 13
    sums = np.array([h.double().sum().item() for h in hs])
    abss = np.array([h.double().abs().sum().item() for h in hs])
    np.testing.assert_allclose(abss, gold[f"{tag}_layer_abs"], rtol=1e-5)
    np.testing.assert_allclose(sums, gold[f"{tag}_layer_sums"], atol=1e-5 * abss.max())
    if tag == "short":
        for i in (0, 6, 12):
            np.testing.assert_allclose(hs[i].numpy(), gold[f"short_hs{i}"], atol=2e-4, rtol=0)
    else:
        np.testing.assert_allclose(hs[12][:, :8].numpy(), gold["s1_hs12"], atol=2e-4, rtol=0)


def test_pos_conv_weight_norm():
    rng = np.random.default_rng(0)
    v = torch.from_numpy(rng.standard_normal((8, 4, 6)).astype(np.float32))
    g = torch.from_numpy(rng.uniform(1, 2, (1, 1, 6)).astype(np.float32))
    w = pos_conv_weight(g, v)
    np.testing.assert_allclose(torch.sqrt((w ** 2).sum(dim=(0, 1))).numpy(), g.flatten().numpy(), rtol=1e-5)


def test_match_length_and_featurizer(sd):
    h = torch.arange(2 * 3 * 4, dtype=torch.float32).view(2, 3, 4)
    m = match_length(h, 1200)  # ceil(1200/320) = 4 frames
    assert m.shape == (2, 4, 4) and torch.equal(m[:, 3], h[:, 2])
    assert match_length(h, 640).shape == (2, 2, 4)
    wav = torch.from_numpy(synth_audio(3, 1, 4000, int16_scale=False))
    with torch.no_grad():
        f = s3prl_frontend(wav, sd)
    assert f.shape == (1, s3prl_num_frames(4000), 768) and torch.isfinite(f).all()


def test_s3prl_min_second_zero_pad(sd):
    """S3PRLUpstream.forward (s3prl>=0.4, MIN_SECOND = 0.05): a batch shorter than
    800 samples runs zero-padded to 800; the output keeps len(range(0, W, 320))
    frames and equals the explicitly padded input's first frames.  Restated from
    s3prl's published source: parity unpinned (s3prl is absent offline)."""
    from oracle.hubert_ref import s3prl_upstream
    for W in (1, 250, 400, 640, 799):
        wav = torch.from_numpy(synth_audio(5, 2, W, int16_scale=False))
        with torch.no_grad():
            got = s3prl_frontend(wav, sd)
            pad = s3prl_frontend(torch.nn.functional.pad(wav, (0, 800 - W)), sd)
            hs = s3prl_upstream(wav, sd)
        assert got.shape == (2, s3prl_num_frames(W), 768)
        assert len(hs) == 13 and all(h.shape == got.shape for h in hs)
        torch.testing.assert_close(got, pad[:, :got.shape[1]], rtol=0, atol=0)
    # at >= 800 samples nothing is padded
    wav = torch.from_numpy(synth_audio(6, 1, 800, int16_scale=False))
    with torch.no_grad():
        hs = hubert_hidden_states(wav, sd)
        torch.testing.assert_close(s3prl_upstream(wav, sd)[12], match_length(hs[12], 800), rtol=0, atol=0)
