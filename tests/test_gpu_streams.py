"""GPU: concurrent sub-batches (model option "streams", model.cpp Model::forward /
hubert_model.cpp forward_frontend_segments).

With streams = n the batch's utterances are split into n contiguous ranges, each
forwarded on its own HIP stream over its own workspace slice.  Every kernel on
the path computes an utterance's rows from that utterance's rows alone (GEMM rows
are independent of the M tiling, pooling / GLOB / CMN statistics are per
utterance), so the outputs must be bit-identical to streams = 1 — including the
HuBERT ragged frame offsets."""
import numpy as np
import pytest
import torch

from wespeaker_hubert_amd.synthetic import synth_audio, synth_feats, synth_state_dict

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _models(arch, streams, **kw):
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    ms, sd = [], None
    for n in streams:
        m = HipSpeakerModel(arch, **kw)
        m.set_option("streams", n)
        if sd is None:
            sd = synth_state_dict(21, m.state_dict_layout())
        m.load_state_dict(sd)
        ms.append(m.to(DEV))
    return ms


@pytest.mark.parametrize("arch,B,T,kw", [
    ("ECAPA_TDNN_c1024", 5, 200, dict(feat_dim=80, embed_dim=192)),
    ("ECAPA_TDNN_GLOB_c512", 4, 77, dict(feat_dim=80, embed_dim=192)),
    ("ECAPA_TDNN_c512", 1, 50, dict(feat_dim=80, embed_dim=192)),  # B < streams: one range
    ("ResNet34", 5, 120, dict(feat_dim=80, embed_dim=256)),
    ("ResNet34", 3, 64, dict(feat_dim=80, embed_dim=256, two_emb_layer=True)),
    ("SimAM_ResNet34_ASP", 3, 64, dict(feat_dim=80, embed_dim=256)),
])
def test_streams_bit_identical(arch, B, T, kw):
    ms = _models(arch, (1, 2, 3), **kw)
    x = torch.from_numpy(synth_feats(7, B, T, 80)).to(DEV)
    ref = ms[0].embed(x).cpu().numpy()
    assert np.all(np.isfinite(ref))
    for m in ms[1:]:
        out = m.embed(x).cpu().numpy()
        assert np.array_equal(out, ref), np.abs(out - ref).max()
    # a second call reuses the per-range workspace slices and the side streams
    out = ms[1].embed(x).cpu().numpy()
    assert np.array_equal(out, ref)


def _frontends(streams):
    from wespeaker_hubert_amd.arch import hubert_params
    from wespeaker_hubert_amd.s3prl_frontend import S3prlFrontend
    sd = synth_state_dict(41, hubert_params())
    out = []
    for n in streams:
        fe = S3prlFrontend({"name": "hubert_base"})
        fe.set_option("streams", n)
        fe.load_state_dict(sd)
        out.append(fe.to(DEV))
    return out


def test_streams_hubert_uniform_and_ragged():
    fes = _frontends((1, 2, 3))
    wav = torch.from_numpy(synth_audio(3, 4, 16000, int16_scale=False)).to(DEV)
    ref = fes[0].extract(wav, cmn=True).cpu().numpy()
    for fe in fes[1:]:
        assert np.array_equal(fe.extract(wav, cmn=True).cpu().numpy(), ref)
    lens = [800, 16000, 3000, 12345, 400]
    wavs = [torch.from_numpy(synth_audio(50 + i, 1, n, int16_scale=False)[0]) for i, n in enumerate(lens)]
    f0, o0 = fes[0].extract_segments(wavs, cmn=True)
    for fe in fes[1:]:
        f, o = fe.extract_segments(wavs, cmn=True)
        assert o == o0
        assert np.array_equal(f.cpu().numpy(), f0.cpu().numpy())
