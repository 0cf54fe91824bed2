"""Host-side logic that needs no GPU: registry, state_dict intake, errors."""
import os

import numpy as np
import pytest
import torch

from wespeaker_hubert_amd import arch as A
from wespeaker_hubert_amd.speaker_model import HipSpeakerModel, get_speaker_model
from wespeaker_hubert_amd.synthetic import synth_state_dict


def test_load_state_dict_accepts_reference_layout_and_reports_extras(caplog):
    m = get_speaker_model("ECAPA_TDNN_GLOB_c512")(feat_dim=80, embed_dim=192)
    sd = synth_state_dict(0, m.state_dict_layout())
    sd = {k: torch.from_numpy(v) for k, v in sd.items()}
    sd["projection.weight"] = torch.zeros(10, 192)   # training-only head in avg_model.pt
    del sd["linear.bias"]
    missing, unexpected = m.load_state_dict(sd)
    assert missing == ["linear.bias"]
    assert unexpected == ["projection.weight"]
    assert "missing tensor: linear.bias" in caplog.text


def test_shape_mismatch_raises():
    m = HipSpeakerModel("ECAPA_TDNN_c512", feat_dim=80, embed_dim=192)
    with pytest.raises(ValueError):
        m.load_state_dict({"layer1.conv.weight": np.zeros((512, 80, 3), np.float32)})


def test_unknown_model_name():
    with pytest.raises(KeyError):
        get_speaker_model("NOPE_c1")


def test_cpu_device_is_refused():
    m = HipSpeakerModel("ECAPA_TDNN_c512", feat_dim=80, embed_dim=192)
    with pytest.raises(RuntimeError):
        m.to("cpu")


def test_flop_count_c1024():
    spec = A.make_spec("ECAPA_TDNN_c1024", feat_dim=80, embed_dim=192)
    assert abs(A.ecapa_gflop_per_utt(spec, 498) - 12.80) < 0.05


def test_s3prl_frontend_intake_and_options(caplog):
    """S3prlFrontend mirror (frontend/s3prl.py:23-93): reference checkpoint names with
    or without the `frontend.` prefix, fairseq-only members ignored silently."""
    from wespeaker_hubert_amd.s3prl_frontend import S3prlFrontend
    fe = S3prlFrontend({"name": "hubert_base"})
    assert fe.output_size() == 768 and fe._options["layer"] == -1
    lay = fe.state_dict_layout()
    sd = {k[len("frontend."):]: np.zeros(s, np.float32) for k, s in lay[:3]}
    sd["upstream.upstream.model.mask_emb"] = np.zeros(768, np.float32)
    sd["upstream.upstream.model.final_proj.weight"] = np.zeros((256, 768), np.float32)
    missing, unexpected = fe.load_state_dict(sd)
    assert unexpected == [] and len(missing) == len(lay) - 3
    assert S3prlFrontend({"name": "hubert_base"}, multilayer_feature=False)._options["layer"] == 12
    assert S3prlFrontend({"name": "hubert"}, multilayer_feature=False, layer=4)._options["layer"] == 4
    with pytest.raises(AssertionError):
        S3prlFrontend({"name": "hubert_base"}, layer=3)
    with pytest.raises(NotImplementedError):
        S3prlFrontend({"name": "wavlm_large"})
    with pytest.raises(RuntimeError):
        fe.to("cpu")


def test_ragged_pack_groups_are_contiguous_and_bounded():
    from wespeaker_hubert_amd.batching import pack, stream_groups
    lens = [16000, 400, 80000, 399 + 160 * 50, 48000, 1600000, 8000]
    frames = [1 + (n - 400) // 160 for n in lens]
    groups = pack(lens, max_frames=600)
    assert groups[0][0] == 0 and groups[-1][1] == len(lens)
    assert all(a[1] == b[0] for a, b in zip(groups, groups[1:]))
    for lo, hi in groups:
        assert hi - lo == 1 or sum(frames[lo:hi]) <= 600
    got = list(stream_groups(((str(i), np.zeros(n)) for i, n in enumerate(lens)), 600))
    assert [len(k) for k, _ in got] == [hi - lo for lo, hi in groups]


# ---------------------------------------------------------------- diarization --
def test_subsegment_matches_reference_fixture():
    """diar.subsegment vs the reference's diar/extract_emb.py:55-83 on the cases in
    tests/golden/diar_subsegment.npz (made by make_golden.py diar)."""
    from wespeaker_hubert_amd.diar import subsegment
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "diar_subsegment.npz"))
    n = 0
    while f"case_{n}" in z:
        seg_id, win, per = z[f"case_{n}"]
        ids, wins = subsegment(z[f"fbank_{n}"], str(seg_id), int(win), int(per), 10)
        assert ids == [str(x) for x in z[f"ids_{n}"]]
        np.testing.assert_array_equal(np.stack(wins), z[f"wins_{n}"])
        n += 1
    assert n == 6


def test_extraction_config_parsing():
    """dataset_args -> fbank / cmvn options (bin/extract.py:66-67,104-106, processor.py:472-476)."""
    import pytest
    from wespeaker_hubert_amd.batching import Cmvn
    from wespeaker_hubert_amd.frontend import FbankArgs
    a = FbankArgs.from_config({"num_mel_bins": 64, "frame_shift": 10, "frame_length": 25, "dither": 1.0},
                              sample_rate=8000)
    assert a == FbankArgs(64, 25.0, 10.0, 8000, "hamming") and a.num_frames(8000) == 98
    with pytest.raises(NotImplementedError):
        FbankArgs.from_config({"use_energy": True})
    assert Cmvn.from_config({}) == Cmvn(True, True, False)
    c = Cmvn.from_config({"cmvn": True, "cmvn_args": {"norm_mean": True, "norm_var": True}})
    assert c.mean and c.var
    c = Cmvn.from_config({"cmvn": False, "cmvn_args": {"norm_var": True}})
    assert not c.mean and not c.var
    with pytest.raises(TypeError):
        Cmvn.from_config({"cmvn_args": {"norm_std": True}})


def test_oracle_apply_cmvn_matches_torch_formula():
    """oracle.fbank_ref.apply_cmvn restates dataset_utils.py:19-26 (torch.var unbiased)."""
    import torch
    from oracle.fbank_ref import apply_cmvn
    x = np.random.default_rng(1).standard_normal((2, 50, 8)).astype(np.float32) * 3 + 2
    t = torch.from_numpy(x).double()
    t = t - t.mean(dim=1, keepdim=True)
    t = t / torch.sqrt(torch.var(t, dim=1, keepdim=True) + 1e-7)
    np.testing.assert_allclose(apply_cmvn(x, True, True), t.numpy(), atol=2e-6)
