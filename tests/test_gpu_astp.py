"""GPU: the fused ASTP head (astp_fused.hip: linear2 on bf16x3 MFMA + softmax
over frames + attentive mean / std, pooling_layers.py:133-144) against the
unfused path (linear2 GEMM writing the logits + the pooling kernel) and the
oracle.  The two paths round the logits' softmax sums in different orders, so
they agree to ~1e-6, not bitwise; the oracle bar (1e-4 / cos 0.9999) holds."""
import numpy as np
import pytest
import torch

from oracle import models_ref
from wespeaker_hubert_amd.synthetic import synth_feats, synth_state_dict

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _pair(arch, seed):
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    ms, sd = [], None
    for fused in (1, 0):
        m = HipSpeakerModel(arch, feat_dim=80, embed_dim=192)
        m.set_option("astp_fused", fused)
        if sd is None:
            sd = synth_state_dict(seed, m.state_dict_layout())
        m.load_state_dict(sd)
        ms.append(m.to(DEV))
    return ms[0], ms[1], sd


@pytest.mark.parametrize("arch,B,T", [("ECAPA_TDNN_c1024", 3, 498), ("ECAPA_TDNN_GLOB_c512", 4, 77),
                                      ("ECAPA_TDNN_c512", 2, 2), ("ECAPA_TDNN_GLOB_c1024", 2, 33)])
def test_astp_fused_matches_unfused_and_oracle(arch, B, T):
    fused, plain, sd = _pair(arch, 21)
    x = torch.from_numpy(synth_feats(6, B, T, 80)).to(DEV)
    a = fused.embed(x).cpu().numpy()
    b = plain.embed(x).cpu().numpy()
    assert np.all(np.isfinite(a))
    assert np.abs(a - b).max() < 2e-5 * max(1.0, np.abs(b).max())
    with torch.no_grad():
        _, ref = models_ref.forward(arch, x.cpu(), {k: torch.from_numpy(v) for k, v in sd.items()})
    assert np.abs(a - ref.numpy()).max() < 1e-4


def test_astp_fused_ragged_equals_batch_of_one():
    fused, _, _ = _pair("ECAPA_TDNN_GLOB_c512", 22)
    frames = [3, 77, 498, 150, 2, 263, 41, 31, 32, 33]
    feats = [synth_feats(500 + i, 1, t, 80)[0] for i, t in enumerate(frames)]
    cat = torch.from_numpy(np.concatenate(feats)).to(DEV)
    off = torch.tensor(np.concatenate([[0], np.cumsum(frames)]), dtype=torch.int32, device=DEV)
    got = fused.embed_segments(cat, off).cpu().numpy()
    for i, f in enumerate(feats):
        one = fused.embed(torch.from_numpy(f[None]).to(DEV)).cpu().numpy()[0]
        assert np.abs(got[i] - one).max() <= 1e-6

