"""GPU: the fused Res2Net chain (res2_chain.hip, one launch per SE_Res2Block,
ecapa_tdnn.py:64-78) against the 7-launch GEMM chain it replaces and the oracle.

Both paths feed the MFMA the same bf16 hi/lo operands in the same k order and
apply the same epilogue, so the embeddings must be bit-identical; the oracle
bar (per-dim 1e-4, cosine 0.9999) applies on top.  Shapes cover window / halo
edges: T = 2 (every tap mostly padding), T < 256 (utterances inside one
window), T = 498 with many blocks, and ragged batches (per-utterance padding
inside a window)."""
import numpy as np
import pytest
import torch

from oracle import models_ref
from wespeaker_hubert_amd.synthetic import synth_feats, synth_state_dict

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _pair(arch, seed, variant=0):
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    ms = []
    sd = None
    for fused in (1, 0):
        m = HipSpeakerModel(arch, feat_dim=80, embed_dim=192)
        m.set_option("res2_fused", fused)
        m.set_option("res2_variant", variant)
        if sd is None:
            sd = synth_state_dict(seed, m.state_dict_layout())
        m.load_state_dict(sd)
        ms.append(m.to(DEV))
    return ms[0], ms[1], sd


@pytest.mark.parametrize("arch,B,T", [("ECAPA_TDNN_c1024", 3, 498), ("ECAPA_TDNN_c1024", 40, 498),
                                      ("ECAPA_TDNN_c512", 5, 263), ("ECAPA_TDNN_GLOB_c512", 3, 77),
                                      ("ECAPA_TDNN_GLOB_c1024", 2, 2), ("ECAPA_TDNN_c512", 7, 31)])
@pytest.mark.parametrize("variant", [0, 2, 3, 4])
def test_res2_fused_equals_chain_and_oracle(arch, B, T, variant):
    """res2_variant 0: 128-row windows, 4 waves of 64 x 64; 3: 8 waves of 64 rows x 32 channels;
    4: halo-free strips (c1024 widths; the c512 models run variant 3)."""
    fused, chain, sd = _pair(arch, 11, variant)
    x = torch.from_numpy(synth_feats(5, B, T, 80)).to(DEV)
    a = fused.embed(x).cpu().numpy()
    b = chain.embed(x).cpu().numpy()
    assert np.all(np.isfinite(a))
    assert np.array_equal(a, b), np.abs(a - b).max()
    rows = list(range(min(B, 3)))
    with torch.no_grad():
        _, ref = models_ref.forward(arch, x[rows].cpu(), {k: torch.from_numpy(v) for k, v in sd.items()})
    assert np.abs(a[rows] - ref.numpy()).max() < 1e-4


@pytest.mark.parametrize("variant", [0, 2, 3, 4])
def test_res2_fused_ragged_equals_chain(variant):
    fused, chain, _ = _pair("ECAPA_TDNN_c1024", 12, variant)
    frames = [3, 77, 498, 150, 2, 263, 41, 300, 9]
    feats = np.concatenate([synth_feats(400 + i, 1, t, 80)[0] for i, t in enumerate(frames)])
    cat = torch.from_numpy(feats).to(DEV)
    off = torch.tensor(np.concatenate([[0], np.cumsum(frames)]), dtype=torch.int32, device=DEV)
    a = fused.embed_segments(cat, off).cpu().numpy()
    b = chain.embed_segments(cat, off).cpu().numpy()
    assert np.array_equal(a, b), np.abs(a - b).max()
