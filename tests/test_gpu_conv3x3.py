"""GPU: the LDS-image 3x3 conv (conv3x3_img.hip, ResNet bottleneck conv2 with
32 / 64 / 128 channels, stride 1; resnet.py:72-107) against the implicit GEMM it
replaces (option conv3x3_img=0) and the oracle.

Both kernels add the same bf16 hi/lo products in the same k order (tap-major,
conv_gemm_x3's 2-D order) with the same epilogue, so the embeddings must be
bit-identical; shapes cover partial time tiles (T not a multiple of 64 / 32),
the stride-2 first block of stage 2 (implicit GEMM) next to its stride-1 blocks,
basic blocks (ResNet18/34: both 3x3 convs, the second with the residual in its
epilogue), and batch independence."""
import numpy as np
import pytest
import torch

from oracle import models_ref
from wespeaker_hubert_amd.synthetic import synth_feats, synth_state_dict

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _pair(arch, seed, img=1):
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    ms, sd = [], None
    for on in (img, 0):
        m = HipSpeakerModel(arch, feat_dim=80, embed_dim=256)
        m.set_option("conv3x3_img", on)
        if not arch.startswith("SimAM"):
            m.set_option("res_tail", 0)  # the image kernel alone (the fused tail: test_res_tail_*)
        if sd is None:
            sd = synth_state_dict(seed, m.state_dict_layout(), residual_tame=True)
        m.load_state_dict(sd)
        ms.append(m.to(DEV))
    return ms[0], ms[1], sd


CASES = [("ResNet50", 3, 100), ("ResNet50", 2, 37), ("ResNet101", 1, 200), ("ResNet293", 2, 64),
         ("ResNet34", 3, 77), ("ResNet18", 2, 9), ("SimAM_ResNet34_ASP", 2, 64)]


# option conv3x3_img: 1 = 32 / 64 channels on the image kernel, 2 / 3 = also 128 channels
# (stage 3 of the ResNets, stage 2 of SimAM-ResNet34; 4 x 32 and 2 x 32 position tiles)
@pytest.mark.parametrize("img", [1, 2, 3])
@pytest.mark.parametrize("arch,B,T", CASES)
def test_conv3x3_img_equals_implicit_gemm_and_oracle(arch, B, T, img):
    img, gemm, sd = _pair(arch, 31, img)
    x = torch.from_numpy(synth_feats(9, B, T, 80)).to(DEV)
    a = img.embed(x).cpu().numpy()
    b = gemm.embed(x).cpu().numpy()
    assert np.all(np.isfinite(a))
    assert np.array_equal(a, b), np.abs(a - b).max()
    rows = list(range(min(B, 2)))
    with torch.no_grad():
        _, ref = models_ref.forward(arch, x[rows].cpu(), {k: torch.from_numpy(v) for k, v in sd.items()})
    assert np.abs(a[rows] - ref.numpy()).max() < 1e-4


@pytest.mark.parametrize("img", [1, 2])
def test_conv3x3_img_batch_rows_equal_batch_of_one(img):
    img, _, _ = _pair("ResNet50", 32, img)
    x = torch.from_numpy(synth_feats(10, 6, 150, 80)).to(DEV)
    full = img.embed(x).cpu().numpy()
    for i in (0, 3, 5):
        one = img.embed(x[i:i + 1]).cpu().numpy()[0]
        assert np.array_equal(full[i], one)


@pytest.mark.parametrize("arch,B,T", [("ResNet293", 2, 64), ("ResNet50", 3, 37), ("ResNet34", 2, 77)])
def test_residual_prefetch_bit_identical(arch, B, T):
    """Option res_prefetch (conv_gemm_x3 ROLE 2: the 1x1 residual convs load their
    residual ahead of the last two k-tiles) changes only when the residual is read:
    same products, same order, same epilogue -> identical embeddings."""
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    outs, sd = [], None
    x = torch.from_numpy(synth_feats(12, B, T, 80)).to(DEV)
    for on in (1, 0):
        m = HipSpeakerModel(arch, feat_dim=80, embed_dim=256)
        m.set_option("res_prefetch", on)
        if sd is None:
            sd = synth_state_dict(33, m.state_dict_layout(), residual_tame=True)
        m.load_state_dict(sd)
        m.to(DEV)
        outs.append(m.embed(x).cpu().numpy())
    assert np.all(np.isfinite(outs[0]))
    assert np.array_equal(outs[0], outs[1])



def _tail_pair(arch, seed, feat_dim, on=1):
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    ms, sd = [], None
    for on in (on, 0):
        m = HipSpeakerModel(arch, feat_dim=feat_dim, embed_dim=256)
        m.set_option("res_tail", on)
        if sd is None:
            sd = synth_state_dict(seed, m.state_dict_layout(), residual_tame=True)
        m.load_state_dict(sd)
        ms.append(m.to(DEV))
    return ms[0], ms[1], sd


# feat_dim 40: stage 3 runs at F = 10, a partial 4-row frequency tile; T = 37 / 100 / 150
# leave partial 32- / 64-frame time tiles (tail2_kernel's 8 / 4 / 2-row frequency tiles divide
# F / 2^s exactly for the valid feat_dim % 8 == 0; tools/tail_check exercises partial ones)
@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("arch,B,T,F", [("ResNet50", 3, 100, 80), ("ResNet50", 2, 37, 40),
                                        ("ResNet101", 1, 150, 80), ("ResNet293", 2, 64, 80),
                                        ("ResNet152", 2, 45, 40)])
def test_res_tail_matches_unfused_and_oracle(arch, B, T, F, mode):
    """Option res_tail (conv3x3_img.hip bottleneck_tail: conv2 + conv3 + residual in one
    launch, conv2's output kept in registers as conv3's A operand with a permuted k
    order; mode 1 also runs the next block's conv1 on the output chunks staged in LDS)
    against the unfused launches (conv3x3_img + conv_gemm_x3) and the oracle.  The same
    bf16x3 products are summed in a different k order inside the MFMAs, so the paths
    agree to fp32 rounding, not bitwise."""
    tail, plain, sd = _tail_pair(arch, 41, F, mode)
    x = torch.from_numpy(synth_feats(19, B, T, F)).to(DEV)
    a = tail.embed(x).cpu().numpy()
    b = plain.embed(x).cpu().numpy()
    assert np.all(np.isfinite(a))
    assert np.abs(a - b).max() <= 2e-5 * max(1.0, float(np.abs(b).max())), np.abs(a - b).max()
    with torch.no_grad():
        _, ref = models_ref.forward(arch, x.cpu(), {k: torch.from_numpy(v) for k, v in sd.items()})
    assert np.abs(a - ref.numpy()).max() < 1e-4


@pytest.mark.parametrize("mode", [1, 2])
def test_res_tail_batch_rows_equal_batch_of_one(mode):
    tail, _, _ = _tail_pair("ResNet50", 42, 80, mode)
    x = torch.from_numpy(synth_feats(20, 5, 123, 80)).to(DEV)
    full = tail.embed(x).cpu().numpy()
    for i in (0, 2, 4):
        assert np.array_equal(full[i], tail.embed(x[i:i + 1]).cpu().numpy()[0])
