"""GPU parity of the HuBERT-base SSL front end and
the C4 chain HuBERT -> CMN -> ECAPA_TDNN_GLOB_c512(feat_dim 768).

Checker: oracle/hubert_ref.py (fp32 torch-CPU restatement, pinned against the
transformers HubertModel proxy fixture tests/golden/hubert_proxy.npz; the s3prl
glue itself is parity-unpinned — s3prl is absent offline).
Tolerances: hidden states / features |delta| <= 2e-4 (LayerNorm-scaled O(1)
values after 12 fp32-class layers); embeddings per-dim |delta| < 1e-4 and
cosine >= 0.9999 (BASELINE.json north_star).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import hubert_ref, models_ref  # noqa: E402
from wespeaker_hubert_amd.arch import hubert_params, s3prl_num_frames  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict  # noqa: E402

DEV = "cuda:0"
FEAT_ATOL = 2e-4
EMB_ATOL = 1e-4
EMB_COS = 0.9999
SEED = 41


@pytest.fixture(scope="module")
def sd_np():
    return synth_state_dict(SEED, hubert_params())


@pytest.fixture(scope="module")
def sd_t(sd_np):
    return {k: torch.from_numpy(v) for k, v in sd_np.items()}


def _frontend(sd_np, layer=-1, precision=1, multilayer=True):
    from wespeaker_hubert_amd.s3prl_frontend import S3prlFrontend
    fe = S3prlFrontend({"name": "hubert_base"}, multilayer_feature=multilayer, layer=layer)
    fe.set_option("precision", precision)
    fe.load_state_dict(sd_np)
    return fe.to(DEV)


def _wav(seed, B, W):
    return synth_audio(seed, B, W, int16_scale=False)


def _cmn(x):
    return x - x.mean(dim=1, keepdim=True)


@pytest.mark.parametrize("layer", [0, 1, 6, 12])
def test_hidden_state_matches_oracle(sd_np, sd_t, layer):
    wav = _wav(7, 2, 16000)
    fe = _frontend(sd_np, layer=layer, multilayer=False)
    got = fe.extract(torch.from_numpy(wav).to(DEV)).cpu()
    with torch.no_grad():
        ref = hubert_ref.s3prl_upstream(torch.from_numpy(wav), sd_t)[layer]
    assert got.shape == ref.shape == (2, 50, 768)
    d = (got - ref).abs().max().item()
    assert d <= FEAT_ATOL, f"layer {layer}: max |delta| {d}"


@pytest.mark.parametrize("precision", [1, 0], ids=["bf16x3", "f32"])
@pytest.mark.parametrize("W", [16000, 12345, 400, 48000, 799, 250, 1])
def test_featurizer_output_matches_oracle(sd_np, sd_t, precision, W):
    wav = _wav(8, 2, W)
    fe = _frontend(sd_np, precision=precision)
    x = torch.from_numpy(wav).to(DEV)
    got = fe.extract(x).cpu()
    got_cmn = fe.extract(x, cmn=True).cpu()
    with torch.no_grad():
        ref = hubert_ref.s3prl_frontend(torch.from_numpy(wav), sd_t)
    assert got.shape == ref.shape == (2, s3prl_num_frames(W), 768)
    assert (got - ref).abs().max().item() <= FEAT_ATOL
    assert (got_cmn - _cmn(ref)).abs().max().item() <= FEAT_ATOL
    feats, lens = fe(x, torch.full((2,), W, dtype=torch.long))
    assert torch.equal(feats.cpu(), got) and lens.tolist() == [s3prl_num_frames(W)] * 2


def test_last_layer_when_not_multilayer(sd_np, sd_t):
    """multilayer_feature=False, layer=-1: featurizer over feats[-1:] (s3prl.py:88-91)."""
    wav = _wav(9, 1, 8000)
    got = _frontend(sd_np, multilayer=False).extract(torch.from_numpy(wav).to(DEV)).cpu()
    with torch.no_grad():
        ref = hubert_ref.s3prl_upstream(torch.from_numpy(wav), sd_t)[-1]
    assert (got - ref).abs().max().item() <= FEAT_ATOL


def test_short_input_is_zero_padded_to_min_second(sd_np, sd_t):
    """s3prl S3PRLUpstream.forward pads batches shorter than MIN_SECOND (800
    samples) with zeros before HuBERT: the padded samples change the features
    (GroupNorm / conv frames), and the output keeps len(range(0, W, 320)) frames."""
    W = 600
    wav = _wav(14, 2, W)
    got = _frontend(sd_np).extract(torch.from_numpy(wav).to(DEV)).cpu()
    with torch.no_grad():
        ref = hubert_ref.s3prl_frontend(torch.from_numpy(wav), sd_t)
        padded = hubert_ref.s3prl_frontend(torch.from_numpy(np.pad(wav, ((0, 0), (0, 200)))), sd_t)
    assert got.shape == (2, 2, 768)
    assert (got - ref).abs().max().item() <= FEAT_ATOL
    assert (got - padded[:, :2]).abs().max().item() <= FEAT_ATOL


def test_batch_rows_independent_and_chunked(sd_np):
    """Size-independent property at the bench shape: a 5 s batch big enough to
    split the feature extractor into utterance chunks gives every row exactly
    what a batch of one gives."""
    B, W = 60, 80000
    wav = torch.from_numpy(_wav(10, B, W)).to(DEV)
    fe = _frontend(sd_np)
    fe.set_option("streams", 1)  # one utterance range: 60 x 15 999 conv0 rows > one 917 504-row chunk
    full = fe.extract(wav, cmn=True)
    for i in (0, 31, B - 1):
        one = fe.extract(wav[i:i + 1].contiguous(), cmn=True)
        d = (full[i] - one[0]).abs().max().item()
        assert d <= 1e-5, f"row {i}: {d}"
    assert torch.isfinite(full).all()


def test_hubert_ecapa_chain_embeddings(sd_np, sd_t):
    """C4: wav -> HuBERT -> CMN -> ECAPA_TDNN_GLOB_c512(feat_dim=768) -> embed."""
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    wav = _wav(11, 3, 24000)
    fe = _frontend(sd_np)
    m = HipSpeakerModel("ECAPA_TDNN_GLOB_c512", feat_dim=768, embed_dim=192)
    sd_e = synth_state_dict(12, m.state_dict_layout())
    m.load_state_dict(sd_e)
    m.to(DEV)
    feats = fe.extract(torch.from_numpy(wav).to(DEV), cmn=True)
    got = m(feats)[-1].cpu().numpy()
    with torch.no_grad():
        f_ref = _cmn(hubert_ref.s3prl_frontend(torch.from_numpy(wav), sd_t))
        ref = models_ref.forward("ECAPA_TDNN_GLOB_c512", f_ref,
                                 {k: torch.from_numpy(v) for k, v in sd_e.items()})[-1].numpy()
    d = np.abs(got - ref).max()
    cos = (got * ref).sum(1) / (np.linalg.norm(got, axis=1) * np.linalg.norm(ref, axis=1))
    assert d < EMB_ATOL, f"max |delta| {d}"
    assert cos.min() >= EMB_COS


@pytest.mark.parametrize("layer,multi", [(-1, True), (3, False)])
def test_ragged_batch_equals_batch_of_one(sd_np, sd_t, layer, multi):
    """wsp_frontend_forward_segments: utterances of different lengths in one launch
    give each utterance's batch-of-one features (and the oracle's)."""
    lens = [400, 12345, 16000, 8007, 48000, 1999, 250, 700]
    wavs = [_wav(40 + i, 1, n)[0] for i, n in enumerate(lens)]
    fe = _frontend(sd_np, layer=layer, multilayer=multi)
    feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs], cmn=True)
    assert offs == list(np.concatenate([[0], np.cumsum([s3prl_num_frames(n) for n in lens])]))
    for i, w in enumerate(wavs):
        one = fe.extract(torch.from_numpy(w[None]).to(DEV), cmn=True)[0]
        got = feats[offs[i]:offs[i + 1]]
        assert (got - one).abs().max().item() <= 1e-5, i
        if i in (0, 3, 6, 7):
            with torch.no_grad():
                if layer < 0:
                    ref = hubert_ref.s3prl_frontend(torch.from_numpy(w[None]), sd_t)
                else:
                    ref = hubert_ref.s3prl_upstream(torch.from_numpy(w[None]), sd_t)[layer]
            ref = _cmn(ref)[0]
            assert (got.cpu() - ref).abs().max().item() <= FEAT_ATOL


@pytest.mark.parametrize("W", [16000, 100000])
@pytest.mark.parametrize("pipe", [1, 0])
def test_lds_attention_matches_oracle(sd_np, sd_t, W, pipe):
    """attn.hip — the persistent pipelined kernel (keys in LDS halves of 128, the next
    half in flight) and the one-block-per-(utterance, head) kernel — against the oracle;
    W = 100000 gives 312 frames: two query blocks and three key halves per (utterance,
    head)."""
    wav = _wav(17, 2, W)
    fe = _frontend(sd_np)
    fe.set_option("attn_pipe", pipe)
    got = fe.extract(torch.from_numpy(wav).to(DEV)).cpu()
    with torch.no_grad():
        ref = hubert_ref.s3prl_frontend(torch.from_numpy(wav), sd_t)
    assert float((got - ref).abs().max()) < FEAT_ATOL


def test_lds_attention_ragged_long_utterances(sd_np):
    fe = _frontend(sd_np)
    lens = [100000, 3200, 90000, 16000]
    wavs = [_wav(60 + i, 1, n)[0] for i, n in enumerate(lens)]
    feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs], cmn=True)
    for i, w in enumerate(wavs):
        one = fe.extract(torch.from_numpy(w[None]).to(DEV), cmn=True)[0]
        np.testing.assert_allclose(feats[offs[i]:offs[i + 1]].cpu().numpy(), one.cpu().numpy(), atol=1e-5, rtol=0)


def test_c4_bench_shape_rows_match_oracle(sd_np, sd_t):
    """C4 at the bench shape: B = 256 x 5 s with the default front-end options (two
    utterance-range streams of 128, each split into 57 / 57 / 14-utterance feature-
    extractor chunks: the 2-GiB conv0 operand cap) -> CMN -> ECAPA_TDNN_GLOB_c512(768).
    Rows at the start, at both chunk boundaries and the stream boundary, and at the end
    equal their batch-of-one embeddings and the oracle chain at the north-star bar."""
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    B, W = 256, 80000
    rows = (0, 56, 57, 127, 128, 255)
    wav = _wav(13, B, W)
    fe = _frontend(sd_np)
    assert fe.get_option("streams") == 2
    m = HipSpeakerModel("ECAPA_TDNN_GLOB_c512", feat_dim=768, embed_dim=192)
    sd_e = synth_state_dict(12, m.state_dict_layout())
    m.load_state_dict(sd_e)
    m.to(DEV)
    wd = torch.from_numpy(wav).to(DEV)
    got = m(fe.extract(wd, cmn=True))[-1].cpu().numpy()
    assert got.shape == (B, 192) and np.all(np.isfinite(got))
    for r in rows:
        one = m(fe.extract(wd[r:r + 1].contiguous(), cmn=True))[-1].cpu().numpy()[0]
        assert np.abs(got[r] - one).max() <= 1e-6, (r, np.abs(got[r] - one).max())
    with torch.no_grad():
        f_ref = _cmn(hubert_ref.s3prl_frontend(torch.from_numpy(wav[list(rows)]), sd_t))
        ref = models_ref.forward("ECAPA_TDNN_GLOB_c512", f_ref,
                                 {k: torch.from_numpy(v) for k, v in sd_e.items()})[-1].numpy()
    g = got[list(rows)]
    d = np.abs(g - ref).max()
    cos = (g * ref).sum(1) / (np.linalg.norm(g, axis=1) * np.linalg.norm(ref, axis=1))
    assert d < EMB_ATOL, f"max |delta| {d}"
    assert cos.min() >= EMB_COS


def test_lds_dma_tile_bit_identical_to_register_staged(sd_np):
    """The front end on x3_variant 7 (default: the GEMMs family 7 takes staged by LDS-DMA, the rest
    on 6) equals x3_variant 6 bit for bit (same products, same MFMA order), ragged batch included
    (LayerNorm fold off: it exists on family 7 only)."""
    lens = [16000, 12345, 48000, 700]
    wavs = [_wav(70 + i, 1, n)[0] for i, n in enumerate(lens)]
    got = []
    for v in (6, 7):
        fe = _frontend(sd_np)
        fe.set_option("x3_variant", v)
        fe.set_option("ln_fold", 0)  # the fold runs on family 7 only (its own test below)
        feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs], cmn=True)
        uni = fe.extract(torch.from_numpy(_wav(75, 3, 32000)).to(DEV), cmn=True)
        got.append((feats.cpu().numpy(), uni.cpu().numpy()))
    for g in got[1:]:
        np.testing.assert_array_equal(got[0][0], g[0])
        np.testing.assert_array_equal(got[0][1], g[1])


@pytest.mark.parametrize("layer", [0, -1])
def test_direct_pos_conv_matches_grouped_gemm_and_oracle(sd_np, sd_t, layer):
    """pos_conv.hip (option pos_conv 1, default: one block per 256 frames x group, the input patch
    split once into LDS) against the grouped implicit GEMM (pos_conv 0, within 5e-5) and the oracle, on a ragged
    batch with utterances of 1 .. 3 frame windows (100000 samples = 312 frames; 700 -> 2 frames)
    and a uniform one.  Hidden state 0 is LayerNorm(x + GELU(pos_conv(x))): the kernel's output one
    LayerNorm away."""
    lens = [100000, 700, 16000, 250000, 12345]
    wavs = [_wav(80 + i, 1, n)[0] for i, n in enumerate(lens)]
    outs = []
    for pc in (1, 0):
        fe = _frontend(sd_np, layer=layer, multilayer=layer < 0)
        fe.set_option("pos_conv", pc)
        assert fe.get_option("pos_conv") == pc
        feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs])
        outs.append((feats.cpu(), offs))
    (a, offs), (b, _) = outs
    # two fp32 summation orders of the same conv, 12 layers downstream: a few ulp-scale 1e-5
    assert (a - b).abs().max().item() <= 5e-5
    for i in (0, 1, 3):
        with torch.no_grad():
            if layer < 0:
                ref = hubert_ref.s3prl_frontend(torch.from_numpy(wavs[i][None]), sd_t)[0]
            else:
                ref = hubert_ref.s3prl_upstream(torch.from_numpy(wavs[i][None]), sd_t)[layer][0]
        assert (a[offs[i]:offs[i + 1]] - ref).abs().max().item() <= FEAT_ATOL, i


@pytest.mark.parametrize("layer", [2, -1])
def test_layernorm_fold_matches_kernels_and_oracle(sd_np, sd_t, layer):
    """Option ln_fold 1: the post-attention LayerNorm folded into the GEMMs — out_proj
    emits per-row (mean, M2) partials, fc1 runs on the un-normalised rows with gamma in its
    weights and applies (acc - mu colsum(W')) rstd + b + W beta, fc2 normalises its residual on
    the fly — against ln_fold 0 (LayerNorm kernels) and the oracle, ragged batch included."""
    lens = [100000, 700, 16000, 48000, 12345]
    wavs = [_wav(90 + i, 1, n)[0] for i, n in enumerate(lens)]
    outs = []
    for lf in (1, 0):
        fe = _frontend(sd_np, layer=layer, multilayer=layer < 0)
        fe.set_option("ln_fold", lf)
        assert fe.get_option("ln_fold") == lf
        feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs])
        outs.append((feats.cpu(), offs))
    (a, offs), (b, _) = outs
    d = (a - b).abs().max().item()
    assert d <= 5e-5, d
    for i in (0, 1, 3):
        with torch.no_grad():
            if layer < 0:
                ref = hubert_ref.s3prl_frontend(torch.from_numpy(wavs[i][None]), sd_t)[0]
            else:
                ref = hubert_ref.s3prl_upstream(torch.from_numpy(wavs[i][None]), sd_t)[layer][0]
        assert (a[offs[i]:offs[i + 1]] - ref).abs().max().item() <= FEAT_ATOL, i


def test_ragged_multichunk_batch_tail_batch(sd_np):
    """a ragged wsp_frontend_forward_segments batch big enough to split the feature
    extractor into utterance chunks (conv0 rows above 2 GiB / 2 KB = 917 504 per chunk): CNN
    layers 4-6 then run batch-wide over global level-3/4/5 offsets with each chunk's rows
    placed at its chunk-relative row3.  Rows on both sides of the chunk boundary equal their
    batch-of-one features, and tail_batch 1 equals tail_batch 0 (per chunk) bit for bit."""
    rng = np.random.default_rng(3)
    lens = [int(n) for n in rng.integers(40000, 120000, 76)]
    wavs = [synth_audio(900 + i, 1, n, int16_scale=False)[0] for i, n in enumerate(lens)]
    t0 = [(n - 10) // 5 + 1 for n in lens]
    cap = (1 << 31) // 8 * 7 // (512 * 4)
    rows, b1 = 0, 0
    while b1 < len(lens) and (b1 == 0 or rows + t0[b1] <= cap):
        rows += t0[b1]
        b1 += 1
    assert 0 < b1 < len(lens), "the batch must span two feature-extractor chunks"
    fe = _frontend(sd_np)
    fe.set_option("streams", 1)  # one utterance range, so the chunking above is the kernel's
    feats, offs = fe.extract_segments([torch.from_numpy(w) for w in wavs], cmn=True)
    assert fe.get_option("tail_batch") == 1
    for i in (0, b1 - 1, b1, len(lens) - 1):
        one = fe.extract(torch.from_numpy(wavs[i][None]).to(DEV), cmn=True)[0]
        d = (feats[offs[i]:offs[i + 1]] - one).abs().max().item()
        assert d <= 1e-5, f"row {i} (chunk boundary at {b1}): {d}"
    fe.set_option("tail_batch", 0)
    feats0, offs0 = fe.extract_segments([torch.from_numpy(w) for w in wavs], cmn=True)
    assert offs0 == offs and torch.equal(feats0, feats)
