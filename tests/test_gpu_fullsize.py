"""GPU parity at the BASELINE.json configuration sizes.

* C5: AS-Norm statistics and trial scores at the vox1-O shape — 4 874 x 192
  eval embeddings, a 10 000-speaker cohort, top-300, 37 611 trials — against
  oracle/scoring_ref (bin/score_norm.py:26-36, 105-107; bin/score.py:38-72).
* C2: ECAPA_TDNN_c1024 on the bench batch (B = 256 x 5 s waveforms through the
  fused fbank + CMN launch): rows 0 / 127 / 255 equal their batch-of-one
  embeddings and the oracle chain (f64 fbank + fp32 torch ECAPA) at the
  north-star bar (per-dim 1e-4, cosine 0.9999).
* C3: ResNet293 at B = 128 x 5 s, which the model runs as two 64-utterance
  chunks (2-GiB operand cap): rows on both sides of the chunk boundary equal
  their batch-of-one embeddings and the oracle.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import fbank_ref, models_ref, scoring_ref  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict  # noqa: E402

DEV = "cuda:0"
EMB_ATOL = 1e-4
EMB_COS = 0.9999


def _assert_emb(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert np.all(np.isfinite(got))
    d = np.abs(got - ref).max()
    cos = (got * ref).sum(-1) / (np.linalg.norm(got, axis=-1) * np.linalg.norm(ref, axis=-1))
    assert d < EMB_ATOL, f"max |delta| {d}"
    assert cos.min() >= EMB_COS, cos.min()


def test_c5_asnorm_vox1o_shape(tmp_path):
    from wespeaker_hubert_amd import scoring
    rng = np.random.default_rng(55)
    Ne, Nc, D, top_n, n_trials = 4874, 10000, 192, 300, 37611
    E = rng.standard_normal((Ne, D)).astype(np.float32)
    C = rng.standard_normal((Nc, D)).astype(np.float32)
    C[17:40] = C[3]  # exact ties inside the score rows
    mean_vec = (0.1 * rng.standard_normal(D)).astype(np.float32)
    Ed = torch.from_numpy(E).to(DEV)
    Cd = torch.from_numpy(C).to(DEV)
    mvd = torch.from_numpy(mean_vec).to(DEV)
    mu, sd = scoring.asnorm_stats(Ed, Cd, top_n, mean_vec=mvd)
    rmu, rsd = scoring_ref.get_mean_std(E - mean_vec, C - mean_vec, top_n)
    np.testing.assert_allclose(mu, rmu, atol=3e-6)
    np.testing.assert_allclose(sd, rsd, atol=3e-6)
    # trials: cosine of mean-subtracted embeddings, then AS-Norm, at {:.5f} like score.py / score_norm.py
    ia = rng.integers(0, Ne, n_trials).astype(np.int32)
    ib = rng.integers(0, Ne, n_trials).astype(np.int32)
    Em = torch.from_numpy(E - mean_vec).to(DEV)
    s = scoring.cosine_pairs(Em, ia, ib)
    Em64 = (E - mean_vec).astype(np.float64)
    nrm = np.linalg.norm(Em64, axis=1)
    ref_s = (Em64[ia] * Em64[ib]).sum(1) / (nrm[ia] * nrm[ib])
    np.testing.assert_allclose(s, ref_s, atol=1e-12)
    s5 = np.array([float(f"{v:.5f}") for v in s])
    r5 = np.array([float(f"{v:.5f}") for v in ref_s])
    ref = scoring_ref.asnorm(r5, rmu[ia], rsd[ia], rmu[ib], rsd[ib])
    # the product's score files: bin/score.py's `{:.5f}` trial scores, then bin/score_norm.py's
    # read-back + AS-Norm combine + `{:.5f}` output (scoring.trials_cosine_score / score_norm)
    keys = [f"id{i:05d}" for i in range(Ne)]
    emb = {k: E[i] for i, k in enumerate(keys)}
    trial = tmp_path / "vox1_O_cleaned.kaldi"
    with open(trial, "w") as f:
        for a, b in zip(ia, ib):
            f.write(f"{keys[a]} {keys[b]} {'target' if a % 7 == b % 7 else 'nontarget'}\n")
    score_file, = scoring.trials_cosine_score(emb, [str(trial)], str(tmp_path / "scores"), mean_vec=mean_vec,
                                              device=DEV)
    norm_file = str(tmp_path / "vox1_O_cleaned.kaldi.asnorm.score")
    scoring.score_norm("asnorm", top_n, score_file, norm_file, {f"spk{i}": C[i] for i in range(Nc)}, emb,
                       mean_vec=mean_vec, device=DEV)
    rows = [ln.split() for ln in open(norm_file)]
    assert len(rows) == n_trials and all(len(r) == 8 for r in rows)
    got = np.array([float(r[2]) for r in rows])
    assert np.abs(got - ref).max() < 1e-3  # AS-Norm scores, written {:.5f} by the reference
    assert np.mean(np.abs(got - ref) < 1.5e-5) > 0.999
    # side columns (score_norm.py:111-115): |e - mean|, |t - mean|, mu_e, mu_t at 4 decimals
    e_mag = np.linalg.norm(Em64, axis=1)
    np.testing.assert_allclose([float(r[4]) for r in rows], e_mag[ia], atol=6e-5)
    np.testing.assert_allclose([float(r[7]) for r in rows], rmu[ib], atol=6e-5)


def test_asnorm_top_n_larger_than_cohort_uses_whole_cohort():
    """score_norm.py:33 slices [:, :top_n]: an oversized top_n means the whole cohort."""
    from wespeaker_hubert_amd import scoring
    rng = np.random.default_rng(56)
    E = torch.from_numpy(rng.standard_normal((9, 64)).astype(np.float32)).to(DEV)
    C = torch.from_numpy(rng.standard_normal((50, 64)).astype(np.float32)).to(DEV)
    a = scoring.asnorm_stats(E, C, 57)
    b = scoring.asnorm_stats(E, C, 50)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])


def _rows_vs_one_and_oracle(arch, B, rows, seed, residual_tame, **kw):
    from wespeaker_hubert_amd.frontend import compute_fbank
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    m = HipSpeakerModel(arch, **kw)
    sd = synth_state_dict(seed, m.state_dict_layout(), residual_tame=residual_tame)
    m.load_state_dict(sd)
    m.to(DEV)
    wav = synth_audio(seed + 1, B, 80000)
    wd = torch.from_numpy(wav).to(DEV)
    feats = compute_fbank(wd, scale=1.0, cmn=True)
    emb = m(feats)[-1].cpu().numpy()
    assert emb.shape[0] == B and np.all(np.isfinite(emb))
    sdt = {k: torch.from_numpy(v) for k, v in sd.items()}
    ref_feats = np.stack([fbank_ref.fbank(wav[r], cmn=True) for r in rows])
    with torch.no_grad():
        _, ref = models_ref.forward(arch, torch.from_numpy(ref_feats), sdt)
    for i, r in enumerate(rows):
        one = m(compute_fbank(wd[r:r + 1].contiguous(), scale=1.0, cmn=True))[-1].cpu().numpy()[0]
        assert np.abs(emb[r] - one).max() <= 1e-6, (r, np.abs(emb[r] - one).max())
    _assert_emb(emb[list(rows)], ref.numpy())


def test_c2_ecapa_c1024_bench_batch_rows():
    _rows_vs_one_and_oracle("ECAPA_TDNN_c1024", 256, (0, 127, 255), 1234, False, feat_dim=80, embed_dim=192)


def test_c3_resnet293_two_chunk_rows():
    _rows_vs_one_and_oracle("ResNet293", 128, (0, 63, 64, 127), 1234, True, feat_dim=80, embed_dim=256)


def test_ecapa_c1024_batch_beyond_2gib_runs_in_chunks():
    """B = 640 x 5 s: the [M][1536] ASTP operands exceed 2 GiB (32-bit buffer offsets), so the
    forward runs two 320-utterance chunks over one chunk-sized workspace; rows on both sides of
    the chunk seam equal their batch-of-one embeddings and the oracle (bin/extract.py:90-120
    feeds batches of any size)."""
    _rows_vs_one_and_oracle("ECAPA_TDNN_c1024", 640, (0, 319, 320, 639), 4321, False, feat_dim=80, embed_dim=192)
