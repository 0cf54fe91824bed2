"""GPU: the north-star EER-delta proxy (BASELINE.json: "vox1-O-clean EER within
+-0.01 % absolute of the reference").  Real VoxCeleb audio and a trained
checkpoint are absent offline, so the delta is measured on speaker-structured
synthetic data whose EER is realistic (~1 %), through the whole scoring path of
local/score.sh / score_norm.sh:

  HIP:    wav -> wsp_fbank (+CMN) -> ECAPA forward -> mean-vector cosine
          (wsp_cosine_pairs, scoring.trials_cosine_score's {:.5f} score file) -> AS-Norm
          top-n (wsp_asnorm_stats) + combine (scoring.score_norm's {:.5f} file) -> EER / minDCF
  oracle: f64 numpy fbank -> fp32 torch-CPU ECAPA -> numpy cosine / AS-Norm ->
          EER / minDCF (oracle/scoring_ref, pinned by tests/golden/scoring.npz)

Scores are rounded to the 5 decimals the reference writes (bin/score.py:69-71,
bin/score_norm.py:113-115) before the metrics, as compute_metrics.py reads them
back.  Bars: |dEER| <= 1e-4 (0.01 % absolute), |dminDCF| <= 1e-3.

Two tiers:
* model level: 40 speakers x 8 utterances of 2 s (the vox1-O speaker count),
  every target pair + 20 000 non-target pairs, a 100-speaker cohort (2 utterances
  each, speaker means as tools/vector_mean.py makes them), top-50;
* scoring level at the vox1-O shape: 4 874 eval embeddings of 40 speakers,
  37 611 trials, a 10 000-speaker cohort, top-300 (embeddings = speaker centres +
  noise, the same inputs for both pipelines).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from oracle import fbank_ref, models_ref, scoring_ref  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_speaker_audio, synth_state_dict  # noqa: E402

DEV = "cuda:0"
P_TARGET, C_MISS, C_FA = 0.01, 1, 1   # local/score.sh:46-50


def _r5(x):
    return np.array([float(f"{v:.5f}") for v in np.asarray(x, np.float64)])


def _metrics(scores, labels, impl):
    fnr, fpr = impl.compute_pmiss_pfa_rbst(np.asarray(scores), np.asarray(labels))
    return impl.compute_eer(fnr, fpr), impl.compute_c_norm(fnr, fpr, P_TARGET, C_MISS, C_FA)


def _trials(rng, spk, n_nontarget):
    n = len(spk)
    ia, ib = np.triu_indices(n, 1)
    tgt = spk[ia] == spk[ib]
    a, b = ia[tgt], ib[tgt]
    na = rng.integers(0, n, 4 * n_nontarget)
    nb = rng.integers(0, n, 4 * n_nontarget)
    keep = spk[na] != spk[nb]
    na, nb = na[keep][:n_nontarget], nb[keep][:n_nontarget]
    ia = np.concatenate([a, na]).astype(np.int32)
    ib = np.concatenate([b, nb]).astype(np.int32)
    lab = np.concatenate([np.ones(len(a), int), np.zeros(len(na), int)])
    return ia, ib, lab


def _hip_scores(E, C, mean_vec, ia, ib, top_n, lab, tmp_path):
    """The product's file path of local/score.sh + local/score_norm.sh: embeddings by
    key, a trials file, scoring.trials_cosine_score (bin/score.py:38-72, `{:.5f}` score
    file), scoring.score_norm (bin/score_norm.py:54-115: the score file read back, AS-Norm
    statistics on the GPU, the combine, `{:.5f}` output) -- both files parsed as
    compute_metrics.py reads them."""
    from wespeaker_hubert_amd import scoring
    keys = [f"u{i:05d}" for i in range(len(E))]
    emb = {k: E[i] for i, k in enumerate(keys)}
    cohort = {f"spk{i:05d}": C[i] for i in range(len(C))}
    trial = tmp_path / "trials"
    with open(trial, "w") as f:
        for a, b, l in zip(ia, ib, lab):
            f.write(f"{keys[a]} {keys[b]} {'target' if l else 'nontarget'}\n")
    score_file, = scoring.trials_cosine_score(emb, [str(trial)], str(tmp_path / "scores"), mean_vec=mean_vec,
                                              device=DEV)
    norm_file = str(tmp_path / "trials.asnorm.score")
    scoring.score_norm("asnorm", top_n, score_file, norm_file, cohort, emb, mean_vec=mean_vec, device=DEV)

    def col(path):
        rows = [ln.split() for ln in open(path)]
        assert [r[0] for r in rows] == [keys[a] for a in ia] and [r[1] for r in rows] == [keys[b] for b in ib]
        return np.array([float(r[2]) for r in rows])
    return col(score_file), col(norm_file)


def _ref_scores(E, C, mean_vec, ia, ib, top_n):
    Em = (E - mean_vec).astype(np.float64)
    nrm = np.linalg.norm(Em, axis=1)
    c5 = _r5((Em[ia] * Em[ib]).sum(1) / (nrm[ia] * nrm[ib]))
    mu, sd = scoring_ref.get_mean_std(E - mean_vec, C - mean_vec, top_n)
    return c5, _r5(scoring_ref.asnorm(c5, mu[ia], sd[ia], mu[ib], sd[ib]))


def _compare(hip, ref, labels, eer_range):
    from wespeaker_hubert_amd import scoring
    out = {}
    for name, h, r in (("cosine", hip[0], ref[0]), ("asnorm", hip[1], ref[1])):
        eh, dh = _metrics(h, labels, scoring)
        er, dr = _metrics(r, labels, scoring_ref)
        assert eer_range[0] < er < eer_range[1], (name, er)
        assert abs(eh - er) <= 1e-4, (name, eh, er)
        assert abs(dh - dr) <= 1e-3, (name, dh, dr)
        out[name] = (eh, er, dh, dr)
    return out


def test_eer_delta_model_level_ecapa(tmp_path):
    from wespeaker_hubert_amd.frontend import compute_fbank
    from wespeaker_hubert_amd.speaker_model import HipSpeakerModel
    arch, n_spk, n_utt, N = "ECAPA_TDNN_c512", 40, 8, 32000
    m = HipSpeakerModel(arch, feat_dim=80, embed_dim=192)
    sd = synth_state_dict(77, m.state_dict_layout())
    m.load_state_dict(sd)
    m.to(DEV)
    wav = synth_speaker_audio(5, range(n_spk), n_utt, N, snr_db=10.0, jitter=0.5)
    coh = synth_speaker_audio(5, range(1000, 1100), 2, N, snr_db=10.0, jitter=0.5)
    allw = np.concatenate([wav, coh])

    # HIP extraction: device fbank + CMN, batched ECAPA forward
    emb = m(compute_fbank(torch.from_numpy(allw).to(DEV), scale=1.0, cmn=True))[-1].cpu().numpy()
    # oracle extraction
    feats = np.stack([fbank_ref.fbank(w, cmn=True) for w in allw])
    with torch.no_grad():
        _, ref = models_ref.forward(arch, torch.from_numpy(feats), {k: torch.from_numpy(v) for k, v in sd.items()})
    ref = ref.numpy()
    assert np.abs(emb - ref).max() < 1e-4

    ne = n_spk * n_utt
    spk = np.repeat(np.arange(n_spk), n_utt)
    ia, ib, lab = _trials(np.random.default_rng(3), spk, 20000)
    res = []
    for E_all in (emb, ref):
        E = E_all[:ne]
        Cu = E_all[ne:]
        mean_vec = Cu.mean(0).astype(np.float32)                  # mean of the cohort set's embeddings
        C = Cu.reshape(100, 2, -1).mean(1).astype(np.float32)     # per-speaker cohort means (vector_mean.py)
        res.append((E, C, mean_vec))
    hip = _hip_scores(*res[0], ia, ib, 50, lab, tmp_path)
    orc = _ref_scores(*res[1], ia, ib, 50)
    _compare(hip, orc, lab, (1e-3, 0.05))


def test_eer_delta_scoring_vox1o_shape(tmp_path):
    rng = np.random.default_rng(11)
    n_spk, Ne, Nc, D, n_trials, top_n = 40, 4874, 10000, 192, 37611, 300
    centres = rng.standard_normal((n_spk, D))
    spk = np.sort(rng.integers(0, n_spk, Ne))
    E = (centres[spk] + 1.45 * rng.standard_normal((Ne, D))).astype(np.float32)
    C = (rng.standard_normal((Nc, D)) + 0.3 * rng.standard_normal(D)).astype(np.float32)
    mean_vec = C.mean(0).astype(np.float32)
    ia, ib, lab = _trials(rng, spk, n_trials)
    keep = np.concatenate([rng.permutation(np.flatnonzero(lab == 1))[:n_trials // 10],
                           np.flatnonzero(lab == 0)[:n_trials - n_trials // 10]])
    ia, ib, lab = ia[keep], ib[keep], lab[keep]
    assert len(lab) == n_trials
    hip = _hip_scores(E, C, mean_vec, ia, ib, top_n, lab, tmp_path)
    orc = _ref_scores(E, C, mean_vec, ia, ib, top_n)
    _compare(hip, orc, lab, (1e-3, 0.05))
