"""GPU tests of the drop-in boundary's configuration space beyond the voxceleb
defaults (VERDICT r5 "what's missing" #2), each through the C-ABI against the
CPU oracle:

  * kaldi.fbank options the recipes pass: num_mel_bins 23 / 40 / 64 / 72 / 80 /
    128 at 8 and 16 kHz (examples/sre/v2,v3/conf/resnet.yaml: 40 / 64 bins at
    8 kHz), the five window types (Speaker.set_window_type, cli/speaker.py:62);
  * apply_cmvn(norm_mean, norm_var) (dataset_utils.py:19-26), cmvn: false
    (bin/extract.py:104-106), uniform and ragged;
  * bin/extract.py with `--data_type feat` (Kaldi FM / CM2 matrices at ark
    offsets, processor.parse_feat) at batch_size 1 and > 1 (random chunks), and
    with an SRE-style 8 kHz 64-bin ResNet config + norm_var.

Tolerances: fbank within 1e-5 (max |log-mel|) of the float64 oracle and no further
from it than the float32 restatement of torchaudio's path (+ 2e-6); CMVN within 2e-6
(relative to the values' scale); embeddings the north-star per-dim 1e-4 / cosine
0.9999.  Fbank parity vs torchaudio itself stays unpinned (torchaudio absent).
"""
import json
import os
import random
import struct

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu

from oracle import fbank_ref, models_ref  # noqa: E402
from wespeaker_hubert_amd import arch as A  # noqa: E402
from wespeaker_hubert_amd.audio import write_wav  # noqa: E402
from wespeaker_hubert_amd.kaldi_io import load_scp_sequential  # noqa: E402
from wespeaker_hubert_amd.synthetic import synth_audio, synth_feats, synth_state_dict  # noqa: E402

DEV = "cuda:0"
FBANK_ATOL = 1e-5


def _cos(a, b):
    a, b = a.astype(np.float64), b.astype(np.float64)
    return float(a @ b / np.linalg.norm(a) / np.linalg.norm(b))


def _assert_emb(got, ref):
    assert np.all(np.isfinite(got))
    assert np.abs(got - ref).max() < 1e-4, np.abs(got - ref).max()
    assert _cos(got.ravel(), ref.ravel()) >= 0.9999


@pytest.mark.parametrize("nb,sr,win", [(40, 8000, "hamming"), (64, 8000, "hamming"), (23, 8000, "povey"),
                                       (72, 16000, "hamming"), (40, 16000, "hamming"), (128, 16000, "hamming"),
                                       (80, 16000, "povey"), (80, 16000, "hanning"), (80, 16000, "rectangular"),
                                       (80, 16000, "blackman"), (64, 8000, "blackman")])
def test_fbank_config_matches_oracle(nb, sr, win):
    from wespeaker_hubert_amd.frontend import FbankArgs, compute_fbank
    args = FbankArgs(nb, sample_rate=sr, window_type=win)
    fl, fs, _ = args.geometry()
    for N in (sr * 5, fl, fl + 3 * fs + 17):
        wav = synth_audio(40 + nb + N, 3, N)
        got = compute_fbank(torch.from_numpy(wav).to(DEV), scale=1.0, cmn=False, args=args).cpu().numpy()
        ref = np.stack([fbank_ref.fbank(w, nb, sample_freq=float(sr), window_type=win) for w in wav])
        ref32 = np.stack([fbank_ref.fbank(w, nb, sample_freq=float(sr), window_type=win, dtype=np.float32)
                          for w in wav])
        assert got.shape == ref.shape == (3, 1 + (N - fl) // fs, nb)
        d = float(np.abs(got - ref).max())
        err32 = float(np.abs(ref32 - ref).max())
        assert d <= FBANK_ATOL and d <= err32 + 2e-6, (N, d, err32)
        got_cmn = compute_fbank(torch.from_numpy(wav.astype(np.int16)).to(DEV), cmn=True, args=args).cpu().numpy()
        ref_cmn = np.stack([fbank_ref.fbank(w, nb, sample_freq=float(sr), window_type=win, cmn=True) for w in wav])
        assert np.abs(got_cmn - ref_cmn).max() <= FBANK_ATOL


def test_fbank_8k_segments_equal_per_utterance():
    from wespeaker_hubert_amd.frontend import FbankArgs, compute_fbank, compute_fbank_segments
    args = FbankArgs(64, sample_rate=8000)
    lens = [200, 8000, 281, 24000, 6173, 40000]
    wavs = [synth_audio(800 + i, 1, n)[0] for i, n in enumerate(lens)]
    feats, off, frames = compute_fbank_segments([torch.from_numpy(w) for w in wavs], device=torch.device(DEV),
                                                args=args)
    off = off.cpu().numpy()
    assert frames == [1 + (n - 200) // 80 for n in lens] and feats.shape[1] == 64
    for i, w in enumerate(wavs):
        one = compute_fbank(torch.from_numpy(w[None]).to(DEV), cmn=True, args=args)[0]
        assert torch.equal(feats[off[i]:off[i + 1]], one), i


def test_fbank_default_args_unchanged_instance():
    """The headline configuration keeps its fixed instance: the explicit default
    FbankArgs and the legacy wsp_fbank entry give identical bytes."""
    from wespeaker_hubert_amd import _lib
    from wespeaker_hubert_amd.frontend import FbankArgs, compute_fbank
    wav = torch.from_numpy(synth_audio(5, 2, 33333)).to(DEV)
    a = compute_fbank(wav, cmn=True, args=FbankArgs()).cpu()
    b = torch.empty_like(a.to(DEV))
    stream = torch.cuda.current_stream().cuda_stream
    _lib.check(_lib.load().wsp_fbank(wav.data_ptr(), _lib.WSP_DTYPE_F32, 2, wav.shape[1], wav.shape[1], 1.0,
                                     b.data_ptr(), 80, 16000, _lib.WSP_WINDOW_HAMMING, 1, stream), "wsp_fbank")
    assert torch.equal(a, b.cpu())


@pytest.mark.parametrize("norm_mean,norm_var", [(True, True), (False, True), (True, False)])
def test_cmvn_matches_oracle(norm_mean, norm_var):
    from wespeaker_hubert_amd.frontend import apply_cmvn
    x = (synth_feats(91, 3, 157, 80) * 3.0 + 7.0).astype(np.float32)
    got = apply_cmvn(torch.from_numpy(x).to(DEV), norm_mean, norm_var).cpu().numpy()
    ref = fbank_ref.apply_cmvn(x, norm_mean, norm_var)
    assert np.abs(got - ref).max() <= 2e-6 * max(1.0, float(np.abs(ref).max()))
    # ragged rows: each utterance equals its own (1, T, D) result; T = 1 gives NaN under norm_var
    lens = [157, 1, 33, 2]
    rows = [synth_feats(92 + i, 1, t, 40)[0] * 2.0 + 1.0 for i, t in enumerate(lens)]
    cat = torch.from_numpy(np.concatenate(rows).astype(np.float32)).to(DEV)
    off = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int32, device=DEV)
    got = apply_cmvn(cat, norm_mean, norm_var, frame_offsets=off).cpu().numpy()
    o = np.concatenate([[0], np.cumsum(lens)])
    for i, r in enumerate(rows):
        one = apply_cmvn(torch.from_numpy(r[None].astype(np.float32)).to(DEV), norm_mean, norm_var).cpu().numpy()[0]
        np.testing.assert_array_equal(got[o[i]:o[i + 1]], one)
        ref = fbank_ref.apply_cmvn(r[None], norm_mean, norm_var)[0]
        if lens[i] == 1 and norm_var:
            assert np.isnan(got[o[i]:o[i + 1]]).all()
        else:
            assert np.abs(got[o[i]:o[i + 1]] - ref).max() <= 2e-6 * max(1.0, float(np.abs(ref).max()))


# ----------------------------------------------------------------- extract --

def _write_kaldi_mats(path, mats, fmt="FM"):
    """Kaldi binary ark of matrices; returns {key: "path:offset"} (kaldiio.WriteHelper layout)."""
    specs = {}
    with open(path, "wb") as f:
        for k, m in mats.items():
            f.write(k.encode() + b" ")
            specs[k] = f"{path}:{f.tell()}"
            m = np.asarray(m, np.float32)
            if fmt == "FM":
                f.write(b"\0BFM \x04" + struct.pack("<i", m.shape[0]) + b"\x04" + struct.pack("<i", m.shape[1]))
                f.write(m.astype("<f4").tobytes())
            else:  # CM2: two-byte row-major with a global range
                mn, mx = float(m.min()), float(m.max())
                q = np.round((m - mn) / (mx - mn) * 65535.0).astype("<u2")
                f.write(b"\0BCM2 " + struct.pack("<ffii", mn, mx - mn, m.shape[0], m.shape[1]) + q.tobytes())
    return specs


def _make_model_dir(d, arch, model_args, dataset_args, seed):
    spec = A.make_spec(arch, **model_args)
    sd = synth_state_dict(seed, A.param_list(spec))
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, d / "avg_model.pt")
    with open(d / "config.yaml", "w") as f:
        yaml.safe_dump({"model": arch, "model_args": model_args, "dataset_args": dataset_args}, f)
    return {k: torch.from_numpy(v) for k, v in sd.items()}


@pytest.mark.parametrize("batch_size", [1, 3])
def test_extract_driver_feat_data_type(tmp_path, batch_size):
    """--data_type feat: JSON {key, feat, spk} lines whose feat is "ark:offset" (FM and CM2
    matrices), whole matrices at batch_size 1 (ragged batches), seeded num_frms chunks above
    (processor.random_chunk(..., 'feat')), then apply_cmvn (norm_mean) and ECAPA."""
    from wespeaker_hubert_amd.bin.extract import extract, get_random_chunk
    from wespeaker_hubert_amd.kaldi_io import load_mat
    arch = "ECAPA_TDNN_c512"
    sd = _make_model_dir(tmp_path, arch, {"feat_dim": 80, "embed_dim": 192, "pooling_func": "ASTP"},
                         {"frontend": "fbank", "num_frms": 50, "fbank_args": {"num_mel_bins": 80}}, 71)
    lens = [120, 37, 298, 60, 211]
    mats = {f"f{i}": synth_feats(600 + i, 1, t, 80)[0] * 4.0 + 1.5 for i, t in enumerate(lens)}
    specs = _write_kaldi_mats(str(tmp_path / "feats.ark"), dict(list(mats.items())[:3]), "FM")
    specs.update(_write_kaldi_mats(str(tmp_path / "feats2.ark"), dict(list(mats.items())[3:]), "CM2"))
    lst = tmp_path / "feat.list"
    with open(lst, "w") as f:
        for k in mats:
            f.write(json.dumps({"key": k, "feat": specs[k], "spk": "s"}) + "\n")
    scp = extract(config=str(tmp_path / "config.yaml"), model_path=str(tmp_path / "avg_model.pt"), data_type="feat",
                  data_list=str(lst), embed_ark=str(tmp_path / "xv.ark"), batch_size=batch_size, num_workers=2)
    got = dict(load_scp_sequential(scp))
    assert list(got) == list(mats)
    rng = random.Random(0)
    for k in mats:
        m = load_mat(specs[k])  # the stored (possibly compressed) values
        if k in ("f0", "f1", "f2"):
            np.testing.assert_array_equal(m, mats[k].astype(np.float32))
        else:
            assert np.abs(m - mats[k]).max() <= (mats[k].max() - mats[k].min()) / 65535.0
        x = m if batch_size == 1 else get_random_chunk(m, 50, rng)
        feats = fbank_ref.apply_cmvn(x[None], True, False)
        with torch.no_grad():
            _, ref = models_ref.forward(arch, torch.from_numpy(feats), sd)
        _assert_emb(got[k], ref[0].numpy())


def test_extract_driver_sre_8k_64bin_resnet_norm_var(tmp_path):
    """examples/sre/v3/conf/resnet.yaml shape: 8 kHz audio, fbank_args num_mel_bins 64,
    ResNet34 (feat_dim 64), plus cmvn_args norm_var: true; whole utterances."""
    from wespeaker_hubert_amd.bin.extract import extract
    arch = "ResNet34"
    margs = {"feat_dim": 64, "embed_dim": 256, "pooling_func": "TSTP", "two_emb_layer": False}
    dargs = {"frontend": "fbank", "resample_rate": 8000, "num_frms": 200,
             "fbank_args": {"num_mel_bins": 64, "frame_shift": 10, "frame_length": 25, "dither": 1.0},
             "cmvn": True, "cmvn_args": {"norm_mean": True, "norm_var": True}}
    sd = _make_model_dir(tmp_path, arch, margs, dargs, 72)
    lens = [8000, 12345, 24000]
    lines = []
    pcms = {}
    for i, n in enumerate(lens):
        pcm = synth_audio(900 + i, 1, n)[0]
        p = str(tmp_path / f"s{i}.wav")
        write_wav(p, pcm, sample_rate=8000)
        pcms[f"s{i}"] = pcm
        lines.append(json.dumps({"key": f"s{i}", "wav": p, "spk": "x"}))
    lst = tmp_path / "raw.list"
    lst.write_text("\n".join(lines) + "\n")
    scp = extract(config=str(tmp_path / "config.yaml"), model_path=str(tmp_path / "avg_model.pt"), data_type="raw",
                  data_list=str(lst), embed_ark=str(tmp_path / "xv.ark"), batch_size=1, num_workers=1)
    got = dict(load_scp_sequential(scp))
    for k, pcm in pcms.items():
        f = fbank_ref.fbank(pcm, 64, sample_freq=8000.0)
        f = fbank_ref.apply_cmvn(f[None], True, True)
        with torch.no_grad():
            _, ref = models_ref.forward(arch, torch.from_numpy(f), sd)
        _assert_emb(got[k], ref[0].numpy())


def test_extract_driver_cmvn_false(tmp_path):
    """dataset_args.cmvn: false — features go to the backbone unnormalised.  No reference
    recipe uses it; with raw log-mels (mean ~10-15) and synthetic weights (whose BN running
    statistics do not absorb that offset) every activation and the embedding itself come out
    ~10x larger than on CMN'd input, so the per-dim bar is taken relative to the embedding's
    largest magnitude (1e-4 x max(1, max|ref|)); cosine >= 0.9999 as everywhere."""
    from wespeaker_hubert_amd.bin.extract import extract
    arch = "ECAPA_TDNN_c512"
    sd = _make_model_dir(tmp_path, arch, {"feat_dim": 40, "embed_dim": 192, "pooling_func": "ASTP"},
                         {"frontend": "fbank", "num_frms": 200, "cmvn": False,
                          "fbank_args": {"num_mel_bins": 40, "frame_shift": 10, "frame_length": 25}}, 73)
    pcm = synth_audio(77, 2, 20000)
    lines = []
    for i in range(2):
        p = str(tmp_path / f"c{i}.wav")
        write_wav(p, pcm[i])
        lines.append(json.dumps({"key": f"c{i}", "wav": p, "spk": "x"}))
    (tmp_path / "raw.list").write_text("\n".join(lines) + "\n")
    scp = extract(config=str(tmp_path / "config.yaml"), model_path=str(tmp_path / "avg_model.pt"), data_type="raw",
                  data_list=str(tmp_path / "raw.list"), embed_ark=str(tmp_path / "xv.ark"), batch_size=1)
    got = dict(load_scp_sequential(scp))
    for i in range(2):
        f = fbank_ref.fbank(pcm[i], 40)[None]
        with torch.no_grad():
            _, ref = models_ref.forward(arch, torch.from_numpy(f), sd)
        ref = ref[0].numpy()
        g = got[f"c{i}"]
        assert np.all(np.isfinite(g)) and _cos(g, ref) >= 0.9999
        assert np.abs(g - ref).max() < 1e-4 * max(1.0, float(np.abs(ref).max())), (np.abs(g - ref).max(),
                                                                                    np.abs(ref).max())


@pytest.mark.parametrize("win", ["povey", "blackman"])
def test_speaker_set_window_type(tmp_path, win):
    """Speaker.set_window_type (cli/speaker.py:62) reaches the kernel: extract_embedding and
    extract_embedding_list equal the oracle chain with that window."""
    from wespeaker_hubert_amd.cli.speaker import load_model
    arch = "ECAPA_TDNN_c512"
    sd = _make_model_dir(tmp_path, arch, {"feat_dim": 80, "embed_dim": 192, "pooling_func": "ASTP"},
                         {"frontend": "fbank"}, 74)
    pcm = synth_audio(78, 2, 24000)
    paths = []
    for i in range(2):
        p = str(tmp_path / f"w{i}.wav")
        write_wav(p, pcm[i])
        paths.append(p)
    spk = load_model(str(tmp_path))
    spk.set_window_type(win)
    e0 = spk.extract_embedding(paths[0]).numpy()
    (tmp_path / "wav.scp").write_text("".join(f"w{i} {p}\n" for i, p in enumerate(paths)))
    names, embs = spk.extract_embedding_list(str(tmp_path / "wav.scp"))
    for i in range(2):
        f = fbank_ref.fbank(pcm[i], window_type=win, cmn=True)[None]
        with torch.no_grad():
            _, ref = models_ref.forward(arch, torch.from_numpy(f), sd)
        _assert_emb(embs[i], ref[0].numpy())
        if i == 0:
            _assert_emb(e0, ref[0].numpy())
    spk.set_window_type("triangle")
    with pytest.raises(ValueError):
        spk.extract_embedding(paths[0])
