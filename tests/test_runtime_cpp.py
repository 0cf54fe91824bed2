"""C++ runtime backend (runtime/: HipSpeakerModel / HipSpeakerEngine, the HIP
sibling of the reference's ONNX / MNN SpeakerModel behind
runtime/core/speaker/speaker_model.h:25-32, and the extract_emb_main /
asv_main CLIs).  CPU: exporter + CLI argument / model-file handling.  GPU: the
engine's chunked, chunk-averaged embeddings vs the oracle chain following
speaker_engine.cc:77-159 (fbank of the whole utterance, 198-frame chunks, tail
topped up from the first chunk, a short utterance repeated, per-chunk CMN)."""
import os
import subprocess

import numpy as np
import pytest
import torch
import yaml

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(REPO, "runtime", "bin")
ARCH = "ECAPA_TDNN_c512"


def _need_bins():
    # make is a no-op when runtime/bin is current (it is built by __graft_entry__.build())
    subprocess.run(["make", "-C", os.path.join(REPO, "runtime")], check=True, capture_output=True)


@pytest.fixture(scope="module")
def exported(tmp_path_factory):
    from wespeaker_hubert_amd import arch as A
    from wespeaker_hubert_amd.bin.export_hip import export
    from wespeaker_hubert_amd.synthetic import synth_state_dict
    d = tmp_path_factory.mktemp("rt")
    sd = synth_state_dict(51, A.param_list(A.make_spec(ARCH, feat_dim=80, embed_dim=192)))
    ckpt = {k: torch.from_numpy(v) for k, v in sd.items()}
    ckpt["projection.weight"] = torch.zeros(3, 192)
    torch.save(ckpt, d / "avg_model.pt")
    with open(d / "config.yaml", "w") as f:
        yaml.safe_dump({"model": ARCH, "model_args": {"feat_dim": 80, "embed_dim": 192}}, f)
    out = export(str(d / "config.yaml"), str(d / "avg_model.pt"), str(d / "model.safetensors"))
    return out, sd, d


def test_export_writes_reference_names_and_metadata(exported):
    from safetensors import safe_open
    path, sd, _ = exported
    with safe_open(path, framework="numpy") as f:
        meta = f.metadata()
        keys = set(f.keys())
        np.testing.assert_array_equal(f.get_tensor("layer1.conv.weight"), sd["layer1.conv.weight"])
    assert meta["arch"] == ARCH and meta["feat_dim"] == "80" and meta["embed_dim"] == "192"
    assert "projection.weight" not in keys and keys <= set(sd)


def test_cli_help_and_bad_model_file(exported, tmp_path):
    _need_bins()
    exe = os.path.join(BIN, "extract_emb_main")
    r = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "speaker_model_path" in r.stdout
    bad = tmp_path / "bad.safetensors"
    bad.write_bytes(b"\x00" * 64)
    wav = tmp_path / "a.wav"
    from wespeaker_hubert_amd.audio import write_wav
    write_wav(str(wav), np.zeros((1, 16000), dtype=np.float32))
    r = subprocess.run([exe, "--speaker_model_path", str(bad), "--wav_path", str(wav)], capture_output=True, text=True)
    assert r.returncode == 2 and "not a safetensors file" in r.stderr
    r = subprocess.run([os.path.join(BIN, "asv_main")], capture_output=True, text=True)
    assert r.returncode == 1 and "enroll_wav" in r.stdout


def _engine_oracle(pcm, sd, samples_per_chunk):
    """speaker_engine.cc:77-159 on the oracle: whole-utterance fbank, chunking, per-chunk CMN, mean."""
    from oracle import fbank_ref, models_ref
    fb = fbank_ref.fbank(pcm, cmn=False).astype(np.float32)
    if samples_per_chunk <= 0:
        chunks = [fb]
    else:
        n = 1 + (samples_per_chunk - 400) // 160
        chunks = [fb[t:t + n] for t in range(0, fb.shape[0] - n + 1, n)]
        tail = fb[len(chunks) * n:]
        if len(tail):
            if not chunks:
                c = np.concatenate([tail] * (n // len(tail)))
                c = np.concatenate([c, c[:n - len(c)]])
            else:
                c = np.concatenate([tail, chunks[0][:n - len(tail)]])
            chunks.append(c)
    x = np.stack([c - c.astype(np.float64).mean(0, keepdims=True) for c in chunks]).astype(np.float32)
    with torch.no_grad():
        _, e = models_ref.forward(ARCH, torch.from_numpy(x), {k: torch.from_numpy(v) for k, v in sd.items()})
    return e.numpy().mean(0)


@pytest.mark.gpu
@pytest.mark.parametrize("spc", [32000, 0])
def test_gpu_extract_emb_main_matches_engine_oracle(exported, spc):
    from wespeaker_hubert_amd.audio import write_wav
    from wespeaker_hubert_amd.synthetic import synth_audio
    _need_bins()
    path, sd, d = exported
    lens = {"short": 9000, "mid": 43210, "long": 80000, "exact": 400 + 395 * 160}
    lines = []
    pcms = {}
    for i, (k, n) in enumerate(lens.items()):
        pcm = synth_audio(700 + i, 1, n)
        write_wav(str(d / f"{k}.wav"), pcm)
        pcms[k] = pcm[0]
        lines.append(f"{k} {d / (k + '.wav')}")
    scp = d / "wav.scp"
    scp.write_text("\n".join(lines) + "\n")
    res = d / f"emb_{spc}.txt"
    r = subprocess.run([os.path.join(BIN, "extract_emb_main"), "--speaker_model_path", path, "--wav_scp", str(scp),
                        "--result", str(res), "--samples_per_chunk", str(spc), "--embedding_size", "192"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    got = {}
    for ln in res.read_text().splitlines():
        parts = ln.split()
        got[parts[0]] = np.array([float(v) for v in parts[1:]], dtype=np.float64)
    assert set(got) == set(lens)
    for k, pcm in pcms.items():
        ref = _engine_oracle(pcm, sd, spc).astype(np.float64)
        e = got[k]
        cos = float(e @ ref / np.linalg.norm(e) / np.linalg.norm(ref))
        assert cos >= 0.9999, (k, cos)
        assert np.abs(e - ref).max() < 1e-4, k  # waveform -> embedding, north-star per-dim bar
    # asv_main: (cos + 1) / 2 of the two engine embeddings
    r = subprocess.run([os.path.join(BIN, "asv_main"), "--speaker_model_path", path, "--enroll_wav",
                        str(d / "mid.wav"), "--test_wav", str(d / "long.wav"), "--SamplesPerChunk", str(spc)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    score = float(r.stdout.split("Cosine score:")[1].split()[0])
    a, b = got["mid"], got["long"]
    assert abs(score - (a @ b / np.linalg.norm(a) / np.linalg.norm(b) + 1) / 2) < 1e-5


@pytest.mark.gpu
def test_gpu_engine_8k_64bin(tmp_path):
    """FeaturePipelineConfig(num_bins, sample_rate) beyond 80 / 16 kHz (feature_pipeline.h:35-39:
    25 / 10 ms frames at the given rate): --fbank_dim 64 --sample_rate 8000 with a 64-dim model,
    chunked like speaker_engine.cc, against the oracle chain at 8 kHz."""
    from oracle import fbank_ref, models_ref
    from wespeaker_hubert_amd import arch as A
    from wespeaker_hubert_amd.audio import write_wav
    from wespeaker_hubert_amd.bin.export_hip import export
    from wespeaker_hubert_amd.synthetic import synth_audio, synth_state_dict
    _need_bins()
    sd = synth_state_dict(52, A.param_list(A.make_spec(ARCH, feat_dim=64, embed_dim=192)))
    torch.save({k: torch.from_numpy(v) for k, v in sd.items()}, tmp_path / "avg_model.pt")
    with open(tmp_path / "config.yaml", "w") as f:
        yaml.safe_dump({"model": ARCH, "model_args": {"feat_dim": 64, "embed_dim": 192}}, f)
    path = export(str(tmp_path / "config.yaml"), str(tmp_path / "avg_model.pt"), str(tmp_path / "m.safetensors"))
    pcm = synth_audio(711, 1, 21000)
    write_wav(str(tmp_path / "a.wav"), pcm, sample_rate=8000)
    (tmp_path / "wav.scp").write_text(f"a {tmp_path / 'a.wav'}\n")
    spc = 16000
    r = subprocess.run([os.path.join(BIN, "extract_emb_main"), "--speaker_model_path", path, "--wav_scp",
                        str(tmp_path / "wav.scp"), "--result", str(tmp_path / "e.txt"), "--samples_per_chunk",
                        str(spc), "--fbank_dim", "64", "--sample_rate", "8000"], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    e = np.array([float(v) for v in (tmp_path / "e.txt").read_text().split()[1:]], dtype=np.float64)
    fb = fbank_ref.fbank(pcm[0], 64, sample_freq=8000.0).astype(np.float32)
    n = 1 + (spc - 200) // 80
    chunks = [fb[t:t + n] for t in range(0, fb.shape[0] - n + 1, n)]
    tail = fb[len(chunks) * n:]
    if len(tail):
        chunks.append(np.concatenate([tail, chunks[0][:n - len(tail)]]))
    x = np.stack([c - c.astype(np.float64).mean(0, keepdims=True) for c in chunks]).astype(np.float32)
    with torch.no_grad():
        _, ref = models_ref.forward(ARCH, torch.from_numpy(x), {k: torch.from_numpy(v) for k, v in sd.items()})
    ref = ref.numpy().mean(0).astype(np.float64)
    assert float(e @ ref / np.linalg.norm(e) / np.linalg.norm(ref)) >= 0.9999
    assert np.abs(e - ref).max() < 1e-4
