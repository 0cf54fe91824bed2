"""WAV front door (audio.py) on CPU: every PCM width / float layout the
reference's torchaudio.load accepts, with its normalize=False / True dtypes and
scaling (cli/speaker.py:123-126, dataset/processor.py:96-110), and the shard
reader no longer dropping or garbling non-16-bit members (bin/extract.py)."""
import io
import tarfile

import numpy as np
import pytest

from wespeaker_hubert_amd import audio


def _roundtrip(x, fmt, sr=16000):
    buf = io.BytesIO()
    audio.write_wav_ext(buf, x, sr, fmt)
    return buf.getvalue()


def test_s16_matches_stdlib_writer(tmp_path):
    x = np.random.default_rng(0).integers(-32768, 32767, (2, 1001)).astype(np.int16)
    p = str(tmp_path / "a.wav")
    audio.write_wav(p, x)
    raw, sr = audio.load_wav(p)
    assert sr == 16000 and raw.dtype == np.int16
    np.testing.assert_array_equal(raw, x)
    nrm, _ = audio.load_wav(p, normalize=True)
    np.testing.assert_array_equal(nrm, x.astype(np.float32) / 32768)
    for fmt in ("s16", "ext_s16"):
        got, _ = audio.decode_wav_bytes(_roundtrip(x, fmt))
        np.testing.assert_array_equal(got, x)


def test_u8_s24_s32_and_float_layouts():
    rng = np.random.default_rng(1)
    u8 = rng.integers(0, 256, (1, 333)).astype(np.uint8)
    got, _ = audio.decode_wav_bytes(_roundtrip(u8, "u8"))
    assert got.dtype == np.uint8
    np.testing.assert_array_equal(got, u8)
    np.testing.assert_allclose(audio.decode_wav_bytes(_roundtrip(u8, "u8"), normalize=True)[0],
                               (u8.astype(np.float32) - 128) / 128)
    s24 = rng.integers(-(1 << 23), 1 << 23, (2, 257))
    got, _ = audio.decode_wav_bytes(_roundtrip(s24, "s24"))
    assert got.dtype == np.int32
    np.testing.assert_array_equal(got, (s24 << 8).astype(np.int32))  # left-justified, as torchaudio
    nrm, _ = audio.decode_wav_bytes(_roundtrip(s24, "s24"), normalize=True)
    np.testing.assert_allclose(nrm, s24 / float(1 << 23), rtol=0, atol=1e-7)
    s32 = rng.integers(-(1 << 31), (1 << 31) - 1, (1, 100)).astype(np.int32)
    got, _ = audio.decode_wav_bytes(_roundtrip(s32, "s32"))
    np.testing.assert_array_equal(got, s32)
    f = rng.uniform(-1, 1, (1, 99)).astype(np.float32)
    for fmt in ("f32", "ext_f32", "f64"):
        got, _ = audio.decode_wav_bytes(_roundtrip(f, fmt))
        assert got.dtype == np.float32
        np.testing.assert_array_equal(got, f)


def test_bad_inputs_raise():
    with pytest.raises(ValueError):
        audio.decode_wav_bytes(b"RIFX0000WAVE")
    with pytest.raises(NotImplementedError):
        audio.load_audio(b"ID3\x04....", fmt="mp3", name="x.mp3")


def test_shard_reader_decodes_every_width(tmp_path):
    from wespeaker_hubert_amd.bin.extract import iter_shard
    rng = np.random.default_rng(2)
    s16 = rng.integers(-32768, 32767, (1, 800)).astype(np.int16)
    s24 = rng.integers(-(1 << 23), 1 << 23, (1, 800))
    tar_path = str(tmp_path / "shard.tar")
    with tarfile.open(tar_path, "w") as tar:
        for name, blob in (("u1.wav", _roundtrip(s16, "s16")), ("u2.wav", _roundtrip(s24, "s24"))):
            ti = tarfile.TarInfo(name)
            ti.size = len(blob)
            tar.addfile(ti, io.BytesIO(blob))
        ti = tarfile.TarInfo("u1.spk")
        ti.size = 2
        tar.addfile(ti, io.BytesIO(b"s1"))
    got = {k: (x, sr) for k, x, sr in iter_shard([tar_path])}
    assert set(got) == {"u1", "u2"}
    np.testing.assert_array_equal(got["u1"][0], s16[0].astype(np.float32))  # int16 scale
    np.testing.assert_allclose(got["u2"][0], s24[0] / 256.0, atol=1e-3)
    tar2 = str(tmp_path / "shard2.tar")
    with tarfile.open(tar2, "w") as tar:
        ti = tarfile.TarInfo("u3.mp3")
        ti.size = 4
        tar.addfile(ti, io.BytesIO(b"ID3\x04"))
    with pytest.raises(NotImplementedError):
        list(iter_shard([tar2]))
