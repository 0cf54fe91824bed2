"""Host FLAC decoder (wespeaker_hubert_amd/native/flac.c) against streams from
tests/flac_writer.py covering every header code, channel mode, subframe type,
residual method / partitioning / escape, wasted bits, variable block size and
multi-byte frame numbers; CRCs pinned by their catalogue check values.  The
decoder's parity with libFLAC / torchaudio is unpinned (neither exists here)."""
import io
import tarfile

import numpy as np
import pytest

from flac_writer import crc8, crc16, encode_flac
from wespeaker_hubert_amd import audio
from wespeaker_hubert_amd.flac import decode_flac


def test_crc_catalogue_check_values():
    assert crc8(b"123456789") == 0xF4      # CRC-8 (poly 0x07, init 0): FLAC frame header
    assert crc16(b"123456789") == 0xFEE8   # CRC-16/BUYPASS (poly 0x8005, init 0): FLAC frame


def _signal(ch, n, bps, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    amp = (1 << (bps - 1)) * 0.6
    x = np.stack([amp * np.sin(2 * np.pi * (0.01 + 0.003 * c) * t) + rng.normal(0, amp * 0.02, n) for c in range(ch)])
    return np.clip(np.round(x), -(1 << (bps - 1)), (1 << (bps - 1)) - 1).astype(np.int64)


CASES = [
    # (channels, bps, sr, block sizes, channel mode, subframe kind, order, residual method, partition order)
    (1, 16, 16000, [4096, 4096, 1000], "independent", "fixed", 2, 0, 0),
    (1, 16, 16000, [192, 576, 1152, 2304, 256, 77], "independent", "fixed", 0, 1, 2),
    (1, 8, 8000, [1024, 300], "independent", "fixed", 1, 0, 1),
    (1, 24, 48000, [2048, 2048], "independent", "lpc", 8, 1, 3),
    (1, 16, 22050, [4608, 1000], "independent", "fixed", 3, 0, 0),
    (2, 16, 44100, [4096, 4096], "left_side", "fixed", 4, 0, 2),
    (2, 16, 44100, [4096, 512], "side_right", "lpc", 4, 0, 1),
    (2, 24, 96000, [1024, 1024], "mid_side", "lpc", 12, 1, 0),
    (2, 16, 12345, [2048, 100], "independent", "verbatim", 0, 0, 0),
    (1, 16, 11000, [1000, 1000], "independent", "lpc", 1, 0, 0),
    (1, 12, 16000, [512, 512], "independent", "fixed", 2, 0, 0),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}ch{c[1]}b{c[2]}_{c[4]}_{c[5]}{c[6]}" for c in CASES])
def test_roundtrip(case):
    ch, bps, sr, bsz, mode, kind, order, method, porder = case
    x = _signal(ch, sum(bsz), bps, 3)
    data = encode_flac(x, sr, bps, bsz, mode, subframe=lambda fi, ci, b: (kind, order),
                       residual=lambda fi, ci: (method, porder if min(bsz) % (1 << porder) == 0 and
                                                (min(bsz) >> porder) >= order else 0, ()))
    y, rate, bits = decode_flac(data)
    assert (rate, bits) == (sr, bps)
    np.testing.assert_array_equal(y, x)


def test_constant_wasted_bits_escape_and_streaminfo_codes():
    n = 3000
    x = _signal(2, n, 16, 5)
    x[0, :1000] = 1234                  # CONSTANT frame on channel 0
    x[1] = (x[1] >> 3) << 3             # 3 wasted bits on channel 1

    def sub(fi, ci, b):
        return ("constant", 0) if (fi == 0 and ci == 0) else ("fixed", 2)
    data = encode_flac(x, 16000, 16, [1000, 1000, 1000], "independent", subframe=sub,
                       residual=lambda fi, ci: (0, 2, (1,) if fi == 1 else ()),
                       wasted=lambda fi, ci: 3 if ci == 1 else 0,
                       header_rate_from_streaminfo=True, header_bps_from_streaminfo=True)
    y, rate, bits = decode_flac(data)
    assert (rate, bits) == (16000, 16)
    np.testing.assert_array_equal(y, x)


def test_variable_blocksize_and_long_frame_numbers():
    sizes = [16] * 200 + [64, 1000, 7]   # > 127 frames: multi-byte UTF-8 numbers
    x = _signal(1, sum(sizes), 16, 7)
    for variable in (False, True):
        if not variable:
            sizes_f = [16] * 300             # fixed-size stream: frame numbers 128..299 are 2-byte
            xf = _signal(1, sum(sizes_f), 16, 8)
            y, _, _ = decode_flac(encode_flac(xf, 16000, 16, sizes_f, subframe=lambda *a: ("fixed", 1)))
            np.testing.assert_array_equal(y, xf)
        else:
            y, _, _ = decode_flac(encode_flac(x, 16000, 16, sizes, variable=True, subframe=lambda *a: ("fixed", 1)))
            np.testing.assert_array_equal(y, x)


def test_corruption_is_detected():
    x = _signal(1, 4096, 16, 9)
    data = bytearray(encode_flac(x, 16000, 16, [4096]))
    bad = bytearray(data)
    bad[-40] ^= 0x10
    with pytest.raises(ValueError, match="CRC|truncated|reserved"):
        decode_flac(bytes(bad))
    with pytest.raises(ValueError, match="fLaC"):
        decode_flac(b"RIFF" + bytes(data[4:]))
    with pytest.raises(ValueError):
        decode_flac(bytes(data[:-10]))



def test_id3_tags_around_the_stream_are_skipped():
    """A leading ID3v2 tag (syncsafe size, with and without its footer flag) and a
    trailing ID3v1 'TAG' block, which common decoders tolerate, decode to the
    untagged stream's samples."""
    x = _signal(1, 3000, 16, 11)
    data = encode_flac(x, 16000, 16, [1000, 1000, 1000])
    body = b"TIT2" + (5).to_bytes(4, "big") + b"\x00\x00" + b"\x00test"   # one text frame
    body += bytes(300)                                                   # padding
    sz = len(body)
    syncsafe = bytes([(sz >> 21) & 0x7F, (sz >> 14) & 0x7F, (sz >> 7) & 0x7F, sz & 0x7F])
    v1 = b"TAG" + bytes(125)
    for flags, footer in ((0x00, b""), (0x10, b"3DI\x04\x00\x10" + syncsafe)):
        tagged = b"ID3\x04\x00" + bytes([flags]) + syncsafe + body + footer + data + v1
        y, rate, bits = decode_flac(tagged)
        assert (rate, bits) == (16000, 16)
        np.testing.assert_array_equal(y, x)
    # padding after the last frame ends the stream once STREAMINFO's count is decoded
    y, _, _ = decode_flac(data + bytes(64))
    np.testing.assert_array_equal(y, x)


def test_load_audio_flac_matches_torchaudio_conventions():
    x16 = _signal(1, 2000, 16, 11)
    d16 = encode_flac(x16, 16000, 16, [2000])
    raw, sr = audio.load_audio(d16, fmt="flac")
    assert raw.dtype == np.int16 and sr == 16000
    np.testing.assert_array_equal(raw, x16)
    norm, _ = audio.load_audio(d16, fmt="flac", normalize=True)
    np.testing.assert_array_equal(norm, (x16 / 32768.0).astype(np.float32))
    x24 = _signal(1, 500, 24, 12)
    raw24, _ = audio.load_audio(encode_flac(x24, 16000, 24, [500]), fmt="flac")
    assert raw24.dtype == np.int32
    np.testing.assert_array_equal(raw24, x24 << 8)   # left-justified, as for 24-bit WAV


def test_shard_with_flac_member_decodes():
    from wespeaker_hubert_amd.bin.extract import iter_shard
    x = _signal(1, 1600, 16, 13)
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tar:
        for name, data in (("utt1.flac", encode_flac(x, 16000, 16, [1600])), ("utt1.spk", b"spk1")):
            ti = tarfile.TarInfo(name)
            ti.size = len(data)
            tar.addfile(ti, io.BytesIO(data))
    import tempfile, os
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "shard.tar")
        open(p, "wb").write(buf.getvalue())
        items = list(iter_shard([p]))
    assert len(items) == 1 and items[0][0] == "utt1" and items[0][2] == 16000
    np.testing.assert_array_equal(items[0][1], (x[0] / 32768.0).astype(np.float32) * np.float32(32768))
