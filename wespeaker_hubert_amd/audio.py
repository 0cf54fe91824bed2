"""Audio decoding for the extraction front door (torchaudio is not a dependency).

Mirrors what the reference gets from torchaudio:

* `torchaudio.load(path, normalize=False)` (cli/speaker.py:123-126): the raw
  integer sample values, shape (channels, N) — int16 for 16-bit PCM, uint8 for
  8-bit, int32 for 32-bit and for 24-bit (left-justified, i.e. the 24-bit value
  << 8, as torchaudio's sox / ffmpeg backends return s24 as s32); IEEE-float
  files are float32 either way.
* `torchaudio.load(path)` (normalize=True, dataset/processor.py:96-110): float32
  in [-1, 1]: int16 / 2^15, int32 (and left-justified 24-bit) / 2^31,
  (uint8 - 128) / 2^7.

Formats: RIFF/WAVE with WAVE_FORMAT_PCM (8/16/24/32-bit), WAVE_FORMAT_IEEE_FLOAT
(32/64-bit) and WAVE_FORMAT_EXTENSIBLE carrying either; FLAC via
`flac.decode_flac` (host C decoder, wespeaker_hubert_amd/native/flac.c).
Other containers (mp3, m4a, ogg, opus, wma) raise NotImplementedError.
Resampling lives in resample.py (device kernel).
"""
from __future__ import annotations

import struct
from typing import BinaryIO, Tuple, Union

import numpy as np

WAVE_FORMAT_PCM = 0x0001
WAVE_FORMAT_IEEE_FLOAT = 0x0003
WAVE_FORMAT_EXTENSIBLE = 0xFFFE

Source = Union[str, bytes, BinaryIO]


def _read_all(src: Source) -> bytes:
    if isinstance(src, (bytes, bytearray, memoryview)):
        return bytes(src)
    if isinstance(src, str):
        with open(src, "rb") as f:
            return f.read()
    return src.read()


def _normalize(x: np.ndarray) -> np.ndarray:
    if x.dtype == np.int16:
        return x.astype(np.float32) / np.float32(1 << 15)
    if x.dtype == np.int32:
        return (x.astype(np.float64) / float(1 << 31)).astype(np.float32)
    if x.dtype == np.uint8:
        return (x.astype(np.float32) - np.float32(128)) / np.float32(128)
    return x.astype(np.float32)


def decode_wav_bytes(data: bytes, name: str = "<wav>", normalize: bool = False) -> Tuple[np.ndarray, int]:
    """RIFF/WAVE bytes -> ((channels, N) array, sample_rate); see module doc for dtypes."""
    if len(data) < 12 or data[:4] != b"RIFF" or data[8:12] != b"WAVE":
        raise ValueError(f"{name}: not a RIFF/WAVE file")
    pos, fmt, payload = 12, None, None
    while pos + 8 <= len(data):
        cid, size = data[pos:pos + 4], struct.unpack_from("<I", data, pos + 4)[0]
        body = data[pos + 8:pos + 8 + size]
        if cid == b"fmt ":
            fmt = body
        elif cid == b"data":
            payload = body
            break
        pos += 8 + size + (size & 1)
    if fmt is None or payload is None:
        raise ValueError(f"{name}: missing fmt or data chunk")
    tag, ch, sr, _, align, bits = struct.unpack_from("<HHIIHH", fmt, 0)
    if tag == WAVE_FORMAT_EXTENSIBLE:
        if len(fmt) < 40:
            raise ValueError(f"{name}: short WAVE_FORMAT_EXTENSIBLE header")
        tag = struct.unpack_from("<H", fmt, 24)[0]  # first two bytes of the sub-format GUID
    if ch < 1 or align < ch:
        raise ValueError(f"{name}: bad channel layout")
    width = align // ch
    n = len(payload) // align
    raw = np.frombuffer(payload[:n * align], dtype=np.uint8).reshape(n, ch, width)
    if tag == WAVE_FORMAT_PCM:
        if width == 1:
            x = raw[:, :, 0].copy()
        elif width == 2:
            x = raw.copy().view("<i2")[:, :, 0]
        elif width == 3:  # left-justified into int32 (value << 8)
            b = raw.astype(np.int32)
            x = ((b[:, :, 0] << 8) | (b[:, :, 1] << 16) | (b[:, :, 2] << 24)).astype(np.int32)
        elif width == 4:
            x = raw.copy().view("<i4")[:, :, 0]
        else:
            raise NotImplementedError(f"{name}: {8 * width}-bit PCM is not supported")
        if bits > 8 * width:
            raise ValueError(f"{name}: {bits} valid bits in {8 * width}-bit containers")
    elif tag == WAVE_FORMAT_IEEE_FLOAT:
        if width == 4:
            x = raw.copy().view("<f4")[:, :, 0]
        elif width == 8:
            x = raw.copy().view("<f8")[:, :, 0].astype(np.float32)
        else:
            raise NotImplementedError(f"{name}: {8 * width}-bit float WAV is not supported")
    else:
        raise NotImplementedError(f"{name}: WAVE format tag 0x{tag:04x} is not supported")
    x = np.ascontiguousarray(x.T)
    return (_normalize(x) if normalize else x), int(sr)


def load_audio(src: Source, fmt: str = "", normalize: bool = False, name: str = "") -> Tuple[np.ndarray, int]:
    """Decode a WAV or FLAC file / bytes / stream: ((channels, N), sample_rate)."""
    data = _read_all(src)
    name = name or (src if isinstance(src, str) else "<audio>")
    ext = (fmt or (name.rpartition(".")[2] if "." in name else "")).lower()
    if data[:4] == b"fLaC" or ext == "flac":
        from .flac import decode_flac
        x, sr, bits = decode_flac(data, name=name)
        if normalize:
            return (x.astype(np.float64) / float(1 << (bits - 1))).astype(np.float32), sr
        return _flac_raw(x, bits), sr
    if data[:4] == b"RIFF" or ext in ("", "wav", "wave"):
        return decode_wav_bytes(data, name, normalize)
    raise NotImplementedError(f"{name}: audio format {ext!r} is not supported (wav and flac are)")


def _flac_raw(x: np.ndarray, bits: int) -> np.ndarray:
    """torchaudio.load(normalize=False) dtypes for FLAC: 16-bit -> int16, 8-bit ->
    uint8 (offset binary), otherwise int32 left-justified to 32 bits."""
    if bits == 16:
        return x.astype(np.int16)
    if bits == 8:
        return (x + 128).astype(np.uint8)
    return (x.astype(np.int64) << (32 - bits)).astype(np.int32)


def load_wav(path: str, normalize: bool = False) -> Tuple[np.ndarray, int]:
    """`torchaudio.load(path, normalize=normalize)` for WAV and FLAC files."""
    return load_audio(path, normalize=normalize, name=path)


def write_wav(path: str, pcm: np.ndarray, sample_rate: int = 16000) -> None:
    """16-bit PCM WAV writer (test fixtures / tools)."""
    import wave
    pcm = np.asarray(pcm)
    if pcm.ndim == 1:
        pcm = pcm[None, :]
    data = np.clip(np.round(pcm), -32768, 32767).astype("<i2").T.tobytes()
    with wave.open(path, "wb") as w:
        w.setnchannels(pcm.shape[0])
        w.setsampwidth(2)
        w.setframerate(sample_rate)
        w.writeframes(data)


def write_wav_ext(path_or_buf, x: np.ndarray, sample_rate: int, fmt: str) -> None:
    """WAV writer for the other layouts (tests): fmt in {'u8', 's16', 's24', 's32', 'f32', 'f64',
    'ext_s16', 'ext_f32'}; x is (channels, N) in the container's raw scale."""
    x = np.asarray(x)
    if x.ndim == 1:
        x = x[None]
    ch, n = x.shape
    ext = fmt.startswith("ext_")
    base = fmt[4:] if ext else fmt
    width = {"u8": 1, "s16": 2, "s24": 3, "s32": 4, "f32": 4, "f64": 8}[base]
    tag = WAVE_FORMAT_IEEE_FLOAT if base[0] == "f" else WAVE_FORMAT_PCM
    inter = x.T
    if base == "u8":
        body = inter.astype(np.uint8).tobytes()
    elif base == "s16":
        body = inter.astype("<i2").tobytes()
    elif base == "s24":
        v = inter.astype(np.int64) & 0xFFFFFF
        body = np.stack([(v & 255), (v >> 8) & 255, (v >> 16) & 255], axis=-1).astype(np.uint8).tobytes()
    elif base == "s32":
        body = inter.astype("<i4").tobytes()
    elif base == "f32":
        body = inter.astype("<f4").tobytes()
    else:
        body = inter.astype("<f8").tobytes()
    if ext:
        guid_tail = b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        fmt_chunk = struct.pack("<HHIIHHHHI", WAVE_FORMAT_EXTENSIBLE, ch, sample_rate, sample_rate * ch * width,
                                ch * width, 8 * width, 22, 8 * width, 0) + struct.pack("<H", tag) + guid_tail
    else:
        fmt_chunk = struct.pack("<HHIIHH", tag, ch, sample_rate, sample_rate * ch * width, ch * width, 8 * width)
    riff = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt_chunk)) + fmt_chunk
    riff += b"data" + struct.pack("<I", len(body)) + body + (b"\x00" if len(body) & 1 else b"")
    out = b"RIFF" + struct.pack("<I", len(riff)) + riff
    if isinstance(path_or_buf, str):
        with open(path_or_buf, "wb") as f:
            f.write(out)
    else:
        path_or_buf.write(out)


__all__ = ["load_wav", "load_audio", "decode_wav_bytes", "write_wav", "write_wav_ext"]
