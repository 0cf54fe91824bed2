"""Kaldi ark/scp embedding I/O without kaldiio (not installed here).

Byte format written by the reference through kaldiio 2.17
(`kaldiio.WriteHelper('ark,scp:X.ark,X.scp')`, used at cli/speaker.py:362-367
and bin/extract.py:90-120) for a 1-D float32 vector:

    <key> SP  '\\0B'  'FV '  '\\x04' <int32 LE dim>  <dim x float32 LE>

and one scp line per record `<key> <ark path>:<byte offset of '\\0B'>`, so
the files are readable by `kaldiio.load_scp_sequential` (bin/score.py:29).
Byte-exact parity with kaldiio is *unpinned* (kaldiio is absent); the format
is fixed by tests/test_kaldi_io.py.
"""
from __future__ import annotations

import os
import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np


class WriteHelper:
    """Subset of kaldiio.WriteHelper: 'ark,scp:<ark>,<scp>' or 'ark:<ark>'."""

    def __init__(self, wspecifier: str):
        kind, _, paths = wspecifier.partition(":")
        kinds = kind.split(",")
        files = paths.split(",")
        if kinds[0] != "ark":
            raise ValueError(f"unsupported wspecifier {wspecifier}")
        self.ark_path = files[0]
        self.scp_path = files[1] if len(kinds) > 1 and kinds[1] == "scp" else None
        self._ark = open(self.ark_path, "wb")
        self._scp = open(self.scp_path, "w", encoding="utf-8") if self.scp_path else None

    def __call__(self, key: str, array) -> None:
        arr = np.asarray(array)
        if arr.ndim != 1:
            raise ValueError("only 1-D embeddings are written")
        if arr.dtype == np.float32:
            tag = b"FV "
        elif arr.dtype == np.float64:
            tag = b"DV "
        else:
            arr = arr.astype(np.float32)
            tag = b"FV "
        self._ark.write(key.encode("utf-8") + b" ")
        offset = self._ark.tell()
        self._ark.write(b"\0B" + tag + b"\x04" + struct.pack("<i", arr.shape[0]))
        self._ark.write(arr.astype(arr.dtype.newbyteorder("<")).tobytes())
        if self._scp is not None:
            self._scp.write(f"{key} {self.ark_path}:{offset}\n")

    def close(self):
        self._ark.close()
        if self._scp is not None:
            self._scp.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _read_vector(f) -> np.ndarray:
    if f.read(2) != b"\0B":
        raise ValueError("not a binary kaldi record")
    tag = f.read(3)
    dtype = {b"FV ": "<f4", b"DV ": "<f8"}.get(tag)
    if dtype is None:
        raise ValueError(f"unsupported kaldi type {tag!r}")
    if f.read(1) != b"\x04":
        raise ValueError("bad size marker")
    (n,) = struct.unpack("<i", f.read(4))
    return np.frombuffer(f.read(n * np.dtype(dtype).itemsize), dtype=dtype).astype(dtype[1:])


# --------------------------------------------------------------- matrices --
# kaldiio.load_mat as the `feat` data type calls it (processor.parse_feat,
# wespeaker/dataset/processor.py:171-196): "<ark path>:<byte offset>" (plus
# kaldiio's optional "[r0:r1]" / "[r0:r1,c0:c1]" slice), or a path alone for the
# first object in the file.  Kaldi's published binary layouts
# (src/matrix/kaldi-matrix.cc Matrix::Read, src/matrix/compressed-matrix.{h,cc}):
#   "\0B" "FM " | "DM "  '\x04' int32 rows  '\x04' int32 cols  rows*cols f32 | f64
#   "\0B" "CM " | "CM2 " | "CM3 "  GlobalHeader {f32 min, f32 range, i32 rows, i32 cols}
#       CM  (kOneByteWithColHeaders): cols x PerColHeader {u16 p0, p25, p75, p100},
#           then rows bytes per column (column-major)
#       CM2 (kTwoByte): rows*cols u16 row-major; CM3 (kOneByte): rows*cols u8 row-major
# and the text form "[ v v v\n v v v ]".  Decoding follows CompressedMatrix::CopyToMat
# in its float arithmetic.  Byte-exact parity with kaldiio is *unpinned* (kaldiio is
# absent); tests/test_kaldi_io.py fixes the layouts from hand-written bytes.

_U16_SCALE = np.float32(1.52590218966964e-05)  # compressed-matrix.cc Uint16ToFloat: 1/65535 as a float literal


def _read_int32(f) -> int:
    if f.read(1) != b"\x04":
        raise ValueError("bad int32 size marker")
    return struct.unpack("<i", f.read(4))[0]


def _char_to_float(p0, p25, p75, p100, v: np.ndarray) -> np.ndarray:
    """CompressedMatrix::CharToFloat: float products times a double reciprocal, rounded to float."""
    v32 = v.astype(np.float32)
    lo = (p0 + ((p25 - p0) * v32).astype(np.float64) * (1 / 64.0))
    mid = (p25 + ((p75 - p25) * (v32 - np.float32(64))).astype(np.float64) * (1 / 128.0))
    hi = (p75 + ((p100 - p75) * (v32 - np.float32(192))).astype(np.float64) * (1 / 63.0))
    return np.where(v <= 64, lo, np.where(v <= 192, mid, hi)).astype(np.float32)


def _read_compressed(f, fmt: bytes) -> np.ndarray:
    mn, rng, rows, cols = struct.unpack("<ffii", f.read(16))
    mn, rng = np.float32(mn), np.float32(rng)
    if rows < 0 or cols < 0:
        raise ValueError("bad compressed matrix header")
    if fmt == b"CM":
        hdr = np.frombuffer(f.read(8 * cols), dtype="<u2").reshape(cols, 4).astype(np.float32)
        pct = (mn + rng * _U16_SCALE * hdr).astype(np.float32)  # Uint16ToFloat per percentile
        data = np.frombuffer(f.read(rows * cols), dtype=np.uint8).reshape(cols, rows)
        out = np.empty((rows, cols), dtype=np.float32)
        for c in range(cols):
            out[:, c] = _char_to_float(pct[c, 0], pct[c, 1], pct[c, 2], pct[c, 3], data[c])
        return out
    if fmt == b"CM2":
        data = np.frombuffer(f.read(2 * rows * cols), dtype="<u2").reshape(rows, cols)
        inc = np.float64(rng) * (1.0 / 65535.0)  # CopyToMat: increment = range * (1.0 / 65535.0)
    elif fmt == b"CM3":
        data = np.frombuffer(f.read(rows * cols), dtype=np.uint8).reshape(rows, cols)
        inc = np.float64(rng) * (1.0 / 255.0)
    else:
        raise ValueError(f"unsupported compressed matrix type {fmt!r}")
    inc = np.float32(inc)
    return (mn + data.astype(np.float32) * inc).astype(np.float32)


def _read_text_matrix(f, first: bytes) -> np.ndarray:
    buf = first
    while b"]" not in buf:
        c = f.read(4096)
        if not c:
            raise ValueError("unterminated text matrix")
        buf += c
    body = buf[buf.index(b"[") + 1:buf.index(b"]")].decode("ascii")
    rows = [ln.split() for ln in body.strip().splitlines() if ln.strip()]
    if not rows:
        return np.zeros((0, 0), dtype=np.float32)
    return np.asarray([[float(v) for v in r] for r in rows], dtype=np.float32)


def read_matrix(f) -> np.ndarray:
    """One Kaldi matrix at the file position (binary FM / DM / CM / CM2 / CM3, or text)."""
    head = f.read(2)
    if head != b"\0B":
        return _read_text_matrix(f, head)
    tok = b""
    while True:
        c = f.read(1)
        if not c:
            raise ValueError("truncated kaldi token")
        if c == b" ":
            break
        tok += c
    if tok in (b"FM", b"DM"):
        rows, cols = _read_int32(f), _read_int32(f)
        dt = "<f4" if tok == b"FM" else "<f8"
        n = rows * cols
        arr = np.frombuffer(f.read(n * np.dtype(dt).itemsize), dtype=dt)
        if arr.size != n:
            raise ValueError("truncated kaldi matrix")
        return arr.reshape(rows, cols).astype(dt[1:])
    if tok in (b"CM", b"CM2", b"CM3"):
        return _read_compressed(f, tok)
    raise ValueError(f"unsupported kaldi matrix type {tok!r}")


def _parse_slice(spec: str):
    """kaldiio's trailing "[r0:r1]" / "[r0:r1,c0:c1]" range."""
    if not spec.endswith("]") or "[" not in spec:
        return spec, None
    base, _, rng = spec[:-1].rpartition("[")
    parts = []
    for p in rng.split(","):
        a, _, b = p.partition(":")
        parts.append(slice(int(a) if a else None, int(b) if b else None))
    return base, tuple(parts)


def load_mat(spec: str) -> np.ndarray:
    """kaldiio.load_mat for "<path>:<offset>[slice]" and "<path>" (first object)."""
    spec, sl = _parse_slice(spec.strip())
    path, off = spec, 0
    head, sep, tail = spec.rpartition(":")
    if sep and tail.isdigit() and head:
        path, off = head, int(tail)
    with open(path, "rb") as f:
        f.seek(off)
        if off == 0:  # an ark file from its start: "<key> " precedes the object
            peek = f.read(2)
            f.seek(0)
            if peek not in (b"\0B",) and not peek.startswith(b"["):
                while f.read(1) not in (b" ", b""):
                    pass
        mat = read_matrix(f)
    return mat[sl] if sl is not None else mat


def load_ark(path: str) -> Iterator[Tuple[str, np.ndarray]]:
    with open(path, "rb") as f:
        while True:
            key = b""
            c = f.read(1)
            if not c:
                return
            while c != b" ":
                key += c
                c = f.read(1)
            yield key.decode("utf-8"), _read_vector(f)


def load_scp_sequential(scp_path: str) -> Iterator[Tuple[str, np.ndarray]]:
    """kaldiio.load_scp_sequential analogue for `key path:offset` lines."""
    handles: Dict[str, object] = {}
    try:
        with open(scp_path, "r", encoding="utf-8") as fin:
            for line in fin:
                if not line.strip():
                    continue
                key, loc = line.strip().split(None, 1)
                path, _, off = loc.rpartition(":")
                f = handles.get(path)
                if f is None:
                    f = handles[path] = open(path, "rb")
                f.seek(int(off))
                yield key, _read_vector(f)
    finally:
        for f in handles.values():
            f.close()


def load_scp_matrix(scp_path: str) -> Tuple[List[str], np.ndarray]:
    """All records of an embedding scp as one (keys, [n][D] array) pair, in scp order.

    The ark bytes are read once per file and the records gathered with numpy (each
    record's '\\0B' + 'FV '/'DV ' + size-4 + dim header checked vectorised); a list of
    vectors of different dims or types falls back to load_scp_sequential.  Same values
    as load_scp_sequential (the scoring stages of the C5 pipeline read 10k-20k
    records per stage: ~8x faster than the per-record reader)."""
    with open(scp_path, "r", encoding="utf-8") as fin:
        recs = [ln.split(None, 1) for ln in fin]
    recs = [r for r in recs if len(r) == 2]
    keys: List[str] = [r[0] for r in recs]
    locs = [r[1].strip().rpartition(":") for r in recs]
    if not keys:
        return keys, np.zeros((0, 0), np.float32)
    off = np.fromiter((int(lc[2]) for lc in locs), np.int64, len(locs))
    uniq: Dict[str, int] = {}
    pidx = np.fromiter((uniq.setdefault(lc[0], len(uniq)) for lc in locs), np.int64, len(locs))
    bufs = [np.fromfile(pth, dtype=np.uint8) for pth in uniq]
    head = np.empty((len(keys), 10), np.uint8)
    for j, buf in enumerate(bufs):
        sel = pidx == j
        if np.any(off[sel] + 10 > buf.size):
            raise ValueError(f"truncated ark {list(uniq)[j]}")
        head[sel] = buf[off[sel, None] + np.arange(10)]
    tags = {b"FV ": "<f4", b"DV ": "<f8"}
    t0 = bytes(head[0, 2:5])
    dims = head[:, 6:10].copy().view("<i4").reshape(-1)
    uniform = (np.all(head[:, 0] == 0) and np.all(head[:, 1] == ord("B")) and t0 in tags
               and np.all(head[:, 2:5] == np.frombuffer(t0, np.uint8)) and np.all(head[:, 5] == 4)
               and np.all(dims == dims[0]))
    if not uniform:
        recs = dict(load_scp_sequential(scp_path))
        return keys, np.stack([recs[k] for k in keys])
    dt = np.dtype(tags[t0])
    nb = int(dims[0]) * dt.itemsize
    raw = np.empty((len(keys), nb), np.uint8)
    for j, buf in enumerate(bufs):
        sel = np.flatnonzero(pidx == j)
        o = off[sel] + 10
        if np.any(o + nb > buf.size):
            raise ValueError(f"truncated ark {list(uniq)[j]}")
        step = np.diff(o)
        if len(o) > 1 and np.all(step == step[0]) and step[0] >= nb:
            # records at a fixed stride (WriteHelper's key + header + data, equal-length keys):
            # one strided view instead of a gather
            raw[sel] = np.lib.stride_tricks.as_strided(buf[o[0]:], shape=(len(o), nb), strides=(int(step[0]), 1))
        else:
            mv = memoryview(buf)
            rows = raw[sel]
            for i, oo in enumerate(o.tolist()):
                rows[i] = mv[oo:oo + nb]
            raw[sel] = rows
    out = raw.view(dt)
    if not dt.isnative:
        out = out.astype(dt.newbyteorder("="))
    return keys, out.reshape(len(keys), int(dims[0]))


def read_scp(scp_file: str) -> List[Tuple[str, str]]:
    """utils/file_utils.py read_scp."""
    out = []
    with open(scp_file, "r", encoding="utf8") as fin:
        for line in fin:
            tokens = line.strip().split()
            if tokens:
                out.append((tokens[0], " ".join(tokens[1:])))
    return out


def read_table(table_file: str) -> List[List[str]]:
    """utils/file_utils.py read_table."""
    with open(table_file, "r", encoding="utf8") as fin:
        return [line.strip().split() for line in fin]


def validate_path(path: str) -> None:
    """utils/utils.py validate_path."""
    d = os.path.dirname(path)
    if d and not os.path.exists(d):
        os.makedirs(d, exist_ok=True)
