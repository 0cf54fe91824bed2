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
