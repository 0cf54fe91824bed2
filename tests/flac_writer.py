"""Minimal FLAC *encoder* for tests of the host decoder (native/flac.c).

Written from the published format specification (RFC 9639) to produce streams
that exercise every decoder path: STREAMINFO + skipped metadata, fixed and
variable block sizes (all block-size / sample-rate / sample-size header codes),
UTF-8 frame / sample numbers, independent / left-side / side-right / mid-side
channels, CONSTANT / VERBATIM / FIXED 0..4 / LPC subframes, wasted bits, Rice
residuals with 4- and 5-bit parameters, partition orders and escape partitions,
CRC-8 / CRC-16.  Both CRCs are pinned by their catalogue check values
(tests/test_flac_cpu.py).  No FLAC tool or library exists in this image, so
the decoder's parity with libFLAC / torchaudio is unpinned beyond this.
"""
from __future__ import annotations

import numpy as np


def crc8(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b
        for _ in range(8):
            c = ((c << 1) ^ 0x07) & 0xFF if c & 0x80 else (c << 1) & 0xFF
    return c


def crc16(data: bytes) -> int:
    c = 0
    for b in data:
        c ^= b << 8
        for _ in range(8):
            c = ((c << 1) ^ 0x8005) & 0xFFFF if c & 0x8000 else (c << 1) & 0xFFFF
    return c


class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v: int, k: int):
        for i in range(k - 1, -1, -1):
            self.bits.append((v >> i) & 1)

    def put_signed(self, v: int, k: int):
        self.put(v & ((1 << k) - 1), k)

    def put_unary(self, q: int):
        self.bits.extend([0] * q)
        self.bits.append(1)

    def align(self):
        while len(self.bits) % 8:
            self.bits.append(0)

    def tobytes(self) -> bytes:
        assert len(self.bits) % 8 == 0
        out = bytearray()
        for i in range(0, len(self.bits), 8):
            v = 0
            for b in self.bits[i:i + 8]:
                v = (v << 1) | b
            out.append(v)
        return bytes(out)


def utf8_number(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for n, lead in ((2, 0xC0), (3, 0xE0), (4, 0xF0), (5, 0xF8), (6, 0xFC), (7, 0xFE)):
        if v < (1 << (5 * n + 1 if n < 7 else 36)):
            out = []
            for _ in range(n - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            out.append(lead | v)
            return bytes(reversed(out))
    raise ValueError(v)


def _rice_param(res, pbits):
    m = float(np.mean(np.abs(res))) if len(res) else 0.0
    k = max(0, int(np.floor(np.log2(m + 1))) if m > 0 else 0)
    return min(k, (1 << pbits) - 2)


def encode_residual(w: BitWriter, res: list, bs: int, order: int, method: int, porder: int, escape_parts=()):
    pbits = 5 if method else 4
    w.put(method, 2)
    w.put(porder, 4)
    i = 0
    for p in range(1 << porder):
        cnt = (bs >> porder) - (order if p == 0 else 0)
        part = res[i:i + cnt]
        i += cnt
        if p in escape_parts:
            nb = max(1, max((abs(int(v)) for v in part), default=0).bit_length() + 1)
            w.put((1 << pbits) - 1, pbits)
            w.put(nb, 5)
            for v in part:
                w.put_signed(int(v), nb)
            continue
        k = _rice_param(part, pbits)
        w.put(k, pbits)
        for v in part:
            v = int(v)
            u = (v << 1) if v >= 0 else ((-v) << 1) - 1
            w.put_unary(u >> k)
            w.put(u & ((1 << k) - 1), k)


FIXED_COEF = {0: [], 1: [1], 2: [2, -1], 3: [3, -3, 1], 4: [4, -6, 4, -1]}


def encode_subframe(w: BitWriter, x: np.ndarray, sbps: int, kind: str, order: int = 0, wasted: int = 0,
                    method: int = 0, porder: int = 0, escape_parts=(), lpc_prec: int = 12, lpc_shift: int = 10):
    x = [int(v) for v in x]
    bs = len(x)
    w.put(0, 1)
    type_code = {"constant": 0, "verbatim": 1}.get(kind)
    if kind == "fixed":
        type_code = 8 + order
    elif kind == "lpc":
        type_code = 32 + order - 1
    w.put(type_code, 6)
    if wasted:
        assert all(v % (1 << wasted) == 0 for v in x)
        w.put(1, 1)
        w.put_unary(wasted - 1)
        x = [v >> wasted for v in x]
    else:
        w.put(0, 1)
    sb = sbps - wasted
    if kind == "constant":
        assert len(set(x)) == 1
        w.put_signed(x[0], sb)
    elif kind == "verbatim":
        for v in x:
            w.put_signed(v, sb)
    elif kind == "fixed":
        for v in x[:order]:
            w.put_signed(v, sb)
        c = FIXED_COEF[order]
        res = [x[i] - sum(c[j] * x[i - 1 - j] for j in range(order)) for i in range(order, bs)]
        encode_residual(w, res, bs, order, method, porder, escape_parts)
    elif kind == "lpc":
        for v in x[:order]:
            w.put_signed(v, sb)
        xf = np.asarray(x, np.float64)
        # least-squares predictor, quantised to lpc_prec bits with lpc_shift
        A = np.stack([xf[order - 1 - j:bs - 1 - j] for j in range(order)], 1)
        coef = np.linalg.lstsq(A, xf[order:], rcond=None)[0] if bs > 2 * order else np.zeros(order)
        lim = (1 << (lpc_prec - 1)) - 1
        q = [int(np.clip(np.round(c * (1 << lpc_shift)), -lim - 1, lim)) for c in coef]
        w.put(lpc_prec - 1, 4)
        w.put_signed(lpc_shift, 5)
        for c in q:
            w.put_signed(c, lpc_prec)
        res = [x[i] - (sum(q[j] * x[i - 1 - j] for j in range(order)) >> lpc_shift) for i in range(order, bs)]
        encode_residual(w, res, bs, order, method, porder, escape_parts)
    else:
        raise ValueError(kind)


BS_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12, 8192: 13,
            16384: 14, 32768: 15}
SR_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9, 48000: 10,
            96000: 11}
SS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def encode_flac(x: np.ndarray, sr: int, bps: int, block_sizes, channel_mode: str = "independent",
                subframe=lambda fi, ci, blk: ("fixed", 2), residual=lambda fi, ci: (0, 0, ()),
                wasted=lambda fi, ci: 0, variable: bool = False, header_rate_from_streaminfo: bool = False,
                header_bps_from_streaminfo: bool = False, extra_metadata: bool = True, lpc=(12, 10)) -> bytes:
    """x: int (channels, N).  block_sizes: the frames' sizes (sum = N)."""
    x = np.asarray(x, np.int64)
    ch, n = x.shape
    assert sum(block_sizes) == n
    out = bytearray(b"fLaC")
    si = BitWriter()
    si.put(min(block_sizes) if variable else max(block_sizes[:-1] or block_sizes), 16)
    si.put(max(block_sizes), 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(sr, 20)
    si.put(ch - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    si.put(0, 128)
    body = si.tobytes()
    out += bytes([0x00 if extra_metadata else 0x80]) + len(body).to_bytes(3, "big") + body
    if extra_metadata:
        pad = b"\x00" * 13
        out += bytes([0x80 | 1]) + len(pad).to_bytes(3, "big") + pad  # PADDING, last
    pos = 0
    for fi, bs in enumerate(block_sizes):
        blk = x[:, pos:pos + bs]
        h = BitWriter()
        h.put(0x3FFE, 14)
        h.put(0, 1)
        h.put(1 if variable else 0, 1)
        tail = BitWriter()
        if bs in BS_CODES:
            h.put(BS_CODES[bs], 4)
        elif bs <= 256:
            h.put(6, 4)
            tail.put(bs - 1, 8)
        else:
            h.put(7, 4)
            tail.put(bs - 1, 16)
        if header_rate_from_streaminfo:
            h.put(0, 4)
        elif sr in SR_CODES:
            h.put(SR_CODES[sr], 4)
        elif sr % 1000 == 0 and sr // 1000 < 256:
            h.put(12, 4)
            tail.put(sr // 1000, 8)
        elif sr < 65536:
            h.put(13, 4)
            tail.put(sr, 16)
        else:
            h.put(14, 4)
            tail.put(sr // 10, 16)
        mode_code = {"independent": ch - 1, "left_side": 8, "side_right": 9, "mid_side": 10}[channel_mode]
        h.put(mode_code, 4)
        h.put(0 if header_bps_from_streaminfo else SS_CODES[bps], 3)
        h.put(0, 1)
        hb = h.tobytes() + utf8_number(pos if variable else fi) + tail.tobytes()
        hb += bytes([crc8(hb)])
        if channel_mode == "independent":
            subs = [(blk[c], bps) for c in range(ch)]
        else:
            l, r = blk[0], blk[1]
            side = l - r
            if channel_mode == "left_side":
                subs = [(l, bps), (side, bps + 1)]
            elif channel_mode == "side_right":
                subs = [(side, bps + 1), (r, bps)]
            else:
                subs = [((l + r) >> 1, bps), (side, bps + 1)]
        w = BitWriter()
        for ci, (s, sbps) in enumerate(subs):
            kind, order = subframe(fi, ci, s)
            method, porder, esc = residual(fi, ci)
            encode_subframe(w, s, sbps, kind, order, wasted(fi, ci), method, porder, esc, lpc[0], lpc[1])
        w.align()
        fb = hb + w.tobytes()
        out += fb + crc16(fb).to_bytes(2, "big")
        pos += bs
    return bytes(out)
