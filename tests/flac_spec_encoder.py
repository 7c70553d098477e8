"""A FLAC encoder written from the format specification (RFC 9639), test infrastructure only.

It exists to check libsuta_audio's decoder (include/suta_audio.h) bit-exactly: every coding tool a
decoder must handle is selectable per frame and per subframe, so the tests can walk all of them:
CONSTANT / VERBATIM / FIXED (orders 0-4) / LPC (orders 1-32) subframes, wasted bits, Rice (4-bit) and
Rice2 (5-bit) parameters, escaped partitions (raw k-bit residuals, k = 0 included), partition orders
0-8, the four channel assignments (independent, left/side, side/right, mid/side), fixed and variable
blocking strategies, every block-size and sample-rate code family (table, 8/16-bit explicit, "from
STREAMINFO"), bits per sample 4-32, extra metadata blocks and an ID3v2 prefix.

It optimises nothing: parameters are whatever the caller (or a simple heuristic) picks.  No real
encoder (libFLAC, ffmpeg) exists in this image, so files made by one are "parity unpinned"; the
round trip here pins the decoder against the specification.
"""
from __future__ import annotations

import hashlib
import struct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

BLOCK_CODES = {192: 1, 576: 2, 1152: 3, 2304: 4, 4608: 5, 256: 8, 512: 9, 1024: 10, 2048: 11, 4096: 12,
               8192: 13, 16384: 14, 32768: 15}
RATE_CODES = {88200: 1, 176400: 2, 192000: 3, 8000: 4, 16000: 5, 22050: 6, 24000: 7, 32000: 8, 44100: 9,
              48000: 10, 96000: 11}
BPS_CODES = {8: 1, 12: 2, 16: 4, 20: 5, 24: 6, 32: 7}


def _crc_table(width, poly):
    top = 1 << (width - 1)
    mask = (1 << width) - 1
    t = []
    for i in range(256):
        c = i << (width - 8)
        for _ in range(8):
            c = ((c << 1) ^ poly) if c & top else (c << 1)
        t.append(c & mask)
    return t


_C8 = _crc_table(8, 0x07)
_C16 = _crc_table(16, 0x8005)


def crc8(b: bytes) -> int:
    c = 0
    for x in b:
        c = _C8[c ^ x]
    return c


def crc16(b: bytes) -> int:
    c = 0
    for x in b:
        c = ((c << 8) & 0xFFFF) ^ _C16[(c >> 8) ^ x]
    return c


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v: int, k: int):
        if k == 0:
            return
        self.acc = (self.acc << k) | (int(v) & ((1 << k) - 1))
        self.n += k
        while self.n >= 8:
            self.n -= 8
            self.out.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def unary(self, q: int):
        while q >= 32:
            self.put(0, 32)
            q -= 32
        self.put(1, q + 1)

    def align(self):
        if self.n:
            self.put(0, 8 - self.n)

    def bytes(self) -> bytes:
        assert self.n == 0
        return bytes(self.out)


def _utf8_number(v: int) -> bytes:
    if v < 0x80:
        return bytes([v])
    for n, bits in ((2, 11), (3, 16), (4, 21), (5, 26), (6, 31), (7, 36)):
        if v < (1 << bits):
            out = []
            for _ in range(n - 1):
                out.append(0x80 | (v & 0x3F))
                v >>= 6
            lead = (0xFF << (8 - n)) & 0xFF if n < 7 else 0xFE
            return bytes([lead | v] + out[::-1])
    raise ValueError("coded number too large")


@dataclass
class Sub:
    """Subframe recipe.  kind: 'constant' | 'verbatim' | 'fixed' | 'lpc'."""
    kind: str = "fixed"
    order: int = 2
    lpc_precision: int = 12
    wasted: Optional[int] = None    # None: detect from the samples
    porder: Optional[int] = None    # residual partition order; None: largest valid <= 4
    rice2: bool = False             # method 1 (5-bit parameters)
    escape: Sequence[int] = ()      # partitions coded raw
    param: Optional[int] = None     # force this Rice parameter on non-escaped partitions


@dataclass
class Frame:
    blocksize: int
    channel_mode: str = "independent"   # independent | left_side | side_right | mid_side
    subs: List[Sub] = field(default_factory=list)
    bs_code: Optional[int] = None       # force the code (6/7: explicit 8/16-bit)
    sr_code: Optional[int] = None       # force (0 = STREAMINFO, 12/13/14 explicit)
    ss_from_streaminfo: bool = False


def _fixed_residual(s: List[int], order: int) -> List[int]:
    if order == 0:
        return s[:]
    pred = {1: lambda i: s[i - 1], 2: lambda i: 2 * s[i - 1] - s[i - 2],
            3: lambda i: 3 * s[i - 1] - 3 * s[i - 2] + s[i - 3],
            4: lambda i: 4 * s[i - 1] - 6 * s[i - 2] + 4 * s[i - 3] - s[i - 4]}[order]
    return [s[i] - pred(i) for i in range(order, len(s))]


def _lpc_coefs(s: List[int], order: int, precision: int):
    """Least-squares predictor quantised to `precision` signed bits with the largest shift <= 15 that
    fits (shift >= 0: RFC 9639 forbids negative shifts)."""
    x = np.asarray(s, np.float64)
    n = len(x)
    if n <= order + 1 or not np.any(x):
        a = np.zeros(order)
    else:
        A = np.stack([x[order - 1 - j:n - 1 - j] for j in range(order)], 1)
        a = np.linalg.lstsq(A, x[order:], rcond=None)[0]
    lim = (1 << (precision - 1)) - 1
    shift = 15
    while shift > 0 and np.max(np.abs(a)) * (1 << shift) > lim:
        shift -= 1
    q = [int(v) for v in np.clip(np.round(a * (1 << shift)), -lim - 1, lim)]
    return q, shift


def _lpc_residual(s, coefs, shift):
    p = len(coefs)
    return [s[i] - (sum(c * s[i - 1 - j] for j, c in enumerate(coefs)) >> shift) for i in range(p, len(s))]


def _put_residual(bw: BitWriter, res: List[int], bs: int, order: int, sub: Sub):
    porder = sub.porder
    if porder is None:
        porder = 0
        while porder < 4 and bs % (1 << (porder + 1)) == 0 and (bs >> (porder + 1)) >= order:
            porder += 1
    assert bs % (1 << porder) == 0 and (bs >> porder) >= order
    assert all(-(1 << 31) <= v < (1 << 31) for v in res), "residual exceeds 32 bits (RFC 9639 9.2.7)"
    method = 1 if sub.rice2 else 0
    bw.put(method, 2)
    bw.put(porder, 4)
    psz = bs >> porder
    pbits, esc = (5, 31) if method else (4, 15)
    k = 0
    for pi in range(1 << porder):
        cnt = psz - order if pi == 0 else psz
        part = res[k:k + cnt]
        k += cnt
        if pi in sub.escape:
            nb = 0
            if any(part):
                nb = max((v.bit_length() if v >= 0 else (-v - 1).bit_length()) + 1 for v in part)
            bw.put(esc, pbits)
            bw.put(nb, 5)
            for v in part:
                bw.put(v, nb)
            continue
        if sub.param is not None:
            param = sub.param
        else:
            m = np.mean([abs(v) for v in part]) if part else 0.0
            param = int(max(0, np.floor(np.log2(m + 1)))) if m > 0 else 0
        param = min(param, esc - 1)
        bw.put(param, pbits)
        for v in part:
            u = (v << 1) if v >= 0 else ((-v) << 1) - 1
            bw.unary(u >> param)
            bw.put(u & ((1 << param) - 1), param)


def _put_subframe(bw: BitWriter, s: List[int], bps: int, sub: Sub):
    w = sub.wasted
    if w is None:
        w = 0
        if any(s):
            while w < bps - 1 and all(((v >> w) & 1) == 0 for v in s):
                w += 1
    if w:
        assert all(v % (1 << w) == 0 for v in s)
        s = [v >> w for v in s]
    eb = bps - w
    code = {"constant": 0, "verbatim": 1}.get(sub.kind)
    if sub.kind == "fixed":
        code = 8 + sub.order
    elif sub.kind == "lpc":
        code = 32 + sub.order - 1
    bw.put(0, 1)
    bw.put(code, 6)
    if w:
        bw.put(1, 1)
        bw.unary(w - 1)
    else:
        bw.put(0, 1)
    bs = len(s)
    if sub.kind == "constant":
        assert all(v == s[0] for v in s)
        bw.put(s[0], eb)
    elif sub.kind == "verbatim":
        for v in s:
            bw.put(v, eb)
    elif sub.kind == "fixed":
        for v in s[:sub.order]:
            bw.put(v, eb)
        _put_residual(bw, _fixed_residual(s, sub.order), bs, sub.order, sub)
    else:
        coefs, shift = _lpc_coefs(s, sub.order, sub.lpc_precision)
        for v in s[:sub.order]:
            bw.put(v, eb)
        bw.put(sub.lpc_precision - 1, 4)
        bw.put(shift, 5)
        for c in coefs:
            bw.put(c, sub.lpc_precision)
        _put_residual(bw, _lpc_residual(s, coefs, shift), bs, sub.order, sub)


def encode(samples: np.ndarray, rate: int, bps: int, frames: Sequence[Frame], variable: bool = False,
           extra_metadata: bool = False, id3: bool = False) -> bytes:
    """samples: (channels, n) integer array within bps bits.  sum(frame.blocksize) must equal n."""
    x = np.asarray(samples, np.int64)
    if x.ndim == 1:
        x = x[None]
    C, n = x.shape
    assert sum(f.blocksize for f in frames) == n
    lo, hi = -(1 << (bps - 1)), (1 << (bps - 1)) - 1
    assert x.min(initial=0) >= lo and x.max(initial=0) <= hi
    body = bytearray()
    pos = 0
    for fi, fr in enumerate(frames):
        bs = fr.blocksize
        blk = [list(map(int, x[c, pos:pos + bs])) for c in range(C)]
        mode = fr.channel_mode
        if mode == "independent":
            chans, cbps, ch_code = blk, [bps] * C, C - 1
        else:
            assert C == 2
            L, R = blk
            side = [a - b for a, b in zip(L, R)]
            if mode == "left_side":
                chans, cbps, ch_code = [L, side], [bps, bps + 1], 8
            elif mode == "side_right":
                chans, cbps, ch_code = [side, R], [bps + 1, bps], 9
            else:
                mid = [(a + b) >> 1 for a, b in zip(L, R)]
                chans, cbps, ch_code = [mid, side], [bps, bps + 1], 10
        bw = BitWriter()
        bw.put(0b111111111111100, 15)
        bw.put(1 if variable else 0, 1)
        bs_code = fr.bs_code if fr.bs_code is not None else BLOCK_CODES.get(bs, 6 if bs <= 256 else 7)
        if bs_code in BLOCK_CODES.values():
            assert BLOCK_CODES.get(bs) == bs_code
        sr_code = fr.sr_code if fr.sr_code is not None else RATE_CODES.get(rate, 0)
        ss_code = 0 if fr.ss_from_streaminfo else BPS_CODES.get(bps, 0)
        bw.put(bs_code, 4)
        bw.put(sr_code, 4)
        bw.put(ch_code, 4)
        bw.put(ss_code, 3)
        bw.put(0, 1)
        for byte in _utf8_number(pos if variable else fi):
            bw.put(byte, 8)
        if bs_code == 6:
            bw.put(bs - 1, 8)
        elif bs_code == 7:
            bw.put(bs - 1, 16)
        if sr_code == 12:
            assert rate % 1000 == 0
            bw.put(rate // 1000, 8)
        elif sr_code == 13:
            bw.put(rate, 16)
        elif sr_code == 14:
            assert rate % 10 == 0
            bw.put(rate // 10, 16)
        hdr = bw.bytes()
        bw.put(crc8(hdr), 8)
        subs = fr.subs or [Sub() for _ in range(C)]
        for c in range(C):
            _put_subframe(bw, chans[c], cbps[c], subs[c])
        bw.align()
        fb = bw.bytes()
        body += fb + struct.pack(">H", crc16(fb))
        pos += bs
    # STREAMINFO
    bsz = [f.blocksize for f in frames] or [4096]
    si = BitWriter()
    si.put(min(bsz) if variable else max(16, max(bsz)), 16)
    si.put(max(16, max(bsz)), 16)
    si.put(0, 24)
    si.put(0, 24)
    si.put(rate, 20)
    si.put(C - 1, 3)
    si.put(bps - 1, 5)
    si.put(n, 36)
    inter = x.T.reshape(-1)
    nbytes = (bps + 7) // 8
    md5 = hashlib.md5(b"".join(int(v).to_bytes(nbytes, "little", signed=True) for v in inter)).digest()
    streaminfo = si.bytes() + md5
    blocks = [(0, streaminfo)]
    if extra_metadata:
        vendor = b"suta-spec-encoder"
        vc = struct.pack("<I", len(vendor)) + vendor + struct.pack("<I", 1) + struct.pack("<I", 7) + b"TITLE=x"
        blocks += [(4, vc), (1, b"\x00" * 37)]
    meta = bytearray(b"fLaC")
    for i, (t, data) in enumerate(blocks):
        last = 0x80 if i == len(blocks) - 1 else 0
        meta += bytes([last | t]) + len(data).to_bytes(3, "big") + data
    out = bytes(meta) + bytes(body)
    if id3:
        tag = b"TIT2\x00\x00\x00\x02\x00\x00\x00x"
        sz = len(tag)
        syn = bytes([(sz >> 21) & 0x7F, (sz >> 14) & 0x7F, (sz >> 7) & 0x7F, sz & 0x7F])
        out = b"ID3\x04\x00\x00" + syn + tag + out
    return out


def simple_frames(n: int, channels: int, blocksize: int = 4096, kind: str = "lpc", order: int = 8,
                  channel_mode: str = "independent") -> List[Frame]:
    """Uniform frames covering n samples (the last one shorter, explicit size code)."""
    out = []
    pos = 0
    while pos < n:
        bs = min(blocksize, n - pos)
        o = min(order, bs - 1) if kind in ("fixed", "lpc") else order
        if kind == "fixed":
            o = min(o, 4)
        out.append(Frame(bs, channel_mode, [Sub(kind, max(o, 0 if kind == "fixed" else 1)) for _ in range(channels)]))
        pos += bs
    return out
