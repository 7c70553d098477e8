"""Writes MPEG-1 Layer III frames bit by bit from a known quantised spectrum (ISO/IEC 11172-3 2.4.1 syntax,
Table B.7 Huffman codes) — the test-side encoder of tests/test_mp3.py.  No psychoacoustics: the spectra are
random integers, the point is that libsuta_audio must parse every field back and reproduce the PCM that
oracle/mp3_np.py computes from the same spectrum.  44.1 kHz, 320 kbit/s, no CRC, main_data_begin = 0.
"""
import os
import re

import numpy as np

SFB_LONG = [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576]
SLEN = [[0, 0, 0, 0, 3, 1, 1, 1, 2, 2, 2, 3, 3, 3, 4, 4], [0, 1, 2, 3, 0, 1, 2, 3, 1, 2, 3, 1, 2, 3, 2, 3]]
QUAD_LEN = [1, 4, 4, 5, 4, 6, 5, 6, 4, 5, 5, 6, 5, 6, 6, 6]
QUAD_COD = [1, 5, 4, 5, 6, 5, 4, 4, 7, 3, 6, 0, 7, 2, 3, 1]
LINBITS = {16: 1, 17: 2, 18: 3, 19: 4, 20: 6, 21: 8, 22: 10, 23: 13,
           24: 4, 25: 5, 26: 6, 27: 7, 28: 8, 29: 9, 30: 11, 31: 13}
SIZE = {1: 2, 2: 3, 3: 3, 5: 4, 6: 4, 7: 6, 8: 6, 9: 6, 10: 8, 11: 8, 12: 8, 13: 16, 15: 16}
FRAME_BYTES = 1044          # 144000 * 320 / 44100, padding 0

_TABLES_H = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "test-time-adaptation-asr-suta_amd",
                         "csrc", "mp3_tables.h")
_HUFF = None


def huff():
    global _HUFF
    if _HUFF is None:
        txt = open(_TABLES_H).read()
        _HUFF = {}
        for t in (1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15, 16, 24):
            lens = [int(v) for v in re.search(r"hlen%d\[\d+\] = \{([^}]*)\}" % t, txt).group(1).split(",")]
            cods = [int(v) for v in re.search(r"hcod%d\[\d+\] = \{([^}]*)\}" % t, txt).group(1).split(",")]
            _HUFF[t] = (lens, cods)
    return _HUFF


def max_value(t):
    return 15 + (1 << LINBITS[t]) - 1 if t in LINBITS else SIZE[t] - 1


class BitWriter:
    def __init__(self):
        self.bits = []

    def put(self, v, n):
        for b in range(n - 1, -1, -1):
            self.bits.append((v >> b) & 1)

    def tobytes(self, nbytes=None):
        bits = self.bits + [0] * (-len(self.bits) % 8)
        out = np.packbits(np.array(bits, np.uint8)).tobytes()
        if nbytes is not None:
            assert len(out) <= nbytes, (len(out), nbytes)
            out += bytes(nbytes - len(out))
        return out


def _regions(g):
    big = 2 * g["big_values"]
    if g["ws"]:
        return [min(36, big), big, big]
    return [min(SFB_LONG[min(g["region0"] + 1, 22)], big), min(SFB_LONG[min(g["region0"] + g["region1"] + 2, 22)], big),
            big]


def random_granule(rng, block_type=0, mixed=0, nbig=None, ncount1=None):
    """A granule dict: random quantised spectrum, scale factors, gains and table selections."""
    g = {"ws": int(block_type != 0), "block_type": block_type, "mixed": mixed if block_type == 2 else 0,
         "gg": int(rng.integers(150, 185)), "sfc": int(rng.integers(0, 16)), "preflag": int(rng.integers(0, 2)),
         "sf_scale": int(rng.integers(0, 2)), "count1_table": int(rng.integers(0, 2)),
         "subblock_gain": [int(v) for v in rng.integers(0, 8, 3)] if block_type else [0, 0, 0],
         "region0": int(rng.integers(0, 16)), "region1": int(rng.integers(0, 8))}
    if g["ws"]:
        g["preflag"] = 0 if block_type == 2 else g["preflag"]
    s1, s2 = SLEN[0][g["sfc"]], SLEN[1][g["sfc"]]
    g["sf_l"] = [int(rng.integers(0, 1 << (s1 if sfb < 11 else s2))) for sfb in range(21)]
    g["sf_s"] = [[int(rng.integers(0, 1 << (s1 if sfb < 6 else s2))) for _ in range(3)] for sfb in range(12)]
    if block_type == 2 and mixed:
        g["sf_l"] = [v if sfb < 8 else 0 for sfb, v in enumerate(
            [int(rng.integers(0, 1 << s1)) for sfb in range(21)])]
        g["sf_s"] = [[0, 0, 0] if sfb < 3 else row for sfb, row in enumerate(g["sf_s"])]
    elif block_type == 2:
        g["sf_l"] = [0] * 21
    else:
        g["sf_s"] = [[0, 0, 0] for _ in range(12)]
    nbig = int(rng.integers(10, 120)) * 2 if nbig is None else nbig
    g["big_values"] = nbig // 2
    tables = [int(t) for t in rng.choice([1, 2, 3, 5, 6, 7, 8, 9, 10, 11, 12, 13, 15] + list(range(16, 32)), 3)]
    g["table"] = tables
    is_ = np.zeros(576, np.int64)
    r = _regions(g)
    starts = [0, r[0], r[1]]
    for reg in range(3):
        a, b = starts[reg], r[reg]
        if b > a:
            mv = min(max_value(tables[reg]), 40)
            is_[a:b] = rng.integers(-mv, mv + 1, b - a)
    nq = int(rng.integers(0, 40)) if ncount1 is None else ncount1
    nq = min(nq, (576 - nbig) // 4)
    is_[nbig:nbig + 4 * nq] = rng.integers(-1, 2, 4 * nq)
    g["is"] = is_
    g["count1_end"] = nbig + 4 * nq
    return g


def write_granule(bw, g):
    """Scale factors (part 2) and Huffman data (part 3) of one granule / channel; returns part2_3_length."""
    n0 = len(bw.bits)
    s1, s2 = SLEN[0][g["sfc"]], SLEN[1][g["sfc"]]
    if g["ws"] and g["block_type"] == 2:
        if g["mixed"]:
            for sfb in range(8):
                bw.put(g["sf_l"][sfb], s1)
        for sfb in range(3 if g["mixed"] else 0, 12):
            for w in range(3):
                bw.put(g["sf_s"][sfb][w], s1 if sfb < 6 else s2)
    else:
        for sfb in range(21):
            bw.put(g["sf_l"][sfb], s1 if sfb < 11 else s2)
    H = huff()
    r = _regions(g)
    i = 0
    for reg in range(3):
        t = g["table"][reg]
        base = t if t < 16 else (16 if t < 24 else 24)
        n = 16 if t >= 16 else SIZE[t]
        lb = LINBITS.get(t, 0)
        lens, cods = H[base]
        while i < r[reg]:
            x, y = int(g["is"][i]), int(g["is"][i + 1])
            ax, ay = abs(x), abs(y)
            idx = min(ax, 15) * n + min(ay, 15) if lb else ax * n + ay
            bw.put(cods[idx], lens[idx])
            if lb and ax >= 15:
                bw.put(ax - 15, lb)
            if ax:
                bw.put(int(x < 0), 1)
            if lb and ay >= 15:
                bw.put(ay - 15, lb)
            if ay:
                bw.put(int(y < 0), 1)
            i += 2
    while i < g["count1_end"]:
        q = [int(v) for v in g["is"][i:i + 4]]
        v = sum((abs(q[k]) & 1) << (3 - k) for k in range(4))
        if g["count1_table"]:
            bw.put(15 - v, 4)
        else:
            bw.put(QUAD_COD[v], QUAD_LEN[v])
        for k in range(4):
            if q[k]:
                bw.put(int(q[k] < 0), 1)
        i += 4
    return len(bw.bits) - n0


def write_frame(granules, channels, ms=False):
    """granules: [gr0, gr1], each a list of per-channel granule dicts -> one MPEG-1 Layer III frame."""
    main = BitWriter()
    p23 = [[write_granule(main, granules[gr][ch]) for ch in range(channels)] for gr in range(2)]
    side = BitWriter()
    side.put(0, 9)                                   # main_data_begin
    side.put(0, 5 if channels == 1 else 3)          # private bits
    for ch in range(channels):
        side.put(0, 4)                               # scfsi
    for gr in range(2):
        for ch in range(channels):
            g = granules[gr][ch]
            side.put(p23[gr][ch], 12)
            side.put(g["big_values"], 9)
            side.put(g["gg"], 8)
            side.put(g["sfc"], 4)
            side.put(g["ws"], 1)
            if g["ws"]:
                side.put(g["block_type"], 2)
                side.put(g["mixed"], 1)
                side.put(g["table"][0], 5)
                side.put(g["table"][1], 5)
                for w in range(3):
                    side.put(g["subblock_gain"][w], 3)
            else:
                for reg in range(3):
                    side.put(g["table"][reg], 5)
                side.put(g["region0"], 4)
                side.put(g["region1"], 3)
            side.put(g["preflag"], 1)
            side.put(g["sf_scale"], 1)
            side.put(g["count1_table"], 1)
    mode = 3 if channels == 1 else 1
    header = bytes([0xFF, 0xFB, (14 << 4) | (0 << 2), (mode << 6) | ((2 if ms else 0) << 4)])
    side_bytes = side.tobytes()
    body = main.tobytes(FRAME_BYTES - 4 - len(side_bytes))
    return header + side_bytes + body
