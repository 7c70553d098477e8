"""Generate csrc/mp3_tables.h: the normative data tables of ISO/IEC 11172-3 Annex B that an MPEG audio
Layer III decoder cannot compute — the big-value Huffman code tables (Table B.7, tables 1-24) and the
synthesis window D[i] (Table B.3).

No copy of the tables exists in this image as text (no libmpg123 / libmad / minimp3 / ffmpeg sources or
headers), but an FFmpeg build is linked into kaleido's Chromium executable (a Python package of the image, not
part of the reference).  FFmpeg keeps the tables as plain arrays in its read-only data (per table: code lengths
as uint8[n*n] followed by the codes as uint16[n*n]; the window as int32[257] = D[i] * 65536).  This script READS
those bytes (the executable is never run or loaded), anchored on the small tables typed below from the
standard, and checks every table it takes:
  * each big-value table is a complete prefix code: Kraft sum == 1, no code a prefix of another, every
    code < 2^len (a mis-read table fails all three);
  * tables 1-7 equal the values typed here from the standard;
  * the window's first and last entries equal Table B.3's D[0..7] and D[256] (1.144989014).
The scale-factor band tables (Annex B.8), count1 tables (B.7 A/B), pretab and the antialias coefficients are
typed in csrc/mp3.cpp directly from the standard; this script checks the band tables against FFmpeg's
band_size_long / band_size_short arrays when those are present.

usage: python tools/mp3_tables.py [path-to-binary] [--check-only]
"""
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "..", "test-time-adaptation-asr-suta_amd", "csrc", "mp3_tables.h")
DEFAULT_BIN = "/usr/local/lib/python3.10/dist-packages/kaleido/executable/bin/kaleido"

# table id -> size n (values 0..n-1 for x and y).  Tables 4 and 14 are not defined by the standard.
SIZES = [(1, 2), (2, 3), (3, 3), (5, 4), (6, 4), (7, 6), (8, 6), (9, 6), (10, 8), (11, 8), (12, 8),
         (13, 16), (15, 16), (16, 16), (24, 16)]

# Typed from ISO/IEC 11172-3 Table B.7 (x-major order: index = x * n + y): anchors and cross-checks.
TYPED = {
    1: ([1, 3, 2, 3], [1, 1, 1, 0]),
    2: ([1, 3, 6, 3, 3, 5, 5, 5, 6], [1, 2, 1, 3, 1, 1, 3, 2, 0]),
    3: ([2, 2, 6, 3, 2, 5, 5, 5, 6], [3, 2, 1, 1, 1, 1, 3, 2, 0]),
    5: ([1, 3, 6, 7, 3, 3, 6, 7, 6, 6, 7, 8, 7, 6, 7, 8], [1, 2, 6, 5, 3, 1, 4, 4, 7, 5, 7, 1, 6, 1, 1, 0]),
    6: ([3, 3, 5, 7, 3, 2, 4, 5, 4, 4, 5, 6, 6, 5, 6, 7], [7, 3, 5, 1, 6, 2, 3, 2, 5, 4, 4, 1, 3, 3, 2, 0]),
    7: ([1, 3, 6, 8, 8, 9, 3, 4, 6, 7, 7, 8, 6, 5, 7, 8, 8, 9, 7, 7, 8, 9, 9, 9, 7, 7, 8, 9, 9, 10, 8, 8, 9, 10,
         10, 10],
        [1, 2, 10, 19, 16, 10, 3, 3, 7, 10, 5, 3, 11, 4, 13, 17, 8, 4, 12, 11, 18, 15, 11, 2, 7, 6, 9, 14, 3, 1,
         6, 4, 5, 3, 2, 0]),
}
# Table B.3: D[0..7] and D[256] in units of 2^-16
WINDOW_HEAD = [0, -1, -1, -1, -1, -1, -1, -2]
WINDOW_CENTER = 75038

# Annex B.8 scale-factor band boundaries (typed in csrc/mp3.cpp too); widths checked against FFmpeg when found.
SFB_LONG = [
    [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576],
    [0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576],
    [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576],
    [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576],
    [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 330, 394, 464, 540, 576],
    [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576],
    [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576],
    [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576],
    [0, 12, 24, 36, 48, 60, 72, 88, 108, 132, 160, 192, 232, 280, 336, 400, 476, 566, 568, 570, 572, 574, 576],
]
SFB_SHORT = [
    [0, 4, 8, 12, 16, 22, 30, 40, 52, 66, 84, 106, 136, 192],
    [0, 4, 8, 12, 16, 22, 28, 38, 50, 64, 80, 100, 126, 192],
    [0, 4, 8, 12, 16, 22, 30, 42, 58, 78, 104, 138, 180, 192],
    [0, 4, 8, 12, 18, 24, 32, 42, 56, 74, 100, 132, 174, 192],
    [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 136, 180, 192],
    [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192],
    [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192],
    [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192],
    [0, 8, 16, 24, 36, 52, 72, 96, 124, 160, 162, 164, 166, 192],
]


def check_prefix_code(lens, codes):
    """Complete prefix code: Kraft sum 1, codes fit their lengths, no code a prefix of another."""
    if any(l <= 0 or l > 19 for l in lens):
        return False
    if any(c >> l for c, l in zip(codes, lens)):
        return False
    if sum(2.0 ** -l for l in lens) != 1.0:
        return False
    words = sorted(format(c, "0%db" % l) for c, l in zip(codes, lens))
    return all(not words[i + 1].startswith(words[i]) for i in range(len(words) - 1))


def extract(blob):
    anchor = bytes(TYPED[1][0]) + struct.pack("<4H", *TYPED[1][1])
    pos = blob.find(anchor)
    if pos < 0:
        raise SystemExit("table 1 anchor not found")
    tables = {}
    cur = pos
    for tid, n in SIZES:
        nn = n * n
        while blob[cur] == 0:  # alignment padding before the next length array (lengths are >= 1)
            cur += 1
        lens = list(blob[cur:cur + nn])
        found = None
        for off in range(cur + nn, cur + nn + 32):
            if off % 2:
                continue
            codes = list(struct.unpack_from("<%dH" % nn, blob, off))
            if check_prefix_code(lens, codes):
                found = (off, codes)
                break
        if found is None:
            raise SystemExit("table %d: no valid code array after its lengths at %d" % (tid, cur))
        tables[tid] = (lens, found[1])
        cur = found[0] + 2 * nn
        if tid in TYPED and tables[tid] != TYPED[tid]:
            raise SystemExit("table %d differs from the values typed from the standard" % tid)
    head = struct.pack("<8i", *WINDOW_HEAD)
    wpos = blob.find(head)
    while wpos >= 0:
        win = list(struct.unpack_from("<257i", blob, wpos))
        if win[256] == WINDOW_CENTER:
            break
        wpos = blob.find(head, wpos + 4)
    if wpos < 0:
        raise SystemExit("synthesis window not found")
    return tables, win


def check_bands(blob):
    """FFmpeg's band_size_long[9][22] / band_size_short[9][13] (uint8 widths) against Annex B.8 typed above."""
    longw = b"".join(bytes(b - a for a, b in zip(t[:-1], t[1:])) for t in SFB_LONG)
    shortw = b"".join(bytes(b - a for a, b in zip(t[:-1], t[1:])) for t in SFB_SHORT)
    # count1 tables A and B (Table B.7, typed in csrc/mp3.cpp): lengths of A, of B, codes of A, of B
    quad = bytes(QUAD_A_LEN + [4] * 16 + QUAD_A_COD + list(range(15, -1, -1)))
    return blob.find(longw) >= 0, blob.find(shortw) >= 0, blob.find(quad) >= 0


QUAD_A_LEN = [1, 4, 4, 5, 4, 6, 5, 6, 4, 5, 5, 6, 5, 6, 6, 6]
QUAD_A_COD = [1, 5, 4, 5, 6, 5, 4, 4, 7, 3, 6, 0, 7, 2, 3, 1]


def emit(tables, win):
    L = ["// Generated by tools/mp3_tables.py -- ISO/IEC 11172-3 Annex B normative data (see that script for the",
         "// source and the checks applied).  Big-value Huffman tables in x-major order (index = x * n + y).",
         "#pragma once", "#include <cstdint>", "", "namespace mp3tab {", ""]
    for tid, n in SIZES:
        lens, codes = tables[tid]
        L.append("static const uint8_t hlen%d[%d] = {%s};" % (tid, n * n, ",".join(map(str, lens))))
        L.append("static const uint16_t hcod%d[%d] = {%s};" % (tid, n * n, ",".join(map(str, codes))))
    L.append("")
    L.append("// Table B.3 synthesis window D[i] * 65536, i = 0..256 (D[512 - i] = D[i] when i % 64 == 0, else -D[i])")
    L.append("static const int32_t window257[257] = {%s};" % ",".join(map(str, win)))
    L.append("")
    L.append("}  // namespace mp3tab")
    return "\n".join(L) + "\n"


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0] if args else DEFAULT_BIN
    with open(path, "rb") as f:
        blob = f.read()
    tables, win = extract(blob)
    bl, bs, bq = check_bands(blob)
    print("huffman tables:", " ".join("%d(%d)" % (t, n) for t, n in SIZES), "-- all complete prefix codes")
    print("tables 1-7 equal the typed values; window D[0..7], D[256] ok")
    print("Annex B.8 long band widths found:", bl, " short:", bs, " count1 tables A/B:", bq)
    text = emit(tables, win)
    if "--check-only" in sys.argv:
        with open(OUT) as f:
            same = f.read() == text
        print("csrc/mp3_tables.h matches:", same)
        sys.exit(0 if same else 1)
    with open(OUT, "w") as f:
        f.write(text)
    print("wrote", os.path.relpath(OUT))


if __name__ == "__main__":
    main()
