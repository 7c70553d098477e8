"""HBM traffic per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), per kernel family.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of wide
(16 B/lane) coalesced reads -> doubled here; WRITE_SIZE is exact for 16-B/lane stores.  Both are in KB.
usage: python tools/pmc_traffic.py FETCH_counter_collection.csv WRITE_counter_collection.csv [out.json]
"""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import suta_loader  # noqa: E402

suta_loader.load()
from suta_amd.flops import kernel_base  # noqa: E402


def load(path, counter):
    per = collections.defaultdict(lambda: [0, 0.0])
    seen = set()
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        key = (r.get("Dispatch_Id"), r.get("Counter_Name"))
        name = kernel_base(r["Kernel_Name"])  # one entry per kernel base name (mangled or demangled)
        v = float(r["Counter_Value"])
        if key not in seen:
            seen.add(key)
            per[name][0] += 1
        per[name][1] += v
    return per


def load_by_grid(path, counter):
    """GEMM-family dispatches grouped by (kernel template, total grid threads): per-shape traffic."""
    per = collections.defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        n = r["Kernel_Name"]
        if not any(k in n for k in ("gemm_", "flash_", "posconv")):
            continue
        base = n.replace("void ", "").replace("(anonymous namespace)::", "")
        tmpl = base.split("(")[0]
        key = (tmpl[:90], int(r["Grid_Size"]))
        per[key][0] += 1
        per[key][1] += float(r["Counter_Value"])
    return per


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    if "--by-grid" in sys.argv:
        fg, wg = load_by_grid(sys.argv[1], "FETCH_SIZE"), load_by_grid(sys.argv[2], "WRITE_SIZE")
        rows = []
        for k in set(fg) | set(wg):
            n = max(fg[k][0], wg[k][0])
            rd = 2.0 * fg[k][1] * 1024 / max(1, fg[k][0])
            wr = wg[k][1] * 1024 / max(1, wg[k][0])
            rows.append((n * (rd + wr), k, n, rd, wr))
        for tot, k, n, rd, wr in sorted(rows, reverse=True)[:40]:
            print(f"{tot/1e9:9.2f} GB total  {n:5d} x  read {rd/1e6:9.2f} MB  write {wr/1e6:9.2f} MB  grid {k[1]:9d}  {k[0]}")
        return
    out = {}
    for k in sorted(set(fetch) | set(write)):
        n = max(fetch[k][0], write[k][0])
        rd = 2.0 * fetch[k][1] * 1024 / max(1, fetch[k][0])
        wr = write[k][1] * 1024 / max(1, write[k][0])
        out[k] = {"launches": n, "read_bytes_per_launch": rd, "write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": rd + wr}
        print(f"{k:28s} {n:6d} launches  read {rd/1e6:9.2f} MB  write {wr/1e6:9.2f} MB per launch")
    if len(sys.argv) > 3:
        json.dump(out, open(sys.argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
