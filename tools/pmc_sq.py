"""Per-kernel SQ breakdown from rocprofv3 --pmc passes (one CSV per pass, any number of passes).

Pass A: SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
        SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
Pass B: SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
        SQ_WAIT_INST_LDS SQ_INSTS_VALU_CVT
WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~= WAVE_CYCLES
(MI355X_MICROARCH.md, PMC slots).

MFMA busy (fraction of the matrix pipe's cycles in use) = SQ_VALU_MFMA_BUSY_CYCLES / (32 x SQ_BUSY_CYCLES):
SQ_VALU_MFMA_BUSY_CYCLES sums, over every SIMD an SQ counter instance serves, the cycles its matrix pipe is busy
(MI355X_MICROARCH.md: "counts cycles (= 32 x N_mfma for 32x32x16 bf16)"; the committed passes show exactly 32 per
v_mfma_f32_32x32x16_bf16 and 64 per v_mfma_f32_32x32x2_f32 instruction, the guide's issue cycles per SIMD), while
SQ_BUSY_CYCLES counts each instance's busy cycles once.  One instance per shader engine: 256 CUs / 32 shader
engines x 4 SIMDs = 32 SIMDs per instance (MI355X_MICROARCH.md, chip-level parameters), hence the 32.  Cross-check:
gemm_glds_kernel in profiles/r3/close_c2_sq.txt reads 0.81 this way against 0.78 of the fp32 MFMA peak from its
timed FLOPs (the clock under load is below the 2.4 GHz the peak assumes).  Instruction counts are per
wave-instruction; VALU counts include the MFMAs (SQ_INSTS_VALU), so valu/mfma below subtracts them.
usage: python tools/pmc_sq.py pass_a.csv [pass_b.csv ...] [--json out.json]
       python tools/pmc_sq.py --from-json committed_sq.json [--json out.json]   (re-derive from the raw sums)
"""
import collections
import csv
import json
import sys


SIMDS_PER_SQ = 32  # 256 CUs x 4 SIMDs / 32 shader engines (one SQ counter instance each)


def short(name):
    return name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]


def main():
    args = sys.argv[1:]
    out_json = None
    if "--json" in args:
        i = args.index("--json")
        out_json = args[i + 1]
        args = args[:i] + args[i + 2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(lambda: collections.defaultdict(set))
    launches_of = {}
    if args and args[0] == "--from-json":
        for k, e in json.load(open(args[1])).items():
            acc[k].update(e["raw"])
            launches_of[k] = e["launches"]
        args = []
    for path in args:
        for r in csv.DictReader(open(path)):
            k = short(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k][r["Counter_Name"]].add(r.get("Dispatch_Id"))
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_INSTS_VALU", 0)))
    res = {}
    print(f"{'kernel':34s} {'launch':>6s} {'parked':>6s} {'stall':>6s} {'active':>6s} {'mfma_busy':>9s} "
          f"{'ldsconf/i':>9s} {'valu/mfma':>9s} {'trans/mfma':>10s} {'lds/mfma':>8s} {'vmem/mfma':>9s}")
    for k, c in rows:
        launches = launches_of.get(k, max((len(v) for v in n[k].values()), default=0))
        wc = c.get("SQ_WAVE_CYCLES", 0)
        busy = c.get("SQ_BUSY_CYCLES", 0)
        mf = c.get("SQ_INSTS_MFMA", 0)
        e = {"launches": launches}
        if wc:
            e.update(parked=c.get("SQ_WAIT_ANY", 0) / wc, stall=c.get("SQ_WAIT_INST_ANY", 0) / wc,
                     active=c.get("SQ_ACTIVE_INST_ANY", 0) / wc)
        if busy:
            e["mfma_busy"] = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (SIMDS_PER_SQ * busy)
        if c.get("SQ_INSTS_LDS"):
            e["lds_conflict_cycles_per_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
        if mf:
            e["valu_per_mfma"] = (c.get("SQ_INSTS_VALU", 0) - mf) / mf
            e["trans_per_mfma"] = c.get("SQ_INSTS_VALU_TRANS_F32", 0) / mf
            e["cvt_per_mfma"] = c.get("SQ_INSTS_VALU_CVT", 0) / mf
            e["salu_per_mfma"] = c.get("SQ_INSTS_SALU", 0) / mf
            e["vmem_per_mfma"] = (c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_VMEM_WR", 0)) / mf
            if c.get("SQ_INSTS_LDS"):
                e["lds_per_mfma"] = c["SQ_INSTS_LDS"] / mf
        e["raw"] = dict(c)
        res[k] = e

        def f(key, w, p=3):
            return f"{e[key]:{w}.{p}f}" if key in e else " " * (w - 1) + "-"
        print(f"{k[:34]:34s} {launches:6d} {f('parked', 6)} {f('stall', 6)} {f('active', 6)} {f('mfma_busy', 9)} "
              f"{f('lds_conflict_cycles_per_inst', 9)} {f('valu_per_mfma', 9, 2)} {f('trans_per_mfma', 10, 2)} "
              f"{f('lds_per_mfma', 8, 2)} {f('vmem_per_mfma', 9, 3)}")
    if out_json:
        json.dump(res, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
