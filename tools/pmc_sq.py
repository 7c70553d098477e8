"""Per-kernel SQ stall breakdown from one rocprofv3 --pmc pass (tools/profile_round2.sh).
WAIT_ANY (parked on s_waitcnt / barrier) + WAIT_INST_ANY (issue stall) + ACTIVE_INST_ANY ~= WAVE_CYCLES
(MI355X_MICROARCH.md, PMC slots); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES x 4 SIMDs) per CU.
usage: python tools/pmc_sq.py <counter_collection.csv>"""
import collections
import csv
import sys


def main():
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        n[name].add(r.get("Dispatch_Id"))
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))
    print(f"{'kernel':28s} {'launches':>8s} {'parked':>7s} {'stall':>7s} {'active':>7s} {'mfma_busy':>9s} {'lds_conf/inst':>13s}")
    for k, c in rows:
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        busy = c.get("SQ_BUSY_CYCLES", 0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (4 * busy) if busy else 0
        li = c.get("SQ_INSTS_LDS", 0)
        print(f"{k:28s} {len(n[k]):8d} {c.get('SQ_WAIT_ANY', 0) / wc:7.3f} {c.get('SQ_WAIT_INST_ANY', 0) / wc:7.3f} "
              f"{c.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.3f} {mf:9.3f} {c.get('SQ_LDS_BANK_CONFLICT', 0) / li if li else 0:13.3f}")


if __name__ == "__main__":
    main()
