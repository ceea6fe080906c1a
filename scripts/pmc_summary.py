"""Per-kernel mean of rocprofv3 --pmc CSV counters (all *counter_collection.csv under a dir).
    python scripts/pmc_summary.py gpurun_out/pmc_attn [kernel-filter]"""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    flt = sys.argv[2] if len(sys.argv) > 2 else ""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if flt in r["Kernel_Name"]:
                agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        m = {c: sum(x) / len(x) for c, x in v.items()}
        print(k)
        for c in sorted(m):
            print(f"    {c:28s} {m[c]:16.0f}")
        if "SQ_INSTS_MFMA" in m and m["SQ_INSTS_MFMA"]:
            print(f"    VALU/MFMA {m.get('SQ_INSTS_VALU', 0) / m['SQ_INSTS_MFMA']:.1f}  "
                  f"LDS/MFMA {m.get('SQ_INSTS_LDS', 0) / m['SQ_INSTS_MFMA']:.2f}  "
                  f"conflicts/LDS {m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_INSTS_LDS', 1)):.2f}")
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            w = m["SQ_WAVE_CYCLES"]
            print(f"    of wave cycles: wait {m.get('SQ_WAIT_ANY', 0) / w:.2f}  issue-stall "
                  f"{m.get('SQ_WAIT_INST_ANY', 0) / w:.2f}  busy-mfma {m.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / 4 / w:.2f}")


if __name__ == "__main__":
    main()
