"""Per-kernel PMC summary of rocprofv3 --pmc CSV output (tools/gpu_pmc_table.sh).
MFMA % = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); LDS conflict % = SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE; L2 hit % = TCC_HIT / (TCC_HIT + TCC_MISS).
Usage: python tools/pmc_summary.py <dir> [top]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, top=8):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        print("no counter_collection.csv under", d)
        return
    agg = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(set)
    for f in files:
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0))[:top]
    print(f"{'kernel':70s} {'disp':>5} {'MFMA%chip':>9} {'LDSconf%':>9} {'L2hit%':>7}")
    for k, c in rows:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs, MFMA busy over the 1024
        # SIMDs: utilisation of the whole chip's matrix pipes while active
        mf = 100 * c["SQ_VALU_MFMA_BUSY_CYCLES"] / max(c["GRBM_GUI_ACTIVE"] / 8 * 1024, 1)
        lc = 100 * c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_LDS_IDX_ACTIVE"], 1)
        hit = 100 * c["TCC_HIT_sum"] / max(c["TCC_HIT_sum"] + c["TCC_MISS_sum"], 1)
        print(f"{k:70s} {len(cnt[k]):5d} {mf:9.1f} {lc:9.2f} {hit:7.1f}")
        print("    raw: " + ", ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
