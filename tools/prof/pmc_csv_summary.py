"""Per-kernel summary of a rocprofv3 --pmc CSV (counter_collection.csv):
counter sums over dispatches, LDS conflict % (SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE) and MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE x CUs / 2): the normalisation of the round-3 PMC tables)."""
import collections
import csv
import glob
import sys

CUS = 256


def main(root, top=12):
    files = glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)
    if not files:
        print("no counter_collection.csv under", root)
        return
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row.get("Kernel_Name", "?")
                agg[k][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[k].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", 0))[:top]
    print(f"{'kernel':70s} {'disp':>5s} {'MFMA%':>6s} {'LDSconf%':>8s}")
    for k, c in rows:
        g = c.get("GRBM_GUI_ACTIVE", 0)
        mf = 100 * c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (g * CUS / 2) if g else 0
        lds = 100 * c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"] if c.get("SQ_LDS_IDX_ACTIVE") else 0
        print(f"{k[:70]:70s} {len(disp[k]):5d} {mf:6.1f} {lds:8.2f}")
        print("    raw: " + ", ".join(f"{n}={v:.3g}" for n, v in sorted(c.items())))


if __name__ == "__main__":
    main(sys.argv[1])
