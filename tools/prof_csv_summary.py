"""Summarise a rocprofv3 CSV kernel trace (tools/gpu_prof_csv.sh):
per-kernel totals, GPU busy (union of kernel intervals) and span.
Usage: python tools/prof_csv_summary.py <dir> [top]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(d, top=15):
    tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    rows = []
    for r in csv.DictReader(open(tr[0])):
        rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    agg = defaultdict(lambda: [0, 0.0])
    for name, s, e in rows:
        short = name.split("(")[0].replace("void ", "")[:80]
        agg[short][0] += 1
        agg[short][1] += (e - s) * 1e-6
    iv = sorted((s, e) for _, s, e in rows)
    busy, cs, ce = 0, None, None
    for s_, e_ in iv:
        if cs is None or s_ > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    busy += ce - cs
    span = iv[-1][1] - iv[0][0]
    tot = sum(v[1] for v in agg.values())
    print(f"dispatches={len(rows)}  sum(kernel ms)={tot:.1f}  span ms={span * 1e-6:.1f}  busy(union) ms={busy * 1e-6:.1f}")
    print(f"{'calls':>7} {'total ms':>10} {'avg us':>9}  kernel")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{c:7d} {ms:10.2f} {1e3 * ms / c:9.1f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 15)
