"""Summarise a rocprofv3 SQLite (.db) kernel trace: per-kernel totals,
plus overall GPU busy span.  Usage: python tools/prof_summary.py <db> [top]"""
import sqlite3
import sys
from collections import defaultdict


def main(path, top=25):
    con = sqlite3.connect(path)
    cur = con.cursor()
    q = """select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id"""
    try:
        rows = cur.execute(q).fetchall()
    except sqlite3.OperationalError:
        rows = cur.execute("select name, start, end from kernels").fetchall()
    agg = defaultdict(lambda: [0, 0.0])
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    for name, s, e in rows:
        short = name.split("(")[0]
        if len(short) > 90:
            short = short[:90]
        agg[short][0] += 1
        agg[short][1] += (e - s) * 1e-6
    tot = sum(v[1] for v in agg.values())
    # union of busy intervals (GPU-busy time, any stream)
    iv = sorted((s, e) for _, s, e in rows)
    busy, cs, ce = 0, None, None
    for s_, e_ in iv:
        if cs is None or s_ > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    if cs is not None:
        busy += ce - cs
    print(f"dispatches={len(rows)}  sum(kernel ms)={tot:.2f}  span ms={(t1 - t0) * 1e-6:.2f}  "
          f"busy(union) ms={busy * 1e-6:.2f}")
    print(f"{'calls':>7} {'total ms':>10} {'avg us':>9}  kernel")
    for k, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{c:7d} {ms:10.3f} {1e3 * ms / c:9.2f}  {k}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
