"""Kernel table from a rocprofv3 rocpd database (run_results.db): calls,
total ms, average us per kernel name, plus span and busy (union) time.
usage: python tools/prof_db_summary.py <run_results.db> [top]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 30
c = sqlite3.connect(db)
rows = list(c.execute("select name, start, end from kernels order by start"))
agg = defaultdict(lambda: [0, 0.0])
busy, cur_s, cur_e = 0.0, None, None
for nm, s, e in rows:
    k = nm.split("(")[0]
    agg[k][0] += 1
    agg[k][1] += (e - s) / 1e6
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += (cur_e - cur_s) / 1e6
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
if cur_e is not None:
    busy += (cur_e - cur_s) / 1e6
span = (rows[-1][2] - rows[0][1]) / 1e6 if rows else 0
print(f"dispatches={len(rows)}  sum(kernel ms)={sum(v[1] for v in agg.values()):.1f}  span ms={span:.1f}  busy(union) ms={busy:.1f}")
print(f"{'calls':>7} {'total ms':>10} {'avg us':>10}  kernel")
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:top]:
    print(f"{n:7d} {t:10.2f} {1e3 * t / n:10.1f}  {k[:110]}")

# --deciles PATTERN: over the span of the LAST factorization (from the first
# kernel whose name contains FIRST, default the pattern itself), the share of
# each tenth covered by kernels matching PATTERN (e.g. gemm_real), by other
# kernels only, and idle
if "--deciles" in sys.argv:
    pat = sys.argv[sys.argv.index("--deciles") + 1]
    first = sys.argv[sys.argv.index("--first") + 1] if "--first" in sys.argv else None
    starts = [i for i, (nm, s, e) in enumerate(rows) if first and first in nm]
    sub = rows[starts[len(starts) // 2]:] if starts else rows
    t0, t1 = sub[0][1], max(e for _, _, e in sub)
    nb = 10
    import numpy as np
    res = 20000
    grid = np.linspace(t0, t1, res + 1)
    g = np.zeros(res, bool)
    o = np.zeros(res, bool)
    for nm, s, e in sub:
        i0, i1 = np.searchsorted(grid, [s, e])
        (g if pat in nm else o)[max(i0 - 1, 0):i1] = True
    print(f"span {(t1 - t0) / 1e6:.1f} ms from kernel #{len(rows) - len(sub)}")
    for d in range(nb):
        a, b = d * res // nb, (d + 1) * res // nb
        gg = g[a:b].mean()
        oo = (o[a:b] & ~g[a:b]).mean()
        print(f"  {10 * d:3d}-{10 * d + 10:3d} %: {pat} {100 * gg:5.1f} %  other-only {100 * oo:5.1f} %  idle {100 * (1 - gg - oo):5.1f} %")
