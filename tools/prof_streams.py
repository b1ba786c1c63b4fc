"""Per-stream timeline summary of a rocprofv3 kernel trace (rocpd SQLite db).

For each HIP stream (or HW queue when stream ids are absent): dispatches,
busy time (union of its kernel intervals), and the top kernels on it; then
the overlap between the two busiest streams (how much of the panel chain
hides under the trailing update) and the idle gaps of the busiest stream.

    python tools/prof_streams.py <db> [top]
"""
import sqlite3
import sys
from collections import defaultdict


def _union(iv):
    busy, cs, ce = 0, None, None
    for s, e in sorted(iv):
        if cs is None or s > ce:
            if cs is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if cs is not None:
        busy += ce - cs
    return busy


def _merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def _inter(a, b):
    i = j = tot = 0
    while i < len(a) and j < len(b):
        s = max(a[i][0], b[j][0])
        e = min(a[i][1], b[j][1])
        if e > s:
            tot += e - s
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main(path, top=8):
    con = sqlite3.connect(path)
    cur = con.cursor()
    cols = [r[1] for r in cur.execute("pragma table_info(rocpd_kernel_dispatch)").fetchall()]
    key = "stream_id" if "stream_id" in cols else ("queue_id" if "queue_id" in cols else None)
    sel = f"d.{key}" if key else "0"
    rows = cur.execute(f"""select s.kernel_name, d.start, d.end, {sel} from rocpd_kernel_dispatch d
                           join rocpd_info_kernel_symbol s on d.kernel_id = s.id""").fetchall()
    t0 = min(r[1] for r in rows)
    t1 = max(r[2] for r in rows)
    print(f"span {(t1 - t0) * 1e-6:.2f} ms, busy(any stream) {_union([(r[1], r[2]) for r in rows]) * 1e-6:.2f} ms,"
          f" {len(rows)} dispatches, grouped by {key}")
    by = defaultdict(list)
    for name, s, e, q in rows:
        by[q].append((name.split("(")[0][:80], s, e))
    order = sorted(by, key=lambda q: -_union([(s, e) for _, s, e in by[q]]))
    merged = {}
    for q in order:
        iv = [(s, e) for _, s, e in by[q]]
        merged[q] = _merge(iv)
        agg = defaultdict(lambda: [0, 0.0])
        for n, s, e in by[q]:
            agg[n][0] += 1
            agg[n][1] += (e - s) * 1e-6
        print(f"\n{key}={q}: {len(iv)} dispatches, busy {_union(iv) * 1e-6:.2f} ms")
        for n, (c, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
            print(f"  {c:6d} {ms:9.3f} ms {1e3 * ms / c:9.2f} us  {n}")
    if len(order) >= 2:
        a, b = merged[order[0]], merged[order[1]]
        ov = _inter(a, b)
        print(f"\noverlap of the two busiest streams: {ov * 1e-6:.2f} ms")
        gaps = [(a[i + 1][0] - a[i][1]) for i in range(len(a) - 1)]
        big = sorted(gaps, reverse=True)[:10]
        print(f"busiest stream: {len(gaps)} gaps, total {sum(gaps) * 1e-6:.2f} ms, largest (us): "
              + ", ".join(f"{g * 1e-3:.0f}" for g in big))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 8)
