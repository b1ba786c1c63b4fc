"""Critical-path model of a lookahead factorization from a rocprofv3
kernel trace (rocpd SQLite DB): splits the trace into runs at the restore
copies, then for the last run reports per stream the busy time, and on the
update stream (the stream with the most kernel time) the idle gaps -- the
time the trailing update waited for the panel chain -- attributed to the
panel-stream kernels running inside each gap.

  python tools/prof/critpath.py gpurun_out/prof_potrf/potrf_results.db [n_gaps]
"""
import collections
import sqlite3
import sys


def main(db, ngaps=12):
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    # a run starts after the last caller-stream (stream 0) kernel that is
    # followed by library-stream kernels (bench.py: restore copy, info fill)
    cuts = [r[3] for i, r in enumerate(rows) if r[1] == 0 and any(x[1] != 0 for x in rows[i + 1:i + 50])]
    t0 = cuts[-1] if cuts else rows[0][2]
    run = [r for r in rows if r[2] >= t0 and r[1] != 0]
    if not run:
        print("no kernels after the last restore copy")
        return
    start, end = min(r[2] for r in run), max(r[3] for r in run)
    busy = collections.defaultdict(float)
    for n, s, a, b in run:
        busy[s] += (b - a) / 1e6
    upd = max(busy, key=busy.get)
    print(f"run span {(end - start) / 1e6:.2f} ms; kernels {len(run)}")
    for s, v in sorted(busy.items()):
        print(f"  stream {s}: busy {v:.2f} ms{'  (update)' if s == upd else ''}")
    u = sorted((a, b) for n, s, a, b in run if s == upd)
    gaps, cur = [], start
    for a, b in u:
        if a > cur:
            gaps.append((cur, a))
        cur = max(cur, b)
    if end > cur:
        gaps.append((cur, end))
    tot = sum(b - a for a, b in gaps) / 1e6
    print(f"update-stream idle: {tot:.2f} ms in {len(gaps)} gaps ({100 * tot / ((end - start) / 1e6):.1f} % of the run)")
    other = [(n, s, a, b) for n, s, a, b in run if s != upd]
    print(f"largest {ngaps} gaps (ms from run start, length, panel kernels inside):")
    for a, b in sorted(gaps, key=lambda g: g[0] - g[1])[:ngaps]:
        inside = collections.Counter()
        for n, s, x, y in other:
            ov = min(b, y) - max(a, x)
            if ov > 0:
                inside[n.split("(")[0].replace("void ", "").replace("slate_hip::", "")[:40]] += ov / 1e3
        desc = ", ".join(f"{k} {v:.0f}us" for k, v in inside.most_common(3))
        print(f"  {(a - start) / 1e6:8.2f}  {(b - a) / 1e3:8.1f} us  {desc}")
    # the first and last kernel of the update stream: lead-in / tail
    print(f"lead-in (run start -> first update kernel): {(u[0][0] - start) / 1e6:.2f} ms; "
          f"tail (last update kernel -> run end): {(end - max(b for a, b in u)) / 1e6:.2f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
