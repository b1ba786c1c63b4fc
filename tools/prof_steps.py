"""Per-factorization critical-path view of a rocprofv3 kernel trace: takes
the LAST `nt` launches of the panel kernel (`--panel`, default potrf_lds) as
the timed factorization and reports, per tenth of its span, the time covered
by trailing-update GEMMs, by other kernels only, and idle; plus the panel
kernel's durations early/late.  python tools/prof_steps.py <dir> [nt] [panel]"""
import csv
import glob
import os
import sys


def main(d, nt=64, panel="potrf_lds"):
    tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(tr))]
    ks.sort()
    pan = [k for k in ks if panel in k[2]]
    t0 = pan[-nt][0]
    t1 = max(e for s, e, n in ks if s >= t0 and ("gemm" in n or panel in n or "trsm" in n))
    win = [(max(s, t0), min(e, t1), n) for s, e, n in ks if e > t0 and s < t1]
    span = t1 - t0
    print(f"factorization span {span / 1e6:.1f} ms (last {nt} '{panel}' launches)")
    for b in range(10):
        a0, a1 = t0 + span * b // 10, t0 + span * (b + 1) // 10
        g = [(max(s, a0), min(e, a1)) for s, e, n in win if "gemm" in n and e > a0 and s < a1]
        o = [(max(s, a0), min(e, a1)) for s, e, n in win if "gemm" not in n and e > a0 and s < a1]

        def union(iv):
            iv = sorted(iv)
            out = []
            for s, e in iv:
                if out and s <= out[-1][1]:
                    out[-1][1] = max(out[-1][1], e)
                else:
                    out.append([s, e])
            return out
        ug, uo = union(g), union(g + o)
        lg = sum(e - s for s, e in ug)
        la = sum(e - s for s, e in uo)
        w = a1 - a0
        print(f"  {b * 10:3d}-{b * 10 + 10:3d} %: GEMM {100 * lg / w:5.1f} %  other-only {100 * (la - lg) / w:5.1f} %"
              f"  idle {100 * (w - la) / w:5.1f} %")
    pd = [(e - s) / 1e3 for s, e, n in pan[-nt:]]
    q = max(1, nt // 4)
    print("  panel us: first quarter avg %.0f, last quarter avg %.0f" % (sum(pd[:q]) / q, sum(pd[-q:]) / q))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 64, sys.argv[3] if len(sys.argv) > 3 else "potrf_lds")
