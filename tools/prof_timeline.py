"""Critical-path view of a rocprofv3 CSV kernel trace: over the last
`--window` ms of the trace (the timed factorization), how much of the time is
covered by the trailing-update GEMMs, how much by other kernels only, and how
much is idle.  python tools/prof_timeline.py <dir> [window_ms]"""
import csv
import glob
import os
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    i = j = 0
    out = []
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def main(d, window_ms=None):
    tr = glob.glob(os.path.join(d, "*kernel_trace.csv"))[0]
    rows = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(tr))]
    end = max(e for _, _, e in rows)
    t0 = end - int(window_ms * 1e6) if window_ms else min(s for _, s, _ in rows)
    rows = [(n, max(s, t0), e) for n, s, e in rows if e > t0]
    gemm = union([[s, e] for n, s, e in rows if "gemm" in n])
    other = union([[s, e] for n, s, e in rows if "gemm" not in n])
    allk = union([[s, e] for _, s, e in rows])
    span = end - t0
    g, a = length(gemm), length(allk)
    ov = length(intersect(gemm, other))
    print(f"window {span * 1e-6:.1f} ms: GEMM running {g * 1e-6:.1f} ms ({100 * g / span:.1f} %), "
          f"other kernels only {(a - g) * 1e-6:.1f} ms ({100 * (a - g) / span:.1f} %), "
          f"idle {(span - a) * 1e-6:.1f} ms; other kernels overlapped with GEMM {ov * 1e-6:.1f} ms")
    # the same per tenth of the window (where in the factorization the GEMM stops covering)
    for k in range(10):
        s0, s1 = t0 + span * k // 10, t0 + span * (k + 1) // 10
        w = [[s0, s1]]
        gg = length(intersect(gemm, w))
        aa = length(intersect(allk, w))
        print(f"  {10 * k:3d}-{10 * k + 10:3d} %: GEMM {100 * gg / (s1 - s0):5.1f} %  other-only {100 * (aa - gg) / (s1 - s0):5.1f} %  idle {100 * (s1 - s0 - aa) / (s1 - s0):5.1f} %")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else None)
