"""Kernels of the last factorization in a rocprofv3 kernel-trace CSV inside a
time window (ms from its start), one line per kernel with stream, start,
duration: python tools/r5/trace_window.py run_kernel_trace.csv T0 T1"""
import csv
import sys


def main(path, t0, t1):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
    marks = [k[0] for k in ks if ("copyBuffer" in k[3] or "copy_words" in k[3]) and k[1] - k[0] > 100000]
    lo = marks[-2] if len(marks) >= 2 else ks[0][0]
    hi = marks[-1] if len(marks) >= 2 else ks[-1][1]
    sel = [k for k in ks if k[0] > lo and k[1] <= hi]
    base = min(k[0] for k in sel)
    for s, e, sid, nm in sel:
        a = (s - base) / 1e6
        if t0 <= a <= t1:
            nm = nm.replace("void ", "").replace("slate_hip::", "").split("(")[0][:60]
            print(f"{a:8.3f} +{(e - s) / 1e3:7.1f}us  s{sid}  {'    ' * (int(sid) - 1)}{nm}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), float(sys.argv[3]))
