"""Per-stream busy time / gaps of the LAST factorization in a rocprofv3
kernel-trace CSV (the timed steps are bracketed by the input-restore
copies): python tools/r5/trace_streams.py run_kernel_trace.csv"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
    # input restores: the long device copies (the loopback's collectives are short copies too)
    marks = [k[0] for k in ks if ("copyBuffer" in k[3] or "copy_words" in k[3]) and k[1] - k[0] > 100000]
    lo = marks[-2] if len(marks) >= 2 else ks[0][0]
    hi = marks[-1] if len(marks) >= 2 else ks[-1][1]
    sel = [k for k in ks if k[0] > lo and k[1] <= hi]
    span = (max(k[1] for k in sel) - min(k[0] for k in sel)) / 1e6
    print(f"last factorization: {len(sel)} kernels, span {span:.1f} ms")
    by = collections.defaultdict(list)
    for k in sel:
        by[k[2]].append(k)
    for sid, L in sorted(by.items()):
        names = collections.Counter()
        for k in L:
            nm = k[3].replace("void ", "").replace("slate_hip::", "")
            names[nm.split("(")[0][:70]] += (k[1] - k[0]) / 1e6
        iv = sorted((k[0], k[1]) for k in L)
        cs, ce = iv[0]
        busy, gaps = 0, []
        for s, e in iv[1:]:
            if s > ce:
                busy += ce - cs
                gaps.append((s - ce) / 1e6)
                cs, ce = s, e
            else:
                ce = max(ce, e)
        busy += ce - cs
        print(f"stream {sid}: {len(L)} kernels, busy {busy / 1e6:.1f} ms, idle gaps {sum(gaps):.1f} ms "
              f"({sum(1 for g in gaps if g > 0.05)} over 50 us)")
        for nm, t in names.most_common(8):
            print(f"    {t:8.1f} ms  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
