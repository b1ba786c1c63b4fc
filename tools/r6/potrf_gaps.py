"""Where the 1-GPU dpotrf loses time: the update stream's idle gaps of the
LAST factorization in a rocprofv3 kernel-trace CSV, placed in the
factorization (fraction of the span) with the kernels the other streams ran
meanwhile.  python tools/r6/potrf_gaps.py run_kernel_trace.csv"""
import collections
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
    marks = [k[0] for k in ks if ("copyBuffer" in k[3] or "copy_words" in k[3]) and k[1] - k[0] > 100000]
    lo = marks[-2] if len(marks) >= 2 else ks[0][0]
    hi = marks[-1] if len(marks) >= 2 else ks[-1][1]
    sel = [k for k in ks if k[0] > lo and k[1] <= hi]
    t0 = min(k[0] for k in sel)
    t1 = max(k[1] for k in sel)
    span = (t1 - t0) / 1e6
    gemm = [k for k in sel if "gemm" in k[3]]
    # the update stream = the stream holding the most GEMM time
    per = collections.Counter()
    for k in gemm:
        per[k[2]] += k[1] - k[0]
    us = per.most_common(1)[0][0]
    U = sorted((k[0], k[1]) for k in sel if k[2] == us)
    print(f"span {span:.2f} ms; update stream {us}: {len(U)} kernels")
    gaps = []
    prev_end = t0
    for s, e in U:
        if s > prev_end:
            gaps.append((prev_end, s))
        prev_end = max(prev_end, e)
    if t1 > prev_end:
        gaps.append((prev_end, t1))
    tot = sum(b - a for a, b in gaps) / 1e6
    print(f"update stream idle {tot:.2f} ms in {len(gaps)} gaps")
    bins = collections.Counter()
    for a, b in gaps:
        bins[int(10 * (a - t0) / (t1 - t0))] += (b - a) / 1e6
    for i in range(10):
        print(f"  {i * 10:3d}-{i * 10 + 10:3d}% of span: idle {bins[i]:6.2f} ms")
    # what ran during the idle time
    during = collections.Counter()
    for a, b in gaps:
        for k in sel:
            if k[2] == us:
                continue
            o = min(b, k[1]) - max(a, k[0])
            if o > 0:
                during[k[3].replace("void ", "").replace("slate_hip::", "").split("(")[0][:60]] += o / 1e6
    print("other streams' kernels inside those gaps (overlap ms):")
    for nm, t in during.most_common(10):
        print(f"  {t:7.2f}  {nm}")
    # GEMM durations on the update stream in the first / middle / last thirds
    names = collections.Counter()
    for k in sel:
        names[(k[2], k[3].replace("void ", "").replace("slate_hip::", "").split("(")[0][:60])] += (k[1] - k[0]) / 1e6
    print("kernel time by stream:")
    for (sid, nm), t in sorted(names.items(), key=lambda x: -x[1])[:14]:
        print(f"  {sid:>4} {t:8.2f} ms  {nm}")


if __name__ == "__main__":
    main(sys.argv[1])
