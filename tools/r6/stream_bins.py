import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]) for r in rows))
marks = [k[0] for k in ks if ("copyBuffer" in k[3] or "copy_words" in k[3]) and k[1] - k[0] > 100000]
lo, hi = marks[-2], marks[-1]
sel = [k for k in ks if k[0] > lo and k[1] <= hi]
t0 = min(k[0] for k in sel); t1 = max(k[1] for k in sel)
B = 10
busy = collections.defaultdict(lambda: collections.Counter())
for s, e, sid, nm in sel:
    nm = nm.replace("void ", "").replace("slate_hip::", "").split("(")[0][:34]
    for b in range(B):
        a0 = t0 + (t1 - t0) * b / B; a1 = t0 + (t1 - t0) * (b + 1) / B
        o = min(e, a1) - max(s, a0)
        if o > 0: busy[(b, sid)][nm] += o / 1e6
for b in range(B):
    for sid in sorted({k[1] for k in busy if k[0] == b}):
        c = busy[(b, sid)]
        tot = sum(c.values())
        top = ", ".join(f"{n} {v:.1f}" for n, v in c.most_common(4))
        print(f"bin {b} stream {sid}: busy {tot:6.1f} ms of {(t1-t0)/1e6/B:.1f} | {top}")
