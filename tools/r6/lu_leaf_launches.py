import csv, collections, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"], r.get("Grid_Size_X", r.get("Grid_Size","")), r.get("Workgroup_Size_X","")) for r in rows))
marks = [k[0] for k in ks if ("copyBuffer" in k[3] or "copy_words" in k[3]) and k[1] - k[0] > 100000]
lo, hi = marks[-2], marks[-1]
sel = [k for k in ks if k[0] > lo and k[1] <= hi]
t0 = min(k[0] for k in sel)
tag = [k for k in sel if "getrf_base_tag" in k[3]]
print(len(tag), "tag launches; keys:", list(rows[0].keys())[:30])
for i in range(0, len(tag), 64):
    grp = tag[i:i+64]
    d = [ (k[1]-k[0])/1e3 for k in grp]
    print(f"launch {i:5d}-{i+len(grp)-1:5d} at {(grp[0][0]-t0)/1e6:7.1f} ms: mean {sum(d)/len(d):6.1f} us  min {min(d):6.1f} max {max(d):6.1f}  {grp[0][3][:40]} grid {grp[0][4]} wg {grp[0][5]}")
print()
for i in (512, 528, 544, 768, 784, 960):
    grp = tag[i:i+16]
    print(f"panel@{i}: " + " ".join(f"{(k[1]-k[0])/1e3:.0f}" for k in grp), " grid", grp[0][4])
# gaps between consecutive tag launches in a panel
for i in (512, 768):
    grp = tag[i:i+16]
    print("gaps us:", " ".join(f"{(grp[j+1][0]-grp[j][1])/1e3:.0f}" for j in range(15)))
