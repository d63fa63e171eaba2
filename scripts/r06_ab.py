import csv,statistics as s,sys,glob
for d in sorted(glob.glob(sys.argv[1]+"/v*/")):
    rows=list(csv.DictReader(open(d+"run_kernel_trace.csv")))
    rows.sort(key=lambda r:int(r["Start_Timestamp"]))
    out=[]
    for k in ["k_mv_gather","k_cg_consume","k_mv_pbfs"]:
        l=[(int(r["End_Timestamp"])-int(r["Start_Timestamp"]))/1e3 for r in rows if k in r["Kernel_Name"]]
        out.append(f"{k} c4 {s.median(l[5:25]):.1f} c5 {s.median(l[28:]) if len(l)>28 else 0:.1f}")
    print(d, " | ".join(out))
