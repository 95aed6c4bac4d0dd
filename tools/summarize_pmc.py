import csv, collections, glob, os, sys
root = sys.argv[1]
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f: continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "segments_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(d.rstrip("/")), " ".join(f"{k}={sum(v)/len(v):.3e}" for k, v in sorted(agg.items())))
