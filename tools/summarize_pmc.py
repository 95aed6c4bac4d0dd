import csv, collections, glob, os, sys
root = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "segments_kernel"  # kernel-name substring; per kernel when not the wheel
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f: continue
    aggs = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f[0])):
        if pat in r["Kernel_Name"]:
            kn = r["Kernel_Name"].replace("(anonymous namespace)", "").split("(")[0].split("::")[-1]
            aggs[kn][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for kn, agg in sorted(aggs.items()):
        print(os.path.basename(d.rstrip("/")), kn, " ".join(f"{k}={sum(v)/len(v):.3e}" for k, v in sorted(agg.items())))
