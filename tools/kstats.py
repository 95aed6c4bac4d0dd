"""Print a rocprofv3 kernel_stats.csv as short name / calls / average ms (profiling aid)."""
import csv, sys
for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"].replace("(anonymous namespace)", "")
        short = n.split("(")[0].split("::")[-1] if "(" in n else n
        print(f"  {short:32s} calls={r['Calls']:>4s} avg_ms={float(r['AverageNs'])/1e6:8.3f} total_ms={float(r['TotalDurationNs'])/1e6:8.3f}")
