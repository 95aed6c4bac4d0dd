"""Print a rocprofv3 kernel_stats.csv compactly: short kernel name, calls, average us, total share."""
import csv, re, sys
for row in list(csv.DictReader(open(sys.argv[1])))[: int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    name = re.sub(r"\(.*", "", row["Name"].replace("dse::(anonymous namespace)::", ""))
    print(f"{name:32s} calls={row['Calls']:>4s} avg_us={float(row['AverageNs'])/1e3:9.1f} pct={float(row['Percentage']):6.2f}")
