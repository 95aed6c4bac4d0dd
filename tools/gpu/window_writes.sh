# HBM write/fetch PMC of the window's bucket kernels (one counter per run, no tracing)
set -u
OUT=gpurun_out/wwrite
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d $OUT/$c -o $c --output-format csv -- python3 tools/window_bench.py > $OUT/$c.log 2>&1
  rc=$?; echo "[$c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    f = glob.glob(f"gpurun_out/wwrite/{c}/**/*counter_collection.csv", recursive=True)[0]
    tot = collections.defaultdict(float); disp = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("dse::(anonymous namespace)::", "").split("(")[0]
        tot[k] += float(r["Counter_Value"]); disp[k].add(r["Dispatch_Id"])
    for k in sorted(tot, key=lambda k: -tot[k])[:8]:
        print(f"{c} {k:40s} dispatches={len(disp[k]):3d} GB/dispatch={tot[k]*1024/len(disp[k])/1e9:7.3f}")
PY
