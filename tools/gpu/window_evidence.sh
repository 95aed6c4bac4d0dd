#!/bin/bash
# Window (BASELINE config 5) evidence of the in-tree library: the bench.py --window line, its
# rocprofv3 kernel stats, one PMC pass each of FETCH_SIZE and WRITE_SIZE (no tracing), and the
# per-slice costs of an 8-GPU run on one GPU (tools/rank_steps.py window 8): OUT=gpurun_out/<dir>
set -o pipefail
OUT=${OUT:-gpurun_out/window_ev}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --window --steps 10 --warmup 3 > $OUT/bench_window.json 2> $OUT/bench_window.err || { tail -20 $OUT/bench_window.err; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/bench_window.json')); r=j['roofline']; print('window', j['ms_per_step'], j['verified'], r['kernel_ms'], r['frac'])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kstats -o run -- python3 bench.py --window --steps 5 --warmup 2 > $OUT/kstats.log 2>&1 || { tail -20 $OUT/kstats.log; exit 1; }
cp "$(find $OUT/kstats -name '*kernel_stats.csv' | head -1)" $OUT/window_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c -d $OUT/pmc_$c -o pmc --output-format csv -- python3 bench.py --window --steps 5 --warmup 2 > $OUT/pmc_$c.log 2>&1
  rc=$?; echo "[$c] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
cp "$(find $OUT/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)" $OUT/pmc_window_fetch.csv
cp "$(find $OUT/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)" $OUT/pmc_window_write.csv
timeout -k 10 240 python tools/rank_steps.py window 8 > $OUT/rank_steps_window.txt 2>&1 || { tail -20 $OUT/rank_steps_window.txt; exit 1; }
tail -3 $OUT/rank_steps_window.txt
