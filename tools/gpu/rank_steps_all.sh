#!/bin/bash
# Per-chunk costs of every multi-chunk BASELINE config on one GPU (tools/rank_steps.py),
# plus the default bench line and the 1-GPU config sweep: OUT=gpurun_out/<dir>
set -o pipefail
OUT=${OUT:-gpurun_out/rank_steps}
mkdir -p $OUT
timeout -k 10 180 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$OUT/bench.json')); print('bench', j['ms_per_step'], j['value'], j['verified'], j['roofline']['kernel_ms'])"
timeout -k 10 300 python tools/config_sweep.py $OUT/configs_1gpu.json > $OUT/configs.log 2>&1 || { tail -20 $OUT/configs.log; exit 1; }
tail -12 $OUT/configs.log
for np in "1e10 2" "1e10 4" "1e10 8" "1e11 2" "1e11 4" "1e11 8" "1e12 8"; do
  timeout -k 10 240 python tools/rank_steps.py $np >> $OUT/rank_steps.txt 2>&1 || { tail -20 $OUT/rank_steps.txt; exit 1; }
done
timeout -k 10 240 python tools/rank_steps.py window 8 >> $OUT/rank_steps.txt 2>&1 || { tail -20 $OUT/rank_steps.txt; exit 1; }
grep -E "critical|^N=|^window" $OUT/rank_steps.txt
