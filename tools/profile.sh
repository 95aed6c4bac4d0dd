#!/bin/bash
# Profile bench.py on the GPU box: kernel trace + stats, then PMC passes
# (one block-limited counter group per run, never combined with tracing).
# Summaries land in gpurun_out/prof_<tag>/summary/ with fixed names:
#   rocprofv3_kernel_stats.csv, pmc_{sq,wait,fetch,write}_sieve_kernel.csv
# Usage (via gpurun): bash tools/profile.sh <tag> [bench args...]
set -u
TAG=${1:-r01}; shift || true
ARGS=${*:---steps 5 --warmup 2 --cpu-baseline off}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT/summary
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 180 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  return $rc
}
run trace --kernel-trace --stats || exit 1
cp "$(find $OUT/trace -name '*kernel_stats.csv' | head -1)" $OUT/summary/rocprofv3_kernel_stats.csv
run pmc_sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run pmc_wait --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE || exit 1
for n in sq wait fetch write; do
  cp "$(find $OUT/pmc_$n -name '*counter_collection.csv' | head -1)" $OUT/summary/pmc_${n}_sieve_kernel.csv
done
grep -h "^{\"metric\"" $OUT/trace.log | tail -1 > $OUT/summary/bench_under_trace.json
echo done
