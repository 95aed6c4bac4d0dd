#!/bin/bash
# Instruction-fetch counters of bench.py's wheel kernel (one small counter
# group per run, never with tracing):
#   OUT=gpurun_out/<dir> N=<n> [LIB=variants/libdse_x.so] bash tools/gpu/pmc_ifetch.sh
set -u
OUT=${OUT:-gpurun_out/ifetch}; N=${N:-1e11}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
[ -n "${LIB:-}" ] && export DSE_LIB=$LIB
ARGS="--steps 4 --warmup 1 --cpu-baseline off --n $N"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL ${TMO:-120} rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] && cp "$(find $OUT/$name -name '*counter_collection.csv' | head -1)" $OUT/$name.csv
  return $rc
}
run pmc_if --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE || exit 1
run pmc_ic1 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES || exit 1
run pmc_ic2 --pmc SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_REQ || exit 1
run pmc_ic3 --pmc SQC_ICACHE_INPUT_VALID_READYB SQC_TC_INST_REQ || exit 1
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
