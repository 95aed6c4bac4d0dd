#!/bin/bash
# Kernel trace + PMC passes of bench.py (one counter group per run, never with tracing):
#   OUT=gpurun_out/<dir> N=<n> [LIB=variants/libdse_x.so] bash tools/gpu/pmc_deep.sh
set -u
OUT=${OUT:-gpurun_out/pmc}; N=${N:-1e11}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
[ -n "${LIB:-}" ] && export DSE_LIB=$LIB
ARGS="--steps 4 --warmup 1 --cpu-baseline off --n $N"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -s KILL ${TMO:-150} rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 bench.py $ARGS \
    > $OUT/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  [ $rc -eq 0 ] && cp "$(find $OUT/$name -name '*counter_collection.csv' -o -name '*kernel_stats.csv' | head -1)" $OUT/$name.csv
  return $rc
}
run trace --kernel-trace --stats || exit 1
run pmc_a --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE || exit 1
run pmc_b --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE || exit 1
run pmc_c --pmc SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_IFETCH SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT || exit 1
run pmc_fetch --pmc FETCH_SIZE || exit 1
run pmc_write --pmc WRITE_SIZE || exit 1
python3 tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
