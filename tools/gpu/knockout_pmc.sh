#!/bin/bash
# One PMC pass of bench.py at N per knockout build (tools/instrument_knockout.py,
# variants/libdse_ko<mask>.so), then the per-class table (tools/knockout_table.py):
#   OUT=gpurun_out/ko N=1e11 bash tools/gpu/knockout_pmc.sh 0 1 2 4 8 16 32 15 63
set -u
OUT=${OUT:-gpurun_out/ko}; N=${N:-1e11}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for m in "$@"; do
  mkdir -p $OUT/ko$m
  DSE_LIB=variants/libdse_ko$m.so timeout -s KILL ${TMO:-120} rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU \
    SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    -d $OUT/ko$m/raw -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --n $N \
    > $OUT/ko$m/run.log 2>&1
  rc=$?
  echo "[ko$m] rc=$rc"
  [ $rc -eq 0 ] || exit 1
  cp "$(find $OUT/ko$m/raw -name '*counter_collection.csv' | head -1)" $OUT/ko$m/pmc_a.csv || exit 1
done
python3 tools/knockout_table.py $OUT "$@" | tee $OUT/table.txt
