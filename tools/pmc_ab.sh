#!/bin/bash
# PMC A/B of library builds on the GPU box: pmc_ab.sh TAG LIB... (one counter pass per lib)
# -> gpurun_out/pmcab_TAG/<libname>/ ; summarize with tools/summarize_pmc.py gpurun_out/pmcab_TAG
set -u
TAG=$1; shift
OUT=gpurun_out/pmcab_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for L in "$@"; do
  n=$(basename $L .so)
  DSE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES \
    -d $OUT/$n -o $n --output-format csv -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $OUT/$n.log 2>&1 || exit 1
  echo "[$n] ok"
done
