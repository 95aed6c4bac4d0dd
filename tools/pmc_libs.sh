#!/bin/bash
# PMC passes of bench.py (N=1e11) for several library builds (profiling aid):
# bash tools/pmc_libs.sh <tag> <lib-name>... ; libs are variants/libdse_<name>.so
# ("prod" = the production library). Counter sets are fixed below, one
# rocprofv3 --pmc pass each.
set -u
TAG=$1; shift
OUT=gpurun_out/pmc_libs_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_LDS_MEM_VIOLATIONS SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES_SAVED SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE"
for name in "$@"; do
  if [ "$name" = prod ]; then LIB=$PWD/distributed-sieve-e_amd/mail_sieve_e/libdse.so; else LIB=$PWD/variants/libdse_$name.so; fi
  for p in 1 2; do
    eval CNT=\$P$p
    DSE_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $CNT -d $OUT/${name}_p$p -o ${name}_p$p --output-format csv \
      -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $OUT/${name}_p$p.log 2>&1
    rc=$?
    echo "[$name p$p] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/summarize_pmc.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
