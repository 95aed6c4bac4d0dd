#!/bin/bash
# Per-phase PMC of the wheel kernel (profiling only): one rocprofv3 --pmc pass
# per phase variant of a -DDSE_PHASE_KNOB build (variants/libdse_knob.so,
# built beforehand on the CPU by tools/build_variant.sh knob -DDSE_PHASE_KNOB).
# Differences between variants attribute LDS cycles, bank conflicts and VALU
# to the A / B / L units. Usage (via gpurun): bash tools/phase_pmc.sh <tag> [N]
set -u
TAG=${1:-phase}; N=${2:-1e11}
OUT=gpurun_out/phase_pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
LIB=${DSE_LIB:-$PWD/variants/libdse_knob.so}
SQ="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
for v in all:127 skel:120 A:121 B:122 L:124 init_expand:40; do
  name=${v%%:*}; ph=${v##*:}
  DSE_LIB=$LIB DSE_PHASES=$ph timeout -s KILL 90 rocprofv3 --pmc $SQ -d $OUT/$name -o $name --output-format csv \
    -- python3 bench.py --steps 3 --warmup 1 --cpu-baseline off --n $N > $OUT/$name.log 2>&1
  rc=$?
  echo "[$name phases=$ph] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/summarize_pmc.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
