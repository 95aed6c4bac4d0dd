#!/bin/bash
# PMC counters per ablation variant (DSE_PHASES); one counter group per run.
set -u
OUT=gpurun_out/prof_phases
mkdir -p $OUT
export TMPDIR=/tmp
export DSE_LIB=${DSE_LIB:-variants/libdse_knob.so}  # knob build: tools/build_variant.sh knob -DDSE_PHASE_KNOB
for v in ${VARIANTS:-127 121 122 124 120}; do
  for grp in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
             "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"; do
    name=v${v}_$(echo $grp | cut -c1-12 | tr ' ' '_')
    DSE_PHASES=$v timeout -k 10 120 rocprofv3 --pmc $grp -d $OUT/$name -o $name --output-format csv -- \
      python3 bench.py --steps 3 --warmup 1 --cpu-baseline off > $OUT/$name.log 2>&1 || { echo "fail $name"; exit 1; }
  done
done
echo done
