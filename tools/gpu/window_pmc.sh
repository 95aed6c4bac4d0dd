# PMC passes of the window (tools/window_bench.py) for prod and variants: bash tools/gpu/window_pmc.sh TAG name...
set -u
TAG=$1; shift
OUT=gpurun_out/wpmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
P1="SQ_LDS_ADDR_CONFLICT SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
P4="FETCH_SIZE GRBM_GUI_ACTIVE"
for name in "$@"; do
  if [ "$name" = prod ]; then LIB=$PWD/distributed-sieve-e_amd/mail_sieve_e/libdse.so; else LIB=$PWD/variants/libdse_$name.so; fi
  for p in 1 2 3 4; do
    eval CNT=\$P$p
    DSE_LIB=$LIB timeout -s KILL 90 rocprofv3 --pmc $CNT -d $OUT/${name}_p$p -o ${name}_p$p --output-format csv \
      -- python3 tools/window_bench.py > $OUT/${name}_p$p.log 2>&1
    rc=$?
    echo "[$name p$p] rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
python3 tools/summarize_pmc.py $OUT bucket_ > $OUT/summary.txt
cat $OUT/summary.txt
