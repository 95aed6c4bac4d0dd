set -o pipefail
bash tools/gpu/window_kstats.sh wk1 wk2 wk3 wk4 wk5 > gpurun_out/wk/summary.txt 2>&1 || { tail -30 gpurun_out/wk/summary.txt; exit 1; }
cat gpurun_out/wk/summary.txt
bash tools/gpu/window_pmc.sh r06 prod > /dev/null 2>&1 || exit 1
grep fill_stage gpurun_out/wpmc_r06/summary.txt
