# Round-4 evidence of the in-tree build: rocprofv3 trace + PMC of the default bench (tools/profile.sh),
# the extra PMC pass groups (tools/gpu/pmc_deep.sh), per-chunk costs of the multi-chunk configs.
set -o pipefail
timeout -k 10 600 bash tools/profile.sh r04 || exit 1
OUT=gpurun_out/pmc_deep N=1e11 bash tools/gpu/pmc_deep.sh > /dev/null 2>&1 || exit 1
tail -30 gpurun_out/pmc_deep/summary.txt
OUT=gpurun_out/rank_steps bash tools/gpu/rank_steps_all.sh || exit 1
