# Round evidence of the in-tree build: the GPU suite, the default bench line (CPU baseline included),
# the 1-rank RCCL bench line, the 1-GPU config sweep and every config's per-rank costs
# (rank_steps_all.sh, window included), rocprofv3 trace + PMC of the bench (tools/profile.sh),
# the extra PMC groups (pmc_deep.sh) and the window's line, kernel stats and PMC (window_evidence.sh).
#   TAG=r06 bash tools/gpu/evidence.sh        (outputs under gpurun_out/ev_$TAG)
set -o pipefail
TAG=${TAG:-r06}
O=gpurun_out/ev_$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
OUT=$O bash tools/gpu/rank_steps_all.sh || exit 1
timeout -k 10 300 python bench.py --rccl-single --cpu-baseline off > $O/bench_rccl_single.json 2> $O/bench_rccl.err || { tail -20 $O/bench_rccl.err; exit 1; }
timeout -k 10 600 bash tools/profile.sh $TAG || exit 1
OUT=$O/pmc_deep N=1e11 bash tools/gpu/pmc_deep.sh > /dev/null 2>&1 || exit 1
tail -22 $O/pmc_deep/summary.txt
OUT=$O/window bash tools/gpu/window_evidence.sh || exit 1
