# Round-5 evidence of the final build: GPU suite, bench line (CPU baseline included), 1-rank RCCL line,
# config sweep, rank steps, rocprofv3 trace + PMC of the bench, extra PMC groups, window kernel stats,
# A/B against the round-start build.
set -o pipefail
O=gpurun_out/ev5f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputest.log 2>&1 || { tail -30 $O/gputest.log; exit 1; }
tail -1 $O/gputest.log
OUT=$O bash tools/gpu/rank_steps_all.sh || exit 1
timeout -k 10 300 python bench.py --rccl-single --cpu-baseline off > $O/bench_rccl_single.json 2> $O/bench_rccl.err || { tail -20 $O/bench_rccl.err; exit 1; }
timeout -k 10 600 bash tools/profile.sh r05 || exit 1
OUT=gpurun_out/pmc_deep5 N=1e11 bash tools/gpu/pmc_deep.sh > /dev/null 2>&1 || exit 1
tail -22 gpurun_out/pmc_deep5/summary.txt
bash tools/gpu/window_kstats.sh || exit 1
for n in 1e11 1e12; do
  OUT=$O N=$n ROUNDS=2 TMO=500 bash tools/gpu/ab.sh prod r04 > /dev/null || exit 1
done
cat $O/ab_*.txt
