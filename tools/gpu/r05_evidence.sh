# Round-5 evidence of the in-tree build: GPU tests, the default bench line (CPU baseline included),
# the 1-rank RCCL bench line, rocprofv3 trace + PMC of the bench (tools/profile.sh), the extra PMC
# groups (tools/gpu/pmc_deep.sh), per-chunk costs + the 1-GPU config sweep, window kernel stats.
set -o pipefail
O=gpurun_out/ev5
mkdir -p $O
# (GPU suite: profiles/r05/gputest_merged.log)

timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json; j=json.load(open('$O/bench.json')); print('bench', j['ms_per_step'], j['value'], j['verified'], j['roofline']['kernel_ms'], j['cpu_baseline']['value'])"
timeout -k 10 300 python bench.py --rccl-single --cpu-baseline off > $O/bench_rccl_single.json 2> $O/bench_rccl.err || { tail -20 $O/bench_rccl.err; exit 1; }
timeout -k 10 600 bash tools/profile.sh r05 || exit 1
OUT=gpurun_out/pmc_deep5 N=1e11 bash tools/gpu/pmc_deep.sh > /dev/null 2>&1 || exit 1
tail -22 gpurun_out/pmc_deep5/summary.txt
OUT=gpurun_out/rank_steps5 bash tools/gpu/rank_steps_all.sh || exit 1
bash tools/gpu/window_kstats.sh || exit 1
