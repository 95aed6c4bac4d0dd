# bucket band split: window/bucket GPU tests, then window timing per split (bucket_split_log2), then kernel stats
set -o pipefail
mkdir -p gpurun_out/s
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "window or bucket" > gpurun_out/s/test.log 2>&1 || { tail -30 gpurun_out/s/test.log; exit 1; }
tail -1 gpurun_out/s/test.log
for k in ${SPLITS:-63 21 24 25 26 27 28}; do
  echo -n "split $k: "; timeout -k 10 120 python tools/window_bench.py bucket_split_log2=$k || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for k in ${PROF_SPLITS:-26}; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s/prof_$k -o run -- python tools/window_bench.py bucket_split_log2=$k > gpurun_out/s/prof_$k.log 2>&1 || exit 1
  echo "== split $k"; python3 tools/kstats.py $(find gpurun_out/s/prof_$k -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -14 || true
done
