set -o pipefail
mkdir -p gpurun_out/w
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window or bucket" > gpurun_out/w/test.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/w/test.log; exit 1; }
tail -2 gpurun_out/w/test.log
for r in 1 2; do
  timeout -k 10 120 python tools/window_bench.py && DSE_LIB=variants/libdse_onelevel.so timeout -k 10 120 python tools/window_bench.py || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/w/prof -o run -- python tools/window_bench.py > gpurun_out/w/prof.log 2>&1 || exit 1
find gpurun_out/w/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-5 | head -14
