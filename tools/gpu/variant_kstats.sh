# window tests on prod, then per library (prod + variants): window timing and rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out/v
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "window or bucket" > gpurun_out/v/test.log 2>&1 || { tail -30 gpurun_out/v/test.log; exit 1; }
tail -1 gpurun_out/v/test.log
for v in prod "$@"; do
  if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
  echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in prod "$@"; do
  if [ "$v" = prod ]; then unset DSE_LIB; else export DSE_LIB=variants/libdse_$v.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/v/prof_$v -o run -- python tools/window_bench.py > gpurun_out/v/prof_$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/kstats.py $(find gpurun_out/v/prof_$v -name "*kernel_stats.csv" | head -1) | grep bucket
done
