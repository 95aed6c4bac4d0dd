# bucket/window GPU tests, then an interleaved window A/B of prod and variants: window_check.sh name ...
set -o pipefail
mkdir -p gpurun_out/wc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "window or bucket or kb_float or scratch" > gpurun_out/wc/gputest.log 2>&1 || { tail -40 gpurun_out/wc/gputest.log; exit 1; }
tail -1 gpurun_out/wc/gputest.log
for r in 1 2 3; do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
  done
done
