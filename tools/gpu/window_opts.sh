# window GPU tests, then interleaved timing of option sets ("a=1,b=2" each; "-" = defaults)
set -o pipefail
mkdir -p gpurun_out/w
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window or bucket" > gpurun_out/w/test.log 2>&1 || { tail -30 gpurun_out/w/test.log; exit 1; }
tail -1 gpurun_out/w/test.log
for r in 1 2; do
  for o in "$@"; do
    if [ "$o" = "-" ]; then A=""; else A=${o//,/ }; fi
    timeout -k 10 120 python tools/window_bench.py $A || exit 1
  done
done
