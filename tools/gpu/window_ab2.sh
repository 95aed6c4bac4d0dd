# window tests, then interleaved timing of prod and variants, then PMC of prod
set -o pipefail
mkdir -p gpurun_out/w
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "window or bucket" > gpurun_out/w/test.log 2>&1 || { tail -30 gpurun_out/w/test.log; exit 1; }
tail -1 gpurun_out/w/test.log
for r in 1 2; do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
  done
done
bash tools/gpu/window_prof.sh
