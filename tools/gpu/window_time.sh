# interleaved window timing (count asserted) of variants: bash tools/gpu/window_time.sh name... (prod = production lib)
set -o pipefail
mkdir -p gpurun_out/w
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
  done
done
