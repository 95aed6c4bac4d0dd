# interleaved window timing of prod and variants, x3 (window_bench checks the count)
set -o pipefail
for r in 1 2 3; do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
  done
done
