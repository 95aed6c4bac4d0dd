# interleaved window timing of prod and variants (no tests, no profile)
set -o pipefail
for r in 1 2; do
  for v in prod "$@"; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    echo -n "$v: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py || exit 1
  done
done
