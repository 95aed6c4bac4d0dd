# window: band split x fill variants (runtime split option), interleaved x2
set -o pipefail
for r in 1 2; do
  for v in ${VARS:-prod rg16}; do
    if [ "$v" = prod ]; then L=""; else L=variants/libdse_$v.so; fi
    for k in ${SPLITS:-26 27 28}; do
      echo -n "$v split $k: "; DSE_LIB=$L timeout -k 10 120 python tools/window_bench.py bucket_split_log2=$k || exit 1
    done
  done
done
