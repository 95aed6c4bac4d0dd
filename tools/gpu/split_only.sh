# window timing per bucket band split (bucket_split_log2), interleaved x2, no tests
set -o pipefail
for r in 1 2; do
  for k in ${SPLITS:-24 25 26 27 28}; do
    echo -n "split $k: "; timeout -k 10 120 python tools/window_bench.py bucket_split_log2=$k || exit 1
  done
done
